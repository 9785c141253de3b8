"""Host helpers of the reference (/root/reference/src/utils.py) that survive the move to HIP.

The device helper `load_fn` (:34-54) folds into the kernels' tile loads; the host varlen
pack/unpack loops (:8-31) are replaced by in-place padded-tensor handling in the kernels plus
`cu_seqlens_from_mask` (device-side, no .item() synchronisation).
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib


def infer_bias_strides(
    bias: Optional[Tensor], batch: int, nheads_q: int, seqlen_q: int, seqlen_k: int
) -> Tuple[int, int, int]:
    """Broadcast strides (batch, head, row) of an additive bias [1|B, 1|Hq, Sq, Sk].

    Same contract as /root/reference/src/utils.py:57-77, except that a per-head bias
    [., Hq, ., .] is accepted (the reference compares stride(1) with nheads_q at :70, which
    rejects it) and is indexed by the query head in forward and backward alike (the reference
    uses the kv head in forward, src/forward/kernel.py:141, and the q head in backward,
    src/backward/kernel.py:143).
    """
    if bias is None:
        return 0, 0, 0
    assert bias.dim() == 4 and bias.size(2) == seqlen_q and bias.size(3) == seqlen_k, f"{bias.shape = }"
    if bias.size(0) == 1:
        stride_bb = 0
    elif bias.size(0) == batch:
        stride_bb = bias.stride(0)
    else:
        raise ValueError(f"Attention bias has {bias.size(0) = } while {batch = }")
    if bias.size(1) == 1:
        stride_bh = 0
    elif bias.size(1) == nheads_q:
        stride_bh = bias.stride(1)
    else:
        raise ValueError(f"Attention bias has {bias.size(1) = } while {nheads_q = }")
    if bias.stride(3) != 1:
        raise ValueError("Attention bias must have a contiguous last dimension")
    return stride_bb, stride_bh, bias.stride(2)


def dropout_mask_words(batch: int, heads_q: int, seqlen_q: int, seqlen_k: int) -> int:
    """int32 words of a dropout keep mask (fa2_dropout_mask_bytes / 4 in include/fa2_amd.h):
    32 x 32 bit tiles, batch * heads_q * ceil(Sq / 32) * ceil(Sk / 32) * 32 words, plus one tile of
    slack (ABI 8: the hand-placed dK/dV reads two key tiles as one run)."""
    return batch * heads_q * ((seqlen_q + 31) // 32) * ((seqlen_k + 31) // 32) * 32 + 32


def check_dropout_mask(mask: torch.Tensor, batch: int, heads_q: int, seqlen_q: int, seqlen_k: int, device) -> None:
    need = dropout_mask_words(batch, heads_q, seqlen_q, seqlen_k)
    assert mask.dtype == torch.int32 and mask.is_contiguous() and mask.device == device, \
        "dropout_mask must be a contiguous int32 tensor on the inputs' device"
    assert mask.numel() >= need, f"dropout_mask has {mask.numel()} words, {need} needed"


def handle_dropout(dropout_p: float, dropout_seed: Optional[int], is_forward: bool) -> int:
    """Seed handling of /root/reference/src/utils.py:80-88.

    The reference raises NotImplementedError for a backward with dropout (:88); here the
    backward kernels regenerate the forward's Philox keep mask,
    so the backward only needs the seed the forward used.
    """
    assert dropout_p >= 0, f"Dropout probability {dropout_p = } must be above 0."
    assert dropout_p < 1, f"Dropout probability {dropout_p = } must be strictly below 1."
    if dropout_p == 0:
        return 0
    if is_forward:
        return torch.randint(low=0, high=2**32, size=(1,)).item() if dropout_seed is None else dropout_seed
    if dropout_seed is None:
        raise ValueError("a backward with dropout needs the dropout_seed its forward used")
    return dropout_seed


def encode_dtype(x: Tensor) -> int:
    """dtype code, /root/reference/src/utils.py:102-109 (also the C ABI's fa2_dtype)."""
    if x.dtype == torch.float16:
        return _lib.FA2_F16
    if x.dtype == torch.bfloat16:
        return _lib.FA2_BF16
    if x.dtype == torch.float32:
        return _lib.FA2_F32
    raise ValueError(x.dtype)


def bshd_strides(x: Tensor) -> Tuple[int, int, int]:
    """(batch, seq, head) element strides of a [B, S, H, D] view with unit last stride (one
    stride() call: each costs ~0.4 us of host time, and a launch makes four of these)."""
    s = x.stride()
    assert s[-1] == 1, "last dimension must be contiguous"
    return s[0], s[1], s[2]


def stream_of(x: Tensor) -> int:
    return torch._C._cuda_getCurrentRawStream(x.device.index)


def launch_on(x: Tensor, call):
    """call(stream) on x's device and current stream.  The device switch is made only when x is
    not on the current device: the context manager and the Stream object cost a few microseconds
    per call, which is ~10 % of cfg2's 46 us forward when launches are back to back."""
    idx = x.device.index
    if idx == torch.cuda.current_device():
        return call(torch._C._cuda_getCurrentRawStream(idx))
    with torch.cuda.device(idx):
        return call(torch._C._cuda_getCurrentRawStream(idx))


def cu_seqlens_from_mask(attention_mask: Tensor) -> Tensor:
    """[B+1] int32 cumulative valid lengths of a right-padded [B, S] mask, computed on device."""
    mask = attention_mask
    if mask.dtype != torch.bool:
        mask = mask != 0
    mask = mask.contiguous()
    batch, seqlen = mask.shape
    cu = torch.empty(batch + 1, dtype=torch.int32, device=mask.device)
    lib = _lib.load()
    _lib.check(lib.fa2_cu_seqlens_from_mask(mask.data_ptr(), mask.stride(0), batch, seqlen, cu.data_ptr(),
                                            stream_of(mask)))
    return cu
