"""Backward host launcher: same contract as /root/reference/src/backward/caller.py:14-178.

`_flash_attn_backward(dO, q, k, v, bias, attention_mask, o, lse, dropout_p, causal,
softmax_scale, dropout_seed) -> (dq, dk, dv)`.  The reference's three steps -- Triton
_compute_delta (:95-114), Triton _bwd_kernel (:122-160) and the host GQA sum of dK/dV over
the q-heads of each group (:162-165) -- become one call of the C ABI `fa2_bwd`, which runs
delta, dK/dV (fp32 group sum in registers) and dQ kernels on the current stream.  dQ is
produced in q.dtype directly (the reference accumulates a fp32 buffer that autograd then casts,
:86); dK/dV come out with Hkv heads.  Varlen rows are handled in place (no trim / pack /
unpack, :29-79, :167-176).
"""
import ctypes
import math
import os
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from .utils import bshd_strides, cu_seqlens_from_mask, encode_dtype, handle_dropout, infer_bias_strides, stream_of


def _fill_args(args, q: Tensor, k: Tensor, v: Tensor, o: Tensor, dO: Tensor, causal: bool) -> None:
    """The fields of fa2_bwd_args that the dS-workspace query reads: pointers, strides, sizes."""
    batch, seqlen_q, nheads_q, head_dim = q.shape
    _, seqlen_k, nheads_kv, _ = k.shape
    args.q, args.k, args.v, args.o, args.dout = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dO.data_ptr()
    args.q_stride[:] = bshd_strides(q)
    args.k_stride[:] = bshd_strides(k)
    args.v_stride[:] = bshd_strides(v)
    args.o_stride[:] = bshd_strides(o)
    args.do_stride[:] = bshd_strides(dO)
    args.batch, args.heads_q, args.heads_kv = batch, nheads_q, nheads_kv
    args.seqlen_q, args.seqlen_k, args.head_dim = seqlen_q, seqlen_k, head_dim
    args.causal = int(bool(causal))


def ds_workspace_bytes(q: Tensor, k: Tensor, v: Tensor, o: Tensor, dO: Tensor, causal: bool) -> int:
    """Bytes of the dS workspace (`fa2_bwd_ds_workspace_bytes`): one 2 KiB tile of rounded dS per
    (batch, q-head, 32-query tile, 32-key tile) with a visible pair (causal: about half the
    grid); 0 where the path does not apply (head_dim not a multiple of 8, <= 64 or > 128, or
    tensors without the 16-byte vector layout: the recompute dQ kernel is used instead)."""
    args = _lib.BwdArgs()
    _fill_args(args, q, k, v, o, dO, causal)
    return int(_lib.load().fa2_bwd_ds_workspace_bytes(ctypes.byref(args)))


def _ds_workspace_cap(device: torch.device) -> int:
    """Largest dS workspace the backward allocates by itself.  The dS path is opt-in: with the
    software-pipelined dK/dV kernel the recompute path is as fast or faster (cfg3 causal bwd
    3.73 vs 3.85 ms, non-causal 6.51 vs 6.49 ms, profiles/r02_ab_bwd_paths.txt) and needs O(S)
    memory, as the reference's backward.  FA2_DS_WORKSPACE_MAX_GB=<GB> enables it under that cap
    (0 disables), =auto under half of the memory available right now (free device memory plus
    what torch's caching allocator holds unused)."""
    env = os.environ.get("FA2_DS_WORKSPACE_MAX_GB")
    if env is None:
        return 0
    if env.strip().lower() != "auto":
        return int(float(env) * (1 << 30))
    free, _ = torch.cuda.mem_get_info(device)
    cached = torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
    return (free + max(cached, 0)) // 2


def alloc_ds_workspace(q: Tensor, k: Tensor, v: Tensor, o: Tensor, dO: Tensor, causal: bool) -> Optional[Tensor]:
    """The dS workspace for a backward of these tensors, or None when the dS path does not
    apply, would exceed the cap, or cannot be allocated: the backward then recomputes S and dP
    in its dQ kernel (O(S) memory, as the reference's backward)."""
    nbytes = ds_workspace_bytes(q, k, v, o, dO, causal)
    if nbytes == 0 or nbytes > _ds_workspace_cap(q.device):
        return None
    try:
        return torch.empty(nbytes, dtype=torch.uint8, device=q.device)
    except torch.OutOfMemoryError:
        return None


def alloc_dkv_workspace(args, device: torch.device) -> Optional[Tensor]:
    """fp32 partial-sum workspace of the dK/dV q-head split (`fa2_bwd_dkv_workspace_bytes`), or
    None when no split applies (Hq == Hkv, or B * Hkv * ceil(Sk / 128) already fills the GPU) or
    it cannot be allocated (the backward then sums each GQA group in one workgroup).  Small by
    construction: it only exists when the key-block grid is small."""
    nbytes = int(_lib.load().fa2_bwd_dkv_workspace_bytes(ctypes.byref(args)))
    if nbytes == 0 or os.environ.get("FA2_DKV_SPLIT", "1") == "0":
        return None
    try:
        return torch.empty(nbytes, dtype=torch.uint8, device=device)
    except torch.OutOfMemoryError:
        return None


def _flash_attn_backward(
    dO: Tensor,
    q: Tensor,
    k: Tensor,
    v: Tensor,
    bias: Optional[Tensor],
    attention_mask: Optional[Tensor],
    o: Tensor,
    lse: Tensor,
    dropout_p: float,
    causal: bool,
    softmax_scale: Optional[float],
    dropout_seed: Optional[int],
    dq_dtype: Optional[torch.dtype] = None,
    _stages: Optional[int] = None,
    _delta: Optional[Tensor] = None,
    _ds_ws: Optional[Tensor] = None,
    _use_ds: Optional[bool] = None,
    bias_grad: bool = False,
):
    """Returns (dq, dk, dv) -- the reference's contract -- or (dq, dk, dv, dbias) with
    `bias_grad=True`: dbias = dL/d(bias) in bias's shape and dtype, the fp32 dS the dK/dV kernel
    writes per (batch, q-head) summed over the bias's broadcast dims (deterministic).  The
    reference has no bias gradient (/root/reference/src/wrapper.py:86 returns None)."""
    if attention_mask is not None:
        assert bias is None, "Attention mask is not supported along with attention bias. Just use bias instead."
        assert q.size(1) == k.size(1), "Attention mask is not supported with seqlen_q != seqlen_k"
    dO = dO if dO.stride(-1) == 1 else dO.contiguous()
    batch, seqlen_q, nheads_q, head_dim = q.shape
    _, seqlen_k, nheads_kv, _ = k.shape
    lse_rows = math.ceil(seqlen_q / 128) * 128
    softmax_scale = 1.0 / math.sqrt(head_dim) if softmax_scale is None else softmax_scale
    assert nheads_q % nheads_kv == 0, f"{nheads_q = } is not divisible by {nheads_kv = }"
    assert lse.shape == (batch, nheads_q, lse_rows) and lse.is_contiguous()
    assert q.stride(-1) == k.stride(-1) == v.stride(-1) == o.stride(-1) == 1
    assert dO.dtype == q.dtype == k.dtype == v.dtype == o.dtype

    stride_bb, stride_bh, stride_bm = infer_bias_strides(bias, batch, nheads_q, seqlen_q, seqlen_k)
    dropout_seed = handle_dropout(dropout_p, dropout_seed, is_forward=False)
    cu_seqlens = cu_seqlens_from_mask(attention_mask) if attention_mask is not None else None

    dq_dtype = q.dtype if dq_dtype is None else dq_dtype
    dq = torch.empty(q.shape, dtype=dq_dtype, device=q.device)
    dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
    dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
    delta = torch.empty_like(lse) if _delta is None else _delta  # workspace: rowsum(O * dO)

    args = _lib.BwdArgs()
    _fill_args(args, q, k, v, o, dO, causal)
    args.lse, args.delta = lse.data_ptr(), delta.data_ptr()
    args.dq, args.dk, args.dv = dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
    args.bias = bias.data_ptr() if bias is not None else None
    args.cu_seqlens = cu_seqlens.data_ptr() if cu_seqlens is not None else None
    args.dq_stride[:] = bshd_strides(dq)
    args.dk_stride[:] = bshd_strides(dk)
    args.dv_stride[:] = bshd_strides(dv)
    args.bias_stride[:] = (stride_bb, stride_bh, stride_bm)
    args.lse_row_stride = lse_rows
    dbias_full = None
    if bias_grad:
        assert bias is not None, "bias_grad needs a bias"
        # [B, Hq, Sq, Sk] fp32, zero where no (query, key) pair is visible
        dbias_full = torch.zeros(batch, nheads_q, seqlen_q, seqlen_k, dtype=torch.float32, device=q.device)
        args.dbias = dbias_full.data_ptr()
        args.dbias_stride[:] = dbias_full.stride()[:3]
    args.dtype = encode_dtype(q)
    args.bias_dtype = encode_dtype(bias) if bias is not None else 0
    args.dq_dtype = encode_dtype(dq)
    args.softmax_scale = float(softmax_scale)
    args.dropout_p = float(dropout_p)
    args.dropout_seed = int(dropout_seed) & 0xFFFFFFFFFFFFFFFF
    # dS workspace: dK/dV stores its rounded dS tiles and dQ = dS K streams them (one GEMM)
    # instead of recomputing S and dP; the caller may pass one (stage-by-stage timing)
    if _use_ds is False:
        ds_ws = None
    else:
        ds_ws = _ds_ws if _ds_ws is not None else alloc_ds_workspace(q, k, v, o, dO, causal)
    if ds_ws is not None:
        args.ds_workspace, args.ds_workspace_bytes = ds_ws.data_ptr(), ds_ws.numel() * ds_ws.element_size()
    dkv_ws = alloc_dkv_workspace(args, q.device)
    if dkv_ws is not None:
        args.dkv_workspace, args.dkv_workspace_bytes = dkv_ws.data_ptr(), dkv_ws.numel()
    stages = _stages if _stages is not None else (7 if ds_ws is not None else 6)
    lib = _lib.load()
    with torch.cuda.device(q.device):
        _lib.check(lib.fa2_bwd_stages(ctypes.byref(args), stages, stream_of(q)))
    if not bias_grad:
        return dq, dk, dv
    dims = [i for i in (0, 1) if bias.size(i) == 1]
    dbias = dbias_full.sum(dim=dims, keepdim=True) if dims else dbias_full
    return dq, dk, dv, dbias.to(bias.dtype)
