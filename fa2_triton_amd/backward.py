"""Backward host launcher: same contract as /root/reference/src/backward/caller.py:14-178.

`_flash_attn_backward(dO, q, k, v, bias, attention_mask, o, lse, dropout_p, causal,
softmax_scale, dropout_seed) -> (dq, dk, dv)`.  The reference's three steps -- Triton
_compute_delta (:95-114), Triton _bwd_kernel (:122-160) and the host GQA sum of dK/dV over
the q-heads of each group (:162-165) -- become one call of the C ABI `fa2_bwd`, which runs
the dQ kernel (which also computes delta) and the dK/dV kernel (fp32 group sum in registers)
on the current stream.  dQ is
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
from .utils import (bshd_strides, check_dropout_mask, cu_seqlens_from_mask, encode_dtype, handle_dropout,
                    infer_bias_strides, launch_on)


def _fill_args(args, q: Tensor, k: Tensor, v: Tensor, o: Tensor, dO: Tensor, causal: bool) -> None:
    """Pointers, strides and sizes of fa2_bwd_args."""
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
    bias_grad: bool = False,
    dropout_mask: Optional[Tensor] = None,
):
    """Returns (dq, dk, dv) -- the reference's contract -- or (dq, dk, dv, dbias) with
    `bias_grad=True`: dbias = dL/d(bias) in bias's shape and dtype.  The library's bias-gradient
    kernel sums dS = P (dP - delta) over the bias's broadcast dims in a fixed order into a fp32
    buffer of the bias's shape (deterministic; no [B, Hq, Sq, Sk] intermediate).  The reference
    has no bias gradient (/root/reference/src/wrapper.py:86 returns None)."""
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

    if bias_grad and bias is not None:
        bias = bias.contiguous()  # a zero stride then means a size-1 (broadcast, summed) dim
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
    dbias32 = None
    if bias_grad:
        assert bias is not None, "bias_grad needs a bias"
        # the bias's shape: dims the bias broadcasts over (stride 0) are summed by the kernel
        dbias32 = torch.empty(batch if stride_bb else 1, nheads_q if stride_bh else 1, seqlen_q, seqlen_k,
                              dtype=torch.float32, device=q.device)
        args.dbias = dbias32.data_ptr()
        args.dbias_stride[:] = dbias32.stride()[:3]
    args.dtype = encode_dtype(q)
    args.bias_dtype = encode_dtype(bias) if bias is not None else 0
    args.dq_dtype = encode_dtype(dq)
    args.softmax_scale = float(softmax_scale)
    args.dropout_p = float(dropout_p)
    args.dropout_seed = int(dropout_seed) & 0xFFFFFFFFFFFFFFFF
    if dropout_mask is not None and dropout_p > 0.0:  # the forward's keep bits, read instead of redrawn
        check_dropout_mask(dropout_mask, batch, nheads_q, seqlen_q, seqlen_k, q.device)
        args.dropout_mask = dropout_mask.data_ptr()
    dkv_ws = alloc_dkv_workspace(args, q.device)
    if dkv_ws is not None:
        args.dkv_workspace, args.dkv_workspace_bytes = dkv_ws.data_ptr(), dkv_ws.numel()
    stages = _stages if _stages is not None else (14 if bias_grad else 6)
    _lib.check(launch_on(q, lambda st: _lib.bwd_stages(args, stages, st)))
    if not bias_grad:
        return dq, dk, dv
    return dq, dk, dv, dbias32.view(bias.shape).to(bias.dtype)
