"""Forward host launcher: same contract as /root/reference/src/forward/caller.py:12-122.

`_flash_attn_forward(q, k, v, attention_mask, bias, dropout_p, causal, softmax_scale,
dropout_seed) -> (o, lse, softmax_scale, dropout_seed)`; q [B, Sq, Hq, D], k/v [B, Sk, Hkv, D],
lse [B, Hq, ceil(Sq/128)*128] fp32 in base-2 units.  The Triton launch (:83-116) becomes one
call of the C ABI `fa2_fwd`; the varlen pack/unpack (:44-63, :118-120) disappears because the
HIP kernel reads the padded tensors in place using device-side cu_seqlens.  Keyword-only
`dropout_mask` (beyond the reference): an int32 buffer of dropout_mask_words(...) words that the
forward fills with the keep bits it drew, for the backward to read instead of regenerating them.
"""
import math
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from .utils import (bshd_strides, check_dropout_mask, cu_seqlens_from_mask, encode_dtype, handle_dropout,
                    infer_bias_strides, launch_on)


def _flash_attn_forward(
    q: Tensor,
    k: Tensor,
    v: Tensor,
    attention_mask: Optional[Tensor],
    bias: Optional[Tensor],
    dropout_p: float = 0.0,
    causal: bool = False,
    softmax_scale: Optional[float] = None,
    dropout_seed: Optional[int] = None,
    *,
    dropout_mask: Optional[Tensor] = None,
) -> Tuple[Tensor, Tensor, float, int]:
    if attention_mask is not None:
        assert bias is None, "Attention mask is not supported along with attention bias. Just use bias instead."
        assert q.size(1) == k.size(1), "Attention mask is not supported with seqlen_q != seqlen_k"
    batch, seqlen_q, nheads_q, head_dim = q.shape
    _, seqlen_k, nheads_kv, _ = k.shape
    expected_kv_shape = (batch, seqlen_k, nheads_kv, head_dim)
    assert nheads_q % nheads_kv == 0, f"{nheads_q = } is not divisible by {nheads_kv = }"
    assert k.shape == expected_kv_shape, f"{k.shape = } <> {expected_kv_shape = }"
    assert v.shape == expected_kv_shape, f"{v.shape = } <> {expected_kv_shape = }"
    assert q.dtype == k.dtype == v.dtype, "All tensors must have the same type"
    assert q.dtype in [torch.float16, torch.bfloat16], "Only support fp16 and bf16"
    assert q.is_cuda and k.is_cuda and v.is_cuda
    assert head_dim <= 256, f"{head_dim = } > 256 is not supported"
    softmax_scale = 1.0 / math.sqrt(head_dim) if softmax_scale is None else softmax_scale

    stride_bb, stride_bh, stride_bm = infer_bias_strides(bias, batch, nheads_q, seqlen_q, seqlen_k)
    dropout_seed = handle_dropout(dropout_p, dropout_seed, is_forward=True)
    cu_seqlens = cu_seqlens_from_mask(attention_mask) if attention_mask is not None else None

    o = torch.empty_like(q)
    if o.stride(-1) != 1:
        o = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    lse_rows = math.ceil(seqlen_q / 128) * 128
    lse = torch.empty((batch, nheads_q, lse_rows), device=q.device, dtype=torch.float32)

    args = _lib.FwdArgs()
    args.q, args.k, args.v, args.o, args.lse = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr()
    args.bias = bias.data_ptr() if bias is not None else None
    args.cu_seqlens = cu_seqlens.data_ptr() if cu_seqlens is not None else None
    args.q_stride[:] = bshd_strides(q)
    args.k_stride[:] = bshd_strides(k)
    args.v_stride[:] = bshd_strides(v)
    args.o_stride[:] = bshd_strides(o)
    args.bias_stride[:] = (stride_bb, stride_bh, stride_bm)
    args.batch, args.heads_q, args.heads_kv = batch, nheads_q, nheads_kv
    args.seqlen_q, args.seqlen_k, args.head_dim = seqlen_q, seqlen_k, head_dim
    args.lse_row_stride = lse_rows
    args.causal = int(bool(causal))
    args.dtype = encode_dtype(q)
    args.bias_dtype = encode_dtype(bias) if bias is not None else 0
    args.softmax_scale = float(softmax_scale)
    args.dropout_p = float(dropout_p)
    args.dropout_seed = int(dropout_seed) & 0xFFFFFFFFFFFFFFFF
    if dropout_mask is not None and dropout_p > 0.0:
        check_dropout_mask(dropout_mask, batch, nheads_q, seqlen_q, seqlen_k, q.device)
        args.dropout_mask = dropout_mask.data_ptr()
    _lib.check(launch_on(q, lambda st: _lib.fwd(args, st)))
    return o, lse, softmax_scale, dropout_seed
