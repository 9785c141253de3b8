"""Public autograd op -- same surface as /root/reference/src/wrapper.py:10-100.

`flash_attn_func(q, k, v, attention_mask=None, attention_bias=None, dropout_p=0.0,
causal=False, softmax_scale=None, dropout_seed=None)` with q [B, Sq, Hq, D], k/v
[B, Sk, Hkv, D] (fp16 / bf16), returns O [B, Sq, Hq, D].  Backward returns (dq, dk, dv) and
no gradient for the mask and scalars, exactly as the reference (:62-86).  Beyond the
reference (which returns None for the bias, :86): when `attention_bias` requires grad, its
gradient dL/d(bias) is returned too.  With dropout the keep
bits drawn by the forward are kept for the backward (see _keep_mask_buffer).
"""
import logging
import os
from typing import Optional

import torch
from torch import Tensor

from .backward import _flash_attn_backward
from .forward import _flash_attn_forward
from .utils import dropout_mask_words


def _keep_mask_buffer(q: Tensor, k: Tensor, v: Tensor, dropout_p: float) -> Optional[Tensor]:
    """With dropout, the forward saves its keep bits (1 bit per score, include/fa2_amd.h) so
    that the backward reads them instead of drawing Philox twice more (dQ and dK/dV).  Above
    FA2_DROPOUT_MASK_MAX_GB (default 4, per call), or when the allocation itself fails, the
    backward regenerates them instead (bitwise the same gradients, tests/test_dropout_bwd.py):
    the mask is an O(S^2) cache, never a reason for a forward that fits in O(S) memory to fail."""
    if not dropout_p > 0.0 or not (q.requires_grad or k.requires_grad or v.requires_grad):  # (inputs of Function.forward)
        return None
    words = dropout_mask_words(q.size(0), q.size(2), q.size(1), k.size(1))
    if words * 4 > float(os.environ.get("FA2_DROPOUT_MASK_MAX_GB", "4")) * 2**30:
        return None
    try:
        return torch.empty(words, dtype=torch.int32, device=q.device)
    except torch.OutOfMemoryError:
        logging.getLogger(__name__).info("dropout keep mask (%d bytes) not allocated: the backward regenerates it",
                                         words * 4)
        return None


class FlashAttnFunc(torch.autograd.Function):
    @staticmethod
    def forward(
        ctx,
        q: Tensor,
        k: Tensor,
        v: Tensor,
        attention_mask: Optional[Tensor] = None,
        attention_bias: Optional[Tensor] = None,
        dropout_p: float = 0.0,
        causal: bool = False,
        softmax_scale: Optional[float] = None,
        dropout_seed: Optional[int] = None,
    ):
        # only the last dimension has to be contiguous (reference :41-43); bias fully (:44)
        q = q if q.stride(-1) == 1 else q.contiguous()
        k = k if k.stride(-1) == 1 else k.contiguous()
        v = v if v.stride(-1) == 1 else v.contiguous()
        attention_bias = None if attention_bias is None else attention_bias.contiguous()
        ctx.dropout_mask = _keep_mask_buffer(q, k, v, dropout_p)
        o, lse, ctx.softmax_scale, ctx.dropout_seed = _flash_attn_forward(
            q=q,
            k=k,
            v=v,
            attention_mask=attention_mask,
            bias=attention_bias,
            dropout_p=dropout_p,
            causal=causal,
            softmax_scale=softmax_scale,
            dropout_seed=dropout_seed,
            dropout_mask=ctx.dropout_mask,
        )
        ctx.save_for_backward(q, k, v, attention_bias, attention_mask, o, lse)
        ctx.causal = causal
        ctx.dropout_p = dropout_p
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, bias, attention_mask, o, lse = ctx.saved_tensors
        bias_grad = bias is not None and ctx.needs_input_grad[4]
        grads = _flash_attn_backward(
            dO=do,
            q=q,
            k=k,
            v=v,
            bias=bias,
            attention_mask=attention_mask,
            o=o,
            lse=lse,
            dropout_p=ctx.dropout_p,
            causal=ctx.causal,
            softmax_scale=ctx.softmax_scale,
            dropout_seed=ctx.dropout_seed,
            bias_grad=bias_grad,
            dropout_mask=ctx.dropout_mask,
        )
        dbias = grads[3] if bias_grad else None
        return grads[0], grads[1], grads[2], None, dbias, None, None, None, None


def flash_attn_func(
    q: Tensor,
    k: Tensor,
    v: Tensor,
    attention_mask: Optional[Tensor] = None,
    attention_bias: Optional[Tensor] = None,
    dropout_p: float = 0.0,
    causal: bool = False,
    softmax_scale: Optional[float] = None,
    dropout_seed: Optional[int] = None,
) -> Tensor:
    return FlashAttnFunc.apply(q, k, v, attention_mask, attention_bias, dropout_p, causal, softmax_scale, dropout_seed)
