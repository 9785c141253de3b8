"""O(S^2) attention oracle (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

A restatement, in plain torch ops, of the reference's correctness oracle
`flash_attn_reference` (/root/reference/src/reference_implementation.py:38-123) and its
mask helper `construct_local_mask` (:8-35).  It works on any device: the GPU parity tests
run it on `cuda` tensors exactly as the reference's own tests do (tests/core.py:31-55 there),
the CPU tests and the bench's `cpu_baseline` leg run it on the host.

Semantics (matching the cited lines):
* layout BSHD: q [B, Sq, Hq, D], k/v [B, Sk, Hkv, D]; GQA by contiguous head groups,
  i.e. `repeat_interleave` of K/V heads (:80-81);
* scores = (q / sqrt(D)) k^T, or q (k / sqrt(D))^T with `reorder_ops` (:82-86);
* optional tanh soft-capping (:87-90, unused by the tests);
* key padding -> -inf (:91-92); local / causal window mask, bottom-right aligned against the
  *valid* lengths of the padding masks (:8-35, :93-102);
* additive bias after masking (:103-104); softmax in the compute dtype (:105);
* rows that the window masks completely -> 0 (:106-108); padded query rows -> 0 (:109-112);
* dropout: masked_fill(~mask) on the probabilities, V scaled by 1/(1-p) (:113-120);
* padded query rows of the output -> 0 (:121-122), cast back to the input dtype (:123).
"""
import math
from typing import Optional, Tuple

import torch
from torch import Tensor

LOG2E = 1.4426950408889634


def window_mask(
    seqlen_q: int,
    seqlen_k: int,
    window_size: Tuple[int, int] = (-1, -1),
    query_padding_mask: Optional[Tensor] = None,
    key_padding_mask: Optional[Tensor] = None,
    device=None,
) -> Tensor:
    """True where (query i, key j) is OUTSIDE the local window.

    Restates construct_local_mask (/root/reference/src/reference_implementation.py:8-35):
    the window is anchored at the bottom-right corner of the *valid* part of each sequence,
    i.e. query i is aligned with key i + (Lk - Lq) where Lq / Lk are the unpadded lengths.
    Returns a [Sq, Sk] mask, or [B, 1, Sq, Sk] when padding masks are given.
    """
    rows = torch.arange(seqlen_q, device=device, dtype=torch.long)[:, None]
    cols = torch.arange(seqlen_k, device=device, dtype=torch.long)[None, :]

    def valid_len(mask: Optional[Tensor], full: int):
        if mask is None:
            return full
        return mask.sum(-1).view(-1, 1, 1, 1)

    lk = valid_len(key_padding_mask, seqlen_k)
    lq = valid_len(query_padding_mask, seqlen_q)
    shift = rows + lk - lq  # the diagonal key of each query row
    left, right = window_size
    if left < 0:
        return cols > shift + right
    lk_t = torch.full_like(cols, seqlen_k) if key_padding_mask is None else lk
    return (cols > torch.minimum(shift + right, lk_t)) | (cols < shift - left)


def attention_reference(
    q: Tensor,
    k: Tensor,
    v: Tensor,
    query_padding_mask: Optional[Tensor] = None,
    key_padding_mask: Optional[Tensor] = None,
    attn_bias: Optional[Tensor] = None,
    dropout_p: float = 0.0,
    dropout_mask: Optional[Tensor] = None,
    causal: bool = False,
    window_size: Tuple[int, int] = (-1, -1),
    softcap: float = 0.0,
    upcast: bool = True,
    reorder_ops: bool = False,
) -> Tensor:
    """Dense attention; see the module docstring for the exact semantics.

    Same argument list and meaning as `flash_attn_reference`
    (/root/reference/src/reference_implementation.py:38-52).
    """
    if causal:
        window_size = (window_size[0], 0)
    out_dtype = q.dtype
    if upcast:
        q, k, v = q.float(), k.float(), v.float()
    b, sq, hq, d = q.shape
    sk, hkv = k.shape[1], k.shape[2]
    group = hq // hkv
    k = torch.repeat_interleave(k, group, dim=2)
    v = torch.repeat_interleave(v, group, dim=2)

    inv = 1.0 / math.sqrt(d)
    if reorder_ops:
        scores = torch.einsum("bqhd,bkhd->bhqk", q, k * inv)
    else:
        scores = torch.einsum("bqhd,bkhd->bhqk", q * inv, k)
    if softcap > 0:
        scores = torch.tanh(scores / softcap) * softcap
    if key_padding_mask is not None:
        scores = scores.masked_fill(~key_padding_mask[:, None, None, :], float("-inf"))
    local = None
    if window_size[0] >= 0 or window_size[1] >= 0:
        local = window_mask(sq, sk, window_size, query_padding_mask, key_padding_mask, q.device)
        scores = scores.masked_fill(local, float("-inf"))
    if attn_bias is not None:
        scores = scores + attn_bias

    probs = torch.softmax(scores, dim=-1).to(v.dtype)
    if local is not None:
        probs = probs.masked_fill(local.all(dim=-1, keepdim=True), 0.0)
    if query_padding_mask is not None:
        probs = probs.masked_fill(~query_padding_mask[:, None, :, None], 0.0)
    if dropout_mask is not None:
        probs = probs.masked_fill(~dropout_mask, 0.0)
    out = torch.einsum("bhqk,bkhd->bqhd", probs, v * (1.0 / (1.0 - dropout_p)))
    if query_padding_mask is not None:
        out = out.masked_fill(~query_padding_mask[:, :, None, None], 0.0)
    return out.to(out_dtype)


def lse2_reference(
    q: Tensor,
    k: Tensor,
    attn_bias: Optional[Tensor] = None,
    causal: bool = False,
    padding_mask: Optional[Tensor] = None,
    softmax_scale: Optional[float] = None,
) -> Tensor:
    """Base-2 logsumexp of the scaled, biased, masked scores: [B, Hq, Sq] fp32.

    The forward kernel stores LSE2 = log2(sum_j 2^(s_ij * log2 e)) = ln(sum_j e^s_ij) * log2 e
    (/root/reference/src/forward/kernel.py:119, compute_row_blocks.py:69-72,100-101; the dead
    test /root/reference/tests/test_logsumexp.py:74 multiplies by 1.44269504089 for the same
    reason).  Rows with no visible key are -inf here (logsumexp of the empty set).
    """
    q, k = q.float(), k.float()
    b, sq, hq, d = q.shape
    sk, hkv = k.shape[1], k.shape[2]
    k = torch.repeat_interleave(k, hq // hkv, dim=2)
    scale = 1.0 / math.sqrt(d) if softmax_scale is None else softmax_scale
    scores = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    if attn_bias is not None:
        scores = scores + attn_bias.float()
    if padding_mask is not None:
        scores = scores.masked_fill(~padding_mask[:, None, None, :], float("-inf"))
    if causal:
        cm = window_mask(sq, sk, (-1, 0), padding_mask, padding_mask, q.device)
        scores = scores.masked_fill(cm, float("-inf"))
    return torch.logsumexp(scores, dim=-1) * LOG2E
