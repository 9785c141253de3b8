"""GPU parity harness -- the reference's tests/core.py + tests/utils.py, Triton-free.

Mirrors /root/reference/tests/core.py:10-78 (_test_core_fn) and the generators of
/root/reference/tests/utils.py: generate_test_data (:9-26, seed 0, N(0, 0.5) Q/K/V, N(0, 1) dO),
generate_attention_mask (:40-56, right padding, one full row), generate_dropout_seed_and_mask
(:169-207, here with the torch Philox of oracle/philox.py instead of a Triton kernel) and the
acceptance rule compare_results_fa (:68-142, oracle/tolerance.py).  The oracle is run on the
same device tensors, fp32-upcast ("ref") and in the input dtype with reordered ops ("pt").
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from oracle.philox import dropout_keep_mask_torch
from oracle.reference import attention_reference
from oracle.tolerance import check_fa_tolerance


def generate_test_data(batch_size, nheads_q, nheads_kv, seqlen_q, seqlen_k, head_dim, dtype, seed=0, device="cuda"):
    torch.manual_seed(seed)
    q = torch.empty((batch_size, seqlen_q, nheads_q, head_dim), dtype=dtype, device=device).normal_(0.0, 0.5)
    k = torch.empty((batch_size, seqlen_k, nheads_kv, head_dim), dtype=dtype, device=device).normal_(0.0, 0.5)
    v = torch.empty((batch_size, seqlen_k, nheads_kv, head_dim), dtype=dtype, device=device).normal_(0.0, 0.5)
    do = torch.randn_like(q)
    return q.requires_grad_(), k.requires_grad_(), v.requires_grad_(), do


def generate_attention_mask(x: Tensor) -> Tensor:
    """Random right padding per batch row, one row unpadded (reference tests/utils.py:40-56)."""
    mask = torch.ones(size=x.shape[:2], dtype=torch.bool, device=x.device)
    if x.size(1) == 1:
        return mask
    padding = torch.randint(low=0, high=x.size(1) - 1, size=(x.size(0),)).tolist()
    padding[torch.randint(low=0, high=x.size(0), size=(1,)).item()] = 0
    for i, pad in enumerate(padding):
        if pad:
            mask[i, -pad:] = False
    return mask


def generate_dropout_seed_and_mask(dropout_p, q, k, attention_mask) -> Tuple[Optional[int], Optional[Tensor]]:
    if dropout_p == 0:
        return None, None
    seed = torch.randint(low=0, high=2**32, size=(1,)).item()
    assert attention_mask is None, "dropout + padding mask is not exercised by the reference tests"
    b, sq, hq, _ = q.shape
    return seed, dropout_keep_mask_torch(seed, dropout_p, b, hq, sq, k.size(1), device=q.device)


def run_case(
    batch_size: int,
    nheads_q: int,
    nheads_kv: int,
    seqlen_q: int,
    seqlen_k: int,
    head_dim: int,
    causal: bool,
    dropout_p: float,
    use_attention: bool,
    use_bias: bool,
    dtype: torch.dtype,
    forward_only: bool,
) -> dict:
    from fa2_triton_amd import flash_attn_func

    q, k, v, do = generate_test_data(batch_size, nheads_q, nheads_kv, seqlen_q, seqlen_k, head_dim, dtype)
    attn_mask = generate_attention_mask(q) if use_attention else None
    attn_bias = torch.rand(size=(1, 1, seqlen_q, seqlen_k), dtype=dtype, device=q.device) if use_bias else None
    dropout_seed, dropout_mask = generate_dropout_seed_and_mask(dropout_p, q, k, attn_mask)
    common = dict(query_padding_mask=attn_mask, key_padding_mask=attn_mask, attn_bias=attn_bias,
                  dropout_p=dropout_p, dropout_mask=dropout_mask, causal=causal)
    out_ref = attention_reference(q, k, v, **common)
    out_pt = attention_reference(q, k, v, upcast=False, reorder_ops=True, **common)
    out = flash_attn_func(q, k, v, attention_mask=attn_mask, attention_bias=attn_bias, dropout_p=dropout_p,
                          causal=causal, softmax_scale=None, dropout_seed=dropout_seed)
    assert out.shape == q.shape and out.dtype == q.dtype
    return check_fa_tolerance(q, k, v, None if forward_only else do, out, out_ref, out_pt)


def unpack_keep_mask(words, b, h, sq, sk):
    """Dense [B, Hq, Sq, Sk] bool view of the tiled keep mask of include/fa2_amd.h (ABI 6; the
    ABI-8 slack tile after the last one is not part of the mask)."""
    nrb, ncw = (sq + 31) // 32, (sk + 31) // 32
    t = words[: b * h * nrb * ncw * 32].view(b, h, nrb, ncw, 32)  # [.., row tile, key word, row in tile]
    bits = (t.unsqueeze(-1) >> torch.arange(32, device=words.device, dtype=torch.int32)) & 1
    dense = bits.permute(0, 1, 2, 4, 3, 5).reshape(b, h, nrb * 32, ncw * 32)
    return dense[:, :, :sq, :sk].bool()


def assert_dropout_dv_vs_oracle(dv_got, dv_other, q, k, v, do, words, p, causal):
    """dV of a dropout backward against the fp32 oracle over the SAME keep bits (the forward's
    saved words, unpacked): the rule of the reference's compare_results_fa for gradients
    (tests/utils.py:127-131, oracle/tolerance.py) with the other backward's dV (the general kernel
    over the same bits) as the baseline: max |dv - ref| <= 3 max |dv_other - ref| + 1e-5.  This
    checks the hand-placed dK/dV's P-pack masking and its one-time 1 / (1 - p) against the exact
    math, not only against the other kernel."""
    b, sq, hq, _ = q.shape
    keep = unpack_keep_mask(words, b, hq, sq, k.size(1))
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    out = attention_reference(qf, kf, vf, dropout_p=p, dropout_mask=keep, causal=causal)
    ref = torch.autograd.grad(out, vf, do.float())[0]
    e_got = (dv_got.float() - ref).abs().max().item()
    e_other = (dv_other.float() - ref).abs().max().item()
    assert e_got <= 3 * e_other + 1e-5, f"dv vs fp32 oracle: {e_got:.3e} > 3 x {e_other:.3e} + 1e-5"


def assert_dropout_grads_match(got, want, names=("dq", "dk", "dv")):
    """Gradients of two dropout backwards over the same keep bits.  dQ and dK are bitwise equal
    whichever kernels ran; dV may come from the hand-placed dK/dV, which packs P M and applies
    1 / (1 - p) once to the fp32 sum where the general kernel rounds P M / (1 - p) per score
    (dkdv_hp_kernel.h): within 4 ulps (of the dtype) of the largest |dV|.  (The difference is the
    rounding of each term, so it grows with the number of terms a dV row sums: under a causal mask
    the first keys are visible to every query row and carry both the largest |dV| and the largest
    difference -- the "key % 64 == 0" pattern of DESIGN.md 5 is key 0 of the sequence, at a relative
    difference of 0.5 % like every other key.  assert_dropout_dv_vs_oracle checks dV against the
    exact math.)"""
    for name, x, y in zip(names, got, want):
        if x is None:
            continue
        assert torch.isfinite(x).all(), name
        if name != "dv":
            assert torch.equal(x, y), f"{name}: max |diff| {(x.float() - y.float()).abs().max().item():.3e}"
            continue
        ulp = 2.0 ** -7 if x.dtype == torch.bfloat16 else 2.0 ** -10
        tol = 4 * ulp * y.float().abs().max().item()
        err = (x.float() - y.float()).abs().max().item()
        assert err <= tol, f"dv: max |diff| {err:.3e} > {tol:.3e}"
