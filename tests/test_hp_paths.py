"""The hand-placed D = 128 kernels against the general kernels of the same launch, and their
persistent multi-unit paths.

* Backward: the hand-placed dK/dV (`dkdv_hp_kernel`) computes the same fp32 sums in the same order
  as `dkdv_kernel` (same math as the reference's loop, /root/reference/src/backward/
  compute_dkdv.py:42-112), so dK and dV must be BITWISE equal with the hand-placed paths on and off
  (the per-call fa2_policy, ABI 9).  The hand-placed dQ (round 6) starts its dP chain from -delta
  (dS = P acc, one multiply; `dq_kernel` subtracts delta after the chain, as the reference's
  compute_dq.py:70-76), so dQ may differ by the rounding of dP - delta (assert_hp_vs_general).
* Forward: `fwd_hp_kernel` and `fwd_pipe_kernel` order the softmax differently (defer-max
  thresholds, tile phases): both within the reference's tolerance of the oracle, LSE2 within 1e-3.
* Persistence: one workgroup per CU walks several work units when the grid is capped
  (grid_cap = 2 or 3: every workgroup runs many units, so the next-unit prefetch, buffer parity
  and the hand-off of Q / dO / keep words across units all run).  Results must be bitwise equal
  to the uncapped launch -- with dropout too (the keep words of the next unit are loaded by the
  previous unit's statement).
"""
import pytest
import torch

from tests.core import (assert_dropout_dv_vs_oracle, assert_dropout_grads_match, generate_attention_mask,
                        generate_test_data)

BWD_CASES = [
    # b, hq, hkv, sq, sk, causal, dtype
    (1, 1, 1, 256, 256, False, torch.bfloat16),
    (1, 1, 1, 256, 256, True, torch.bfloat16),
    (2, 4, 2, 512, 512, True, torch.bfloat16),
    (2, 4, 4, 1024, 1024, False, torch.float16),
    (1, 2, 1, 300, 700, True, torch.bfloat16),
    (1, 2, 2, 777, 333, True, torch.float16),
    (1, 4, 1, 129, 257, False, torch.bfloat16),
    (2, 8, 8, 2048, 2048, True, torch.bfloat16),
    # dK/dV steps (32 query rows of one q-head) per block: odd totals and 1-3 steps per head, so the
    # two-step barrier pairs straddle head changes and blocks end on either phase
    (1, 4, 1, 96, 512, False, torch.bfloat16),
    (1, 4, 1, 32, 300, True, torch.float16),
    (2, 3, 1, 160, 160, True, torch.bfloat16),
]


@pytest.fixture
def policy():
    from fa2_triton_amd import _lib as L

    yield L
    L.set_path_policy(0, 0)


def assert_hp_vs_general(hp, gen):
    """out, dK, dV bitwise; dQ within one ulp of the dtype per element (the -delta seed)."""
    for name, a, c in zip(("out", "dq", "dk", "dv"), hp, gen):
        assert torch.isfinite(a).all(), name
        if name != "dq":
            assert torch.equal(a, c), f"{name}: max |diff| {(a.float() - c.float()).abs().max().item():.3e}"
            continue
        # the seed moves dP - delta by an fp32 rounding, which can flip the rounding of a dS element
        # packed to the dtype (2^-8 of |dS|) and so move a dQ element by that term's share of the
        # sum, independent of the element's own size: two ulps of |x| (a binade edge) plus a
        # quarter ulp of the largest |dQ|; a wrong dS element moves dQ by far more
        ulp = 2.0 ** -7 if a.dtype == torch.bfloat16 else 2.0 ** -10
        err = (a.float() - c.float()).abs()
        tol = 2 * ulp * c.float().abs() + 0.25 * ulp * c.float().abs().max().item() + 1e-6
        assert bool((err <= tol).all()), f"dq: {int((err > tol).sum())} elements over one ulp, max |diff| {err.max().item():.3e}"


def _fwd_bwd(q, k, v, do, causal, mask=None, dropout_p=0.0, seed=None, policy=None, disable=0, cap=0):
    from fa2_triton_amd import flash_attn_func

    policy.set_path_policy(disable, cap)
    try:
        out = flash_attn_func(q, k, v, mask, None, dropout_p, causal, None, seed)
        grads = torch.autograd.grad(out, (q, k, v), do)
        torch.cuda.synchronize()
    finally:
        policy.set_path_policy(0, 0)
    return [t.detach().clone() for t in (out,) + tuple(grads)]


@pytest.mark.gpu
@pytest.mark.parametrize("b,hq,hkv,sq,sk,causal,dtype", BWD_CASES, ids=lambda x: str(x).replace("torch.", ""))
def test_hand_placed_backward_bitwise_equals_general(b, hq, hkv, sq, sk, causal, dtype, policy):
    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, 128, dtype)
    # the forward from the general kernel in both arms, so dQ / dK / dV see the same O and LSE2
    hp = _fwd_bwd(q, k, v, do, causal, policy=policy, disable=policy.PATH_FWD_HP)
    gen = _fwd_bwd(q, k, v, do, causal, policy=policy,
                   disable=policy.PATH_FWD_HP | policy.PATH_DQ_HP | policy.PATH_DKDV_HP)
    assert_hp_vs_general(hp, gen)


@pytest.mark.gpu
@pytest.mark.parametrize("b,hq,hkv,sq,sk,causal,dtype", [c for c in BWD_CASES if c[1] > c[2]],
                         ids=lambda x: str(x).replace("torch.", ""))
def test_hand_placed_backward_whole_group_per_block(b, hq, hkv, sq, sk, causal, dtype, policy, monkeypatch):
    """As above with the dK/dV q-head split off (FA2_DKV_SPLIT=0): one workgroup sums the whole GQA
    group, so a key block's step sequence runs several heads back to back and a head's dead causal
    steps (the classes D / Ds / E / F of hp_gen.DkdvGen) hand over to the next head's first step,
    whose S the last dead step computes (the small grids here would otherwise split the group)."""
    monkeypatch.setenv("FA2_DKV_SPLIT", "0")
    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, 128, dtype)
    hp = _fwd_bwd(q, k, v, do, causal, policy=policy, disable=policy.PATH_FWD_HP)
    gen = _fwd_bwd(q, k, v, do, causal, policy=policy,
                   disable=policy.PATH_FWD_HP | policy.PATH_DQ_HP | policy.PATH_DKDV_HP)
    assert_hp_vs_general(hp, gen)


@pytest.mark.gpu
@pytest.mark.parametrize("b,hq,hkv,sq,sk,causal,dtype", BWD_CASES[:6], ids=lambda x: str(x).replace("torch.", ""))
def test_hand_placed_forward_matches_pipelined(b, hq, hkv, sq, sk, causal, dtype, policy):
    from fa2_triton_amd.forward import _flash_attn_forward
    from oracle.reference import attention_reference, lse2_reference

    q, k, v, _ = generate_test_data(b, hq, hkv, sq, sk, 128, dtype)
    res = {}
    for tag, dis in (("hp", 0), ("pipe", policy.PATH_FWD_HP)):
        policy.set_path_policy(dis, 0)
        o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        res[tag] = (o.float(), lse[:, :, :sq].float())
    policy.set_path_policy(0, 0)
    ref = attention_reference(q, k, v, causal=causal).float()
    pt = attention_reference(q, k, v, causal=causal, upcast=False, reorder_ops=True).float()
    lref = lse2_reference(q, k, causal=causal)
    fin = torch.isfinite(lref)
    ept = (pt - ref).abs().max().item()
    for tag, (o, lse) in res.items():
        assert (o - ref).abs().max().item() <= 2 * ept + 5e-5, tag
        assert torch.equal(torch.isfinite(lse), fin), tag
        if fin.any():
            assert (lse[fin] - lref[fin]).abs().max().item() <= 1e-3 * (1 + lref[fin].abs().max().item()), tag


GRID_CASES = [
    # b, hq, hkv, s, causal, dtype, varlen
    (2, 8, 2, 1024, True, torch.bfloat16, False),
    (2, 8, 8, 1024, False, torch.float16, False),
    (3, 4, 2, 777, True, torch.bfloat16, True),
    (2, 6, 2, 416, True, torch.bfloat16, False),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [2, 3])
@pytest.mark.parametrize("b,hq,hkv,s,causal,dtype,varlen", GRID_CASES, ids=lambda x: str(x).replace("torch.", ""))
def test_persistent_units_bitwise_equal_any_grid(b, hq, hkv, s, causal, dtype, varlen, cap, policy):
    q, k, v, do = generate_test_data(b, hq, hkv, s, s, 128, dtype)
    mask = generate_attention_mask(q) if varlen else None
    full = _fwd_bwd(q, k, v, do, causal, mask, policy=policy)
    capped = _fwd_bwd(q, k, v, do, causal, mask, policy=policy, cap=cap)
    for name, a, c in zip(("out", "dq", "dk", "dv"), full, capped):
        assert torch.isfinite(a).all(), name
        assert torch.equal(a, c), name


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [0, 2])
@pytest.mark.parametrize("causal", [True, False])
def test_dropout_hand_placed_dq_multi_unit(causal, cap, policy):
    """The hand-placed dropout dQ reads the forward's saved keep words; several units per workgroup
    (cap 2) must give the dQ of the general kernel regenerating the keep bits with Philox (dK / dV
    from the hand-placed dK/dV: assert_dropout_grads_match)."""
    from fa2_triton_amd.backward import _flash_attn_backward
    from fa2_triton_amd.forward import _flash_attn_forward
    from fa2_triton_amd.utils import dropout_mask_words

    b, hq, hkv, s, p = 2, 4, 2, 1024, 0.2
    q, k, v, do = generate_test_data(b, hq, hkv, s, s, 128, torch.bfloat16)
    words = torch.empty(dropout_mask_words(b, hq, s, s), dtype=torch.int32, device="cuda")
    o, lse, scale, seed = _flash_attn_forward(q, k, v, None, None, p, causal, None, 1234, dropout_mask=words)
    policy.set_path_policy(0, cap)
    hp = _flash_attn_backward(do, q, k, v, None, None, o, lse, p, causal, scale, seed, dropout_mask=words)
    policy.set_path_policy(policy.PATH_DQ_HP | policy.PATH_DKDV_HP, 0)
    regen = _flash_attn_backward(do, q, k, v, None, None, o, lse, p, causal, scale, seed, dropout_mask=None)
    policy.set_path_policy(0, 0)
    assert_dropout_grads_match(hp[:3], regen[:3])
    assert_dropout_dv_vs_oracle(hp[2], regen[2], q, k, v, do, words, p, causal)


DROP_CASES = [
    # b, hq, hkv, s_q, s_k, causal, p, dtype
    (2, 4, 2, 1024, 1024, True, 0.1, torch.bfloat16),
    (2, 4, 4, 1024, 1024, False, 0.2, torch.float16),
    (1, 8, 2, 777, 333, True, 0.17, torch.bfloat16),
    (1, 2, 1, 300, 700, False, 0.3, torch.bfloat16),
    (2, 2, 2, 129, 257, True, 0.1, torch.float16),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [0, 3])
@pytest.mark.parametrize("b,hq,hkv,sq,sk,causal,p,dtype", DROP_CASES, ids=lambda x: str(x).replace("torch.", ""))
def test_dropout_hand_placed_dkdv(b, hq, hkv, sq, sk, causal, p, dtype, cap, policy):
    """The hand-placed dK/dV with the forward's saved keep words (ABI 8) against the general
    dK/dV over the same words: dK bitwise (dS = P (dP kp - delta) in the same operations), dV as
    assert_dropout_grads_match; one and several blocks per workgroup (cap 3), ragged and GQA."""
    from fa2_triton_amd.backward import _flash_attn_backward
    from fa2_triton_amd.forward import _flash_attn_forward
    from fa2_triton_amd.utils import dropout_mask_words

    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, 128, dtype)
    words = torch.empty(dropout_mask_words(b, hq, sq, sk), dtype=torch.int32, device="cuda")
    o, lse, scale, seed = _flash_attn_forward(q, k, v, None, None, p, causal, None, 4321, dropout_mask=words)
    policy.set_path_policy(0, cap)
    hp = _flash_attn_backward(do, q, k, v, None, None, o, lse, p, causal, scale, seed, dropout_mask=words)
    policy.set_path_policy(policy.PATH_DKDV_HP, 0)
    gen = _flash_attn_backward(do, q, k, v, None, None, o, lse, p, causal, scale, seed, dropout_mask=words)
    policy.set_path_policy(0, 0)
    assert_dropout_grads_match(hp[:3], gen[:3])
    assert_dropout_dv_vs_oracle(hp[2], gen[2], q, k, v, do, words, p, causal)


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [0, 2])
@pytest.mark.parametrize("b,hq,hkv,sq,sk,causal,p,dtype", DROP_CASES, ids=lambda x: str(x).replace("torch.", ""))
def test_dropout_hand_placed_forward(b, hq, hkv, sq, sk, causal, p, dtype, cap, policy):
    """The dropout forward at D = 128 (round 6): dropout_mask_kernel draws the keep words (integer
    threshold on the Philox word), fwd_hp_kernel's dropout statement reads them and zeroes the
    dropped P halves after the row sums.  The words equal the Philox oracle's mask on every visible
    element; O and LSE2 against the fp32 oracle over those bits (O = (P * M / (1 - p)) V / l,
    compute_row_blocks.py:76-79), within the bound of the general kernel reading the same words;
    several units per workgroup (cap 2) bitwise equal to one unit each."""
    from fa2_triton_amd.forward import _flash_attn_forward
    from fa2_triton_amd.utils import dropout_mask_words
    from oracle.philox import dropout_keep_mask_torch
    from oracle.reference import attention_reference, lse2_reference
    from tests.core import unpack_keep_mask

    q, k, v, _ = generate_test_data(b, hq, hkv, sq, sk, 128, dtype)
    res = {}
    for tag, dis, cp in (("hp", 0, cap), ("hp1", 0, 0), ("gen", policy.PATH_FWD_HP, 0)):
        words = torch.full((dropout_mask_words(b, hq, sq, sk),), -1, dtype=torch.int32, device=q.device)
        policy.set_path_policy(dis, cp)
        o, lse, _, seed = _flash_attn_forward(q, k, v, None, None, p, causal, None, 777, dropout_mask=words)
        policy.set_path_policy(0, 0)
        res[tag] = (o, lse[:, :, :sq].float(), words)
    assert torch.equal(res["hp"][0], res["hp1"][0]) and torch.equal(res["hp"][1], res["hp1"][1])
    keep = unpack_keep_mask(res["hp"][2], b, hq, sq, sk)
    vis = torch.ones(sq, sk, dtype=torch.bool, device=q.device)
    if causal:
        vis = torch.arange(sk, device=q.device)[None, :] <= torch.arange(sq, device=q.device)[:, None] + (sk - sq)
    want = dropout_keep_mask_torch(seed, p, b, hq, sq, sk, device=q.device)
    assert torch.equal(keep[:, :, vis], want[:, :, vis])
    ref = attention_reference(q, k, v, dropout_p=p, dropout_mask=keep, causal=causal).float()
    e_gen = (res["gen"][0].float() - ref).abs().max().item()
    e_hp = (res["hp"][0].float() - ref).abs().max().item()
    assert e_hp <= 2 * e_gen + 5e-5, f"hp {e_hp:.3e} vs general {e_gen:.3e}"
    lref = lse2_reference(q, k, causal=causal)
    fin = torch.isfinite(lref)
    lse = res["hp"][1]
    assert torch.equal(torch.isfinite(lse), fin)
    if fin.any():
        assert (lse[fin] - lref[fin]).abs().max().item() <= 1e-3 * (1 + lref[fin].abs().max().item())
