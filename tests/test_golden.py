"""Golden vectors: pin the oracle (CPU) and check the HIP kernels against the same fixtures (GPU).

tests/golden/attention_golden.npz was produced by tests/golden/make_golden.py from the
reference's own flash_attn_reference (/root/reference/src/reference_implementation.py:38-123)
imported in the build container; tests/golden/philox_kat.npz by make_philox_kat.py from
Triton 3.6's tl.rand (interpreter).  Neither script runs here or on the GPU box.
"""
import os

import numpy as np
import pytest
import torch

from oracle.philox import dropout_keep_mask, rand, rand_torch
from oracle.reference import attention_reference, lse2_reference

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "attention_golden.npz"))
KAT = np.load(os.path.join(HERE, "golden", "philox_kat.npz"))
CASES = sorted({k.split("/")[0] for k in GOLD.files})


def case(name):
    g = {k.split("/", 1)[1]: GOLD[k] for k in GOLD.files if k.startswith(name + "/")}
    b, hq, hkv, sq, sk, d, causal, use_bias, use_pad = (int(x) for x in g["meta"])
    return g, dict(b=b, hq=hq, hkv=hkv, sq=sq, sk=sk, d=d, causal=bool(causal), bias=bool(use_bias), pad=bool(use_pad),
                   p=float(g["dropout"][0]), seed=int(g["seed"][0]))


# ---------------------------------------------------------------------------------- CPU ----
@pytest.mark.parametrize("name", sorted(k[: -len("_meta")] for k in KAT.files if k.endswith("_meta")))
def test_philox_matches_triton_kat(name):
    seed, base, n = (int(x) for x in KAT[name + "_meta"])
    offs = np.arange(base, base + n, dtype=np.uint64)
    assert np.array_equal(rand(seed, offs), KAT[name])
    assert np.array_equal(rand_torch(seed, torch.from_numpy(offs.astype(np.int64))).numpy(), KAT[name])


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_golden(name):
    g, m = case(name)
    q, k, v = (torch.from_numpy(g[x]).requires_grad_() for x in ("q", "k", "v"))
    bias = torch.from_numpy(g["bias"]) if "bias" in g else None
    pad = torch.from_numpy(g["pad"]) if "pad" in g else None
    keep = None
    if m["p"] > 0:
        keep = torch.from_numpy(dropout_keep_mask(m["seed"], m["p"], m["b"], m["hq"], m["sq"], m["sk"]))
        assert np.array_equal(keep.numpy(), g["keep"])
    out = attention_reference(q, k, v, query_padding_mask=pad, key_padding_mask=pad, attn_bias=bias,
                              dropout_p=m["p"], dropout_mask=keep, causal=m["causal"])
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), torch.from_numpy(g["do"]))
    for name_, got in (("out", out), ("dq", dq), ("dk", dk), ("dv", dv)):
        np.testing.assert_allclose(got.detach().numpy(), g[name_], rtol=1e-5, atol=1e-5, err_msg=name_)
    lse = lse2_reference(q.detach(), k.detach(), bias, m["causal"], pad)
    np.testing.assert_allclose(lse.numpy(), g["lse2"], rtol=1e-5, atol=1e-5)


# ---------------------------------------------------------------------------------- GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("name", CASES)
def test_kernels_match_golden(name, dtype):
    """HIP fwd+bwd on the fixture inputs vs the reference oracle's fp32 outputs.

    Tolerance: the reference tests' rule, with the 'pt' error measured by running the oracle
    in `dtype` (upcast=False, reorder_ops=True) on the same inputs; LSE2 within 1e-3 abs/rel
    on rows that see at least one key.
    """
    from fa2_triton_amd import forward as fwd_mod
    from fa2_triton_amd import flash_attn_func

    g, m = case(name)
    dev = "cuda"
    q, k, v = (torch.from_numpy(g[x]).to(dev, dtype).requires_grad_() for x in ("q", "k", "v"))
    do = torch.from_numpy(g["do"]).to(dev, dtype)
    bias = torch.from_numpy(g["bias"]).to(dev, dtype) if "bias" in g else None
    pad = torch.from_numpy(g["pad"]).to(dev) if "pad" in g else None
    keep = torch.from_numpy(g["keep"]).to(dev) if "keep" in g else None
    out = flash_attn_func(q, k, v, attention_mask=pad, attention_bias=bias, dropout_p=m["p"], causal=m["causal"],
                          dropout_seed=m["seed"] if m["p"] > 0 else None)
    pt = attention_reference(q, k, v, query_padding_mask=pad, key_padding_mask=pad, attn_bias=bias, dropout_p=m["p"],
                             dropout_mask=keep, causal=m["causal"], upcast=False, reorder_ops=True)
    ref_out = torch.from_numpy(g["out"]).to(dev)
    err = (out.float() - ref_out).abs().max().item()
    err_pt = (pt.float() - ref_out).abs().max().item()
    assert err <= 2 * err_pt + 5e-5, (err, err_pt)
    # gradients, with dropout too: the backward regenerates the forward's keep mask
    grads = torch.autograd.grad(out, (q, k, v), do)
    grads_pt = torch.autograd.grad(pt, (q, k, v), do)
    for nm, gg, gp in zip(("dq", "dk", "dv"), grads, grads_pt):
        ref = torch.from_numpy(g[nm]).to(dev)
        e, ep = (gg.float() - ref).abs().max().item(), (gp.float() - ref).abs().max().item()
        assert e <= 3 * ep + 1e-5, (nm, e, ep)
    # LSE2 (base-2 logsumexp) from the forward launcher itself
    with torch.no_grad():
        _, lse, _, _ = fwd_mod._flash_attn_forward(q, k, v, pad, bias, 0.0, m["causal"], None, None)
    ref_lse = torch.from_numpy(g["lse2"]).to(dev)
    got = lse[:, :, : m["sq"]]
    finite = torch.isfinite(ref_lse)
    if pad is not None:
        finite &= pad[:, None, :]
    assert torch.allclose(got[finite], ref_lse[finite], rtol=1e-3, atol=1e-3), (got[finite] - ref_lse[finite]).abs().max()
    assert torch.all(torch.isneginf(got[~torch.isfinite(ref_lse)]))
