"""Generate the golden attention vectors (run once, in the build container; outputs committed).

Oracle of record: the reference's own `flash_attn_reference`
(/root/reference/src/reference_implementation.py:38-123), imported standalone by file path
(the package `src` does not import under Triton 3.6).  For every case below
we store the seeded inputs (rounded to bf16 so the GPU tests can feed them bit-exactly), the
fp32 output O of the reference oracle, dQ/dK/dV by fp32 autograd through it for a seeded dO,
and LSE2 = logsumexp(scores) * log2(e) computed from the same fp32 scores.

Inputs follow the reference tests' generators (/root/reference/tests/utils.py:9-26): N(0, 0.5)
Q/K/V, N(0, 1) dO; bias is U[0,1) of shape [1,1,Sq,Sk] (/root/reference/tests/core.py:28);
padding masks are right-padded with one full row (/root/reference/tests/utils.py:40-56);
dropout masks come from oracle/philox.py (pinned separately against Triton's tl.rand).

Usage:  python tests/golden/make_golden.py [out.npz]
"""
import importlib.util
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle.philox import dropout_keep_mask  # noqa: E402

REF_FILE = "/root/reference/src/reference_implementation.py"

# name: (B, Hq, Hkv, Sq, Sk, D, causal, bias, padding, dropout_p)
CASES = {
    "cfg1_b2h4s128d64": (2, 4, 4, 128, 128, 64, False, False, False, 0.0),
    "causal_sq_lt_sk_gqa": (2, 4, 2, 113, 203, 40, True, False, False, 0.0),
    "causal_sq_gt_sk": (2, 2, 2, 203, 113, 64, True, False, False, 0.0),
    "bias_noncausal_d111": (2, 3, 3, 127, 130, 111, False, True, False, 0.0),
    "bias_causal_gqa": (1, 4, 1, 96, 160, 32, True, True, False, 0.0),
    "varlen_causal": (3, 2, 2, 97, 97, 64, True, False, True, 0.0),
    "varlen_noncausal_gqa": (3, 4, 2, 80, 80, 128, False, False, True, 0.0),
    "sq1": (2, 2, 1, 1, 239, 64, False, False, False, 0.0),
    "sq1_causal": (2, 2, 2, 1, 67, 32, True, False, False, 0.0),
    "dropout_bias": (2, 2, 2, 64, 96, 64, False, True, False, 0.17),
    "dropout_causal": (1, 3, 3, 100, 100, 48, True, False, False, 0.1),
    "d256_causal": (1, 2, 2, 70, 70, 256, True, False, False, 0.0),
}


def load_reference():
    spec = importlib.util.spec_from_file_location("fa2_reference_impl", REF_FILE)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.flash_attn_reference


def bf16_round(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).float()


def make_case(ref_fn, seed, b, hq, hkv, sq, sk, d, causal, use_bias, use_pad, p):
    g = torch.Generator().manual_seed(seed)
    q = bf16_round(torch.randn(b, sq, hq, d, generator=g) * 0.5)
    k = bf16_round(torch.randn(b, sk, hkv, d, generator=g) * 0.5)
    v = bf16_round(torch.randn(b, sk, hkv, d, generator=g) * 0.5)
    do = bf16_round(torch.randn(b, sq, hq, d, generator=g))
    bias = bf16_round(torch.rand(1, 1, sq, sk, generator=g)) if use_bias else None
    pad = None
    if use_pad:
        assert sq == sk
        pad = torch.ones(b, sq, dtype=torch.bool)
        lens = torch.randint(1, sq + 1, (b,), generator=g)
        lens[int(torch.randint(0, b, (1,), generator=g))] = sq
        for i in range(b):
            pad[i, int(lens[i]):] = False
    seed_drop, keep = 0, None
    if p > 0:
        seed_drop = int(torch.randint(0, 2**32, (1,), generator=g, dtype=torch.int64))
        keep = torch.from_numpy(dropout_keep_mask(seed_drop, p, b, hq, sq, sk))
    qq, kk, vv = (t.clone().requires_grad_() for t in (q, k, v))
    out = ref_fn(qq, kk, vv, query_padding_mask=pad, key_padding_mask=pad, attn_bias=bias,
                 dropout_p=p, dropout_mask=keep, causal=causal)
    dq, dk, dv = torch.autograd.grad(out, (qq, kk, vv), do)
    # LSE2 from the same fp32 scores (scale 1/sqrt(D), bias, key padding, causal window).
    kr = k.repeat_interleave(hq // hkv, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", q / math.sqrt(d), kr)
    if bias is not None:
        s = s + bias
    if pad is not None:
        s = s.masked_fill(~pad[:, None, None, :], float("-inf"))
    if causal:
        lq = pad.sum(-1).view(-1, 1, 1, 1) if pad is not None else sq
        lk = lq if pad is not None else sk
        rows = torch.arange(sq)[:, None]
        cols = torch.arange(sk)[None, :]
        s = s.masked_fill(cols > rows + lk - lq, float("-inf"))
    lse2 = torch.logsumexp(s, dim=-1) * 1.4426950408889634
    arrays = dict(q=q, k=k, v=v, do=do, out=out.detach(), dq=dq, dk=dk, dv=dv, lse2=lse2)
    if bias is not None:
        arrays["bias"] = bias
    if pad is not None:
        arrays["pad"] = pad
    if keep is not None:
        arrays["keep"] = keep
    res = {kname: t.numpy() for kname, t in arrays.items()}
    res["meta"] = np.array([b, hq, hkv, sq, sk, d, int(causal), int(use_bias), int(use_pad)], dtype=np.int64)
    res["dropout"] = np.array([p], dtype=np.float64)
    res["seed"] = np.array([seed_drop], dtype=np.uint64)
    return res


def main(path):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref_fn = load_reference()
    out = {}
    for i, (name, cfg) in enumerate(CASES.items()):
        arrays = make_case(ref_fn, 1000 + i, *cfg)
        for kname, a in arrays.items():
            out[f"{name}/{kname}"] = a
    np.savez_compressed(path, **out)
    print(f"wrote {len(CASES)} cases to {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "attention_golden.npz"))
