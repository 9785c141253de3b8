"""Host-overhead A/B of the forward launch path at cfg2 (B=8 Hq=16 S=1024 D=64): back-to-back
flash_attn_func forwards, wall time per call with the old (four stride() calls) and the new (one
stride() call) bshd_strides, alternating.  usage: python scripts/ab_host.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import fa2_triton_amd.backward as B
import fa2_triton_amd.forward as F
from fa2_triton_amd import flash_attn_func
from fa2_triton_amd.utils import bshd_strides as new


def old(x):
    assert x.stride(-1) == 1
    return x.stride(0), x.stride(1), x.stride(2)


q = torch.randn(8, 1024, 16, 64, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
res = {"old": [], "new": []}
for rep in range(6):
    for name, fn in (("old", old), ("new", new)) if rep % 2 == 0 else (("new", new), ("old", old)):
        F.bshd_strides = B.bshd_strides = fn
        for _ in range(50):
            flash_attn_func(q, k, v)
        torch.cuda.synchronize()
        t = time.perf_counter()
        n = 1000
        for _ in range(n):
            flash_attn_func(q, k, v)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t) / n * 1e6)
for name, xs in res.items():
    print(f"{name}: us per forward call {sorted(xs)}")
