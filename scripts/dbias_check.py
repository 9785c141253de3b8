"""Bitwise comparison of the bias gradient across libfa2_amd.so builds (A/B of dbias_kernel
variants whose per-element arithmetic is unchanged).  usage: python scripts/dbias_check.py base.so cand.so [...]
Shapes: cfg3-like [1,1,S,S] broadcast (summed over every pair), [B,1,S,S], [1,H,S,S], ragged S,
GQA, causal and not."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fa2_triton_amd._lib as L  # noqa: E402
from fa2_triton_amd.backward import _flash_attn_backward  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402

libs = [(os.path.basename(os.path.dirname(p)), L.bind(ctypes.CDLL(os.path.abspath(p)))) for p in sys.argv[1:]]
cases = [  # B, Hq, Hkv, Sq, Sk, bias batch, bias heads, causal
    (2, 8, 8, 1024, 1024, 1, 1, True), (2, 8, 8, 1024, 1024, 1, 1, False),
    (2, 8, 2, 777, 1031, 2, 1, True), (3, 6, 3, 333, 200, 1, 6, False), (2, 4, 4, 4096, 4096, 1, 1, True),
    (1, 4, 1, 190, 270, 1, 4, True),
]
bad = 0
for (b, hq, hkv, sq, sk, bb, bh, causal) in cases:
    torch.manual_seed(0)
    q = torch.randn(b, sq, hq, 128, device="cuda", dtype=torch.bfloat16) * 0.5
    k = torch.randn(b, sk, hkv, 128, device="cuda", dtype=torch.bfloat16) * 0.5
    v = torch.randn(b, sk, hkv, 128, device="cuda", dtype=torch.bfloat16) * 0.5
    do = torch.randn_like(q)
    bias = torch.randn(bb, bh, sq, sk, device="cuda", dtype=torch.bfloat16)
    outs = []
    for name, lib in libs:
        L._lib = lib
        o, lse, scale, _ = _flash_attn_forward(q, k, v, None, bias, 0.0, causal, None, None)
        g = _flash_attn_backward(do, q, k, v, bias, None, o, lse, 0.0, causal, scale, None, bias_grad=True)
        torch.cuda.synchronize()
        outs.append((name, g[3].float()))
    for name, g in outs[1:]:
        same = torch.equal(g, outs[0][1])
        diff = (g - outs[0][1]).abs().max().item()
        bad += not same
        print(f"{(b, hq, hkv, sq, sk, bb, bh, causal)} {name}: {'bitwise equal' if same else 'DIFFERS'} max|d|={diff:.3g}")
print("ALL EQUAL" if not bad else f"{bad} DIFFER")
sys.exit(1 if bad else 0)
