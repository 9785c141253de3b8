"""Same-process A/B of the hand-placed kernels against the general ones (_lib.set_path_policy: the per-call fa2_policy):
forward times for a few shapes.  usage: python scripts/ab_policy.py [D]"""
import sys

import torch

from fa2_triton_amd import _lib as L
from fa2_triton_amd.forward import _flash_attn_forward

d = int(sys.argv[1]) if len(sys.argv) > 1 else 64
shapes = [(8, 16, 1024, False), (2, 16, 4096, False), (8, 32, 4096, True), (4, 16, 2048, True), (16, 16, 512, False)]
for b, h, s, causal in shapes:
    q = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16) * 0.5
    k = torch.randn_like(q) * 0.5
    v = torch.randn_like(q) * 0.5
    flops = 4 * b * h * s * s * d * (0.5 if causal else 1.0)
    res = {}
    for tag, dis in (("hp", 0), ("gen", L.PATH_FWD_HP)):
        L.set_path_policy(dis, 0)
        for _ in range(3):
            _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        torch.cuda.synchronize()
        ts = []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        res[tag] = ts[len(ts) // 2]
    L.set_path_policy(0, 0)
    print(f"B={b} H={h} S={s} D={d} causal={causal}: hp {res['hp']*1e3:.1f} us ({flops/res['hp']/1e9:.0f} TF)  "
          f"general {res['gen']*1e3:.1f} us ({flops/res['gen']/1e9:.0f} TF)", flush=True)
