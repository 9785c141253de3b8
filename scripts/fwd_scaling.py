"""Forward time vs sequence length (fixed B*H), to separate per-tile from per-workgroup costs."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--tokens", type=int, default=32768, help="B*S, constant over the sweep")
ap.add_argument("--seqlens", default="1024,2048,4096,8192")
ap.add_argument("--causal", default="0,1")
args = ap.parse_args()
h, d = args.heads, args.d
for causal in [bool(int(c)) for c in args.causal.split(",")]:
    for s in [int(x) for x in args.seqlens.split(",")]:
        bb = max(1, args.tokens // s)  # keep B*S constant: same number of query blocks
        q = torch.empty(bb, s, h, d, device="cuda", dtype=torch.bfloat16).normal_(0, 0.5)
        k = torch.empty_like(q).normal_(0, 0.5)
        v = torch.empty_like(q).normal_(0, 0.5)
        fn = lambda: _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 10
        fl = 4 * bb * h * s * s * d * (0.5 if causal else 1.0)
        tiles = bb * h * (s // 128) * (s // 64) * (0.5 if causal else 1.0)
        print(f"causal={causal} B={bb} S={s}: {t:.3f} ms {fl / t / 1e9:.0f} TFLOP/s  "
              f"{t * 1e3 / (bb * h * (s // 128)) * 512:.2f} us per WG-slot-item, {t * 1e6 / tiles * 512:.3f} us per tile-slot")
