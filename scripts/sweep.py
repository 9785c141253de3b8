"""Throughput sweep of the operator over sequence length, head dim and masking (context for
DESIGN.md; the headline number is bench.py's).  Total tokens per call fixed at 32k (B = 32768 /
S) with 32 heads, bf16, inputs resident in HBM; fwd and fwd+bwd through flash_attn_func, medians
of HIP-event-timed calls; TFLOP/s use the algorithmic count (fwd 4 B H S^2 D, x0.5 causal;
bwd 2.5x fwd).

usage: python scripts/sweep.py [--reps 10] [--dims 64,128] [--seqlens 1024,...]   (one JSON line per point)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd import flash_attn_func  # noqa: E402


def timed(fn, reps, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--dims", default="64,128", help="head dims")
    ap.add_argument("--seqlens", default="1024,2048,4096,8192,16384")
    args = ap.parse_args()
    h = 32
    for d in [int(x) for x in args.dims.split(",")]:
        for s in [int(x) for x in args.seqlens.split(",")]:
            b = max(1, args.tokens // s)
            for causal in (False, True):
                torch.manual_seed(0)
                q = torch.empty(b, s, h, d, device="cuda", dtype=torch.bfloat16).normal_(0, 0.5).requires_grad_()
                k = torch.empty_like(q).normal_(0, 0.5).requires_grad_()
                v = torch.empty_like(q).normal_(0, 0.5).requires_grad_()
                do = torch.randn_like(q)
                fl = 4.0 * b * h * s * s * d * (0.5 if causal else 1.0)

                def fwd():
                    with torch.no_grad():
                        flash_attn_func(q, k, v, causal=causal)

                def fwdbwd():
                    o = flash_attn_func(q, k, v, causal=causal)
                    torch.autograd.grad(o, (q, k, v), do)

                tf, tfb = timed(fwd, args.reps), timed(fwdbwd, args.reps)
                print(json.dumps({"B": b, "H": h, "S": s, "D": d, "causal": causal, "fwd_ms": round(tf, 4),
                                  "fwd_tflops": round(fl / tf / 1e9, 1), "fwdbwd_ms": round(tfb, 4),
                                  "fwdbwd_tflops": round(3.5 * fl / tfb / 1e9, 1)}), flush=True)
                del q, k, v, do


if __name__ == "__main__":
    main()
