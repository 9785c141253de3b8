"""Per-launch time of the forward, dQ and dK/dV kernels over sequence length at a fixed token
count (B S = 32768, H = 32, D = 128, bf16): t(S) = a S + b separates the per-tile cost (a) from
the per-work-item cost (b).  Dev tool.  usage: python scripts/hp_scaling.py [--causal 0|1]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd.backward import _flash_attn_backward  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--causal", type=int, default=1)
ap.add_argument("--seqlens", default="512,1024,2048,4096,8192,16384")
ap.add_argument("--tokens", type=int, default=32768)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
causal = bool(a.causal)


def timed(fn, reps):
    fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    return ts[len(ts) // 2]


for s in [int(x) for x in a.seqlens.split(",")]:
    b = max(1, a.tokens // s)
    torch.manual_seed(0)
    q = torch.randn(b, s, 32, 128, device="cuda", dtype=torch.bfloat16) * 0.5
    k = torch.randn(b, s, 32, 128, device="cuda", dtype=torch.bfloat16) * 0.5
    v = torch.randn(b, s, 32, 128, device="cuda", dtype=torch.bfloat16) * 0.5
    do = torch.randn_like(q)
    o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
    delta = torch.empty_like(lse)
    rec = {"S": s, "B": b, "causal": causal}
    rec["fwd_ms"] = timed(lambda: _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None), a.reps)
    rec["dq_ms"] = timed(lambda: _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.0, causal, None, None,
                                                      _stages=4, _delta=delta), a.reps)
    rec["dkdv_ms"] = timed(lambda: _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.0, causal, None, None,
                                                        _stages=2, _delta=delta), a.reps)
    f = 4.0 * b * 32 * s * s * 128 * (0.5 if causal else 1.0)
    rec["fwd_tf"] = round(f / rec["fwd_ms"] / 1e9, 1)
    rec["dq_exec_tf"] = round(1.5 * f / rec["dq_ms"] / 1e9, 1)
    rec["dkdv_tf"] = round(2 * f / rec["dkdv_ms"] / 1e9, 1)
    print(json.dumps(rec), flush=True)
