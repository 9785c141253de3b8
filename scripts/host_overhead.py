"""Host-side cost of one operator call (the cfg2 step is ~46 us of GPU time, so the Python path
around the launch matters): wall time per call of back-to-back launches on a tiny problem, and
the pieces of the forward launcher timed on their own.  usage: python scripts/host_overhead.py"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd import _lib, flash_attn_func  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402
from fa2_triton_amd.utils import stream_of  # noqa: E402


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


q = torch.randn(1, 128, 1, 64, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
res = {
    "_flash_attn_forward": per_call(lambda: _flash_attn_forward(q, k, v, None, None, 0.0, False, None, None)),
    "flash_attn_func (no grad)": per_call(lambda: flash_attn_func(q, k, v)),
    "torch.empty x2": per_call(lambda: (torch.empty_like(q), torch.empty((1, 1, 128), device=q.device, dtype=torch.float32))),
    "current_stream().cuda_stream": per_call(lambda: torch.cuda.current_stream(q.device).cuda_stream),
    "stream_of (raw)": per_call(lambda: stream_of(q)),
    "torch.cuda.device ctx": per_call(lambda: torch.cuda.device(q.device).__enter__()),
    "FwdArgs()": per_call(lambda: _lib.FwdArgs()),
}
with torch.no_grad():
    qg = q.clone().requires_grad_()
    res["flash_attn_func (grad)"] = per_call(lambda: flash_attn_func(qg, k, v))
for kk, vv in res.items():
    print(f"{kk:28s} {vv:7.2f} us per call")
