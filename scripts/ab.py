"""A/B timing of several libfa2_amd.so builds in ONE process (interleaved rounds), cfg3 causal.

usage: python scripts/ab.py lib_a.so lib_b.so[:ENV=VAL,...] [...]   (env CAUSAL=0 for non-causal, WHAT=fwd,bwd,
       SHAPE=B,H,S,D, DROPOUT=p (the forward saves its keep words, the backward reads them); a
       ":ENV=VAL" suffix sets those variables while that arm runs)
WHAT: fwd | dkdv, dq (backward stages) | bwd (whole backward) | dqb, dkdvb (the stages with a
      [1,1,S,S] bf16 bias) | dbias (bias-gradient stage alone,
      [1,1,S,S] bias summed over every (batch, head) pair)
"""
import ctypes
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fa2_triton_amd._lib as L  # noqa: E402
from fa2_triton_amd.backward import _flash_attn_backward  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402
from fa2_triton_amd.utils import dropout_mask_words  # noqa: E402

libs = []
envs = {}
for arg in sys.argv[1:]:
    path, _, env = arg.partition(":")
    lib = ctypes.CDLL(os.path.abspath(path))
    lib = L.bind(lib)
    name = os.path.join(os.path.basename(os.path.dirname(os.path.abspath(path))), os.path.basename(path)) + (":" + env if env else "")
    envs[name] = dict(kv.split("=", 1) for kv in env.split(",")) if env else {}
    libs.append((name, lib))

b, h, s, d = (int(x) for x in os.environ.get("SHAPE", "8,32,4096,128").split(","))  # B, H, S, D
causal = os.environ.get("CAUSAL", "1") == "1"
what = os.environ.get("WHAT", "fwd,dkdv,dq").split(",")
torch.manual_seed(0)
q = torch.empty(b, s, h, d, device="cuda", dtype=torch.bfloat16).normal_(0, 0.5)
k = torch.empty(b, s, h, d, device="cuda", dtype=torch.bfloat16).normal_(0, 0.5)
v = torch.empty(b, s, h, d, device="cuda", dtype=torch.bfloat16).normal_(0, 0.5)
do = torch.randn_like(q)
pd = float(os.environ.get("DROPOUT", "0"))
seed = 1234 if pd > 0 else None
kmask = torch.empty(dropout_mask_words(b, h, s, s), dtype=torch.int32, device="cuda") if pd > 0 else None
F = 4 * b * h * s * s * d * (0.5 if causal else 1.0)
flops = {"fwd": F, "dkdv": 2 * F, "dq": 1.5 * F, "bwd": 2.5 * F, "dbias": F, "dqb": 1.5 * F, "dkdvb": 2 * F}
bias = torch.randn(1, 1, s, s, device="cuda", dtype=torch.bfloat16) if {"dbias", "dqb", "dkdvb"} & set(what) else None
results = {(n, w): [] for n, _ in libs for w in what}
for rnd in range(5):
    for name, lib in libs:
        L._lib = lib
        for kv in envs.values():
            for k_ in kv:
                os.environ.pop(k_, None)
        os.environ.update(envs[name])
        fw = dict(dropout_mask=kmask)
        # (with a bias arm the saved O / LSE are the biased forward's, as in training)
        o, lse, scale, _ = _flash_attn_forward(q, k, v, None, bias, pd, causal, None, seed, **fw)
        delta = torch.empty_like(lse)
        _flash_attn_backward(do, q, k, v, bias, None, o, lse, pd, causal, scale, seed, _stages=1, _delta=delta, **fw)
        calls = {
            "fwd": lambda: _flash_attn_forward(q, k, v, None, None, pd, causal, None, seed, **fw),
            "dkdv": lambda: _flash_attn_backward(do, q, k, v, None, None, o, lse, pd, causal, scale, seed, _stages=2, _delta=delta, **fw),
            "dq": lambda: _flash_attn_backward(do, q, k, v, None, None, o, lse, pd, causal, scale, seed, _stages=4, _delta=delta, **fw),
            "bwd": lambda: _flash_attn_backward(do, q, k, v, None, None, o, lse, pd, causal, scale, seed, **fw),
            "dqb": lambda: _flash_attn_backward(do, q, k, v, bias, None, o, lse, pd, causal, scale, seed, _stages=4, _delta=delta, **fw),
            "dkdvb": lambda: _flash_attn_backward(do, q, k, v, bias, None, o, lse, pd, causal, scale, seed, _stages=2, _delta=delta, **fw),
            "dbias": lambda: _flash_attn_backward(do, q, k, v, bias, None, o, lse, pd, causal, scale, seed, _stages=8,
                                                  _delta=delta, bias_grad=True, **fw),
        }
        for w in what:
            calls[w]()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                calls[w]()
            e1.record()
            torch.cuda.synchronize()
            results[(name, w)].append(e0.elapsed_time(e1) / 5)
for (name, w), ts in results.items():
    ts = sorted(ts)
    med = ts[len(ts) // 2]
    print(f"{name:28s} {w:5s} median {med:.3f} ms  min {ts[0]:.3f}  {flops[w] / med / 1e9:.0f} TFLOP/s executed")
