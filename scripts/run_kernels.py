"""Run the forward and/or backward launchers a few times at the bench workload (for profilers)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd.backward import _flash_attn_backward  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--what", default="fwd,bwd")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--b", type=int, default=8)
ap.add_argument("--h", type=int, default=32)
ap.add_argument("--hkv", type=int, default=0)
ap.add_argument("--s", type=int, default=4096)
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--causal", type=int, default=1)
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--disable", type=int, default=0, help="fa2_policy.disable bits (PATH_FWD_HP = 1, ...)")
a = ap.parse_args()
if a.disable:
    from fa2_triton_amd import _lib as L
    L.set_path_policy(a.disable, 0)
dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
hkv = a.hkv or a.h
torch.manual_seed(0)
q = torch.empty(a.b, a.s, a.h, a.d, device="cuda", dtype=dt).normal_(0, 0.5)
k = torch.empty(a.b, a.s, hkv, a.d, device="cuda", dtype=dt).normal_(0, 0.5)
v = torch.empty(a.b, a.s, hkv, a.d, device="cuda", dtype=dt).normal_(0, 0.5)
do = torch.randn_like(q)
o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, bool(a.causal), None, None)
for _ in range(a.reps):
    if "fwd" in a.what:
        _flash_attn_forward(q, k, v, None, None, 0.0, bool(a.causal), None, None)
    if "bwd" in a.what:
        _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.0, bool(a.causal), None, None)
torch.cuda.synchronize()
print("ok")
