"""Time the forward launcher at the bench workload with HIP events (for A/B of library builds)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd.backward import _flash_attn_backward  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402

b, h, s, d = 8, 32, 4096, 128
causal = os.environ.get("CAUSAL", "1") == "1"
torch.manual_seed(0)
q = torch.empty(b, s, h, d, device="cuda", dtype=torch.bfloat16).normal_(0, 0.5)
k = torch.empty(b, s, h, d, device="cuda", dtype=torch.bfloat16).normal_(0, 0.5)
v = torch.empty(b, s, h, d, device="cuda", dtype=torch.bfloat16).normal_(0, 0.5)
do = torch.randn_like(q)
f = 4 * b * h * s * s * d * (0.5 if causal else 1.0)
o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
for name, fn, flops in (("fwd", lambda: _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None), f),
                        ("bwd", lambda: _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.0, causal, None, None), 2.5 * f)):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10
    print(f"{os.environ.get('FA2_AMD_LIB', 'default')} {name}: {t:.3f} ms  {flops / t / 1e9:.1f} TFLOP/s")
