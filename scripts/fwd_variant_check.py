"""Dev check: a forward variant (library B, with its env) against the default forward (library A)
on the same inputs -- O and LSE2 max differences over causal / non-causal, Sq != Sk, ragged and
GQA shapes.  The default forward is itself pinned to the oracle by the GPU suite.

usage: python scripts/fwd_variant_check.py base.so variant.so:ENV=VAL[,...]
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fa2_triton_amd._lib as L  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402


def load(arg):
    path, _, env = arg.partition(":")
    lib = L.bind(ctypes.CDLL(os.path.abspath(path)))
    return lib, dict(kv.split("=", 1) for kv in env.split(",")) if env else {}


(la, ea), (lb, eb) = load(sys.argv[1]), load(sys.argv[2])
shapes = [  # B, Hq, Hkv, Sq, Sk, D, causal
    (2, 4, 4, 4096, 4096, 128, True), (2, 4, 4, 4096, 4096, 128, False),
    (1, 8, 2, 1000, 1000, 128, True), (1, 8, 2, 1000, 1000, 128, False),
    (2, 3, 3, 300, 777, 128, True), (2, 3, 3, 777, 300, 128, True), (2, 3, 3, 777, 300, 128, False),
    (1, 2, 1, 1, 513, 128, True), (1, 2, 2, 257, 257, 128, True), (3, 2, 2, 64, 64, 128, False),
    (1, 2, 2, 8192, 8192, 128, True),
    (2, 4, 4, 1024, 1024, 64, False), (1, 4, 2, 777, 513, 64, False), (2, 2, 2, 100, 1000, 64, True),
]
worst = 0.0
for dt in (torch.bfloat16, torch.float16):
    for (B, Hq, Hkv, Sq, Sk, D, causal) in shapes:
        torch.manual_seed(0)
        q = torch.randn(B, Sq, Hq, D, device="cuda", dtype=dt) * 0.5
        k = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=dt) * 0.5
        v = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=dt) * 0.5
        outs = []
        for lib, env in ((la, ea), (lb, eb)):
            L._lib = lib
            for k_ in set(ea) | set(eb):
                os.environ.pop(k_, None)
            os.environ.update(env)
            o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
            torch.cuda.synchronize()
            outs.append((o.float(), lse[:, :, :Sq].float()))
        (oa, sa), (ob, sb) = outs
        do = (oa - ob).abs().max().item()
        fin = torch.isfinite(sa)
        same_inf = bool((fin == torch.isfinite(sb)).all())
        ds = (sa[fin] - sb[fin]).abs().max().item() if fin.any() else 0.0
        nan = bool(torch.isnan(ob).any())
        ref = oa.abs().max().item()
        worst = max(worst, do / max(ref, 1e-6))
        print(f"{str(dt):15s} B={B} Hq={Hq} Hkv={Hkv} Sq={Sq} Sk={Sk} causal={causal}: max|dO| {do:.3e} "
              f"(max|O| {ref:.3f}) max|dLSE2| {ds:.3e} inf-pattern-equal {same_inf} nan {nan}", flush=True)
        if nan or not same_inf or do > 2e-2 * max(ref, 1e-3) or ds > 1e-3:
            print("MISMATCH")
            sys.exit(1)
print(f"OK worst rel {worst:.3e}")
