"""Where a hand-placed kernel's time goes, from s_memtime stamps (dev tool).

Needs the stamp build:  FA2_HIPCC_FLAGS=-DFA2_HP_STAMPS=1 FA2_BUILD_DIR=fa2_triton_amd/_build_stamps
FA2_LIB_OUT=fa2_triton_amd/libfa2_amd_stamps.so python -m fa2_triton_amd.build
Run: python scripts/hp_stamps.py   (loads libfa2_amd_stamps.so through FA2_AMD_LIB)
Per wave and unit (cycles of the shader clock): the statement, its prologue wait, the period-end
waits (own LDS reads + DMA), the barrier waits, and the epilogue after the statement.
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("FA2_AMD_LIB", os.path.join(HERE, "..", "fa2_triton_amd", "libfa2_amd_stamps.so"))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from fa2_triton_amd import _lib  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402

lib = _lib.load()
rd = lib.fa2_debug_hp_stamps
rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]


def stamps():
    buf = (ctypes.c_ulonglong * 16)()
    assert rd(buf) == 0
    return list(buf)


for causal in (True, False):
    for S, B in ((4096, 8), (16384, 2)):
        torch.manual_seed(0)
        q, k, v = (torch.randn(B, S, 32, 128, device="cuda", dtype=torch.bfloat16) * 0.5 for _ in range(3))
        _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        torch.cuda.synchronize()
        stamps()
        reps = 5
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        e1.record()
        torch.cuda.synchronize()
        st = stamps()
        units = st[5] / 4  # per wave
        nmb = S // 256
        tiles = B * 32 * (sum(mb + 1 for mb in range(nmb)) * 4 if causal else nmb * S // 64) * reps
        rec = {"kernel": "fwd_hp", "S": S, "B": B, "causal": causal, "ms": round(e0.elapsed_time(e1) / reps, 4),
               "units_per_wave_launches": units / reps}
        for name, i in (("dma_lds_wait", 0), ("barrier_wait", 1), ("prologue_wait", 2), ("statement", 3), ("epilogue", 4)):
            rec[name + "_cyc_per_unit"] = round(st[i] / st[5], 1)
        rec["periods_per_unit"] = round(tiles / (st[5] / 4), 2)
        rec["statement_cyc_per_period"] = round(st[3] / st[5] / rec["periods_per_unit"], 1)
        rec["dma_lds_wait_frac"] = round(st[0] / st[3], 4)
        rec["barrier_wait_frac"] = round(st[1] / st[3], 4)
        rec["prologue_wait_frac"] = round(st[2] / st[3], 4)
        rec["epilogue_over_statement"] = round(st[4] / st[3], 4)
        print(json.dumps(rec), flush=True)
