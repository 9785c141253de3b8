"""Where the hand-placed forward's time goes, from s_memtime stamps (dev tool).

Needs a stamp build (scripts/fwd_stamp_abl.sh builds them, with optional timing ablations):
  FA2_HIPCC_FLAGS=-DFA2_HP_STAMPS=1 ... -> ab_libs/NAME.so
Run: python scripts/hp_stamps.py ab_libs/NAME.so [...]   (each library in a child process)
Per wave and unit (cycles of the shader clock): the statement, its phases -- X (QK^T(i+1) with the
exponentials of tile i: from the period start to the first PV MFMA's region), Y (PV(i) with the row
sums and the next tile's mask / row max, then the vote), the period-end waits + barrier (plus the
unit's prologue wait) -- and the epilogue after the statement.
"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def run_one(lib_path, cases):
    os.environ["FA2_AMD_LIB"] = os.path.abspath(lib_path)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch

    from fa2_triton_amd import _lib
    from fa2_triton_amd.forward import _flash_attn_forward

    lib = _lib.load()
    rd = lib.fa2_debug_hp_stamps
    rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]

    def stamps():
        buf = (ctypes.c_ulonglong * 16)()
        assert rd(buf) == 0
        return list(buf)

    for causal, S, B in cases:
        torch.manual_seed(0)
        q, k, v = (torch.randn(B, S, 32, 128, device="cuda", dtype=torch.bfloat16) * 0.5 for _ in range(3))
        for _ in range(3):
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
        nmb = S // 256
        tiles = B * 32 * (sum(mb + 1 for mb in range(nmb)) * 4 if causal else nmb * S // 64) * reps
        waves = st[5]  # units x waves
        periods = tiles / (waves / 4)
        rec = {"lib": os.path.basename(lib_path), "S": S, "B": B, "causal": causal,
               "ms": round(e0.elapsed_time(e1) / reps, 4), "periods_per_unit": round(periods, 2)}
        for name, i in (("phase_x", 0), ("phase_y", 1), ("waits", 2), ("statement", 3), ("epilogue", 4)):
            rec[name + "_cyc_per_period"] = round(st[i] / waves / periods, 1)
        rec["rest_cyc_per_unit"] = round((st[3] - st[0] - st[1] - st[2]) / waves, 1)
        rec["epilogue_cyc_per_unit"] = round(st[4] / waves, 1)
        # the epilogue's parts: accumulator read-out, then each 32-row block (1 / l, LSE, staging, stores)
        for name, i in (("readout", 6), ("block0", 7), ("block1", 8), ("pack_ldswrite", 9), ("readback", 10),
                        ("stores", 11)):
            rec[name + "_cyc_per_unit"] = round(st[i] / waves, 1)
        # cycles per SIMD per launch (one wave per SIMD) over the launch time: the in-kernel clock
        rec["clock_ghz"] = round((st[3] + st[4]) / 1024 / reps / (rec["ms"] * 1e6), 3)
        print(json.dumps(rec), flush=True)


CASES = [(False, 4096, 8), (False, 16384, 2), (True, 4096, 8)]

if __name__ == "__main__":
    if len(sys.argv) > 2 or (len(sys.argv) == 2 and sys.argv[1] != "--child"):
        rc = 0
        for lib in sys.argv[1:]:
            r = subprocess.run([sys.executable, __file__, "--child"], env=dict(os.environ, FA2_STAMP_LIB=lib))
            rc = rc or r.returncode
            if r.returncode:
                break
        sys.exit(rc)
    run_one(os.environ.get("FA2_STAMP_LIB", os.path.join(HERE, "..", "fa2_triton_amd", "libfa2_amd_stamps.so")), CASES)
