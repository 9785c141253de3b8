"""Build libfa2_amd.so (gfx950) in-tree with hipcc.

The kernels are templates (dtype x head-dim tile x causal x bias x dropout x aligned); each
(dtype, head-dim tile) pair is instantiated in its own generated translation unit so that
the compile runs in parallel.  Usage: `python -m fa2_triton_amd.build [--force] [-j N]`.
"""
import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
GEN = os.path.join(CSRC, "gen")
OBJ = os.environ.get("FA2_BUILD_DIR", os.path.join(HERE, "_build"))
LIB = os.environ.get("FA2_LIB_OUT", os.path.join(HERE, "libfa2_amd.so"))
# the C ABI header: the repo's include/, or a copy inside the package (scripts/export_to_liger.py)
INCLUDE = next((d for d in (os.path.join(HERE, "include"), os.path.join(os.path.dirname(HERE), "include"))
                if os.path.exists(os.path.join(d, "fa2_amd.h"))), os.path.join(os.path.dirname(HERE), "include"))
ARCH = os.environ.get("FA2_OFFLOAD_ARCH", "gfx950")

DTYPES = {"bf16": "true", "f16": "false"}
TILES = (32, 64, 128, 256)


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm at /opt/rocm)")


def generated_sources():
    os.makedirs(GEN, exist_ok=True)
    srcs = []
    for kind in ("fwd", "bwd"):
        for dname, flag in DTYPES.items():
            for dt in TILES:
                path = os.path.join(GEN, f"{kind}_{dname}_d{dt}.hip")
                extra = ", int" if kind == "bwd" else ""
                body = (
                    f'#include "../{kind}_kernel.h"\n'
                    f"namespace fa2 {{\n"
                    f"template hipError_t launch_{kind}_dt<{flag}, {dt}>(const fa2_{kind}_args&, bool{extra}, hipStream_t);\n"
                    f"}}\n"
                )
                if not os.path.exists(path) or open(path).read() != body:
                    with open(path, "w") as f:
                        f.write(body)
                srcs.append(path)
    return srcs


def generated_headers():
    """The hand-placed instruction streams (hp_gen.py -> csrc/gen/*.h), rewritten only on change."""
    sys.path.insert(0, os.path.dirname(HERE))
    try:
        from fa2_triton_amd import hp_gen
    finally:
        sys.path.pop(0)
    return hp_gen.write_headers()


def deps_mtime() -> float:
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hip"))]
    files += [os.path.join(GEN, f) for f in os.listdir(GEN) if f.endswith(".h")]
    files.append(os.path.join(HERE, "hp_gen.py"))
    files.append(os.path.join(INCLUDE, "fa2_amd.h"))
    files.append(os.path.abspath(__file__))
    return max(os.path.getmtime(f) for f in files)


def compile_one(src: str, force: bool, dep_t: float) -> str:
    obj = os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o"))
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(dep_t, os.path.getmtime(src)):
        return obj
    # development A/B builds: FA2_BUILD_ONLY=fwd_bf16_d128,... recompiles only those units and
    # keeps every other existing object as it is
    only = os.environ.get("FA2_BUILD_ONLY")
    if only and os.path.exists(obj) and not any(tok in os.path.basename(src) for tok in only.split(",")):
        return obj
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
           "-I", CSRC, "-I", INCLUDE, "-Wno-unused-result"]
    # MFMA accumulators in arch VGPRs (where the softmax VALU reads them)
    cmd += ["-mllvm", "-amdgpu-mfma-vgpr-form=true",
           # no SLP packing of the softmax adds into v_pk_add_f32: packed f32 VALU beside MFMAs
           # costs more issue cycles than the scalar pair (MI355X_MICROARCH.md, filler prices)
           "-fno-slp-vectorize"]
    extra = os.environ.get("FA2_HIPCC_FLAGS")
    if extra:
        cmd += extra.split()
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return obj


DEFAULT_LIB = os.path.join(HERE, "libfa2_amd.so")


def check_dev_env():
    """Development builds (timing ablations FA2_HPGEN_ABL, whose outputs are wrong; the stamp or
    dev variants -DFA2_HP_STAMPS / -DFA2_HP_DEV) never overwrite the shipped library or its objects."""
    dev = [k for k in ("FA2_HPGEN_ABL",) if os.environ.get(k)]
    flags = os.environ.get("FA2_HIPCC_FLAGS", "")
    dev += [f for f in ("FA2_HP_STAMPS", "FA2_HP_DEV") if f in flags]
    if dev and (os.path.abspath(LIB) == os.path.abspath(DEFAULT_LIB) or
                os.path.abspath(OBJ) == os.path.abspath(os.path.join(HERE, "_build"))):
        raise RuntimeError(f"development build ({', '.join(dev)}) must set FA2_LIB_OUT and FA2_BUILD_DIR away from "
                           f"the shipped library ({DEFAULT_LIB}) and its objects")


def build(force: bool = False, jobs: int = 0) -> str:
    check_dev_env()
    os.makedirs(OBJ, exist_ok=True)
    generated_headers()
    srcs = [os.path.join(CSRC, "api.hip"), os.path.join(CSRC, "misc.hip")] + generated_sources()
    dep_t = deps_mtime()
    jobs = jobs or min(16, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: compile_one(s, force, dep_t), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, LIB)
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=0)
    args = ap.parse_args(argv)
    print(build(args.force, args.j))


if __name__ == "__main__":
    sys.exit(main())
