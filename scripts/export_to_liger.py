"""Package the operator as Liger-Kernel's `liger_kernel.ops.flash_attention`.

The reference ships its Triton sources into a Liger-Kernel checkout the same way
(/root/reference/export_to_liger.py:6-34: copy src/** except other_implementations/ to
src/liger_kernel/ops/flash_attention/, rewriting `from src.` imports).  Here the package already
uses relative imports, so nothing is rewritten; what is copied is the Python host layer, the HIP
sources with their build script, the C ABI header (into the package's include/, where build.py
finds it) and the built gfx950 library when present -- the oracle and tests stay behind.

usage: python scripts/export_to_liger.py LIGER_CHECKOUT [--no-lib] [--force]
then:  import liger_kernel.ops.flash_attention as fa; fa.flash_attn_func(q, k, v, causal=True)
       (rebuild in place with `python -m liger_kernel.ops.flash_attention.build` if needed)
"""
import argparse
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fa2_triton_amd")
FA_DIR_IN_LIGER = os.path.join("src", "liger_kernel", "ops", "flash_attention")


MANIFEST = ".fa2_export_manifest"


def export(liger_root: str, with_lib: bool = True, force: bool = False) -> list:
    """Copy the package into the checkout.  A directory left by an earlier export (it holds the
    manifest of the files that export wrote) is refreshed: exactly those files are removed first,
    anything else in it is kept.  A directory without a manifest is someone else's: refused
    unless `force`, and even then only overwritten file by file, never deleted."""
    dst = os.path.join(liger_root, FA_DIR_IN_LIGER)
    manifest = os.path.join(dst, MANIFEST)
    root = os.path.realpath(dst)
    if os.path.exists(manifest):
        for rel in open(manifest).read().split():
            path = os.path.realpath(os.path.join(dst, rel))
            # only files inside the export directory: an absolute or '..' entry is ignored
            if os.path.commonpath([root, path]) == root and path != root and os.path.isfile(path):
                os.remove(path)
    elif os.path.exists(dst) and os.listdir(dst) and not force:
        raise SystemExit(f"{dst} exists and was not written by this script; pass --force to overwrite files in it")
    os.makedirs(os.path.join(dst, "csrc"), exist_ok=True)
    os.makedirs(os.path.join(dst, "include"), exist_ok=True)
    written, adopted = [], []

    def put(src, path):
        # a file that was there before this export (someone else's, reachable only with --force) is
        # overwritten but not adopted into the manifest, so a later refresh never deletes it
        (adopted if os.path.exists(path) else written).append(path)
        shutil.copy2(src, path)

    for name in sorted(os.listdir(PKG)):
        if name.endswith(".py") or (with_lib and name == "libfa2_amd.so"):
            put(os.path.join(PKG, name), os.path.join(dst, name))
    for name in sorted(os.listdir(os.path.join(PKG, "csrc"))):
        if name.endswith((".h", ".hip")):  # generated per-instantiation units are rebuilt by build.py
            put(os.path.join(PKG, "csrc", name), os.path.join(dst, "csrc", name))
    put(os.path.join(ROOT, "include", "fa2_amd.h"), os.path.join(dst, "include", "fa2_amd.h"))
    with open(manifest, "w") as f:
        f.write("\n".join(os.path.relpath(p, dst) for p in written) + "\n")
    return written + adopted


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("liger_root")
    ap.add_argument("--no-lib", action="store_true", help="do not copy the built libfa2_amd.so")
    ap.add_argument("--force", action="store_true", help="overwrite files in a directory this script did not write")
    args = ap.parse_args(argv)
    for path in export(args.liger_root, not args.no_lib, args.force):
        print(path)


if __name__ == "__main__":
    sys.exit(main())
