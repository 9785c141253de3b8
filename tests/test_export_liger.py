"""Liger-style packaging (/root/reference/export_to_liger.py:6-34).

The exported `liger_kernel.ops.flash_attention` must import on its own (relative imports, the
library next to it), expose the reference's entry points, and bind the same C ABI.
"""
import importlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_export_imports_as_liger_op(tmp_path):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "export_to_liger.py"), str(tmp_path)],
                         capture_output=True, text=True, check=True).stdout.split()
    dst = tmp_path / "src" / "liger_kernel" / "ops" / "flash_attention"
    assert str(dst / "wrapper.py") in out and (dst / "include" / "fa2_amd.h").exists()
    assert (dst / "csrc" / "bwd_kernel.h").exists() and (dst / "build.py").exists()
    assert not any("oracle" in p or "tests" in p for p in out)
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import liger_kernel.ops.flash_attention as fa\n"
        "from liger_kernel.ops.flash_attention import _lib\n"
        "assert callable(fa.flash_attn_func) and fa.FlashAttnFunc.apply\n"
        "assert _lib.LIB_PATH.startswith(%r)\n"
        "lib = _lib.load(); [getattr(lib, s) for s in _lib.EXPORTED_SYMBOLS]\n"
        "from liger_kernel.ops.flash_attention import build\n"
        "assert build.INCLUDE == %r\n"
        "print('ok')\n" % (str(tmp_path / "src"), str(dst), str(dst / "include"))
    )
    env = {k: v for k, v in os.environ.items() if k != "FA2_AMD_LIB"}
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=str(tmp_path))
    assert res.returncode == 0 and "ok" in res.stdout, res.stderr


def test_export_never_deletes_foreign_files(tmp_path):
    """A re-export refreshes only the files its manifest lists; a directory the script did not
    write is refused without --force (the old export ran rmtree on it)."""
    script = os.path.join(ROOT, "scripts", "export_to_liger.py")
    dst = tmp_path / "src" / "liger_kernel" / "ops" / "flash_attention"
    dst.mkdir(parents=True)
    (dst / "mine.py").write_text("x = 1\n")
    res = subprocess.run([sys.executable, script, str(tmp_path), "--no-lib"], capture_output=True, text=True)
    assert res.returncode != 0 and "--force" in res.stderr
    subprocess.run([sys.executable, script, str(tmp_path), "--no-lib", "--force"], check=True, capture_output=True)
    assert (dst / "mine.py").read_text() == "x = 1\n" and (dst / "wrapper.py").exists()
    (dst / "wrapper.py").write_text("stale\n")
    subprocess.run([sys.executable, script, str(tmp_path), "--no-lib"], check=True, capture_output=True)
    assert (dst / "mine.py").exists() and (dst / "wrapper.py").read_text() != "stale\n"


def test_export_manifest_cannot_reach_outside_or_adopt_foreign_files(tmp_path):
    """manifest entries that leave the export directory ('..', absolute paths) are
    ignored on refresh, and a --force export does not adopt the foreign files it overwrote (so a
    later refresh does not delete them)."""
    script = os.path.join(ROOT, "scripts", "export_to_liger.py")
    dst = tmp_path / "src" / "liger_kernel" / "ops" / "flash_attention"
    dst.mkdir(parents=True)
    (dst / "utils.py").write_text("foreign = True\n")  # same name as a package file
    subprocess.run([sys.executable, script, str(tmp_path), "--no-lib", "--force"], check=True, capture_output=True)
    manifest = (dst / ".fa2_export_manifest").read_text().split()
    assert "utils.py" not in manifest and "wrapper.py" in manifest
    outside = tmp_path / "outside.txt"
    outside.write_text("keep\n")
    (dst / ".fa2_export_manifest").write_text("\n".join(manifest + ["../../../../outside.txt", str(outside)]) + "\n")
    subprocess.run([sys.executable, script, str(tmp_path), "--no-lib"], check=True, capture_output=True)
    assert outside.read_text() == "keep\n"
    assert (dst / "utils.py").exists()
