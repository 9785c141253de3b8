"""pytest configuration: the `gpu` marker and the repo root on sys.path.

`-m "not gpu"` tests run on the CPU (oracle vs golden vectors, host logic, C-ABI exports,
gloo multi-rank logic); `-m gpu` tests need an MI355X and call the HIP kernels through the
C ABI.  The oracle in `oracle/` is imported here only as the checker.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
