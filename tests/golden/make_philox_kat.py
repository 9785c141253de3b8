"""Capture a Philox known-answer vector from Triton's own `tl.rand` (run once, in the build
container only; the output tests/golden/philox_kat.npz is committed).

The reference's dropout mask is `tl.rand(seed, offsets) > p`
(/root/reference/src/forward/compute_row_blocks.py:78, /root/reference/tests/utils.py:193-207).
Triton 3.6.0 is installed here but there is no GPU, so this runs the Triton interpreter
(TRITON_INTERPRET=1) on a tiny kernel of our own that stores `tl.rand` for a range of int32 and
int64 offsets.  The numpy restatement in oracle/philox.py is checked against it by
tests/test_oracle.py.
"""
import os
import sys

os.environ["TRITON_INTERPRET"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402
import triton  # noqa: E402
import triton.language as tl  # noqa: E402


@triton.jit
def _rand_kernel(out_ptr, seed, base, n, BLOCK: tl.constexpr):
    offs = tl.program_id(0) * BLOCK + tl.arange(0, BLOCK)
    vals = tl.rand(seed, base + offs)
    tl.store(out_ptr + offs, vals, mask=offs < n)


def capture(seed: int, base: int, n: int) -> np.ndarray:
    out = torch.empty(n, dtype=torch.float32)
    blk = 256
    _rand_kernel[(triton.cdiv(n, blk),)](out, seed, base, n, BLOCK=blk)
    return out.numpy()


def main(path: str) -> None:
    cases = {
        # (seed, base offset, count): int32 offsets, a seed above 2^31, and int64 offsets
        "s123456789_b0": (123456789, 0, 4096),
        "s3000000000_b1000": (3000000000, 1000, 2048),
        "s42_b4294967000": (42, 4294967000, 1024),
        "s7_b8589934592": (7, 8589934592, 512),
    }
    arrays = {}
    for name, (seed, base, n) in cases.items():
        arrays[name] = capture(seed, base, n)
        arrays[name + "_meta"] = np.array([seed, base, n], dtype=np.uint64)
    np.savez_compressed(path, **arrays)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "philox_kat.npz"))
