"""Philox4x32-10 exactly as Triton's `tl.rand` (TEST INFRASTRUCTURE ONLY).

The reference's dropout draws `keep = tl.rand(seed, off) > p`
(/root/reference/src/forward/compute_row_blocks.py:76-79) with the flat offset
off = Sk * (cu_q + Sq * (h + Hq * b)) + m * Sk + n (/root/reference/src/forward/kernel.py:146-148),
and its test builds the same mask over a dense (B, Hq, Sq, Sk) tensor
(/root/reference/tests/utils.py:169-207).  `tl.rand` is third-party code: Triton 3.6.0 as
installed in this image, triton/language/random.py --
  philox_impl :13-43    10 rounds, round mults A=0xD2511F53 / B=0xCD9E8D57,
                        key bumps 0x9E3779B9 / 0xBB67AE85;
  philox      :46-70    key = (seed_lo, seed_hi) of the 64-bit seed;
  randint4x   :89-111   counter = (off_lo, off_hi, 0, 0); the first output word is used;
  uint_to_uniform_float :127-144   bitcast to int32 x, x<0 -> -x-1, times 4.6566127342e-10 (f32).
This module restates that algorithm in numpy.  It is pinned by a known-answer vector captured
from the Triton interpreter (tests/golden/philox_kat.npz, tests/golden/make_philox_kat.py).
"""
import numpy as np

ROUND_A = np.uint64(0xD2511F53)
ROUND_B = np.uint64(0xCD9E8D57)
KEY_A = np.uint32(0x9E3779B9)
KEY_B = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox_first_word(seed: int, offsets: np.ndarray, rounds: int = 10) -> np.ndarray:
    """First uint32 output word of Philox4x32 for counters (off_lo, off_hi, 0, 0)."""
    off = np.asarray(offsets, dtype=np.uint64)
    c0 = (off & MASK32).astype(np.uint32)
    c1 = (off >> np.uint64(32)).astype(np.uint32)
    c2 = np.zeros_like(c0)
    c3 = np.zeros_like(c0)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32(seed >> 32)
    with np.errstate(over="ignore"):
        for _ in range(rounds):
            pa = ROUND_A * c0.astype(np.uint64)   # A * c0 (64-bit product)
            pb = ROUND_B * c2.astype(np.uint64)   # B * c2
            n0 = (pb >> np.uint64(32)).astype(np.uint32) ^ c1 ^ k0
            n2 = (pa >> np.uint64(32)).astype(np.uint32) ^ c3 ^ k1
            n1 = (pb & MASK32).astype(np.uint32)
            n3 = (pa & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = n0, n1, n2, n3
            k0 = np.uint32((int(k0) + int(KEY_A)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(KEY_B)) & 0xFFFFFFFF)
    return c0


def uint_to_uniform(x: np.ndarray) -> np.ndarray:
    """Triton's uint32 -> [0, 1) float32 conversion (random.py:127-144)."""
    xi = x.view(np.int32).astype(np.int64)
    xi = np.where(xi < 0, -xi - 1, xi)
    return xi.astype(np.float32) * np.float32(4.6566127342e-10)


def rand(seed: int, offsets: np.ndarray) -> np.ndarray:
    """numpy `tl.rand(seed, offsets)`."""
    return uint_to_uniform(philox_first_word(seed, offsets))


def dropout_keep_mask(seed: int, p: float, batch: int, heads: int, seqlen_q: int, seqlen_k: int) -> np.ndarray:
    """Dense (B, Hq, Sq, Sk) keep-mask over the flat index, as tests/utils.py:169-207 there."""
    n = batch * heads * seqlen_q * seqlen_k
    u = rand(seed, np.arange(n, dtype=np.uint64))
    return (u > np.float32(p)).reshape(batch, heads, seqlen_q, seqlen_k)


# ---------------------------------------------------------------------------------------------
# The same generator in torch int64 arithmetic, so GPU tests can build large masks on the device.
_M32 = 0xFFFFFFFF


def _mulhilo32(a: int, c):
    """(hi32, lo32) of a * c for a python uint32 constant and an int64 tensor of uint32 values."""
    c_lo = c & 0xFFFF
    c_hi = c >> 16
    t = a * c_lo            # < 2^48
    u = a * c_hi            # < 2^48
    hi = (u + (t >> 16)) >> 16
    lo = (t + ((u & 0xFFFF) << 16)) & _M32
    return hi & _M32, lo


def rand_torch(seed: int, offsets):
    """torch `tl.rand(seed, offsets)` for an int64 tensor of non-negative offsets (any device)."""
    import torch

    off = offsets.to(torch.int64)
    c0 = off & _M32
    c1 = (off >> 32) & _M32
    c2 = torch.zeros_like(c0)
    c3 = torch.zeros_like(c0)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0, k1 = seed & _M32, seed >> 32
    for _ in range(10):
        hb, lb = _mulhilo32(0xCD9E8D57, c2)
        ha, la = _mulhilo32(0xD2511F53, c0)
        c0, c1, c2, c3 = hb ^ c1 ^ k0, lb, ha ^ c3 ^ k1, la
        k0 = (k0 + 0x9E3779B9) & _M32
        k1 = (k1 + 0xBB67AE85) & _M32
    x = torch.where(c0 >= 2**31, c0 - 2**32, c0)      # bitcast to int32
    x = torch.where(x < 0, -x - 1, x)
    return x.to(torch.float32) * 4.6566127342e-10


def dropout_keep_mask_torch(seed: int, p: float, batch: int, heads: int, seqlen_q: int, seqlen_k: int, device=None):
    import torch

    n = batch * heads * seqlen_q * seqlen_k
    u = rand_torch(seed, torch.arange(n, dtype=torch.int64, device=device))
    return (u > torch.tensor(p, dtype=torch.float32, device=device)).view(batch, heads, seqlen_q, seqlen_k)
