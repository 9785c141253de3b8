"""Forward-only parity grid with bias and dropout -- /root/reference/tests/test_fwd_only.py:7-63.

Same 1280-case grid (bias always on, dropout {0, 0.1}); the dropout keep-mask the oracle
applies comes from oracle/philox.py (bit-identical to Triton's tl.rand, the RNG of the
reference kernel and of its test mask), so dropout parity is exact, not statistical.
All of it by default; FA2_GRID_STRIDE=N runs a deterministic 1-in-N subset.
"""
import itertools
import os
import zlib

import pytest
import torch

from tests.core import run_case

STRIDE = int(os.environ.get("FA2_GRID_STRIDE", "1"))

SEQLENS = [(1, 239), (3, 799), (127, 512), (127, 513), (113, 203), (128, 217), (113, 211), (108, 256), (256, 512),
           (1023, 1024)]
GRID = list(itertools.product([torch.float16, torch.bfloat16], [0, 0.1], [False, True], [32, 40, 59, 64, 80, 96, 111, 128],
                              [(False, False, True), (True, False, True)], SEQLENS, [9], [4]))
def case_id(c) -> str:
    dt = "f16" if c[0] == torch.float16 else "bf16"
    sw, att, bias = c[4]
    mode = ("swap" if sw else "") + ("mask" if att else "") + ("bias" if bias else "") or "plain"
    heads = c[6] if isinstance(c[6], tuple) else (c[6], c[6])
    return f"{dt}-p{c[1]}-{'causal' if c[2] else 'full'}-d{c[3]}-{mode}-s{c[5][0]}x{c[5][1]}-h{heads[0]}x{heads[1]}"


SELECTED = [c for c in GRID if zlib.crc32(repr(c).encode()) % STRIDE == 0]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,dropout_p,causal,head_dim,mode,seqlens,num_heads,batch_size", SELECTED, ids=[case_id(c) for c in SELECTED])
def test_fwd_only(dtype, dropout_p, causal, head_dim, mode, seqlens, num_heads, batch_size):
    swap_seqlens, use_attention, use_bias = mode
    seqlen_q, seqlen_k = seqlens
    if swap_seqlens:
        seqlen_q, seqlen_k = seqlen_k, seqlen_q
    if use_attention:
        seqlen_q = seqlen_k
    run_case(batch_size, num_heads, num_heads, seqlen_q, seqlen_k, head_dim, causal, dropout_p, use_attention, use_bias,
             dtype, forward_only=True)
