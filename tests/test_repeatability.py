"""Bitwise run-to-run determinism -- /root/reference/tests/test_repeatability.py:18-96.

The reference compares masked checksums of O, dQ, dK, dV over 10 repeats (:40-51) on its
active grid (:76-84: fp16, non-causal, padding mask, D=32, Sk=16, Sq in 20..300, B=3, H=1).
Here the comparison is stricter -- `torch.equal` on the whole tensors, NaN-free -- and the grid
adds causal, bf16, GQA and a multi-tile size, since the HIP backward is deterministic by
construction (no atomics: dK/dV and dQ each have exactly one writer per element).
"""
import pytest
import torch

from tests.core import generate_attention_mask, generate_test_data

REF_GRID = [(3, 1, 1, sq, 16, 32, True, False, torch.float16) for sq in (20, 32, 64, 79, 100, 164, 200, 239, 300)]
EXTRA = [
    (2, 4, 2, 517, 517, 128, False, True, torch.bfloat16),
    (2, 8, 2, 1024, 1024, 128, False, True, torch.bfloat16),
    (2, 4, 4, 300, 700, 64, False, False, torch.float16),
    (1, 2, 1, 2048, 2048, 256, False, True, torch.bfloat16),
    # causal D = 128 on the hand-placed kernels with several units per persistent workgroup
    (4, 32, 8, 2048, 2048, 128, False, True, torch.bfloat16),
    (2, 16, 16, 1536, 1536, 128, True, True, torch.float16),
]


def _run(q, k, v, do, mask, causal):
    from fa2_triton_amd import flash_attn_func

    out = flash_attn_func(q, k, v, mask, None, 0.0, causal)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), do)
    return [t.detach().clone() for t in (out, dq, dk, dv)]


@pytest.mark.gpu
@pytest.mark.parametrize("b,hq,hkv,sq,sk,d,attention,causal,dtype", REF_GRID + EXTRA,
                         ids=lambda x: str(x).replace("torch.", ""))
def test_repeatability(b, hq, hkv, sq, sk, d, attention, causal, dtype):
    if attention:
        sk = sq
    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, d, dtype)
    mask = generate_attention_mask(q) if attention else None
    first = _run(q, k, v, do, mask, causal)
    for t, name in zip(first, ("out", "dq", "dk", "dv")):
        assert not torch.isnan(t).any(), name
    for _ in range(9):
        again = _run(q, k, v, do, mask, causal)
        for a, b_, name in zip(first, again, ("out", "dq", "dk", "dv")):
            assert torch.equal(a, b_), name
