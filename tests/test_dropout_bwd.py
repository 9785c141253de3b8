"""Backward with dropout -- SURVEY.md section 8(f) rank 2 (the reference raises, src/utils.py:88).

The forward draws its keep mask with Philox (tl.rand semantics, oracle/philox.py); the backward
kernels regenerate the same bits from the seed the forward returned and differentiate
O = (P * M / (1 - p)) V exactly.  The oracle applies the identical mask (dropout_keep_mask_torch),
so the acceptance rule is the reference tests' compare_results_fa on O, dQ, dK, dV, as for the
no-dropout grid.  Also checked: two backward passes from the same forward are bitwise equal.
"""
import pytest
import torch

from tests.core import generate_test_data, run_case

CASES = [
    # b, hq, hkv, sq, sk, d, causal, p, dtype
    (2, 4, 4, 128, 128, 64, False, 0.1, torch.float16),
    (2, 4, 2, 239, 301, 128, True, 0.17, torch.bfloat16),
    (1, 3, 3, 1, 239, 40, False, 0.1, torch.float16),
    (2, 2, 1, 512, 512, 128, True, 0.3, torch.bfloat16),
    (3, 2, 2, 127, 513, 96, False, 0.1, torch.bfloat16),
    (1, 2, 2, 203, 113, 256, True, 0.1, torch.float16),
    (2, 8, 2, 1024, 1024, 128, True, 0.1, torch.float16),
]


@pytest.mark.gpu
@pytest.mark.parametrize("b,hq,hkv,sq,sk,d,causal,p,dtype", CASES, ids=lambda x: str(x).replace("torch.", ""))
def test_fwd_bwd_with_dropout(b, hq, hkv, sq, sk, d, causal, p, dtype):
    run_case(b, hq, hkv, sq, sk, d, causal, p, False, False, dtype, forward_only=False)


@pytest.mark.gpu
def test_dropout_backward_is_deterministic():
    from fa2_triton_amd import flash_attn_func

    q, k, v, do = generate_test_data(2, 4, 2, 333, 333, 128, torch.bfloat16)
    out = flash_attn_func(q, k, v, None, None, 0.2, True, None, 4242)
    g1 = torch.autograd.grad(out, (q, k, v), do, retain_graph=True)
    g2 = torch.autograd.grad(out, (q, k, v), do)
    for a, b_ in zip(g1, g2):
        assert torch.equal(a, b_)
