"""LSE2 returned by the forward launcher -- /root/reference/tests/test_logsumexp.py:1-77.

The reference's test imports `_flash_attn_forward` (:5) and compares its second output, the
base-2 logsumexp of the scaled (biased, masked) scores, with a dense recomputation scaled by
log2 e (:74); its own body is dead code (`raise NotImplementedError` at :27).  Here it runs:
the default configuration of that file (B=1, H=1, D=32, S=256, causal, dropout 0.17, fp16 --
dropout does not change the LSE, it uses the pre-dropout normaliser) plus GQA, padding masks,
bias, bottom-right causal with Sq > Sk (fully-masked rows -> -inf) and every head-dim tile.
Tolerance: 1e-3 abs/rel against oracle/reference.py:lse2_reference in fp32 on rows that see at
least one key; -inf exactly on rows that see none and on the padding rows beyond Sq.
"""
import pytest
import torch

from oracle.reference import lse2_reference
from tests.core import generate_attention_mask, generate_test_data

CASES = [
    # b, hq, hkv, sq, sk, d, causal, dropout, attention, bias, dtype
    (1, 1, 1, 256, 256, 32, True, 0.17, False, False, torch.float16),
    (2, 8, 2, 333, 333, 128, True, 0.0, True, False, torch.bfloat16),
    (2, 4, 4, 200, 77, 64, True, 0.0, False, False, torch.float16),
    (3, 2, 1, 129, 1000, 96, False, 0.1, False, True, torch.bfloat16),
    (1, 4, 2, 1024, 1024, 256, True, 0.0, False, False, torch.bfloat16),
    (2, 3, 3, 1, 239, 40, False, 0.0, False, True, torch.float16),
]


@pytest.mark.gpu
@pytest.mark.parametrize("b,hq,hkv,sq,sk,d,causal,p,attention,bias,dtype", CASES,
                         ids=lambda x: str(x).replace("torch.", ""))
def test_logsumexp(b, hq, hkv, sq, sk, d, causal, p, attention, bias, dtype):
    from fa2_triton_amd.forward import _flash_attn_forward

    if attention:
        sk = sq
    q, k, v, _ = generate_test_data(b, hq, hkv, sq, sk, d, dtype)
    mask = generate_attention_mask(q) if attention else None
    attn_bias = torch.rand(size=(1, 1, sq, sk), dtype=dtype, device=q.device) if bias else None
    seed = 1234 if p > 0 else None
    with torch.no_grad():
        _, lse, scale, _ = _flash_attn_forward(q, k, v, mask, attn_bias, p, causal, None, seed)
    assert lse.dtype == torch.float32 and lse.shape == (b, hq, ((sq + 127) // 128) * 128)
    ref = lse2_reference(q, k, attn_bias, causal, mask, scale)
    got = lse[:, :, :sq]
    seen = torch.isfinite(ref)
    if mask is not None:
        seen &= mask[:, None, :]
    torch.testing.assert_close(got[seen], ref[seen], rtol=1e-3, atol=1e-3)
    empty = ~torch.isfinite(ref)
    if mask is not None:
        empty &= mask[:, None, :]
    assert torch.all(torch.isneginf(got[empty]))
    assert torch.all(torch.isneginf(lse[:, :, sq:]))
