"""GPU parity for the surfaces the reference grids do not reach.

Each case runs the HIP operator through `flash_attn_func` and checks O, dQ, dK, dV against the
oracle (oracle/reference.py) with the reference tests' acceptance rule (oracle/tolerance.py):
* per-head bias [B, Hq, Sq, Sk], [1, Hq, Sq, Sk], [B, 1, Sq, Sk] with GQA, indexed by the query
  head in forward and backward (the reference uses the kv head in forward,
  /root/reference/src/forward/kernel.py:141, and rejects per-head bias, src/utils.py:70);
* an fp32 bias (bias_dtype 32, /root/reference/src/utils.py:102-109);
* BHSD tensors passed as `x.transpose(1, 2)` views (no copies: unit head_dim stride only,
  /root/reference/src/wrapper.py:41-43);
* a data pointer 2 bytes past a 16-byte boundary (the scalar-load path of an aligned head dim);
* K and V with different sequence strides (the unpipelined forward, the unaligned backward);
* empty sides: Sk = 0 (O = 0, LSE = -inf, dQ = 0) and Sq = 0 (empty O, dK = dV = 0).
"""
import pytest
import torch

from fa2_triton_amd import flash_attn_func
from fa2_triton_amd.forward import _flash_attn_forward
from oracle.reference import attention_reference, lse2_reference
from oracle.tolerance import check_fa_tolerance
from tests.core import generate_test_data


def _check(q, k, v, do, causal, bias=None, grads_of=None):
    out = flash_attn_func(q, k, v, None, bias, 0.0, causal)
    ref = attention_reference(q, k, v, attn_bias=bias, causal=causal)
    pt = attention_reference(q, k, v, attn_bias=bias, causal=causal, upcast=False, reorder_ops=True)
    grads = None
    if grads_of is not None:
        grads = torch.autograd.grad(out, grads_of, do, retain_graph=True)
    return check_fa_tolerance(q, k, v, do, out, ref, pt, grads=grads)


BIAS_SHAPES = ["b_hq", "1_hq", "b_1", "1_1"]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "fp16"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", BIAS_SHAPES)
@pytest.mark.parametrize("bias_dtype", ["same", "fp32"])
@pytest.mark.parametrize("d", [64, 128])
def test_bias_shapes_gqa(dtype, causal, shape, bias_dtype, d):
    b, hq, hkv, sq, sk = 2, 4, 2, 200, 331
    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, d, dtype)
    bb, bh = {"b_hq": (b, hq), "1_hq": (1, hq), "b_1": (b, 1), "1_1": (1, 1)}[shape]
    bdt = dtype if bias_dtype == "same" else torch.float32
    bias = torch.rand(bb, bh, sq, sk, device=q.device, dtype=bdt) * 2 - 1
    _check(q, k, v, do, causal, bias)
    # every head really sees its own bias: LSE2 against the oracle's
    with torch.no_grad():
        _, lse, _, _ = _flash_attn_forward(q, k, v, None, bias, 0.0, causal, None, None)
    ref_lse = lse2_reference(q, k, attn_bias=bias, causal=causal)
    fin = torch.isfinite(ref_lse)
    torch.testing.assert_close(lse[:, :, :sq][fin], ref_lse[fin], rtol=1e-3, atol=1e-3)


PIPE_BIAS_CASES = [
    # b, hq, hkv, sq, sk, d: key counts multiples of 8, so the bias rows are 16-byte aligned and
    # the forward runs the pipelined kernel with LDS-staged bias tiles (fwd_pipe_kernel BIASK)
    (2, 4, 2, 512, 512, 128),
    (1, 3, 3, 384, 640, 64),
    (2, 2, 1, 1000, 1000, 80),
    (1, 2, 2, 129, 256, 128),
    (1, 2, 2, 700, 136, 64),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", PIPE_BIAS_CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "fp16"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", ["b_hq", "1_1", "1_hq"])
@pytest.mark.parametrize("bias_dtype", ["same", "other16"])
def test_bias_pipelined_forward(case, dtype, causal, shape, bias_dtype):
    """The 16-bit, 16-byte-aligned bias path of the pipelined forward (bf16 and fp16 bias in
    either input dtype), O / dQ / dK / dV under the reference rule and LSE2 against the oracle."""
    b, hq, hkv, sq, sk, d = case
    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, d, dtype)
    bb, bh = {"b_hq": (b, hq), "1_hq": (1, hq), "1_1": (1, 1)}[shape]
    bdt = dtype if bias_dtype == "same" else ({torch.bfloat16: torch.float16, torch.float16: torch.bfloat16}[dtype])
    bias = (torch.rand(bb, bh, sq, sk, device=q.device) * 4 - 2).to(bdt)
    _check(q, k, v, do, causal, bias, grads_of=(q, k, v))
    with torch.no_grad():
        _, lse, _, _ = _flash_attn_forward(q, k, v, None, bias, 0.0, causal, None, None)
    ref_lse = lse2_reference(q, k, attn_bias=bias, causal=causal)
    fin = torch.isfinite(ref_lse)
    torch.testing.assert_close(lse[:, :, :sq][fin], ref_lse[fin], rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 96, 128])
def test_bhsd_transposed_views(causal, d):
    b, hq, hkv, sq, sk = 2, 4, 2, 257, 190
    torch.manual_seed(0)
    dev, dt = "cuda", torch.bfloat16
    qb = torch.empty(b, hq, sq, d, device=dev, dtype=dt).normal_(0, 0.5)
    kb = torch.empty(b, hkv, sk, d, device=dev, dtype=dt).normal_(0, 0.5)
    vb = torch.empty(b, hkv, sk, d, device=dev, dtype=dt).normal_(0, 0.5)
    q, k, v = (t.transpose(1, 2).requires_grad_() for t in (qb, kb, vb))  # BSHD views of BHSD memory
    assert not q.is_contiguous() and q.stride(-1) == 1
    do = torch.randn(b, hq, sq, d, device=dev, dtype=dt).transpose(1, 2)
    _check(q, k, v, do, causal, grads_of=(q, k, v))


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 128])
def test_misaligned_data_pointer(causal, d):
    b, hq, hkv, sq, sk = 2, 4, 4, 150, 150
    q0, k0, v0, do = generate_test_data(b, hq, hkv, sq, sk, d, torch.float16)

    def shifted(t):  # same values, data pointer 2 bytes past a 16-byte boundary
        buf = torch.empty(t.numel() + 1, device=t.device, dtype=t.dtype)
        x = buf[1:].view(t.shape)
        x.copy_(t.detach())
        assert x.data_ptr() % 16 == 2
        return x.requires_grad_()

    q, k, v = shifted(q0), shifted(k0), shifted(v0)
    _check(q, k, v, do, causal, grads_of=(q, k, v))


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_kv_unequal_seq_strides(causal):
    b, hq, hkv, sq, sk, d = 2, 4, 2, 300, 260, 128
    q, k0, v, do = generate_test_data(b, hq, hkv, sq, sk, d, torch.bfloat16)
    wide = torch.zeros(b, sk, 2 * hkv, d, device=q.device, dtype=q.dtype)
    wide[:, :, :hkv] = k0.detach()
    k = wide[:, :, :hkv].requires_grad_()  # seq stride 2 Hkv D, V's is Hkv D
    assert k.stride(1) != v.stride(1)
    _check(q, k, v, do, causal, grads_of=(q, k, v))


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_empty_key_side(causal):
    q, k, v, do = generate_test_data(2, 4, 2, 70, 0, 128, torch.bfloat16)
    out = flash_attn_func(q, k, v, None, None, 0.0, causal)
    assert out.shape == q.shape and (out == 0).all()
    with torch.no_grad():
        _, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
    assert torch.isneginf(lse[:, :, :70]).all()
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), do)
    assert (dq == 0).all() and dk.shape == k.shape and dv.shape == v.shape


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_empty_query_side(causal):
    q, k, v, do = generate_test_data(2, 4, 2, 0, 90, 64, torch.float16)
    out = flash_attn_func(q, k, v, None, None, 0.0, causal)
    assert out.shape == q.shape
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), do)
    assert dq.shape == q.shape and (dk == 0).all() and (dv == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "fp16"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", BIAS_SHAPES)
@pytest.mark.parametrize("bias_dtype", ["same", "fp32"])
@pytest.mark.parametrize("dropout_p", [0.0, 0.17])
def test_bias_gradient(dtype, causal, shape, bias_dtype, dropout_p):
    """dL/d(bias) (beyond the reference, which returns None) against autograd through the oracle,
    with the acceptance rule of the other gradients: err <= 3 err_pt + 1e-5, where err_pt is the
    low-precision PyTorch oracle's error; broadcast dims are summed.  With dropout the oracle
    applies the forward's Philox keep mask (oracle/philox.py), as in test_dropout_bwd.py."""
    from oracle.philox import dropout_keep_mask_torch

    b, hq, hkv, sq, sk, d = 2, 4, 2, 190, 270, 128
    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, d, dtype)
    bb, bh = {"b_hq": (b, hq), "1_hq": (1, hq), "b_1": (b, 1), "1_1": (1, 1)}[shape]
    bdt = dtype if bias_dtype == "same" else torch.float32
    bias = (torch.rand(bb, bh, sq, sk, device=q.device, dtype=bdt) * 2 - 1).requires_grad_()
    seed = 1234 if dropout_p else None
    mask = dropout_keep_mask_torch(seed, dropout_p, b, hq, sq, sk, device=q.device) if dropout_p else None
    out = flash_attn_func(q, k, v, None, bias, dropout_p, causal, None, seed)
    dq, dk, dv, dbias = torch.autograd.grad(out, (q, k, v, bias), do)
    assert dbias.shape == bias.shape and dbias.dtype == bias.dtype
    ref = attention_reference(q, k, v, attn_bias=bias, causal=causal, dropout_p=dropout_p, dropout_mask=mask)
    pt = attention_reference(q, k, v, attn_bias=bias, causal=causal, upcast=False, reorder_ops=True,
                             dropout_p=dropout_p, dropout_mask=mask)
    g_ref = torch.autograd.grad(ref, bias, do, retain_graph=True)[0]
    g_pt = torch.autograd.grad(pt, bias, do, retain_graph=True)[0]
    err = (dbias.float() - g_ref.float()).abs().max().item()
    err_pt = (g_pt.float() - g_ref.float()).abs().max().item()
    assert err <= 3 * err_pt + 1e-5, (err, err_pt)
    check_fa_tolerance(q, k, v, do, out, ref, pt, grads=(dq, dk, dv))


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_bias_gradient_memory_and_determinism(causal):
    """A broadcast [1, 1, S, S] bias at B=8 H=32 S=4096 (cfg3 shape): the bias gradient is summed
    over batch and heads inside the library, so the backward allocates O(bias) memory -- less than
    3x the bias's fp32 size on top of dQ/dK/dV -- where a [B, Hq, S, S] fp32 dS buffer would be
    17 GB.  Two backward passes give bitwise equal gradients."""
    b, h, s, d = 8, 32, 4096, 128
    q, k, v, do = generate_test_data(b, h, h, s, s, d, torch.bfloat16)
    bias = (torch.rand(1, 1, s, s, device=q.device, dtype=torch.bfloat16) - 0.5).requires_grad_()
    out = flash_attn_func(q, k, v, None, bias, 0.0, causal)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    g1 = torch.autograd.grad(out, (q, k, v, bias), do, retain_graph=True)
    torch.cuda.synchronize()
    grads_bytes = sum(t.numel() * t.element_size() for t in g1)
    extra = torch.cuda.max_memory_allocated() - base - grads_bytes
    lse_delta = 2 * b * h * s * 4  # the LSE-shaped delta workspace
    assert extra <= 3 * s * s * 4 + lse_delta, extra
    g2 = torch.autograd.grad(out, (q, k, v, bias), do)
    for x, y in zip(g1, g2):
        assert torch.equal(x, y)
    assert torch.isfinite(g1[3]).all()


def _dbias_vs_oracle(q, k, v, do, bias, causal, rows=None):
    """dL/d(bias) from the library against autograd through the fp32 oracle (and the low-precision
    oracle for the tolerance), on all rows or the row slice `rows` of the bias gradient."""
    out = flash_attn_func(q, k, v, None, bias, 0.0, causal)
    dbias = torch.autograd.grad(out, bias, do)[0]
    assert dbias.shape == bias.shape and torch.isfinite(dbias).all()
    ref = attention_reference(q, k, v, attn_bias=bias, causal=causal)
    pt = attention_reference(q, k, v, attn_bias=bias, causal=causal, upcast=False, reorder_ops=True)
    g_ref = torch.autograd.grad(ref, bias, do, retain_graph=True)[0]
    g_pt = torch.autograd.grad(pt, bias, do)[0]
    sl = (slice(None), slice(None), rows if rows is not None else slice(None))
    err = (dbias[sl].float() - g_ref[sl].float()).abs().max().item()
    err_pt = (g_pt[sl].float() - g_ref[sl].float()).abs().max().item()
    assert err <= 3 * err_pt + 1e-5, (err, err_pt)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [32, 64, 256])
def test_bias_gradient_head_dims(d, causal):
    """The bias-gradient kernel's other head-dim tiles (only D = 128 was checked
    against the oracle): the 3-tile K/V ring (D <= 128) and the 2-tile ring of D = 256."""
    q, k, v, do = generate_test_data(2, 4, 2, 190, 270, d, torch.bfloat16)
    bias = (torch.rand(1, 4, 190, 270, device=q.device, dtype=torch.bfloat16) * 2 - 1).requires_grad_()
    _dbias_vs_oracle(q, k, v, do, bias, causal)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_bias_gradient_square_order_ragged(causal):
    """The XCD 8 x 8 square block order of the bias gradient (taken when the bias has >= 32 row
    blocks and >= 32 key tiles) with Sq, Sk not multiples of its squares: padded squares and edge
    tiles.  Row slices at the start, the square seams and the ragged end."""
    sq, sk = 4100, 4200
    q, k, v, do = generate_test_data(1, 1, 1, sq, sk, 128, torch.bfloat16)
    bias = (torch.rand(1, 1, sq, sk, device=q.device, dtype=torch.bfloat16) * 2 - 1).requires_grad_()
    rows = torch.cat([torch.arange(0, 64), torch.arange(1000, 1064), torch.arange(4032, 4100)]).to(q.device)
    _dbias_vs_oracle(q, k, v, do, bias, causal, rows=rows)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("sk,bdt", [(264, torch.bfloat16), (270, torch.bfloat16), (270, torch.float32)],
                         ids=["bf16_rows16", "bf16_unaligned", "fp32"])
def test_bias_at_the_end_of_its_allocation(sk, bdt, causal):
    """A bias whose last row ends exactly where its buffer's NaN canary starts (VERDICT r04 weak 2,
    ADVICE r03: the 16-bit bias tiles are staged by LDS-DMA whose range must end at the last valid
    key).  Any read past the bias would pull a NaN into O, dQ, dK, dV or dBias: results must be
    finite and bitwise equal to the same bias in a plain allocation."""
    b, hq, sq, d = 2, 4, 190, 128
    q, k, v, do = generate_test_data(b, hq, 2, sq, sk, d, torch.bfloat16)
    plain = torch.rand(1, hq, sq, sk, device=q.device, dtype=bdt) * 2 - 1
    n = plain.numel()
    buf = torch.full((n + 4096,), float("nan"), device=q.device, dtype=bdt)
    buf[:n] = plain.flatten()
    guarded = buf[:n].view(1, hq, sq, sk)
    res = []
    for bias in (plain.clone().requires_grad_(), guarded.requires_grad_()):
        out = flash_attn_func(q, k, v, None, bias, 0.0, causal)
        grads = torch.autograd.grad(out, (q, k, v, bias), do)
        res.append([out.detach()] + [g.detach() for g in grads])
    for name, a, c in zip(("out", "dq", "dk", "dv", "dbias"), *res):
        assert torch.isfinite(a).all() and torch.isfinite(c).all(), name
        assert torch.equal(a, c), name
