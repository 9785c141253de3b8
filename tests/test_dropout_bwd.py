"""Backward with dropout -- SURVEY.md section 8(f) rank 2 (the reference raises, src/utils.py:88).

The forward draws its keep mask with Philox (tl.rand semantics, oracle/philox.py) and, through the
autograd op, saves the bits (ABI 6 keep mask); the backward kernels read them -- or, without a
saved mask, regenerate the same bits from the seed -- and differentiate O = (P * M / (1 - p)) V
exactly.  The oracle applies the identical mask (dropout_keep_mask_torch),
so the acceptance rule is the reference tests' compare_results_fa on O, dQ, dK, dV, as for the
no-dropout grid.  Also checked: two backward passes from the same forward are bitwise equal.
"""
import pytest
import torch

from tests.core import assert_dropout_grads_match, generate_test_data, run_case, unpack_keep_mask

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


MASK_CASES = [
    # b, hq, hkv, sq, sk, d, causal, p, dtype
    (2, 4, 2, 239, 301, 128, True, 0.17, torch.bfloat16),
    (3, 2, 2, 127, 513, 64, False, 0.1, torch.float16),
    (2, 8, 2, 1024, 1024, 128, True, 0.1, torch.bfloat16),
    (1, 2, 2, 333, 200, 96, True, 0.25, torch.bfloat16),
]


@pytest.mark.gpu
@pytest.mark.parametrize("b,hq,hkv,sq,sk,d,causal,p,dtype", MASK_CASES, ids=lambda x: str(x).replace("torch.", ""))
def test_saved_keep_mask_matches_philox_and_regeneration(b, hq, hkv, sq, sk, d, causal, p, dtype):
    """The forward's saved keep bits equal the oracle's Philox mask on every visible element, and a
    backward that reads them matches one that regenerates them (dQ, dK, dBias bitwise; dV as
    assert_dropout_grads_match: the D = 128 saved-mask dK/dV runs on the hand-placed kernel)."""
    from fa2_triton_amd.backward import _flash_attn_backward
    from fa2_triton_amd.forward import _flash_attn_forward
    from fa2_triton_amd.utils import dropout_mask_words
    from oracle.philox import dropout_keep_mask_torch
    from oracle.reference import attention_reference

    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, d, dtype)
    seed = 1234
    words = torch.full((dropout_mask_words(b, hq, sq, sk),), -1, dtype=torch.int32, device=q.device)
    o, lse, scale, seed = _flash_attn_forward(q, k, v, None, None, p, causal, None, seed, dropout_mask=words)
    o_ref, _, _, _ = _flash_attn_forward(q, k, v, None, None, p, causal, None, seed)
    keep = unpack_keep_mask(words, b, hq, sq, sk)
    want = dropout_keep_mask_torch(seed, p, b, hq, sq, sk, device=q.device)
    vis = torch.ones(sq, sk, dtype=torch.bool, device=q.device)
    if causal:  # bottom-right aligned: key j visible to row i iff j <= i + sk - sq
        vis = torch.arange(sk, device=q.device)[None, :] <= torch.arange(sq, device=q.device)[:, None] + (sk - sq)
    assert torch.equal(keep[:, :, vis], want[:, :, vis])
    if d == 128:
        # with a keep-mask buffer the D = 128 forward is dropout_mask_kernel + the hand-placed
        # kernel reading its words; without one fwd_kernel draws the bits in its softmax: the same
        # keep mask, O within the general kernel's error against the fp32 oracle over it
        ref = attention_reference(q, k, v, dropout_p=p, dropout_mask=keep, causal=causal).float()
        e_ref = (o_ref.float() - ref).abs().max().item()
        assert (o.float() - ref).abs().max().item() <= 2 * e_ref + 5e-5
    else:  # both fwd_kernel (reading the words / drawing them): the same operations
        assert torch.equal(o, o_ref)
    bias = (torch.randn(1, hq, sq, sk, device=q.device) * 0.5).to(dtype)
    for bb in (None, bias):
        o2, lse2, _, _ = _flash_attn_forward(q, k, v, None, bb, p, causal, None, seed, dropout_mask=words)
        g_mask = _flash_attn_backward(do, q, k, v, bb, None, o2, lse2, p, causal, scale, seed,
                                      bias_grad=bb is not None, dropout_mask=words)
        g_regen = _flash_attn_backward(do, q, k, v, bb, None, o2, lse2, p, causal, scale, seed,
                                       bias_grad=bb is not None)
        assert_dropout_grads_match(g_mask, g_regen, ("dq", "dk", "dv", "dbias"))


def test_keep_mask_layout_unpacks_a_known_pattern():
    """CPU check of the tiled layout helper: bit j % 32 of word [bh][i/32][j/32][i % 32]."""
    b, h, sq, sk = 1, 2, 40, 70
    nrb, ncw = 2, 3
    words = torch.zeros(b * h * nrb * ncw * 32, dtype=torch.int32)
    dense = torch.zeros(b, h, sq, sk, dtype=torch.bool)
    for (hh, i, j) in [(0, 0, 0), (1, 39, 69), (0, 33, 31), (1, 5, 64)]:
        dense[0, hh, i, j] = True
        wi = ((hh * nrb + i // 32) * ncw + j // 32) * 32 + i % 32
        words[wi] |= torch.tensor(1 << (j % 32), dtype=torch.int64).to(torch.int32)
    assert torch.equal(unpack_keep_mask(words, b, h, sq, sk), dense)


def test_keep_mask_allocation_falls_back_on_oom(monkeypatch):
    """CPU: an OutOfMemoryError while allocating the keep mask means 'no saved mask' (the backward
    regenerates the bits), never a failed forward (the mask is O(S^2) per call)."""
    from fa2_triton_amd import wrapper

    q = torch.zeros(1, 64, 2, 16, requires_grad=True)
    k = torch.zeros(1, 64, 2, 16, requires_grad=True)
    assert wrapper._keep_mask_buffer(q, k, k, 0.1) is not None

    def oom(*a, **kw):
        raise torch.OutOfMemoryError("forced")

    monkeypatch.setattr(wrapper.torch, "empty", oom)
    assert wrapper._keep_mask_buffer(q, k, k, 0.1) is None
    monkeypatch.undo()
    monkeypatch.setenv("FA2_DROPOUT_MASK_MAX_GB", "0")
    assert wrapper._keep_mask_buffer(q, k, k, 0.1) is None


@pytest.mark.gpu
def test_forced_mask_fallback_gives_bitwise_equal_gradients(monkeypatch):
    """The autograd op with its keep-mask allocation failing (forced OOM) returns the same O and
    bitwise the same dQ, dK, dV as with the saved mask.  (The hand-placed forward needs the mask
    buffer, so both arms run the general forward here -- reading the words vs drawing them in the
    softmax, the same operations; the hand-placed dropout forward: test_hp_paths.py.)"""
    from fa2_triton_amd import _lib as L
    from fa2_triton_amd import flash_attn_func, wrapper

    q, k, v, do = generate_test_data(2, 4, 2, 300, 300, 128, torch.bfloat16)
    L.set_path_policy(L.PATH_FWD_HP, 0)
    try:
        out = flash_attn_func(q, k, v, None, None, 0.15, True, None, 777)
        g_mask = torch.autograd.grad(out, (q, k, v), do)
        real_empty = torch.empty

        def empty_oom(*a, **kw):
            if kw.get("dtype") is torch.int32:
                raise torch.OutOfMemoryError("forced")
            return real_empty(*a, **kw)

        monkeypatch.setattr(wrapper.torch, "empty", empty_oom)
        out2 = flash_attn_func(q, k, v, None, None, 0.15, True, None, 777)
        monkeypatch.undo()
        g_regen = torch.autograd.grad(out2, (q, k, v), do)
    finally:
        L.set_path_policy(0, 0)
    assert torch.equal(out, out2)
    assert_dropout_grads_match(g_mask, g_regen)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_varlen_dropout_saved_mask(causal):
    """Dropout with a right-padded attention_mask (varlen, cu_seqlens): the saved keep bits equal
    Philox at the reference's packed offsets (kernel.py:146-148 with cu_seqlens) on every visible
    element of every sequence, and a backward reading them is bitwise equal to one regenerating
    them (this combination was unpinned)."""
    from fa2_triton_amd.backward import _flash_attn_backward
    from fa2_triton_amd.forward import _flash_attn_forward
    from fa2_triton_amd.utils import dropout_mask_words
    from oracle.philox import rand_torch

    b, hq, hkv, s, d, p = 3, 4, 2, 300, 128, 0.2
    q, k, v, do = generate_test_data(b, hq, hkv, s, s, d, torch.bfloat16)
    lens = [300, 173, 1]
    mask = torch.zeros(b, s, dtype=torch.bool, device=q.device)
    for i, n in enumerate(lens):
        mask[i, :n] = True
    seed = 99
    words = torch.full((dropout_mask_words(b, hq, s, s),), -1, dtype=torch.int32, device=q.device)
    o, lse, scale, seed = _flash_attn_forward(q, k, v, mask, None, p, causal, None, seed, dropout_mask=words)
    keep = unpack_keep_mask(words, b, hq, s, s)
    cu = 0
    for i, n in enumerate(lens):
        rows = torch.arange(n, device=q.device)
        for h in range(hq):
            # packed offset of (row, key) of sequence i, head h: Lk (cu + Lq h) + Lq... as the forward
            off = n * (cu + n * h) + rows[:, None] * n + rows[None, :]
            want = rand_torch(seed, off) > p
            vis = torch.ones(n, n, dtype=torch.bool, device=q.device)
            if causal:
                vis = rows[None, :] <= rows[:, None]
            assert torch.equal(keep[i, h, :n, :n][vis], want[vis]), (i, h)
        cu += n
    g_mask = _flash_attn_backward(do, q, k, v, None, mask, o, lse, p, causal, scale, seed, dropout_mask=words)
    g_regen = _flash_attn_backward(do, q, k, v, None, mask, o, lse, p, causal, scale, seed)
    assert_dropout_grads_match(g_mask, g_regen)
