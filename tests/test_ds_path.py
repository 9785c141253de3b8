"""The dS-workspace backward (dkdv_kernel stores its rounded dS tiles, dq_ds_kernel computes
dQ = dS K from them) against the recompute backward (dq_kernel) and the oracle.

Every other GPU test with head_dim in {72..128, multiple of 8} already runs the dS path (the
backward allocates the workspace by itself); here the two paths are run side by side on the
same inputs -- causal / non-causal, Sq != Sk (bottom-right causal, fully masked rows), GQA,
padding masks, bias, dropout and an fp32 dQ -- and both are checked with the reference tests'
acceptance rule (oracle/tolerance.py).  dQ of the two paths differs only by the rounding of dS
(S and dP come from differently ordered MFMA sums) and dK by the order of the delta row sum,
so they must agree to a few bf16/fp16 ulps; dV is bitwise equal.
"""
import pytest
import torch

from fa2_triton_amd import flash_attn_func
from fa2_triton_amd.backward import _flash_attn_backward, ds_workspace_bytes
from fa2_triton_amd.forward import _flash_attn_forward
from tests.core import generate_attention_mask, generate_dropout_seed_and_mask, generate_test_data, run_case

CASES = [
    # b, hq, hkv, sq, sk, d, causal, mask, bias, dropout, dtype
    (2, 4, 4, 256, 256, 128, True, False, False, 0.0, torch.bfloat16),
    (2, 4, 2, 517, 517, 128, False, False, False, 0.0, torch.bfloat16),
    (1, 4, 1, 1000, 333, 96, True, False, False, 0.0, torch.float16),
    (1, 2, 2, 203, 1100, 128, True, False, False, 0.0, torch.float16),
    (3, 4, 2, 300, 300, 128, True, True, False, 0.0, torch.bfloat16),
    (2, 2, 2, 160, 96, 128, False, False, True, 0.0, torch.bfloat16),
    (2, 4, 4, 128, 200, 80, False, False, False, 0.2, torch.float16),
    (1, 2, 2, 64, 64, 72, True, False, False, 0.0, torch.bfloat16),
    # non-causal query tails (Sq mod 64 over 1..63) on the two-query-tiles-per-wave dQ path, and
    # causal tails / Sq > Sk / Sq < Sk on the causal-compact workspace layout
    (1, 2, 1, 513, 513, 128, False, False, False, 0.0, torch.bfloat16),
    (1, 2, 2, 545, 300, 128, False, False, False, 0.0, torch.float16),
    (1, 2, 2, 575, 575, 96, False, False, False, 0.0, torch.bfloat16),
    (1, 2, 2, 607, 1024, 128, False, False, False, 0.0, torch.bfloat16),
    (1, 2, 2, 1087, 1087, 128, False, True, False, 0.0, torch.bfloat16),
    (1, 2, 2, 591, 591, 128, True, False, False, 0.0, torch.bfloat16),
    (1, 2, 2, 1000, 37, 128, True, False, False, 0.0, torch.bfloat16),
    (1, 2, 2, 37, 1000, 128, True, False, False, 0.0, torch.float16),
    (1, 2, 2, 129, 95, 128, True, False, False, 0.0, torch.bfloat16),
]


def _grads(q, k, v, do, mask, bias, dropout_p, seed, causal, use_ds, dq_dtype=None):
    with torch.no_grad():
        o, lse, scale, seed = _flash_attn_forward(q, k, v, mask, bias, dropout_p, causal, None, seed)
        ws = torch.empty(ds_workspace_bytes(q, k, v, o, do, causal), dtype=torch.uint8, device=q.device) if use_ds else None
        if use_ds:
            ws.fill_(0xFF)  # NaN bf16/fp16 pattern: any chunk read but never written would show
        return _flash_attn_backward(do, q, k, v, bias, mask, o, lse, dropout_p, causal, scale, seed,
                                    dq_dtype=dq_dtype, _stages=7 if use_ds else 6, _ds_ws=ws, _use_ds=use_ds)


@pytest.mark.gpu
@pytest.mark.parametrize("b,hq,hkv,sq,sk,d,causal,use_mask,use_bias,dropout_p,dtype", CASES,
                         ids=lambda x: str(x).replace("torch.", ""))
def test_ds_path_matches_recompute_path(b, hq, hkv, sq, sk, d, causal, use_mask, use_bias, dropout_p, dtype):
    qm, km = torch.empty(b, sq, hq, d, device="meta"), torch.empty(b, sk, hkv, d, device="meta")
    assert ds_workspace_bytes(qm, km, km, qm, qm, causal) > 0
    q, k, v, do = generate_test_data(b, hq, hkv, sq, sk, d, dtype)
    mask = generate_attention_mask(q) if use_mask else None
    bias = torch.rand(1, 1, sq, sk, device=q.device, dtype=dtype) if use_bias else None
    seed = 1234567 if dropout_p > 0 else None
    with_ds = _grads(q, k, v, do, mask, bias, dropout_p, seed, causal, True)
    without = _grads(q, k, v, do, mask, bias, dropout_p, seed, causal, False)
    for a, r, name in zip(with_ds, without, ("dq", "dk", "dv")):
        assert torch.isfinite(a).all(), name
        if name == "dv":  # P^T dO: the same products, summed over the query tiles in ascending
            # order on the dS path and descending on the recompute path: within one rounding
            torch.testing.assert_close(a.float(), r.float(), rtol=1e-2, atol=1e-3 * r.float().abs().max().item())
        else:  # dQ: dS rounding; dK: delta = rowsum(O dO) summed in another order (delta_kernel
            # here, dq_kernel's fused row sum there)
            torch.testing.assert_close(a.float(), r.float(), rtol=2e-2, atol=2e-3 * r.float().abs().max().item())


@pytest.mark.gpu
def test_ds_path_fp32_dq():
    q, k, v, do = generate_test_data(2, 4, 2, 384, 384, 128, torch.bfloat16)
    a = _grads(q, k, v, do, None, None, 0.0, None, True, True, dq_dtype=torch.float32)[0]
    r = _grads(q, k, v, do, None, None, 0.0, None, True, False, dq_dtype=torch.float32)[0]
    assert a.dtype == torch.float32
    torch.testing.assert_close(a, r, rtol=2e-2, atol=2e-3 * r.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("use_mask", [False, True])
def test_ds_path_vs_oracle(causal, use_mask, monkeypatch):
    # run_case goes through flash_attn_func, whose backward allocates the workspace itself once
    # the (opt-in) dS path is enabled
    monkeypatch.setenv("FA2_DS_WORKSPACE_MAX_GB", "auto")
    run_case(2, 8, 2, 700, 700, 128, causal, 0.0, use_mask, False, torch.bfloat16, False)


def test_ds_path_is_opt_in(monkeypatch):
    """Default backward: the O(S)-memory recompute path (no dS workspace is allocated)."""
    from fa2_triton_amd.backward import _ds_workspace_cap

    monkeypatch.delenv("FA2_DS_WORKSPACE_MAX_GB", raising=False)
    assert _ds_workspace_cap(torch.device("cpu")) == 0
    monkeypatch.setenv("FA2_DS_WORKSPACE_MAX_GB", "1.5")
    assert _ds_workspace_cap(torch.device("cpu")) == 3 << 29


@pytest.mark.gpu
def test_ds_path_disabled_by_cap(monkeypatch):
    monkeypatch.setenv("FA2_DS_WORKSPACE_MAX_GB", "0")
    from fa2_triton_amd.backward import alloc_ds_workspace

    q, k, v, do = generate_test_data(1, 2, 2, 128, 128, 128, torch.bfloat16)
    assert alloc_ds_workspace(q, k, v, q, do, True) is None
    out = flash_attn_func(q, k, v, None, None, 0.0, True)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), do)
    assert torch.isfinite(dq).all()


def _fill_device_memory(leave_bytes: int):
    """Allocate everything but `leave_bytes` of device memory (returned tensor holds it)."""
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    return torch.empty(max(free - leave_bytes, 0), dtype=torch.uint8, device="cuda")


def _check_vs_oracle(q, k, v, do, grads, causal):
    from oracle.reference import attention_reference
    from oracle.tolerance import check_fa_tolerance

    out = flash_attn_func(q, k, v, None, None, 0.0, causal)
    ref = attention_reference(q, k, v, causal=causal)
    pt = attention_reference(q, k, v, causal=causal, upcast=False, reorder_ops=True)
    check_fa_tolerance(q, k, v, do, out, ref, pt, grads=grads)


@pytest.mark.gpu
def test_ds_workspace_capped_by_free_memory(monkeypatch):
    """With less free memory than twice the workspace, the backward takes the O(S) recompute
    path instead of the dS path -- never an OOM where the reference's backward would run."""
    import fa2_triton_amd.backward as bw

    monkeypatch.setenv("FA2_DS_WORKSPACE_MAX_GB", "auto")
    q, k, v, do = generate_test_data(4, 32, 32, 1024, 1024, 128, torch.bfloat16)
    need = ds_workspace_bytes(q, k, v, q, do, True)
    assert need > 100 << 20
    calls = []
    orig = bw.alloc_ds_workspace
    monkeypatch.setattr(bw, "alloc_ds_workspace", lambda *a: calls.append(orig(*a)) or calls[-1])
    out = flash_attn_func(q, k, v, None, None, 0.0, True)
    filler = _fill_device_memory(160 << 20)  # grads need 3 x 32 MiB; the cap is then ~80 MiB
    grads = torch.autograd.grad(out, (q, k, v), do)
    torch.cuda.synchronize()
    del filler
    assert calls and calls[-1] is None
    _check_vs_oracle(q, k, v, do, grads, True)


@pytest.mark.gpu
def test_ds_workspace_oom_falls_back_to_recompute(monkeypatch):
    """An allocation failure of the workspace (cap lifted) is caught: the backward takes the
    recompute path.  The failure is injected (torch.empty of the workspace raises
    torch.OutOfMemoryError) so the test does not depend on the allocator's free-memory view."""
    import fa2_triton_amd.backward as bw

    monkeypatch.setenv("FA2_DS_WORKSPACE_MAX_GB", "100000")
    q, k, v, do = generate_test_data(2, 8, 2, 600, 600, 128, torch.bfloat16)
    need = ds_workspace_bytes(q, k, v, q, do, True)
    assert need > 0
    real_empty = torch.empty

    def empty(*size, **kw):
        if kw.get("dtype") is torch.uint8 and size == (need,):
            raise torch.OutOfMemoryError("injected: workspace allocation fails")
        return real_empty(*size, **kw)

    calls = []
    orig = bw.alloc_ds_workspace
    monkeypatch.setattr(bw, "alloc_ds_workspace", lambda *a: calls.append(orig(*a)) or calls[-1])
    out = flash_attn_func(q, k, v, None, None, 0.0, True)
    monkeypatch.setattr(torch, "empty", empty)
    grads = torch.autograd.grad(out, (q, k, v), do)
    monkeypatch.setattr(torch, "empty", real_empty)
    assert calls and calls[-1] is None
    _check_vs_oracle(q, k, v, do, grads, True)
