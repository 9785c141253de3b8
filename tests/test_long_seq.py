"""Long sequences (64k keys): the regime where a 32-bit row or element offset would overflow.

The O(S^2) oracle cannot run at 64k x 64k, so the checks are exact sub-problems computed in fp32
torch on the same device tensors:
* sampled query rows (first, middle, last 128): O, LSE2 and dQ of those rows depend on their own
  Q / dO rows and all keys only, so a [128 x Sk] score block per head gives them exactly;
* sampled key columns (first, middle, last 128): dK and dV of those keys are sums over all query
  rows of P (dP - delta) Q and P dO, computed from the kernel's own LSE2 and O (both checked on
  the sampled rows above), summed over the GQA group.
Causal masks are bottom-right aligned (key j visible to row i iff j <= i + Sk - Sq), as in the
reference (/root/reference/src/reference_implementation.py:8-35).  Acceptance: max |x - ref| <=
2e-2 max |ref| per tensor, about four bf16 ulps of the largest element.
"""
import math

import pytest
import torch

from tests.core import generate_test_data

LOG2E = 1.4426950408889634


def _close(x, ref, tag):
    x, ref = x.float(), ref.float()
    assert torch.isfinite(x).all(), tag
    err = (x - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 2e-2 * scale + 1e-6, f"{tag}: max err {err:.3e} vs max |ref| {scale:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("sq,sk,causal", [(65536, 65536, True), (65536, 65536, False), (1000, 65536, True)])
def test_long_sequence_sampled_rows_and_keys(sq, sk, causal):
    from fa2_triton_amd import flash_attn_func
    from fa2_triton_amd.forward import _flash_attn_forward

    hq, hkv, d = 2, 1, 128
    q, k, v, do = generate_test_data(1, hq, hkv, sq, sk, d, torch.bfloat16)
    scale = 1.0 / math.sqrt(d)
    with torch.no_grad():
        _, lse2, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
    out = flash_attn_func(q, k, v, None, None, 0.0, causal)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), do)
    out = out.detach()
    qf, kf, vf, dof, of = (t.detach()[0].float() for t in (q, k, v, do, out))  # [S, H, D]
    group = hq // hkv
    diag = sk - sq

    def visible(rows, cols):  # [len(rows), len(cols)] bool
        if not causal:
            return torch.ones(len(rows), len(cols), dtype=torch.bool, device=q.device)
        return cols[None, :] <= rows[:, None] + diag

    # sampled query rows: O, LSE2, dQ
    for r0 in sorted({0, (sq // 2) & ~127, max(0, sq - 128)}):
        rows = torch.arange(r0, min(r0 + 128, sq), device=q.device)
        cols = torch.arange(sk, device=q.device)
        vis = visible(rows, cols)
        for h in range(hq):
            hk = h // group
            s = (qf[rows, h] @ kf[:, hk].T) * scale
            s = s.masked_fill(~vis, float("-inf"))
            lse = torch.logsumexp(s, dim=-1)
            p = torch.exp(s - lse[:, None])
            o_ref = p @ vf[:, hk]
            _close(out[0, rows, h], o_ref, f"O rows {r0} head {h}")
            _close(lse2[0, h, rows], lse * LOG2E, f"LSE2 rows {r0} head {h}")
            dp = dof[rows, h] @ vf[:, hk].T
            delta = (dof[rows, h] * o_ref).sum(-1)
            dq_ref = (p * (dp - delta[:, None])) @ kf[:, hk] * scale
            _close(dq[0, rows, h], dq_ref, f"dQ rows {r0} head {h}")

    # sampled key columns: dK, dV summed over the q-heads of the group
    rows = torch.arange(sq, device=q.device)
    for c0 in sorted({0, (sk // 2) & ~127, sk - 128}):
        cols = torch.arange(c0, c0 + 128, device=q.device)
        vis = visible(rows, cols)
        for hk in range(hkv):
            dk_ref = torch.zeros(128, d, device=q.device)
            dv_ref = torch.zeros(128, d, device=q.device)
            for h in range(hk * group, (hk + 1) * group):
                s = (qf[:, h] @ kf[cols, hk].T) * scale
                lse_nat = lse2[0, h, :sq].float() / LOG2E
                p = torch.where(vis, torch.exp(s - lse_nat[:, None]), torch.zeros_like(s))
                p = torch.nan_to_num(p, nan=0.0)  # rows with no visible key (LSE -inf)
                dv_ref += p.T @ dof[:, h]
                dp = dof[:, h] @ vf[cols, hk].T
                delta = (dof[:, h] * of[:, h]).sum(-1)
                dk_ref += (p * (dp - delta[:, None])).T @ qf[:, h] * scale
            _close(dv[0, cols, hk], dv_ref, f"dV keys {c0}")
            _close(dk[0, cols, hk], dk_ref, f"dK keys {c0}")
