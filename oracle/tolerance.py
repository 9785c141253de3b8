"""The reference tests' acceptance rule (TEST INFRASTRUCTURE ONLY).

Restates compare_results_fa (/root/reference/tests/utils.py:68-142): the error of the
operator under test against the fp32 oracle must be within a small multiple of the error a
plain low-precision PyTorch implementation (oracle with upcast=False, reorder_ops=True) makes:
  output : max|out - ref| <= 2 * max|pt - ref| + 5e-5          (:93)
  dQ, dK : max|g - ref|   <= 3 * max|g_pt - ref| + 1e-5        (:127, :130)
  dV     : same bound, or sum|dv - ref| < 1e-4 (with a warning) (:131-140)
One addition, for degenerate cases only: when the low-precision PyTorch run happens to be
exact (its error against the fp32 oracle is 0, e.g. one visible key per row, so P == 1 and dV
is a plain column sum), the rule above collapses to bit-equality with one particular BLAS
summation order.  Only then is a result also accepted if it is *faithfully rounded*: every
element within one unit in the last place (of the output dtype, at that element's magnitude)
of the fp32 oracle.

The report also carries the north-star figure (BASELINE.json: "fwd+bwd outputs within 1e-3
rtol of the reference"): rtol = max|x - ref| / max|ref| per tensor, under the key
`<name>_rtol`.
"""
import warnings
from typing import Optional, Sequence

import torch
from torch import Tensor


def _maxdiff(a: Tensor, b: Tensor) -> float:
    return (a.float() - b.float()).abs().max().item() if a.numel() else 0.0


def _rtol(err: float, ref: Tensor) -> float:
    """max|x - ref| / max|ref| (0 for an all-zero reference matched exactly)."""
    m = ref.float().abs().max().item() if ref.numel() else 0.0
    return err / m if m > 0 else (0.0 if err == 0 else float("inf"))


def within_one_ulp(x: Tensor, ref: Tensor) -> bool:
    """Every element of x is within 1 ulp (of x.dtype, at |ref|'s binade) of the fp32 ref."""
    if x.dtype not in (torch.float16, torch.bfloat16):
        return False
    mant = 10 if x.dtype == torch.float16 else 7
    r = ref.float()
    tiny = torch.finfo(x.dtype).tiny
    exp = torch.floor(torch.log2(r.abs().clamp_min(tiny)))
    ulp = torch.exp2(exp - mant)
    return bool(((x.float() - r).abs() <= ulp).all().item())


# How often each escape beyond the reference's rule decided a check (reported by tests/conftest.py
# at the end of a run, so the 1-ulp branch cannot widen silently): "ulp" = err > mul * err_pt +
# bias accepted only because err_pt == 0 and every element is within one ulp; "dv_sum" = the
# reference's own small-dV-sum escape (tests/utils.py of the reference).
ESCAPES = {"checks": 0, "ulp": 0, "dv_sum": 0}


def check_fa_tolerance(
    q: Tensor,
    k: Tensor,
    v: Tensor,
    do: Optional[Tensor],
    out: Tensor,
    out_ref: Tensor,
    out_pt: Tensor,
    out_error_mul: float = 2.0,
    out_error_bias: float = 5e-5,
    grad_error_mul: float = 3.0,
    grad_error_bias: float = 1e-5,
    grads: Optional[Sequence[Tensor]] = None,
) -> dict:
    """Raise AssertionError when the rule above is violated; return the measured errors."""
    report = {"out": _maxdiff(out, out_ref), "out_pt": _maxdiff(out_pt, out_ref)}
    report["out_rtol"] = _rtol(report["out"], out_ref)
    ESCAPES["checks"] += 1
    rule = report["out"] <= out_error_mul * report["out_pt"] + out_error_bias
    ulp = not rule and report["out_pt"] == 0 and within_one_ulp(out, out_ref)
    ESCAPES["ulp"] += int(ulp)
    assert rule or ulp, f"Output {report}"
    if do is None:
        return report
    if grads is None:
        grads = torch.autograd.grad(out, (q, k, v), do, retain_graph=True)
    g_ref = torch.autograd.grad(out_ref, (q, k, v), do, retain_graph=True)
    g_pt = torch.autograd.grad(out_pt, (q, k, v), do, retain_graph=True)
    for name, g, gr, gp in zip(("dq", "dk", "dv"), grads, g_ref, g_pt):
        err, err_pt = _maxdiff(g, gr), _maxdiff(gp, gr)
        report[name], report[name + "_pt"] = err, err_pt
        report[name + "_rtol"] = _rtol(err, gr)
        ESCAPES["checks"] += 1
        ok = err <= grad_error_mul * err_pt + grad_error_bias
        if not ok and err_pt == 0 and within_one_ulp(g, gr):
            ESCAPES["ulp"] += 1
            ok = True
        if not ok and name == "dv":
            total = (g.float() - gr.float()).abs().sum().item()
            if total < 1e-4:
                warnings.warn(f"small dV errors summing to {total}", stacklevel=2)
                ESCAPES["dv_sum"] += 1
                ok = True
        assert ok, f"Gradient of {name}: {report}"
    return report
