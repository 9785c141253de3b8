"""GPU dev check of the hand-placed forward (fwd_hp_kernel) against fwd_pipe_kernel and the oracle.

For each shape: O and LSE2 with the hand-placed forward on and off (_lib.set_path_policy: the per-call fa2_policy) in one process, max |diff| between them, and
each one's max |O - O_fp32 oracle|.  usage: python tests/hp_check.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd import _lib as L  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402
from oracle.reference import attention_reference, lse2_reference  # noqa: E402

CASES = [
    # b, hq, hkv, sq, sk, causal, dtype
    (1, 1, 1, 256, 256, False, torch.bfloat16),
    (1, 1, 1, 256, 256, True, torch.bfloat16),
    (2, 4, 2, 512, 512, True, torch.bfloat16),
    (2, 4, 4, 1024, 1024, False, torch.float16),
    (1, 2, 1, 300, 700, True, torch.bfloat16),
    (1, 2, 2, 777, 333, True, torch.float16),
    (1, 2, 2, 1, 129, False, torch.bfloat16),
    (2, 8, 8, 2048, 2048, True, torch.bfloat16),
]


def run(case):
    b, hq, hkv, sq, sk, causal, dt = case
    torch.manual_seed(0)
    q = torch.randn(b, sq, hq, 128, device="cuda", dtype=dt) * 0.5
    k = torch.randn(b, sk, hkv, 128, device="cuda", dtype=dt) * 0.5
    v = torch.randn(b, sk, hkv, 128, device="cuda", dtype=dt) * 0.5
    res = {}
    for hp in ("1", "0"):
        L.set_path_policy(0 if hp == "1" else L.PATH_FWD_HP, 0)
        o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        torch.cuda.synchronize()
        res[hp] = (o.float(), lse[:, :, :sq].float())
    L.set_path_policy(0, 0)
    ref = attention_reference(q, k, v, causal=causal).float()
    pt = attention_reference(q, k, v, causal=causal, upcast=False, reorder_ops=True).float()
    lref = lse2_reference(q, k, causal=causal)
    fl = torch.isfinite(lref)
    e_l1 = (res["1"][1][fl] - lref[fl]).abs().max().item() if fl.any() else 0.0
    e_l0 = (res["0"][1][fl] - lref[fl]).abs().max().item() if fl.any() else 0.0
    d_o = (res["1"][0] - res["0"][0]).abs().max().item()
    fin = torch.isfinite(res["0"][1])
    d_l = (res["1"][1][fin] - res["0"][1][fin]).abs().max().item() if fin.any() else 0.0
    same_inf = torch.equal(torch.isfinite(res["1"][1]), fin)
    e1 = (res["1"][0] - ref).abs().max().item()
    e0 = (res["0"][0] - ref).abs().max().item()
    ept = (pt - ref).abs().max().item()
    ok = e1 <= 2 * ept + 5e-5 and same_inf and e_l1 <= 1e-3 + 1e-3 * lref[fl].abs().max().item()
    print(f"{case}: hp-pipe |dO| {d_o:.3e} |dLSE2| {d_l:.3e} inf-pattern {same_inf} | err hp {e1:.3e} pipe {e0:.3e} "
          f"pt {ept:.3e} | LSE2 err hp {e_l1:.2e} pipe {e_l0:.2e} {'OK' if ok else 'FAIL'}", flush=True)
    return ok


BWD_CASES = [
    # b, hq, hkv, sq, sk, causal, dtype
    (1, 1, 1, 256, 256, False, torch.bfloat16),
    (1, 1, 1, 256, 256, True, torch.bfloat16),
    (2, 4, 2, 512, 512, True, torch.bfloat16),
    (2, 4, 4, 1024, 1024, False, torch.float16),
    (1, 2, 1, 300, 700, True, torch.bfloat16),
    (1, 2, 2, 777, 333, True, torch.float16),
    (1, 4, 1, 129, 257, False, torch.bfloat16),
    (2, 8, 8, 2048, 2048, True, torch.bfloat16),
]


def run_bwd(case):
    from fa2_triton_amd.backward import _flash_attn_backward

    b, hq, hkv, sq, sk, causal, dt = case
    torch.manual_seed(1)
    q = (torch.randn(b, sq, hq, 128, device="cuda", dtype=dt) * 0.5).requires_grad_()
    k = (torch.randn(b, sk, hkv, 128, device="cuda", dtype=dt) * 0.5).requires_grad_()
    v = (torch.randn(b, sk, hkv, 128, device="cuda", dtype=dt) * 0.5).requires_grad_()
    do = torch.randn(b, sq, hq, 128, device="cuda", dtype=dt)
    L.set_path_policy(L.PATH_FWD_HP, 0)
    o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
    res = {}
    for hp in ("1", "0"):
        L.set_path_policy(L.PATH_FWD_HP | (0 if hp == "1" else L.PATH_DQ_HP | L.PATH_DKDV_HP), 0)
        g = _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.0, causal, None, None)
        torch.cuda.synchronize()
        res[hp] = [x.float() for x in g[:3]]
    L.set_path_policy(0, 0)
    ref = attention_reference(q, k, v, causal=causal)
    gref = torch.autograd.grad(ref, (q, k, v), do.float())
    pt = attention_reference(q, k, v, causal=causal, upcast=False, reorder_ops=True)
    gpt = torch.autograd.grad(pt, (q, k, v), do)
    ok = True
    msg = []
    for name, i in (("dQ", 0), ("dK", 1), ("dV", 2)):
        d = (res["1"][i] - res["0"][i]).abs().max().item()
        e1 = (res["1"][i] - gref[i].float()).abs().max().item()
        e0 = (res["0"][i] - gref[i].float()).abs().max().item()
        ept = (gpt[i].float() - gref[i].float()).abs().max().item()
        good = e1 <= 3 * ept + 1e-5 and bool(torch.isfinite(res["1"][i]).all())
        ok &= good
        msg.append(f"{name}: hp-old {d:.3e} err hp {e1:.3e} old {e0:.3e} pt {ept:.3e}")
    print(f"bwd {case}: " + " | ".join(msg) + f" {'OK' if ok else 'FAIL'}", flush=True)
    return ok


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "fwd,bwd"
    bad = []
    if "fwd" in which:
        bad += [c for c in CASES if not run(c)]
    if "bwd" in which:
        bad += [c for c in BWD_CASES if not run_bwd(c)]
    sys.exit(1 if bad else 0)
