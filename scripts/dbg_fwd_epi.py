"""Debug: where the hand-placed forward's output differs from the pipelined one (rows / blocks)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd import _lib as L
from fa2_triton_amd.forward import _flash_attn_forward

for (b, hq, hkv, s, causal, cap) in [(2, 4, 2, 512, True, 0), (2, 4, 2, 512, False, 0), (1, 1, 1, 1024, True, 1), (1, 1, 1, 1024, False, 1)]:
    torch.manual_seed(0)
    q = (torch.randn(b, s, hq, 128, device="cuda") * 0.5).to(torch.bfloat16)
    k = (torch.randn(b, s, hkv, 128, device="cuda") * 0.5).to(torch.bfloat16)
    v = (torch.randn(b, s, hkv, 128, device="cuda") * 0.5).to(torch.bfloat16)
    res = {}
    for tag, dis in (("hp", 0), ("pipe", L.PATH_FWD_HP)):
        L.set_path_policy(dis, cap)
        o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        torch.cuda.synchronize()
        res[tag] = (o.float(), lse.float())
    L.set_path_policy(0, 0)
    d = (res["hp"][0] - res["pipe"][0]).abs()
    bad = ~(d <= 0.05)  # NaN or large
    print((b, hq, hkv, s, causal, cap), "bad elements", int(bad.sum()), "of", bad.numel())
    if bad.any():
        idx = bad.nonzero()
        rows = idx[:, 1]
        print("  rows % 256 hist (by 32):", torch.bincount(rows % 256 // 32, minlength=8).tolist())
        print("  rows // 256:", torch.bincount(rows // 256).tolist(), " heads:", torch.bincount(idx[:, 2]).tolist(), " batch:", torch.bincount(idx[:, 0]).tolist())
        print("  cols hist (by 16):", torch.bincount(idx[:, 3] // 16, minlength=8).tolist())
        print("  nan:", int(torch.isnan(res["hp"][0]).sum()))
    ld = (res["hp"][1][:, :, :s] - res["pipe"][1][:, :, :s]).abs()
    print("  lse bad:", int((~(ld <= 1e-2)).sum()))
