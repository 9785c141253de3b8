"""Development diagnostic: hand-placed dropout dK/dV against the general kernel (dV pattern)."""
import torch

from fa2_triton_amd import _lib as L
from fa2_triton_amd.backward import _flash_attn_backward
from fa2_triton_amd.forward import _flash_attn_forward
from fa2_triton_amd.utils import dropout_mask_words
from tests.core import generate_test_data

for (b, hq, hkv, s, causal, p) in [(1, 1, 1, 256, False, 0.2), (1, 1, 1, 256, False, 0.0001), (2, 4, 2, 1024, True, 0.2)]:
    q, k, v, do = generate_test_data(b, hq, hkv, s, s, 128, torch.bfloat16)
    words = torch.empty(dropout_mask_words(b, hq, s, s), dtype=torch.int32, device="cuda")
    o, lse, scale, seed = _flash_attn_forward(q, k, v, None, None, p, causal, None, 4321, dropout_mask=words)
    L.set_path_policy(0, 0)
    hp = _flash_attn_backward(do, q, k, v, None, None, o, lse, p, causal, scale, seed, dropout_mask=words)
    L.set_path_policy(L.PATH_DKDV_HP, 0)
    gen = _flash_attn_backward(do, q, k, v, None, None, o, lse, p, causal, scale, seed, dropout_mask=words)
    L.set_path_policy(0, 0)
    dvh, dvg = hp[2].float(), gen[2].float()
    err = (dvh - dvg).abs()
    print((b, hq, hkv, s, causal, p), "dk equal", torch.equal(hp[1], gen[1]), "dv max err", err.max().item(),
          "max", dvg.abs().max().item())
    # error per key (row of dV) and per head-dim column
    ek = err.amax(dim=(0, 2, 3))  # [S]
    ed = err.amax(dim=(0, 1, 2))  # [D]
    print("  keys with err > 1e-2:", (ek > 1e-2).nonzero().flatten()[:40].tolist())
    print("  key err by key%64 :", [round(x, 3) for x in ek.view(-1, 64).amax(0).tolist()][:64])
    print("  d err by d%32:", [round(x, 3) for x in ed.view(-1, 32).amax(0).tolist()])
    r = (dvh / dvg.where(dvg.abs() > 1e-3, torch.ones_like(dvg)))
    print("  ratio quantiles", torch.quantile(r.flatten()[:100000], torch.tensor([0.01, 0.5, 0.99], device="cuda")).tolist())
