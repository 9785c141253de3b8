"""Debug: the hand-placed dropout forward's effective keep pattern (V = identity over keys)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd import _lib as L
from fa2_triton_amd.forward import _flash_attn_forward
from fa2_triton_amd.utils import dropout_mask_words
from tests.core import unpack_keep_mask

b, h, s, d, p = 1, 1, 128, 128, 0.5
torch.manual_seed(0)
q = (torch.randn(b, s, h, d, device="cuda") * 0.1).to(torch.bfloat16)
k = (torch.randn(b, s, h, d, device="cuda") * 0.1).to(torch.bfloat16)
v = torch.eye(s, d, device="cuda").to(torch.bfloat16).view(b, s, h, d)
for causal in (False, True):
    out = {}
    for tag, dis in (("hp", 0), ("gen", L.PATH_FWD_HP)):
        w = torch.full((dropout_mask_words(b, h, s, s),), -1, dtype=torch.int32, device="cuda")
        L.set_path_policy(dis, 0)
        o, lse, _, seed = _flash_attn_forward(q, k, v, None, None, p, causal, None, 5, dropout_mask=w)
        L.set_path_policy(0, 0)
        out[tag] = (o[0, :, 0, :].float(), w)
    keep = unpack_keep_mask(out["hp"][1], b, h, s, s)[0, 0]
    assert torch.equal(out["hp"][1], out["gen"][1])
    for tag in ("hp", "gen"):
        nz = out[tag][0] != 0
        bad = nz != keep
        if causal:
            vis = torch.arange(s, device="cuda")[None, :] <= torch.arange(s, device="cuda")[:, None]
            bad = bad & vis
        print(causal, tag, "mismatches", int(bad.sum()), "of", int(keep.numel()))
        if bad.any():
            idx = bad.nonzero()[:24].tolist()
            print("  first (row, key):", idx)
            keys = bad.nonzero()[:, 1]
            print("  key % 32 histogram:", torch.bincount(keys % 32, minlength=32).tolist())
            rows = bad.nonzero()[:, 0]
            print("  row % 64 histogram:", torch.bincount(rows % 64, minlength=64).tolist())
