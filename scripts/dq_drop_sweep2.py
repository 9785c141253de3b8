import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd.backward import _flash_attn_backward  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402
from fa2_triton_amd.utils import dropout_mask_words  # noqa: E402
# debug build: the dropout variant computes dS without the keep bits -> compare with the plain kernel
for causal in (False, True):
    for s in (64, 256):
        torch.manual_seed(0)
        q, k, v = (torch.randn(1, s, 1, 128, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        do = torch.randn_like(q)
        words = torch.full((dropout_mask_words(1, 1, s, s),), -1, dtype=torch.int32, device="cuda")
        o, lse, scale, seed = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        a = _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.0, causal, scale, None)[0].float()
        c = _flash_attn_backward(do, q, k, v, None, None, o, lse, 1e-30, causal, scale, 5, dropout_mask=words)[0].float()
        d = (a - c).abs()[0, :, 0, :].amax(dim=1)
        print("causal", causal, "S", s, "rb max diff", [round(x, 4) for x in d.view(-1, 32).amax(dim=1).tolist()], flush=True)
