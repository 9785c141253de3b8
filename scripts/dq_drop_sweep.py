"""Dev: hand-placed dropout dQ vs dq_kernel over small shapes (which fail, which row blocks)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd.backward import _flash_attn_backward  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402
from fa2_triton_amd.utils import dropout_mask_words  # noqa: E402

for causal in (False, True):
    for s in (64, 128, 256, 320, 512):
        b, hq = 1, 1
        torch.manual_seed(0)
        q, k, v = (torch.randn(b, s, hq, 128, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        do = torch.randn_like(q)
        words = torch.full((dropout_mask_words(b, hq, s, s),), -1, dtype=torch.int32, device="cuda")
        o, lse, scale, seed = _flash_attn_forward(q, k, v, None, None, 0.2, causal, None, 99, dropout_mask=words)
        r = []
        for env in ("1", "0"):
            os.environ["FA2_DQ_HP"] = env
            r.append(_flash_attn_backward(do, q, k, v, None, None, o, lse, 0.2, causal, scale, seed, dropout_mask=words)[0].float())
        d = (r[0] - r[1]).abs()[0, :, 0, :].amax(dim=1)
        bad = [i for i, x in enumerate(d.view(-1, 32).amax(dim=1).tolist()) if x > 0]
        print("causal", causal, "S", s, "bad row blocks", bad, flush=True)
