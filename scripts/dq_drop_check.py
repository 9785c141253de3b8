"""Dev check: hand-placed dQ with dropout (saved keep words) vs dq_kernel (saved words, and
Philox regeneration), bitwise, on a few shapes incl. varlen."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd.backward import _flash_attn_backward  # noqa: E402
from fa2_triton_amd.forward import _flash_attn_forward  # noqa: E402
from fa2_triton_amd.utils import dropout_mask_words  # noqa: E402

for (b, hq, hkv, s, causal, lens) in ((1, 2, 2, 512, False, None), (1, 2, 2, 512, True, None), (2, 4, 2, 300, False, None),
                                     (3, 4, 2, 300, False, [300, 173, 1]), (3, 4, 2, 300, True, [300, 173, 1])):
    torch.manual_seed(0)
    q, k, v = (torch.randn(b, s, h, 128, device="cuda", dtype=torch.bfloat16) for h in (hq, hkv, hkv))
    do = torch.randn_like(q)
    mask = None
    if lens:
        mask = torch.zeros(b, s, dtype=torch.bool, device="cuda")
        for i, n in enumerate(lens):
            mask[i, :n] = True
    words = torch.full((dropout_mask_words(b, hq, s, s),), -1, dtype=torch.int32, device="cuda")
    o, lse, scale, seed = _flash_attn_forward(q, k, v, mask, None, 0.2, causal, None, 99, dropout_mask=words)
    res = {}
    for tag, env, w in (("hp", "1", words), ("old", "0", words), ("regen", "0", None)):
        os.environ["FA2_DQ_HP"] = env
        res[tag] = _flash_attn_backward(do, q, k, v, None, mask, o, lse, 0.2, causal, scale, seed, dropout_mask=w)
    os.environ.pop("FA2_DQ_HP")
    out = []
    for name, i in (("dq", 0), ("dk", 1), ("dv", 2)):
        a, bb, c = res["hp"][i].float(), res["old"][i].float(), res["regen"][i].float()
        out.append(f"{name}: hp-old {(a - bb).abs().max().item():.3e} ({(a != bb).sum().item()} diff) old-regen {(bb - c).abs().max().item():.3e}")
    print((b, hq, hkv, s, causal, lens), " | ".join(out), flush=True)

# where do hp and old differ (non-causal S=512)?
torch.manual_seed(0)
b, hq, s = 1, 1, 512
q, k, v = (torch.randn(b, s, hq, 128, device="cuda", dtype=torch.bfloat16) for _ in range(3))
do = torch.randn_like(q)
words = torch.full((dropout_mask_words(b, hq, s, s),), -1, dtype=torch.int32, device="cuda")
o, lse, scale, seed = _flash_attn_forward(q, k, v, None, None, 0.2, False, None, 99, dropout_mask=words)
os.environ["FA2_DQ_HP"] = "1"
a = _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.2, False, scale, seed, dropout_mask=words)[0].float()
os.environ["FA2_DQ_HP"] = "0"
c = _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.2, False, scale, seed, dropout_mask=words)[0].float()
os.environ["FA2_DQ_HP"] = "1"
z = torch.zeros(dropout_mask_words(b, hq, s, s), dtype=torch.int32, device="cuda") - 1  # keep everything
d = (a - c).abs()[0, :, 0, :].amax(dim=1)
print("rows with diff:", (d > 0).nonzero().flatten().tolist()[:80])
print("row-block max diff:", [round(x, 4) for x in d.view(-1, 32).amax(dim=1).tolist()])
# synthetic keep words: all kept / only key tile t kept, to see which tiles' words go wrong
for name, fill in (("all", None), ("tile0", 0), ("tile1", 1), ("tile3", 3)):
    wz = torch.full_like(words, -1 if fill is None else 0)
    if fill is not None:
        nrb, ncw = (s + 31) // 32, (s + 31) // 32
        wv = wz.view(b * hq, nrb, ncw, 32)
        wv[:, :, 2 * fill: 2 * fill + 2, :] = -1
    os.environ["FA2_DQ_HP"] = "1"
    a = _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.2, False, scale, seed, dropout_mask=wz)[0].float()
    os.environ["FA2_DQ_HP"] = "0"
    c = _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.2, False, scale, seed, dropout_mask=wz)[0].float()
    d = (a - c).abs()[0, :, 0, :].amax(dim=1)
    print(name, "row-block max diff:", [round(x, 4) for x in d.view(-1, 32).amax(dim=1).tolist()])

# which one is right: fp32 torch reference with the saved keep bits (non-causal S=512, H=1)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_dropout_bwd import _unpack_keep_mask  # noqa: E402
keep = _unpack_keep_mask(words, b, hq, s, s).float()  # [B, H, S, S]
qf, kf, vf = (t.detach().float().transpose(1, 2).requires_grad_() for t in (q, k, v))
pr = torch.softmax(qf @ kf.transpose(-1, -2) * scale, dim=-1)
out = (pr * keep / (1 - 0.2)) @ vf
gq, = torch.autograd.grad(out, (qf,), do.float().transpose(1, 2))
gq = gq.transpose(1, 2)
os.environ["FA2_DQ_HP"] = "1"
a = _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.2, False, scale, seed, dropout_mask=words)[0].float()
os.environ["FA2_DQ_HP"] = "0"
c = _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.2, False, scale, seed, dropout_mask=words)[0].float()
for tag, x in (("hp", a), ("old", c)):
    d = (x - gq).abs()[0, :, 0, :].amax(dim=1)
    print(tag, "vs fp32 ref, row-block max err:", [round(y, 4) for y in d.view(-1, 32).amax(dim=1).tolist()])
