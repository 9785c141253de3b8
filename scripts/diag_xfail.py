"""Diagnose the strict xfail (bf16 MQA 16:1, causal, Sq=Sk=777): where its one-ulp dV miss comes
from.  Prints, at the element the tolerance rule flags, the fp32 oracle dV, the oracle's bf16 value,
the low-precision PyTorch run (the rule's err_pt baseline), this library's dV, and an fp32
emulation of the kernel's arithmetic (P rounded to bf16 before the P^T dO product, as the MFMA
operand is, fp32 accumulation over the 16 q-heads x 777 rows).  Dev tool (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd import flash_attn_func  # noqa: E402
from oracle.reference import attention_reference  # noqa: E402
from tests.core import generate_test_data  # noqa: E402

b, hq, hkv, s, d = 1, 16, 1, 777, 128
q, k, v, do = generate_test_data(b, hq, hkv, s, s, d, torch.bfloat16)
common = dict(causal=True)
out_ref = attention_reference(q, k, v, **common)
out_pt = attention_reference(q, k, v, upcast=False, reorder_ops=True, **common)
out = flash_attn_func(q, k, v, causal=True)
dv_ref, = torch.autograd.grad(out_ref, (v,), do, retain_graph=True)
dv_pt, = torch.autograd.grad(out_pt, (v,), do, retain_graph=True)
dv, = torch.autograd.grad(out, (v,), do)
err = (dv.float() - dv_ref.float()).abs()
err_pt = (dv_pt.float() - dv_ref.float()).abs()
idx = tuple(int(x) for x in torch.nonzero(err == err.max())[0])
print("max err", err.max().item(), "at", idx, " err_pt max", err_pt.max().item(),
      " rule: err <= 3 err_pt + 1e-5 ->", err.max().item() <= 3 * err_pt.max().item() + 1e-5)

# fp32 dV of that key row two ways: exact P (oracle) and P rounded to bf16 (the kernel's MFMA operand)
qf, kf, vf, dof = (t.detach().float()[0].transpose(0, 1) for t in (q, k, v, do))  # [H, S, D]
kf, vf = kf.expand(hq, -1, -1), vf.expand(hq, -1, -1)
sc = qf @ kf.transpose(-1, -2) / d ** 0.5
sc = sc.masked_fill(torch.ones(s, s, device=sc.device).triu(1).bool(), float("-inf"))
p = torch.softmax(sc, dim=-1)
j, c = idx[1], idx[3]
exact = (p[:, :, j] * dof[:, :, c]).sum().item()
emul = (p[:, :, j].bfloat16().float() * dof[:, :, c]).sum().item()
print(f"dV[{j},{c}]: oracle fp32 {exact:.6f} -> bf16 {torch.tensor(exact).bfloat16().item()}; "
      f"bf16-P emulation fp32 {emul:.6f} -> bf16 {torch.tensor(emul).bfloat16().item()}; "
      f"library {dv[0, j, 0, c].item()}; PyTorch low-precision run {dv_pt[0, j, 0, c].item()}; "
      f"bf16 rounding boundary between -16.5 and -16.625: -16.5625")
