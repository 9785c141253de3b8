import os, sys, torch
sys.path.insert(0, os.getcwd())
from fa2_triton_amd import flash_attn_func
from oracle.reference import attention_reference
from tests.core import generate_test_data
for case in [(1,16,1,777,777,128,True), (1,16,1,777,901,128,False), (1,8,1,512,512,128,True)]:
    b,hq,hkv,sq,sk,d,causal = case
    q,k,v,do = generate_test_data(b,hq,hkv,sq,sk,d,torch.bfloat16)
    ref = attention_reference(q,k,v,causal=causal)
    gr = torch.autograd.grad(ref,(q,k,v),do)
    pt = attention_reference(q,k,v,causal=causal,upcast=False,reorder_ops=True)
    gp = torch.autograd.grad(pt,(q,k,v),do)
    for mode in ["1","0"]:
        os.environ["FA2_DKV_SPLIT"]=mode
        out = flash_attn_func(q,k,v,None,None,0.0,causal)
        g = torch.autograd.grad(out,(q,k,v),do)
        for n,x,y,z in zip("qkv",g,gr,gp):
            e=(x.float()-y.float()).abs(); i=e.argmax()
            print(case, "split" if mode=="1" else "nosplit", "d"+n, "err", e.max().item(), "at ref", y.flatten()[i].item(), "ours", x.flatten()[i].item(), "pt err", (z.float()-y.float()).abs().max().item(), "max|ref|", y.abs().max().item())
