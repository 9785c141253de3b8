"""Context numbers: this operator vs torch SDPA and torch FlexAttention on ROCm.

SURVEY.md section 8(f) rank 4.  The reference's comparison harness
(/root/reference/benchmarks/utils.py:22-93) times "Liger" (this operator) against "Flex":
`torch.compile(flex_attention, dynamic=False, mode="max-autotune-no-cudagraphs")` with a
`q_idx >= kv_idx` block mask when causal (/root/reference/src/other_implementations/
flex_attention.py:9-26).  The same leg is timed here (--flex-mode picks the compile mode; the
default "default" skips the autotuning sweep, which takes minutes per shape), beside
F.scaled_dot_product_attention.  Flex and SDPA get contiguous [B, H, S, D] tensors (their native
layout; the reference's harness transposes the same way, benchmarks/utils.py:66-69), ours the
reference's [B, S, H, D].  All legs see the same synthetic N(0, 0.5) inputs resident in HBM.
Times are medians of HIP-event-timed calls after warmup; TFLOP/s use the algorithmic count of
SURVEY.md section 8(d) (fwd 4 B H S^2 D, x0.5 causal; bwd 2.5x fwd).

usage: python scripts/compare_sdpa.py [--reps 20] [--no-flex] [--flex-mode default]
       (prints one JSON line per config)
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fa2_triton_amd import flash_attn_func  # noqa: E402

CONFIGS = [
    # name, B, Hq, Hkv, S, D, causal, dtype
    ("cfg2", 8, 16, 16, 1024, 64, False, torch.bfloat16),
    ("cfg3", 8, 32, 32, 4096, 128, True, torch.bfloat16),
    ("cfg3-noncausal", 8, 32, 32, 4096, 128, False, torch.bfloat16),
    ("cfg5-gqa", 2, 32, 8, 8192, 128, True, torch.float16),
    # MQA at batch 1: 32 dK/dV key blocks without the q-head split (tests/test_gqa_split.py)
    ("mqa-b1", 1, 32, 1, 4096, 128, True, torch.bfloat16),
]


def timed(fn, reps, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-flex", action="store_true")
    ap.add_argument("--flex-mode", default="default")
    ap.add_argument("--only", default="", help="comma-separated config names")
    args = ap.parse_args()
    torch.manual_seed(0)
    flex = None
    if not args.no_flex:
        try:
            from torch.nn.attention.flex_attention import create_block_mask, flex_attention

            torch._dynamo.config.cache_size_limit = 1000
            flex = torch.compile(flex_attention, dynamic=False, mode=args.flex_mode)
        except Exception as exc:  # no inductor backend on this build
            print(json.dumps({"flex_unavailable": f"{type(exc).__name__}: {exc}"[:200]}), flush=True)
    for name, b, hq, hkv, s, d, causal, dtype in CONFIGS:
        if args.only and name not in args.only.split(","):
            continue
        fl = 4 * b * hq * s * s * d * (0.5 if causal else 1.0)
        q = torch.empty(b, s, hq, d, device="cuda", dtype=dtype).normal_(0, 0.5).requires_grad_()
        k = torch.empty(b, s, hkv, d, device="cuda", dtype=dtype).normal_(0, 0.5).requires_grad_()
        v = torch.empty(b, s, hkv, d, device="cuda", dtype=dtype).normal_(0, 0.5).requires_grad_()
        do = torch.randn_like(q)
        qs, ks, vs = (t.detach().transpose(1, 2).contiguous().requires_grad_() for t in (q, k, v))
        dos = do.transpose(1, 2).contiguous()
        gqa = {"enable_gqa": True} if hkv != hq else {}

        def ours_fwd():
            with torch.no_grad():
                flash_attn_func(q, k, v, None, None, 0.0, causal)

        def ours_fwdbwd():
            o = flash_attn_func(q, k, v, None, None, 0.0, causal)
            torch.autograd.grad(o, (q, k, v), do)

        def sdpa_fwd():
            with torch.no_grad():
                F.scaled_dot_product_attention(qs, ks, vs, is_causal=causal, **gqa)

        def sdpa_fwdbwd():
            o = F.scaled_dot_product_attention(qs, ks, vs, is_causal=causal, **gqa)
            torch.autograd.grad(o, (qs, ks, vs), dos)

        block_mask = None
        if flex is not None and causal:
            block_mask = create_block_mask(lambda b_, h_, qi, ki: qi >= ki, B=None, H=None, Q_LEN=s, KV_LEN=s)
        fkw = {"enable_gqa": True} if hkv != hq else {}

        def flex_fwd():
            with torch.no_grad():
                flex(qs, ks, vs, block_mask=block_mask, **fkw)

        def flex_fwdbwd():
            o = flex(qs, ks, vs, block_mask=block_mask, **fkw)
            torch.autograd.grad(o, (qs, ks, vs), dos)

        legs = [("ours_fwd", ours_fwd, 1.0), ("ours_fwdbwd", ours_fwdbwd, 3.5),
                ("sdpa_fwd", sdpa_fwd, 1.0), ("sdpa_fwdbwd", sdpa_fwdbwd, 3.5)]
        if flex is not None:
            legs += [("flex_fwd", flex_fwd, 1.0), ("flex_fwdbwd", flex_fwdbwd, 3.5)]
        row = {"config": name, "B": b, "Hq": hq, "Hkv": hkv, "S": s, "D": d, "causal": causal,
               "dtype": str(dtype).replace("torch.", "")}
        if flex is not None:
            row["flex_mode"] = args.flex_mode
        for tag, fn, mult in legs:
            try:
                ms = timed(fn, args.reps)
                row[tag + "_ms"] = round(ms, 4)
                row[tag + "_tflops"] = round(fl * mult / ms / 1e9, 1)
            except Exception as exc:  # e.g. a backend without GQA support
                row[tag + "_error"] = f"{type(exc).__name__}: {exc}"[:200]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
