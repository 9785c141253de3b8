"""Benchmark: attention TFLOP/s (fwd & fwd+bwd) at S=4096 D=128 bf16 and % of MFMA peak.

Workload (BASELINE.json configs[2], the config the metric is quoted on): per GPU
B=8 H=32 S=4096 D=128 bf16, causal, forward + backward through the autograd op
`fa2_triton_amd.flash_attn_func` on synthetic N(0, 0.5) inputs resident in HBM.  One step =
one forward + one backward of that batch.  With N GPUs each rank runs its own B=8 shard
(configs[3]: B=64 over 8 GPUs), no collectives on the data path (weak scaling).

FLOPs are algorithmic: fwd = 4 B H S^2 D / 2 (causal), bwd = 2.5 fwd.

Besides the step time, every launch of the path -- the forward, and the backward's delta,
dK/dV (+ dS tiles) and dQ = dS K kernels (fa2_bwd_stages; without the dS workspace: the
recompute dQ kernel, which also computes delta, and dK/dV) -- is timed with HIP events on the
stream it runs on.  `roofline`
is the dominant (longest) kernel, `roofline_fwd` the north-star forward kernel, each with its
algorithmic FLOPs per launch and the HBM bytes per launch from the committed rocprofv3 PMC
summary (profiles/*_pmc.json).  Rank 0 also times the CPU oracle (oracle/reference.py, fp32,
torch CPU threads) on a bounded slice of the same workload for `cpu_baseline`.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import math
import os
import sys
import time

import torch

PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md: ~8 TB/s)
METRIC = "attention TFLOP/s (fwd & fwd+bwd) at S=4096 D=128 bf16; % of MFMA peak"


def attn_flops(b, h, sq, sk, d, causal):
    f = 4.0 * b * h * sq * sk * d
    return f * 0.5 if causal else f


def reduce_elapsed(elapsed: float, dist, device) -> float:
    """Slowest rank's wall time: the job is done when every shard is (max over ranks)."""
    if dist is None:
        return elapsed
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def job_throughput(f_fwd: float, steps: int, world: int, elapsed: float):
    """Whole-job algorithmic TFLOP/s (fwd + bwd = 3.5 fwd per step per rank) and ms per step."""
    return 3.5 * f_fwd * steps * world / elapsed / 1e12, elapsed / steps * 1e3


def shard_batch(global_batch: int, world: int, rank: int):
    """Batch rows [lo, hi) of this rank (configs[3]: B=64 over 8 GPUs -> 8 per rank)."""
    per = global_batch // world
    return rank * per, rank * per + per


def load_pmc():
    """HBM bytes per launch from the latest committed rocprofv3 PMC summary (profiles/*_pmc.json,
    FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md), valid for the default workload only."""
    import glob

    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*_pmc.json")))
    if not files:
        return {}
    data = json.load(open(files[-1]))
    return {k.replace("fa2::", ""): v for k, v in data.items()}


def cpu_baseline(b, h, s, d, causal, budget_s=20.0):
    """Time the fp32 oracle (fwd+bwd) on the host; slice of the same workload."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle.reference import attention_reference

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    heads = h
    # bound memory/time: one batch element, shrink heads until a rep fits the budget
    best = None
    while heads >= 1:
        q = (torch.randn(1, s, heads, d, generator=g) * 0.5).requires_grad_()
        k = (torch.randn(1, s, heads, d, generator=g) * 0.5).requires_grad_()
        v = (torch.randn(1, s, heads, d, generator=g) * 0.5).requires_grad_()
        do = torch.randn(1, s, heads, d, generator=g)
        t0 = time.perf_counter()
        out = attention_reference(q, k, v, causal=causal)
        torch.autograd.grad(out, (q, k, v), do)
        dt = time.perf_counter() - t0
        best = (heads, dt)
        if dt <= budget_s:
            break
        heads //= 2
    heads, dt = best
    reps = 1
    while dt * reps < 10.0 and reps < 8:  # about 10 s of CPU work in total
        t0 = time.perf_counter()
        out = attention_reference(q, k, v, causal=causal)
        torch.autograd.grad(out, (q, k, v), do)
        dt = (dt * reps + time.perf_counter() - t0) / (reps + 1)
        reps += 1
    flops = 3.5 * attn_flops(1, heads, s, s, d, causal)
    return {
        "value": flops / dt / 1e12,
        "unit": "TFLOP/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle fp32 fwd+bwd, B=1 H={heads} S={s} D={d} causal={causal} (slice of the workload), "
                  f"mean of {reps} reps, {dt:.2f} s each",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--seqlen", type=int, default=4096)
    ap.add_argument("--head-dim", type=int, default=128)
    ap.add_argument("--no-causal", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)

    from fa2_triton_amd import flash_attn_func
    from fa2_triton_amd.backward import _flash_attn_backward, alloc_ds_workspace
    from fa2_triton_amd.forward import _flash_attn_forward

    # weak scaling: the global batch is --batch per GPU; this rank owns rows [lo, hi) of it
    lo, hi = shard_batch(args.batch * world, world, rank)
    b, h, s, d = hi - lo, args.heads, args.seqlen, args.head_dim
    causal = not args.no_causal
    dtype = torch.bfloat16
    torch.manual_seed(1234 + rank)
    q = torch.empty(b, s, h, d, device=device, dtype=dtype).normal_(0, 0.5).requires_grad_()
    k = torch.empty(b, s, h, d, device=device, dtype=dtype).normal_(0, 0.5).requires_grad_()
    v = torch.empty(b, s, h, d, device=device, dtype=dtype).normal_(0, 0.5).requires_grad_()
    do = torch.randn(b, s, h, d, device=device, dtype=dtype)

    def step():
        out = flash_attn_func(q, k, v, causal=causal)
        torch.autograd.grad(out, (q, k, v), do)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = reduce_elapsed(time.perf_counter() - t0, dist, device)

    f_fwd = attn_flops(b, h, s, s, d, causal)
    value, ms_per_step = job_throughput(f_fwd, args.steps, world, elapsed)

    # ---- per-launch timing with HIP events on the launch stream ---------------------------
    # fwd: one launch; bwd: its launches timed one by one (fa2_bwd_stages).  With the dS
    # workspace (the default at this size): delta, dK/dV (+ dS tiles), dQ = dS K; without it:
    # dQ (recomputes S, dP; also writes delta), then dK/dV.
    reps = max(5, args.steps)
    stream = torch.cuda.current_stream(device)
    with torch.no_grad():
        o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        delta = torch.empty_like(lse)  # shared by the stage calls: written first, read by dK/dV
        ws = alloc_ds_workspace(q, k)  # shared too: dK/dV writes the dS tiles dQ reads

        def bwd(stages):
            return lambda: _flash_attn_backward(do, q, k, v, None, None, o, lse, 0.0, causal, None, None,
                                                _stages=stages, _delta=delta, _ds_ws=ws, _use_ds=ws is not None)

        calls = {"fwd_kernel": lambda: _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)}
        if ws is not None:
            calls.update(delta_kernel=bwd(1), dkdv_kernel=bwd(2), dq_kernel=bwd(4))
        else:
            calls.update(dq_kernel=bwd(4), dkdv_kernel=bwd(2))
        times = {}
        for name, fn in calls.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            times[name] = e0.elapsed_time(e1) / reps * 1e-3
        del ws
    t_fwd = times["fwd_kernel"]
    t_bwd = sum(t for n, t in times.items() if n != "fwd_kernel")
    fwd_tf = f_fwd / t_fwd / 1e12
    bwd_tf = 2.5 * f_fwd / t_bwd / 1e12
    # Algorithmic FLOPs per launch: fwd = F; the backward's 5 GEMM-units
    # (2.5 F) are split as S, dP, dV, dK -> dK/dV kernel (2 F) and dQ -> dQ kernel (0.5 F).
    # The recompute dQ kernel also recomputes S and dP (1 F executed but not algorithmic); the
    # dS-path dQ kernel executes exactly its 0.5 F, and is bound by HBM (the dS stream).
    ds_path = "delta_kernel" in times
    algo = {"fwd_kernel": f_fwd, "dkdv_kernel": 2.0 * f_fwd, "dq_kernel": 0.5 * f_fwd, "delta_kernel": 0.0}
    executed = dict(algo, dq_kernel=(0.5 if ds_path else 1.5) * f_fwd)
    # HBM bytes the dS-path dQ kernel must move: the dS tiles it reads (2 KiB per visited
    # 32 x 32 (query, key) tile) + K once + dQ written
    nt = -(-s // 32)
    tiles = nt * (nt + 1) // 2 if causal else nt * nt
    dq_bytes = b * h * tiles * 2048 + b * s * h * d * 2 * 2
    kernels = {
        name: {
            "ms": round(t * 1e3, 4),
            "algorithmic_tflops": round(algo[name] / t / 1e12, 1),
            "executed_mfma_tflops": round(executed[name] / t / 1e12, 1),
        }
        for name, t in times.items()
    }
    if ds_path:
        kernels["dq_kernel"]["hbm_gbps"] = round(dq_bytes / times["dq_kernel"] / 1e9, 1)
    pmc = load_pmc()
    pmc["_workload_ok"] = (b, h, s, d, causal) == (8, 32, 4096, 128, True)
    dominant = max(("fwd_kernel", "dkdv_kernel", "dq_kernel"), key=lambda n: times[n])

    # device symbols the default workload dispatches to (aligned D, no bias, no dropout)
    symbol = {"fwd_kernel": "fwd_pipe_kernel", "dkdv_kernel": "dkdv_kernel", "delta_kernel": "delta_kernel",
              "dq_kernel": "dq_ds_kernel" if ds_path else "dq_kernel"}

    def roofline(name):
        traffic = pmc.get(symbol[name], {}).get("hbm_bytes_per_launch") if pmc.get("_workload_ok") else None
        if name == "dq_kernel" and ds_path:
            ach = dq_bytes / times[name] / 1e9
            return {"bound": "hbm", "kernel": f"fa2::{symbol[name]}", "achieved": round(ach, 1), "peak": PEAK_HBM_GBPS,
                    "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBPS, 4), "traffic": traffic,
                    "algorithmic_bytes_per_launch": dq_bytes}
        ach = algo[name] / times[name] / 1e12
        return {
            "bound": "mfma",
            "kernel": f"fa2::{symbol[name]}",
            "achieved": round(ach, 2),
            "peak": PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(ach / PEAK_TFLOPS, 4),
            "traffic": traffic,
            "algorithmic_flop_per_launch": algo[name],
        }

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(b, h, s, d, causal)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic N(0,0.5) Q/K/V, N(0,1) dO, resident in HBM",
        "config": {
            "workload": f"B={b} H={h} S={s} D={d} bf16 {'causal' if causal else 'non-causal'} fwd+bwd per GPU "
                        "(BASELINE.json configs[2]; configs[3] when batch-sharded over 8 GPUs)",
            "global_batch": b * world,
            "seq_len": s,
            "heads": h,
            "head_dim": d,
            "causal": causal,
            "parallelism": f"batch-sharded x{world}, independent per-GPU launches, no collectives",
        },
        "fwd_tflops": round(fwd_tf, 2),
        "bwd_tflops": round(bwd_tf, 2),
        "fwd_ms": round(t_fwd * 1e3, 4),
        "bwd_ms": round(t_bwd * 1e3, 4),
        "pct_of_peak_fwd": round(100 * fwd_tf / PEAK_TFLOPS, 2),
        "pct_of_peak_fwd_bwd": round(100 * value / world / PEAK_TFLOPS, 2),
        "roofline": roofline(dominant),
        "roofline_fwd": roofline("fwd_kernel"),
        "roofline_dq": roofline("dq_kernel"),
        "bwd_path": "dS workspace (delta, dK/dV + dS tiles, dQ = dS K)" if ds_path else "recompute dQ",
        "kernels": kernels,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
