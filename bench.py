"""Benchmark: attention TFLOP/s (fwd & fwd+bwd) at S=4096 D=128 bf16 and % of MFMA peak.

Workload (BASELINE.json configs[2], the config the metric is quoted on): per GPU
B=8 H=32 S=4096 D=128 bf16, causal, forward + backward through the autograd op
`fa2_triton_amd.flash_attn_func` on synthetic N(0, 0.5) inputs resident in HBM.  One step =
one forward + one backward of that batch.

Multi-GPU (BASELINE.json configs[3]: B=64 over 8 GPUs): one process
per GPU, each running its own batch shard with no collective on the data path; the only
collectives are the barriers around the timed region and the max-reduction of its duration.
  * weak scaling (default): every rank runs B=--batch (8) -> global batch 8 N;
  * strong scaling (--strong): the global batch --global-batch (64) is split B/N per rank.
`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N rank
processes itself (children of this process, which never touches the GPU) and relays rank 0's
line; under torchrun (WORLD_SIZE set) it is one of the ranks.

FLOPs are algorithmic: fwd = 4 B H S^2 D / 2 (causal), bwd = 2.5 fwd.

Besides the step time, every launch of the path -- the forward, and the backward's kernels
(fa2_bwd_stages) -- is timed with HIP events on the stream it runs on.  `roofline` is the
dominant (longest) kernel, `roofline_fwd` the north-star forward kernel, `roofline_dq` the dQ
kernel, each with its algorithmic FLOPs per launch against the bf16 MFMA peak; `traffic` (HBM
bytes per launch) and `mfma_busy_pct` come from the rocprofv3 PMC summary committed under
profiles/ for the same kernel and workload (named in `pmc_source`).  Rank 0 also times the CPU
oracle (oracle/reference.py, fp32, torch CPU threads) on a bounded slice of the same workload,
after the timed region, for `cpu_baseline`.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--strong] [--no-cpu-baseline]
       torchrun --nproc-per-node N bench.py --gpus N ...
       python bench.py --gpus 2 --dry-run      (CPU/gloo: sharding + timing plumbing only)
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md: ~8 TB/s)
N_SIMDS = 1024  # 256 CUs x 4 SIMDs
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


def job_throughput(f_fwd_total: float, steps: int, elapsed: float):
    """Whole-job algorithmic TFLOP/s (fwd + bwd = 3.5 fwd per step, summed over every rank's
    shard) and ms per step."""
    return 3.5 * f_fwd_total * steps / elapsed / 1e12, elapsed / steps * 1e3


def shard_batch(global_batch: int, world: int, rank: int):
    """Batch rows [lo, hi) of this rank: an even split, the first global_batch % world ranks
    one row more (configs[3]: B=64 over 8 GPUs -> rows 8 r .. 8 r + 8)."""
    per, extra = divmod(global_batch, world)
    lo = rank * per + min(rank, extra)
    return lo, lo + per + (1 if rank < extra else 0)


def plan(args, world: int, rank: int):
    """(global batch, this rank's [lo, hi), scaling mode) for weak (default) or strong scaling."""
    if args.strong:
        gb = args.global_batch
        if gb < world:
            raise SystemExit(f"--global-batch {gb} < {world} ranks")
        return gb, shard_batch(gb, world, rank), "strong"
    gb = args.batch * world
    return gb, shard_batch(gb, world, rank), "weak"


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Run this script as n rank processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, rendezvous
    on 127.0.0.1) and wait for them; exits with the first non-zero status.  The parent only
    spawns: it never initialises the GPU (children are started, never exec'd into)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    for p in procs:
        code = p.wait()
        rc = rc or code
    return rc


def cpu_info() -> dict:
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        affinity = os.cpu_count() or 1
    return {"cpu_model": model, "cpus_visible": os.cpu_count(), "cpus_in_affinity": affinity}


def cpu_threads() -> int:
    """Every CPU this process may run on, capped by the box's stated share (OMP_NUM_THREADS,
    set to the GPU box's per-GPU CPU share) when that is set."""
    n = cpu_info()["cpus_in_affinity"]
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(h, s, d, causal, budget_s=20.0):
    """Time the fp32 oracle (fwd+bwd) on the host on a slice of the same workload (one batch
    row, heads halved until one rep fits the budget), about 10-30 s of CPU work in all."""
    sys.path.insert(0, ROOT)
    from oracle.reference import attention_reference

    threads = cpu_threads()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    heads = h
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
    while dt * reps < 10.0 and reps < 8:
        t0 = time.perf_counter()
        out = attention_reference(q, k, v, causal=causal)
        torch.autograd.grad(out, (q, k, v), do)
        dt = (dt * reps + time.perf_counter() - t0) / (reps + 1)
        reps += 1
    flops = 3.5 * attn_flops(1, heads, s, s, d, causal)
    info = cpu_info()
    return {
        "value": flops / dt / 1e12,
        "unit": "TFLOP/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle fp32 fwd+bwd (oracle/reference.py), B=1 H={heads} S={s} D={d} causal={causal} "
                  f"(slice of the workload), mean of {reps} reps, {dt:.2f} s each, {threads} torch threads",
        **info,
    }


def load_pmc():
    """The latest committed rocprofv3 PMC summary (profiles/*_pmc.json; HBM bytes per launch =
    FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md; MFMA-busy cycles; GRBM_GUI_ACTIVE),
    recorded for the default workload only.  Returns (dict by kernel symbol, file name)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    if not files:
        return {}, None
    data = json.load(open(files[-1]))
    return {k.replace("fa2::", ""): v for k, v in data.items()}, os.path.relpath(files[-1], ROOT)


def pmc_fields(rec: dict, launch_s: float) -> dict:
    """traffic / MFMA-busy / effective clock of one kernel from its PMC record."""
    out = {"traffic": rec.get("hbm_bytes_per_launch")}
    grbm = rec.get("GRBM_GUI_ACTIVE")
    busy = rec.get("SQ_VALU_MFMA_BUSY_CYCLES")
    if grbm and busy is not None:
        out["mfma_busy_pct"] = round(100.0 * busy / (N_SIMDS * grbm / 8.0), 1)
    if grbm and launch_s:
        out["clock_ghz"] = round(grbm / 8.0 / launch_s / 1e9, 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="per-GPU batch (weak scaling)")
    ap.add_argument("--strong", action="store_true", help="split --global-batch over the GPUs")
    ap.add_argument("--global-batch", type=int, default=64)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--seqlen", type=int, default=4096)
    ap.add_argument("--head-dim", type=int, default=128)
    ap.add_argument("--no-causal", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo: sharding + timing plumbing, no kernels")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    dist = None
    if args.dry_run:
        device = torch.device("cpu")
        if world > 1:
            import torch.distributed as dist

            dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        device = torch.device("cuda", local_rank)
        if world > 1:
            import torch.distributed as dist

            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=device)

    global_batch, (lo, hi), scaling = plan(args, world, rank)
    b, h, s, d = hi - lo, args.heads, args.seqlen, args.head_dim
    causal = not args.no_causal
    f_fwd_total = attn_flops(global_batch, h, s, s, d, causal)  # every rank's shard
    f_fwd = attn_flops(b, h, s, s, d, causal)                   # this rank's shard

    if args.dry_run:
        if dist:
            dist.barrier()
        elapsed = reduce_elapsed(0.001 * (1 + rank), dist, device)
        shards = [(lo, hi)]
        if dist:
            shards = [None] * world
            dist.all_gather_object(shards, (lo, hi))
        if rank == 0:
            value, ms = job_throughput(f_fwd_total, args.steps, elapsed)
            print(json.dumps({"dry_run": True, "n_gpus": world, "scaling": scaling, "global_batch": global_batch,
                              "shards": shards, "elapsed": elapsed, "value": value, "ms_per_step": ms}), flush=True)
        if dist:
            dist.destroy_process_group()
        return

    from fa2_triton_amd import flash_attn_func
    from fa2_triton_amd.backward import _flash_attn_backward, alloc_ds_workspace
    from fa2_triton_amd.forward import _flash_attn_forward

    dtype = torch.bfloat16
    # this rank's rows of the synthetic global batch (seeded per shard start)
    torch.manual_seed(1234 + lo)
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
    value, ms_per_step = job_throughput(f_fwd_total, args.steps, elapsed)

    # ---- per-launch timing with HIP events on the launch stream ---------------------------
    # fwd: one launch; bwd: its launches timed one by one (fa2_bwd_stages).  With the dS
    # workspace: delta, dK/dV (+ dS tiles), dQ = dS K; without it: dQ (recomputes S, dP; also
    # writes delta), then dK/dV.
    reps = max(5, args.steps)
    stream = torch.cuda.current_stream(device)
    with torch.no_grad():
        o, lse, _, _ = _flash_attn_forward(q, k, v, None, None, 0.0, causal, None, None)
        delta = torch.empty_like(lse)  # shared by the stage calls: written first, read by dK/dV
        ws = alloc_ds_workspace(q, k, v, o, do, causal)  # shared too: dK/dV writes the dS tiles dQ reads

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
        ws_bytes = 0 if ws is None else ws.numel()
        del ws
    t_fwd = times["fwd_kernel"]
    t_bwd = sum(t for n, t in times.items() if n != "fwd_kernel")
    fwd_tf = f_fwd / t_fwd / 1e12
    bwd_tf = 2.5 * f_fwd / t_bwd / 1e12
    # Algorithmic FLOPs per launch: fwd = F; the backward's 5
    # GEMM-units (2.5 F) are split as S, dP, dV, dK -> dK/dV kernel (2 F) and dQ -> dQ kernel
    # (0.5 F).  The recompute dQ kernel also recomputes S and dP (1 F executed, not
    # algorithmic); the dS-path dQ kernel executes exactly its 0.5 F and streams the dS tiles
    # dK/dV wrote -- bytes of the implementation's choosing, reported as `extra_bytes`, never
    # as the roofline's denominator.
    ds_path = "delta_kernel" in times
    algo = {"fwd_kernel": f_fwd, "dkdv_kernel": 2.0 * f_fwd, "dq_kernel": 0.5 * f_fwd, "delta_kernel": 0.0}
    executed = dict(algo, dq_kernel=(0.5 if ds_path else 1.5) * f_fwd)
    nt = -(-s // 32)
    ds_tiles = nt * (nt + 1) // 2 if causal else nt * nt
    ds_bytes = b * h * ds_tiles * 2048  # dS tiles written by dK/dV and read by dQ (dS path)
    kernels = {
        name: {
            "ms": round(t * 1e3, 4),
            "algorithmic_tflops": round(algo[name] / t / 1e12, 1),
            "executed_mfma_tflops": round(executed[name] / t / 1e12, 1),
        }
        for name, t in times.items()
    }
    if ds_path:
        # delta reads O and dO, writes delta; dQ reads the dS stream + K, writes dQ
        kernels["delta_kernel"]["hbm_gbps"] = round((2 * b * s * h * d * 2 + b * h * s * 4) / times["delta_kernel"] / 1e9, 1)
        kernels["dq_kernel"]["hbm_gbps"] = round((ds_bytes + 2 * b * s * h * d * 2) / times["dq_kernel"] / 1e9, 1)
    pmc, pmc_file = load_pmc()
    workload_ok = (b, h, s, d, causal) == (8, 32, 4096, 128, True)
    dominant = max(("fwd_kernel", "dkdv_kernel", "dq_kernel"), key=lambda n: times[n])

    # device symbols the default workload dispatches to (aligned D, no bias, no dropout)
    symbol = {"fwd_kernel": "fwd_pipe_kernel", "dkdv_kernel": "dkdv_kernel", "delta_kernel": "delta_kernel",
              "dq_kernel": "dq_ds_kernel" if ds_path else "dq_kernel"}

    def roofline(name):
        ach = algo[name] / times[name] / 1e12
        rec = pmc.get(symbol[name], {}) if workload_ok else {}
        r = {
            "bound": "mfma",
            "kernel": f"fa2::{symbol[name]}",
            "achieved": round(ach, 2),
            "peak": PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(ach / PEAK_TFLOPS, 4),
            "algorithmic_flop_per_launch": algo[name],
            "executed_flop_per_launch": executed[name],
            "launch_ms": round(times[name] * 1e3, 4),
        }
        r.update(pmc_fields(rec, times[name]) if rec else {"traffic": None})
        if r["traffic"] is not None:
            r["traffic_ratio"] = None
        if name == "fwd_kernel":
            algo_bytes = 4 * b * s * h * d * 2 + b * h * s * 4  # Q, K, V read, O written, LSE
        elif name == "dkdv_kernel":
            algo_bytes = 6 * b * s * h * d * 2 + 2 * b * h * s * 4  # Q K V dO read, dK dV written, LSE, delta
            if ds_path:
                r["extra_bytes"] = ds_bytes  # dS tiles written for dQ (dS path)
        else:
            algo_bytes = 3 * b * s * h * d * 2 + b * h * s * 4 * 2  # (dQ alone) Q or K, dO, dQ + LSE, delta
            if ds_path:
                r["extra_bytes"] = ds_bytes  # dS tiles streamed from HBM (dS path)
        r["algorithmic_bytes_per_launch"] = algo_bytes
        if r["traffic"]:
            r["traffic_ratio"] = round(r["traffic"] / algo_bytes, 2)
        if rec:
            r["pmc_source"] = pmc_file
        return r

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(h, s, d, causal)
    if dist:
        dist.barrier()  # ranks > 0 wait here while rank 0 times the CPU baseline
    if rank != 0:
        dist.destroy_process_group()
        return
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic N(0,0.5) Q/K/V, N(0,1) dO, resident in HBM",
        "config": {
            "workload": f"B={b} H={h} S={s} D={d} bf16 {'causal' if causal else 'non-causal'} fwd+bwd per GPU "
                        f"(BASELINE.json configs[2]; configs[3] = B=64 batch-sharded over 8 GPUs)",
            "global_batch": global_batch,
            "per_gpu_batch": b,
            "seq_len": s,
            "heads": h,
            "head_dim": d,
            "causal": causal,
            "parallelism": f"batch-sharded x{world} ({scaling} scaling), independent per-GPU launches, "
                           "no data-path collectives",
        },
        "fwd_tflops": round(fwd_tf, 2),
        "bwd_tflops": round(bwd_tf, 2),
        "fwd_ms": round(t_fwd * 1e3, 4),
        "bwd_ms": round(t_bwd * 1e3, 4),
        "pct_of_peak_fwd": round(100 * fwd_tf / PEAK_TFLOPS, 2),
        "pct_of_peak_bwd": round(100 * bwd_tf / PEAK_TFLOPS, 2),
        "pct_of_peak_fwd_bwd": round(100 * value / world / PEAK_TFLOPS, 2),
        "roofline": roofline(dominant),
        "roofline_fwd": roofline("fwd_kernel"),
        "roofline_dq": roofline("dq_kernel"),
        "bwd_path": "dS workspace (delta, dK/dV + dS tiles, dQ = dS K)" if ds_path else "recompute dQ",
        "ds_workspace_bytes": ws_bytes,
        "kernels": kernels,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
