"""Benchmark: attention TFLOP/s (fwd & fwd+bwd) at S=4096 D=128 bf16 and % of MFMA peak.

Workload (BASELINE.json configs[2], the config the metric is quoted on; `--config cfg3`, the
default): per GPU B=8 H=32 S=4096 D=128 bf16, causal, forward + backward through the autograd op
`fa2_triton_amd.flash_attn_func` on synthetic N(0, 0.5) inputs resident in HBM.  One step = one
forward + one backward of that batch.  The other BASELINE configs have presets too:
  --config cfg2   B=8 H=16 S=1024 D=64 bf16 non-causal, forward only (configs[1]);
  --config cfg5   B=2 Hq=32 Hkv=8 S=8192 D=128 fp16 causal fwd+bwd (configs[4]; B=2 assumed,
                  SURVEY.md section 8.0);
  --config refbench  B=4 H=32 S=4096 D=128 fp16 non-causal forward only (the reference's own
                  benchmarks/targetted_bench.py shape);
and every field can be overridden (--batch --heads --heads-kv --seqlen --head-dim --dtype
--no-causal --fwd-only).  `--bias` adds the reference tests' additive bias (a [1, 1, Sq, Sk]
tensor in the input dtype, /root/reference/tests/core.py:28) and `--dropout P` dropout with a
fixed seed: both leave the algorithmic FLOPs unchanged (dropout runs the general forward and the
hand-placed dQ / dK/dV over the saved keep words; a 16-bit bias the pipelined forward and the
general backward kernels).  Warm-up (untimed) defaults to >= ~20 ms of GPU work so the timed
region starts at the sustained clock: 5 steps, 25 for refbench, 400 for cfg2 (1000 timed).

Multi-GPU (BASELINE.json configs[3]: B=64 over 8 GPUs): one process
per GPU, each running its own batch shard with no collective on the data path.  The ranks meet
only on a host-side gloo process group (a barrier around the timed region, the max-reduction
of its duration, the gather of the per-rank times): RCCL is never initialised.
  * weak scaling (default): every rank runs B=--batch -> global batch B N;
  * strong scaling (--strong): the global batch --global-batch (64) is split B/N per rank.
`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N rank
processes itself (children of this process, which never touches the GPU), polls them, and on
the first failure terminates the others and exits non-zero; under torchrun (WORLD_SIZE set) it
is one of the ranks.

FLOPs are algorithmic: fwd = 4 B H S^2 D (/2 causal), bwd = 2.5 fwd.

Besides the step time, every launch of the path -- the forward, and the backward's kernels
(fa2_bwd_stages) -- is timed with HIP events on the stream it runs on.  `roofline` is the
dominant (longest) kernel, `roofline_fwd` the north-star forward kernel, `roofline_dq` the dQ
kernel, each with its algorithmic FLOPs per launch against the bf16 MFMA peak; `traffic` (HBM
bytes per launch), `mfma_busy_pct` and `clock_ghz` come from the rocprofv3 PMC summary committed
under profiles/ for the same kernel and the default workload (named in `pmc_source`; the clock
is that profile's own GRBM_GUI_ACTIVE over the same dispatches' durations).  Rank 0 also times
the CPU oracle (oracle/reference.py, fp32, torch CPU threads) on a bounded slice of the same
workload, after the timed region, for `cpu_baseline`.

Usage: python bench.py [--config cfg2|cfg3|cfg5] [--gpus N] [--steps K] [--warmup W] [--strong]
                       [--bias] [--dropout P] [--no-cpu-baseline]
       torchrun --nproc-per-node N bench.py --gpus N ...
       python bench.py --gpus 2 --dry-run      (CPU/gloo: sharding + timing plumbing only)
"""
import argparse
import datetime
import json
import os
import platform
import signal
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PEAK_TFLOPS = 2500.0  # MI355X dense bf16/fp16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)
# Philox4x32-10 draws per second over the whole chip: dropout_mask_kernel (misc.hip: all VALU, 38
# instructions per draw, full occupancy) alone on the non-causal cfg3 mask, 4.29e9 draws in 4.331 ms
# (profiles/r06i_dropout_fwd_kernel_trace.jsonl; round 4's philox_uniform microbench:
# 8.92e11, profiles/r04g_philox_rate.txt) -- the VALU bound of the dropout forward, which draws one
# uniform per visible (row, key) as the reference's tl.rand does
PHILOX_DRAWS_PER_S = 9.918e11
PHILOX_SOURCE = "dropout_mask_kernel alone, non-causal cfg3 (profiles/r06i_dropout_fwd_kernel_trace.jsonl)"
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md: ~8 TB/s)
N_SIMDS = 1024  # 256 CUs x 4 SIMDs
METRIC = "attention TFLOP/s (fwd & fwd+bwd) at S=4096 D=128 bf16; % of MFMA peak"

CONFIGS = {
    "cfg2": dict(batch=8, heads=16, heads_kv=16, seqlen=1024, head_dim=64, dtype="bf16", causal=False, fwd_only=True,
                 ref="BASELINE.json configs[1]"),
    "cfg3": dict(batch=8, heads=32, heads_kv=32, seqlen=4096, head_dim=128, dtype="bf16", causal=True, fwd_only=False,
                 ref="BASELINE.json configs[2]; configs[3] = B=64 batch-sharded over 8 GPUs"),
    "cfg5": dict(batch=2, heads=32, heads_kv=8, seqlen=8192, head_dim=128, dtype="fp16", causal=True, fwd_only=False,
                 ref="BASELINE.json configs[4], B=2 assumed (SURVEY.md section 8.0)"),
    # the reference's own benchmark shape (/root/reference/benchmarks/targetted_bench.py:11-19)
    "refbench": dict(batch=4, heads=32, heads_kv=32, seqlen=4096, head_dim=128, dtype="fp16", causal=False,
                     fwd_only=True, ref="the reference's benchmarks/targetted_bench.py shape (fp16, non-causal, fwd)"),
}
DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16}
DROPOUT_SEED = 20241008


def attn_flops(b, h, sq, sk, d, causal):
    f = 4.0 * b * h * sq * sk * d
    return f * 0.5 if causal else f


def reduce_elapsed(elapsed: float, dist, device=None) -> float:
    """Slowest rank's wall time: the job is done when every shard is (max over ranks).  The
    reduction runs on the host (gloo): `device` is accepted for the old signature only."""
    if dist is None:
        return elapsed
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def gather_elapsed(elapsed: float, dist, world: int):
    """Every rank's wall time (host-side gather), for the line."""
    if dist is None:
        return [elapsed]
    t = torch.zeros(world, dtype=torch.float64)
    t[dist.get_rank()] = elapsed
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def job_throughput(f_total: float, steps: int, elapsed: float, mult: float = 3.5):
    """Whole-job algorithmic TFLOP/s (fwd + bwd = 3.5 fwd per step, fwd alone = 1, summed over
    every rank's shard) and ms per step."""
    return mult * f_total * steps / elapsed / 1e12, elapsed / steps * 1e3


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


def _stop(procs, grace: float = 5.0) -> None:
    """SIGTERM every child still running, SIGKILL what is left after `grace` seconds."""
    for p in procs:
        if p.poll() is None:
            p.terminate()
    end = time.time() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.0, end - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def launch_ranks(n: int, argv, timeout_s: float = 1800.0) -> int:
    """Run this script as n rank processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, rendezvous
    on 127.0.0.1) and poll them: returns 0 when all exit 0; on the first non-zero exit (or after
    timeout_s) the other ranks are terminated and that status (124 on timeout) is returned, so a
    rank that dies never leaves its siblings blocked in a barrier.  The parent only spawns: it
    never initialises the GPU (children are started, never exec'd into)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))

    def on_signal(signum, frame):  # the parent itself is being stopped: take the ranks with it
        _stop(procs)
        sys.exit(128 + signum)

    old = signal.signal(signal.SIGTERM, on_signal)
    deadline = time.time() + timeout_s
    try:
        while True:
            codes = [p.poll() for p in procs]
            failed = [c for c in codes if c not in (None, 0)]
            if failed:
                _stop(procs)
                return failed[0] if failed[0] > 0 else 128 - failed[0]
            if all(c == 0 for c in codes):
                return 0
            if time.time() > deadline:
                print(f"bench.py: ranks still running after {timeout_s:.0f} s, terminating", file=sys.stderr)
                _stop(procs)
                return 124
            time.sleep(0.1)
    finally:
        signal.signal(signal.SIGTERM, old)


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


def cpu_baseline(h, hkv, s, d, causal, fwd_only=False, budget_s=20.0):
    """Time the fp32 oracle on the host on a slice of the same workload: one batch row and as
    many q-heads (whole GQA groups) as fit the time budget at ~0.15 TFLOP/s and 4 GiB per
    [1, H, S, S] fp32 score tensor; about 10-30 s of CPU work in all."""
    sys.path.insert(0, ROOT)
    from oracle.reference import attention_reference

    threads = cpu_threads()
    torch.set_num_threads(threads)
    group = h // hkv
    mult = 1.0 if fwd_only else 3.5
    per_head = mult * attn_flops(1, 1, s, s, d, causal)
    heads = int(min(h, budget_s * 0.15e12 / per_head, (4 << 30) / (s * s * 4)))
    heads = max(group, heads - heads % group)
    g = torch.Generator().manual_seed(0)
    q = (torch.randn(1, s, heads, d, generator=g) * 0.5).requires_grad_(not fwd_only)
    k = (torch.randn(1, s, heads // group, d, generator=g) * 0.5).requires_grad_(not fwd_only)
    v = (torch.randn(1, s, heads // group, d, generator=g) * 0.5).requires_grad_(not fwd_only)
    do = torch.randn(1, s, heads, d, generator=g)

    def run():
        if fwd_only:
            with torch.no_grad():
                attention_reference(q, k, v, causal=causal)
        else:
            out = attention_reference(q, k, v, causal=causal)
            torch.autograd.grad(out, (q, k, v), do)

    t0 = time.perf_counter()
    run()
    dt = time.perf_counter() - t0
    reps = 1
    while dt * reps < 10.0 and reps < 8:
        t0 = time.perf_counter()
        run()
        dt = (dt * reps + time.perf_counter() - t0) / (reps + 1)
        reps += 1
    flops = mult * attn_flops(1, heads, s, s, d, causal)
    info = cpu_info()
    return {
        "value": flops / dt / 1e12,
        "unit": "TFLOP/s",
        "cores": threads,
        "cores_note": "torch threads = every CPU in this process's affinity, capped by OMP_NUM_THREADS when set "
                      "(the GPU box sets it to its per-GPU CPU share, 16, and asks workloads to stay within it)",
        "kind": "port",
        "sample": f"oracle fp32 {'fwd' if fwd_only else 'fwd+bwd'} (oracle/reference.py), B=1 Hq={heads} "
                  f"Hkv={heads // group} S={s} D={d} causal={causal} (slice of the workload), mean of {reps} reps, "
                  f"{dt:.2f} s each, {threads} torch threads",
        **info,
    }


def load_pmc():
    """The latest committed rocprofv3 PMC summary (profiles/*_pmc.json; HBM bytes per launch =
    FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md; MFMA-busy cycles; the effective clock of
    the profiled dispatches), recorded for the default workload only.  Returns (dict by kernel
    symbol, file name)."""
    import glob

    # by name: the round tags (r01.., r02a.., r03a..) order them; file times do not survive a checkout
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    if not files:
        return {}, None
    data = json.load(open(files[-1]))
    return {k.replace("fa2::", ""): v for k, v in data.items()}, os.path.relpath(files[-1], ROOT)


def pmc_fields(rec: dict) -> dict:
    """traffic / MFMA-busy / effective clock of one kernel from its PMC record (all from the same
    profile run: the clock is GRBM_GUI_ACTIVE / 8 over those dispatches' own durations)."""
    out = {"traffic": rec.get("hbm_bytes_per_launch")}
    grbm = rec.get("GRBM_GUI_ACTIVE")
    busy = rec.get("SQ_VALU_MFMA_BUSY_CYCLES")
    if grbm and busy is not None:
        out["mfma_busy_pct"] = round(100.0 * busy / (N_SIMDS * grbm / 8.0), 1)
    if rec.get("clock_ghz"):
        out["clock_ghz"] = round(rec["clock_ghz"], 3)
    return out


def resolve(args):
    """Fill the workload fields left unset from the --config preset."""
    preset = CONFIGS[args.config]
    if args.steps is None:
        args.steps = 1000 if args.config == "cfg2" else 20
    if args.warmup is None:
        # untimed warm-up of >= ~20 ms of GPU work, so the timed region starts at the sustained
        # clock (cfg3's 5 steps are 21 ms; five 46-us cfg2 steps would leave it ramping up)
        args.warmup = {"cfg2": 400, "refbench": 25}.get(args.config, 5)
    for key in ("batch", "heads", "heads_kv", "seqlen", "head_dim", "dtype"):
        if getattr(args, key) is None:
            setattr(args, key, preset[key])
    if args.heads_kv is None or args.heads % args.heads_kv:
        raise SystemExit(f"--heads {args.heads} is not divisible by --heads-kv {args.heads_kv}")
    args.causal = preset["causal"] if args.causal is None else args.causal
    args.fwd_only = preset["fwd_only"] or args.fwd_only
    return preset


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg3")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 20; 1000 for cfg2's 46 us step)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 5; 400 for cfg2, 25 for refbench)")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (weak scaling)")
    ap.add_argument("--strong", action="store_true", help="split --global-batch over the GPUs")
    ap.add_argument("--global-batch", type=int, default=64)
    ap.add_argument("--heads", type=int, default=None)
    ap.add_argument("--heads-kv", type=int, default=None)
    ap.add_argument("--seqlen", type=int, default=None)
    ap.add_argument("--head-dim", type=int, default=None)
    ap.add_argument("--dtype", choices=sorted(DTYPES), default=None)
    ap.add_argument("--causal", dest="causal", action="store_true", default=None)
    ap.add_argument("--no-causal", dest="causal", action="store_false")
    ap.add_argument("--fwd-only", action="store_true")
    ap.add_argument("--bias", action="store_true", help="[1, 1, Sq, Sk] additive bias in the input dtype")
    ap.add_argument("--bias-grad", action="store_true",
                    help="--bias that requires grad: the backward also computes dBias (library extension)")
    ap.add_argument("--dropout", type=float, default=0.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo: sharding + timing plumbing, no kernels")
    ap.add_argument("--launch-timeout", type=float, default=1800.0, help="seconds before a self-launch gives up")
    args = ap.parse_args()
    preset = resolve(args)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # test hooks (tests/test_multigpu_gloo.py): this rank dies / hangs at start-up
    if os.environ.get("FA2_BENCH_FAIL_RANK") == str(rank):
        sys.exit(3)
    if os.environ.get("FA2_BENCH_HANG_RANK") == str(rank):
        time.sleep(3600)

    dist = None
    if world > 1:
        # host-side process group for the barrier and the timer reductions only: the data path
        # has no collective, so RCCL is never needed (nor initialised) on the GPU box
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
    # one GPU per rank; on a box with fewer GPUs than ranks (a rehearsal of the multi-rank path on
    # one card) the ranks share them round-robin -- device_count() does not initialise the GPU
    device = torch.device("cpu") if args.dry_run else torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))

    global_batch, (lo, hi), scaling = plan(args, world, rank)
    b, h, hkv, s, d = hi - lo, args.heads, args.heads_kv, args.seqlen, args.head_dim
    causal, fwd_only = args.causal, args.fwd_only
    mult = 1.0 if fwd_only else 3.5
    f_fwd_total = attn_flops(global_batch, h, s, s, d, causal)  # every rank's shard
    f_fwd = attn_flops(b, h, s, s, d, causal)                   # this rank's shard

    if args.dry_run:
        if dist:
            dist.barrier()
        elapsed = 0.001 * (1 + rank)
        per_rank = gather_elapsed(elapsed, dist, world)
        elapsed = reduce_elapsed(elapsed, dist)
        shards = [(lo, hi)]
        if dist:
            shards = [None] * world
            dist.all_gather_object(shards, (lo, hi))
        if rank == 0:
            value, ms = job_throughput(f_fwd_total, args.steps, elapsed, mult)
            print(json.dumps({"dry_run": True, "n_gpus": world, "scaling": scaling, "global_batch": global_batch,
                              "shards": shards, "elapsed": elapsed, "rank_elapsed_s": per_rank, "value": value,
                              "ms_per_step": ms}), flush=True)
        if dist:
            dist.destroy_process_group()
        return

    torch.cuda.set_device(device)
    from fa2_triton_amd import flash_attn_func
    from fa2_triton_amd.backward import _flash_attn_backward
    from fa2_triton_amd.utils import dropout_mask_words
    from fa2_triton_amd.forward import _flash_attn_forward

    dtype = DTYPES[args.dtype]
    # this rank's rows of the synthetic global batch (seeded per shard start)
    torch.manual_seed(1234 + lo)
    q = torch.empty(b, s, h, d, device=device, dtype=dtype).normal_(0, 0.5).requires_grad_(not fwd_only)
    k = torch.empty(b, s, hkv, d, device=device, dtype=dtype).normal_(0, 0.5).requires_grad_(not fwd_only)
    v = torch.empty(b, s, hkv, d, device=device, dtype=dtype).normal_(0, 0.5).requires_grad_(not fwd_only)
    do = torch.randn(b, s, h, d, device=device, dtype=dtype)
    if args.bias_grad:
        args.bias = True
    bias = torch.rand(1, 1, s, s, device=device, dtype=dtype) if args.bias else None
    if bias is not None and args.bias_grad and not fwd_only:
        bias.requires_grad_(True)
    grad_inputs = (q, k, v, bias) if bias is not None and bias.requires_grad else (q, k, v)
    p_drop = args.dropout
    seed = DROPOUT_SEED if p_drop > 0 else None

    def step():
        if fwd_only:
            with torch.no_grad():
                flash_attn_func(q, k, v, None, bias, p_drop, causal, None, seed)
        else:
            out = flash_attn_func(q, k, v, None, bias, p_drop, causal, None, seed)
            torch.autograd.grad(out, grad_inputs, do)

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
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    per_rank = gather_elapsed(elapsed, dist, world)
    elapsed = reduce_elapsed(elapsed, dist)
    value, ms_per_step = job_throughput(f_fwd_total, args.steps, elapsed, mult)

    # ---- per-launch timing with HIP events on the launch stream ---------------------------
    # fwd: one launch; bwd: dQ (recomputes S, dP; also writes delta), then dK/dV, each timed
    # alone through fa2_bwd_stages with a shared delta workspace.
    # every launch timed on its own (event pair on the launch stream), median of >= 50
    reps = max(50, args.steps)
    stream = torch.cuda.current_stream(device)
    with torch.no_grad():
        # with dropout, as in the autograd op: the forward saves its keep bits, the backward reads them
        kmask = None
        if p_drop > 0:
            kmask = torch.empty(dropout_mask_words(b, h, s, s), dtype=torch.int32, device=device)
        o, lse, _, _ = _flash_attn_forward(q, k, v, None, bias, p_drop, causal, None, seed, dropout_mask=kmask)
        delta = torch.empty_like(lse)  # shared by the stage calls: written by dQ, read by dK/dV

        def bwd(stages):
            return lambda: _flash_attn_backward(do, q, k, v, bias, None, o, lse, p_drop, causal, None, seed,
                                                _stages=stages, _delta=delta, dropout_mask=kmask,
                                                bias_grad=stages == 8)

        calls = {"fwd_kernel": lambda: _flash_attn_forward(q, k, v, None, bias, p_drop, causal, None, seed,
                                                           dropout_mask=kmask)}
        if not fwd_only:
            calls.update(dq_kernel=bwd(4), dkdv_kernel=bwd(2))
            if bias is not None and bias.requires_grad:
                calls.update(dbias_kernel=bwd(8))
        times, spread = {}, {}
        for name, fn in calls.items():
            fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in ev:
                e0.record(stream)
                fn()
                e1.record(stream)
            torch.cuda.synchronize()
            ts = sorted(e0.elapsed_time(e1) * 1e-3 for e0, e1 in ev)
            times[name] = ts[len(ts) // 2]
            spread[name] = {"reps": reps, "mean_ms": round(sum(ts) / len(ts) * 1e3, 4),
                            "min_ms": round(ts[0] * 1e3, 4), "max_ms": round(ts[-1] * 1e3, 4)}
    t_fwd = times["fwd_kernel"]
    t_bwd = sum(t for n, t in times.items() if n != "fwd_kernel")
    fwd_tf = f_fwd / t_fwd / 1e12
    bwd_tf = 2.5 * f_fwd / t_bwd / 1e12 if t_bwd else None
    # Algorithmic FLOPs per launch: fwd = F; the backward's 5
    # GEMM-units (2.5 F) are split as S, dP, dV, dK -> dK/dV kernel (2 F) and dQ -> dQ kernel
    # (0.5 F).  The dQ kernel also recomputes S and dP (1 F executed, not algorithmic).
    algo = {"fwd_kernel": f_fwd, "dkdv_kernel": 2.0 * f_fwd, "dq_kernel": 0.5 * f_fwd}
    executed = dict(algo, dq_kernel=1.5 * f_fwd)
    if "dbias_kernel" in times:  # dBias (extension): S and dP recomputed, counted as its own work
        algo["dbias_kernel"] = executed["dbias_kernel"] = f_fwd
    kernels = {
        name: {
            "ms": round(t * 1e3, 4),
            "timing": "median of per-launch HIP-event times",
            **spread[name],
            "algorithmic_tflops": round(algo[name] / t / 1e12, 1),
            "executed_mfma_tflops": round(executed[name] / t / 1e12, 1),
        }
        for name, t in times.items()
    }
    plain = bias is None and p_drop == 0.0 and d % 8 == 0
    pmc, pmc_file = load_pmc()
    workload_ok = (b, h, hkv, s, d, causal, dtype, fwd_only, plain) == (8, 32, 32, 4096, 128, True, torch.bfloat16, False,
                                                                       True)
    dominant = max(times, key=lambda n: times[n])
    # device symbols the workload dispatches to, by the library's own conditions (the bench's tensors
    # are contiguous, so every row is 16-byte aligned): forward -- fwd_hp_ok (D = 128, no bias; with
    # dropout only with a keep-mask buffer, which this bench passes: dropout_mask_kernel, then
    # fwd_hp_kernel reading its words), else fwd_pipe_kernel (D in {64, 128}, no dropout, no bias
    # or a 16-bit one: bias16_rows), else fwd_kernel (after dropout_mask_kernel with dropout);
    # dQ / dK-dV -- dq_hp_ok / dkdv_hp_ok (D = 128, no bias; with dropout only through the
    # forward's saved keep words)
    hp_fwd = d == 128 and bias is None
    pipe_fwd = d in (64, 128) and p_drop == 0.0 and (bias is None or bias.dtype in (torch.float16, torch.bfloat16))
    hp_bwd = d == 128 and bias is None
    symbol = {"fwd_kernel": "fwd_hp_kernel" if hp_fwd else ("fwd_pipe_kernel" if pipe_fwd else "fwd_kernel"),
              "dkdv_kernel": "dkdv_hp_kernel" if hp_bwd else "dkdv_kernel",
              "dq_kernel": "dq_hp_kernel" if hp_bwd else "dq_kernel", "dbias_kernel": "dbias_kernel"}
    esz = q.element_size()

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
        r.update(pmc_fields(rec) if rec else {"traffic": None})
        qo = b * s * h * d * esz  # Q (or O, dO, dQ) bytes
        kv = b * s * hkv * d * esz  # K (or V, dK, dV) bytes
        rows = b * h * s * 4  # one fp32 row statistic (LSE or delta)
        if name == "fwd_kernel":
            algo_bytes = 2 * qo + 2 * kv + rows  # Q, K, V read, O written, LSE
        elif name == "dkdv_kernel":
            algo_bytes = 2 * qo + 4 * kv + 2 * rows  # Q, dO, K, V read, dK, dV written, LSE, delta
        else:
            algo_bytes = 3 * qo + 2 * kv + 2 * rows  # Q, dO, O (delta) read, dQ written, K, V, LSE, delta
        if bias is not None:
            algo_bytes += bias.numel() * bias.element_size()
        r["algorithmic_bytes_per_launch"] = algo_bytes
        r["traffic_ratio"] = round(r["traffic"] / algo_bytes, 2) if r["traffic"] else None
        if rec:
            r["pmc_source"] = pmc_file
        return r

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(h, hkv, s, d, causal, fwd_only)
    if dist:
        dist.barrier()  # ranks > 0 wait here while rank 0 times the CPU baseline
    if rank != 0:
        dist.destroy_process_group()
        return
    workload = (f"B={b} Hq={h} Hkv={hkv} S={s} D={d} {args.dtype} {'causal' if causal else 'non-causal'} "
                f"{'fwd only' if fwd_only else 'fwd+bwd'} per GPU ({preset['ref']})")
    extras = []
    if bias is not None:
        extras.append("bias [1,1,S,S]")
    if p_drop:
        extras.append(f"dropout {p_drop}")
    if extras:
        workload += " + " + ", ".join(extras)
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
        "dtype": args.dtype,
        "data": "synthetic N(0,0.5) Q/K/V, N(0,1) dO, resident in HBM",
        "config": {
            "workload": workload,
            "config": args.config,
            "global_batch": global_batch,
            "per_gpu_batch": b,
            "seq_len": s,
            "heads": h,
            "heads_kv": hkv,
            "head_dim": d,
            "causal": causal,
            "fwd_only": fwd_only,
            "bias": bias is not None,
            "dropout_p": p_drop,
            "parallelism": f"batch-sharded x{world} ({scaling} scaling), independent per-GPU launches, "
                           "no data-path collectives (host gloo barrier + timer reduction only)",
        },
        "rank_elapsed_s": [round(t, 6) for t in per_rank],
        "fwd_tflops": round(fwd_tf, 2),
        "bwd_tflops": round(bwd_tf, 2) if bwd_tf else None,
        "fwd_ms": round(t_fwd * 1e3, 4),
        "bwd_ms": round(t_bwd * 1e3, 4) if t_bwd else None,
        "pct_of_peak_fwd": round(100 * fwd_tf / PEAK_TFLOPS, 2),
        "pct_of_peak_bwd": round(100 * bwd_tf / PEAK_TFLOPS, 2) if bwd_tf else None,
        "pct_of_peak_step": round(100 * value / world / PEAK_TFLOPS, 2),
        "roofline": roofline(dominant),
        "roofline_fwd": roofline("fwd_kernel"),
        "kernels": kernels,
        "cpu_baseline": cpu,
    }
    if not fwd_only:
        line["roofline_dq"] = roofline("dq_kernel")
    if p_drop > 0:
        # visible (row, key) pairs of one forward launch: one Philox draw each
        vis = s * (s + 1) // 2 if causal else s * s
        draws = b * h * vis
        rate = draws / t_fwd
        line["roofline_valu"] = {"bound": "valu", "kernel": f"fa2::dropout_mask_kernel + fa2::{symbol['fwd_kernel']}",
                                 "achieved": round(rate, 1),
                                 "peak": PHILOX_DRAWS_PER_S, "unit": "Philox draws/s",
                                 "frac": round(rate / PHILOX_DRAWS_PER_S, 4), "draws_per_launch": draws,
                                 "bound_ms": round(draws / PHILOX_DRAWS_PER_S * 1e3, 4),
                                 "peak_source": PHILOX_SOURCE}
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
