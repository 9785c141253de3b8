"""Multi-rank logic of bench.py on CPU (gloo, world_size 2): batch sharding with no data-path
collective, max-over-ranks timing, whole-job throughput (weak and strong scaling), and the
self-launch of `bench.py --gpus N` (N rank processes, rank 0 prints the line).  The GPU path uses the
same functions and the same host-side gloo group; only the barrier and the timer reductions are
collectives (RCCL is never initialised).  A rank that dies makes the launcher stop the others and
exit non-zero at once instead of leaving them blocked in a barrier."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = bench.shard_batch(64, world, rank)
        # each rank "runs" its shard; elapsed differs per rank, the job time is the max
        elapsed = bench.reduce_elapsed(1.0 + rank, dist, torch.device("cpu"))
        dist.barrier()
        out[rank] = (lo, hi, elapsed)
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_and_timing():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    assert res[0][:2] == (0, 32) and res[1][:2] == (32, 64)
    assert res[0][2] == res[1][2] == 2.0  # max over ranks


def test_job_throughput_is_whole_job_aggregate():
    f = bench.attn_flops(8, 32, 4096, 4096, 128, True)
    one, ms1 = bench.job_throughput(f, 10, 0.05)
    eight, ms8 = bench.job_throughput(8 * f, 10, 0.05)  # 8 shards of B=8 in the same time
    assert eight == pytest.approx(8 * one) and ms1 == ms8 == pytest.approx(5.0)
    assert f == pytest.approx(1.0995e12, rel=1e-4)  # BASELINE.md cfg3 fwd FLOP


def test_shard_batch_covers_uneven_batches():
    for gb, world in ((64, 8), (64, 3), (7, 4), (8, 8)):
        shards = [bench.shard_batch(gb, world, r) for r in range(world)]
        assert shards[0][0] == 0 and shards[-1][1] == gb
        assert all(a[1] == b[0] for a, b in zip(shards, shards[1:]))
        assert max(h - l for l, h in shards) - min(h - l for l, h in shards) <= 1


def _bench_dry_run(*extra):
    """`python bench.py --gpus 2 --dry-run ...` exactly as a user runs it: the script launches
    its own 2 rank processes (host-side gloo coordination, here as on the GPU box: RCCL is never
    initialised, the data path has no collective) and rank 0 prints one line."""
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    res = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--dry-run", *extra], capture_output=True,
                         text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout  # one line, from rank 0 only
    return json.loads(lines[0])


def test_bench_gpus_2_launches_two_ranks_weak():
    line = _bench_dry_run()
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["global_batch"] == 16
    assert [tuple(s) for s in line["shards"]] == [(0, 8), (8, 16)]
    assert line["elapsed"] == pytest.approx(0.002)  # max over the two ranks' timers
    assert line["rank_elapsed_s"] == pytest.approx([0.001, 0.002])


def test_bench_gpus_2_strong_splits_global_batch():
    line = _bench_dry_run("--strong", "--global-batch", "64")
    assert line["scaling"] == "strong" and line["global_batch"] == 64
    assert [tuple(s) for s in line["shards"]] == [(0, 32), (32, 64)]


def test_bench_launcher_stops_siblings_when_a_rank_dies():
    """Rank 1 dies at start-up (FA2_BENCH_FAIL_RANK=1) while rank 0 waits for it in the
    process-group rendezvous: the parent must return non-zero within seconds and leave no child."""
    import subprocess
    import sys
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FA2_BENCH_FAIL_RANK"] = "1"
    t0 = time.time()
    parent = subprocess.Popen([sys.executable, bench.__file__, "--gpus", "2", "--dry-run"], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    out, err = parent.communicate(timeout=120)
    assert parent.returncode == 3, (parent.returncode, err)
    assert time.time() - t0 < 60
    # no rank process of this launch is left: the launcher's children carry the parent's pid
    ps = subprocess.run(["ps", "-eo", "pid,ppid,args"], capture_output=True, text=True).stdout
    orphans = [ln for ln in ps.splitlines()[1:] if ln.split()[1] == str(parent.pid)]
    assert not orphans, orphans
    assert "dry_run" not in out


def test_bench_launcher_times_out(monkeypatch):
    """A launch that does not finish within its timeout (rank 1 hangs) is stopped: status 124."""
    import time

    monkeypatch.setenv("FA2_BENCH_HANG_RANK", "1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    t0 = time.time()
    assert bench.launch_ranks(2, ["--gpus", "2", "--dry-run"], timeout_s=10.0) == 124
    assert time.time() - t0 < 40
