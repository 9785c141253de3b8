"""Multi-rank logic of bench.py on CPU (gloo, world_size 2): batch sharding with no data-path
collective, max-over-ranks timing, whole-job throughput (weak scaling).  The GPU path uses the
same functions with the nccl (RCCL) backend; only the barrier and the timer reduction are
collectives."""
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


def test_job_throughput_is_weak_scaling_aggregate():
    f = bench.attn_flops(8, 32, 4096, 4096, 128, True)
    one, ms1 = bench.job_throughput(f, 10, 1, 0.05)
    eight, ms8 = bench.job_throughput(f, 10, 8, 0.05)
    assert eight == pytest.approx(8 * one) and ms1 == ms8 == pytest.approx(5.0)
    assert f == pytest.approx(1.0995e12, rel=1e-4)  # BASELINE.md cfg3 fwd FLOP
