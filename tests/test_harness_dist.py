"""The bench's multi-rank timing path (npge_amd/harness.py) with world_size 2
over gloo on CPU: barrier-bracketed steps, max-over-ranks time, whole-job
throughput, distinct per-rank replica seeds."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import time
    import torch.distributed as dist
    from npge_amd import harness
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def step():
        time.sleep(0.01 * (rank + 1))  # rank 1 is the slow one
        calls.append(1)
        return {"rank": rank}

    dt, info = harness.timed_steps(step, steps=4, warmup=2, dist=dist)
    out[rank] = (dt, len(calls), info["rank"], harness.rank_seed(7, rank, "C2"))
    dist.destroy_process_group()


def test_two_ranks_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    (dt0, n0, r0, s0), (dt1, n1, r1, s1) = out[0], out[1]
    assert n0 == n1 == 6                  # warmup + timed steps on every rank
    assert (r0, r1) == (0, 1)
    assert dt0 == dt1                     # every rank reports the max
    assert dt0 >= 4 * 0.02                # at least the slow rank's time
    assert s0 != s1                       # replicas get distinct genome sets
    from npge_amd import harness
    assert harness.throughput(100, world, 4, 2.0) == 400.0
