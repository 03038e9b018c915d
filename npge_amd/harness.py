"""Timing harness of bench.py (the driver's contract): W untimed warmup steps,
then K timed steps bracketed by a barrier and a device synchronisation on both
sides; the job time is the maximum over ranks and the reported value is the
work of ALL ranks over that time.

Kept free of any GPU call so the multi-rank path is testable with the gloo
backend on CPU (tests/test_harness_dist.py); bench.py passes
torch.cuda.synchronize as `sync` and runs one rank per GPU over RCCL.
"""
import time


def rank_seed(base, rank, config):
    """Per-rank genome-set seed: replicas process distinct synthetic sets."""
    return base + 1000 * rank + sum(map(ord, config))


def timed_steps(step, steps, warmup, dist=None, sync=lambda: None, device=None):
    """Runs warmup + steps calls of step(); returns (max-over-ranks seconds of
    the timed steps, the last step's return value)."""
    import torch
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    info = None
    for _ in range(steps):
        info = step()
    sync()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, info


def throughput(units_per_rank, world, steps, seconds):
    """Whole-job units per second (all ranks' work over the max-over-ranks time)."""
    return units_per_rank * world * steps / seconds
