#!/usr/bin/env python3
"""Headline benchmark: anchored+aligned Mbp/s on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one synthetic genome set already
resident in HBM: AnchorFinder (k=20, fp=0.1, max 100000 fragments) followed by
the block build on its anchors (DraftPangenome-equivalent).
value = input bp of all ranks / max-over-ranks wall time of the K timed steps.

Multi-GPU (torch.distributed.run, one rank per GPU over RCCL), two modes:
  --mode replicas (default): every rank processes its own genome set (same
    config, rank-specific seed) -- weak scaling, no data-path collective;
  --mode sharded: ONE genome set, the AnchorFinder windows and the aligner jobs
    split over the ranks with RCCL exchanges (npge_amd/comm.py) -- strong
    scaling; value = that set's bp / time.
(DESIGN.md "Multi-GPU").

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--mode", choices=("replicas", "sharded"), default="replicas")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL, one rank per GPU) or gloo (rehearsal: ranks may share a GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", default="C2", help="synthetic config timed for cpu_baseline")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    if args.dist_backend == "gloo":  # rehearsal on fewer GPUs than ranks
        local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(args.dist_backend)

    from npge_amd import _capi, harness, synth
    from npge_amd import pipeline

    _capi.check(_capi.lib().npgx_set_device(local_rank))
    sharded = args.mode == "sharded" and world > 1
    seed = harness.rank_seed(synth.BASE_SEED, 0 if sharded else rank, args.config)
    names, seqs = synth.genome_set(args.config, seed=seed)
    bp = synth.total_bp(seqs)
    ss = _capi.SeqSet(seqs, names)          # resident in HBM before timing
    comm = None
    if sharded:
        from npge_amd.comm import TorchComm
        comm = TorchComm(dist, staging="cuda")
    job = pipeline.BlockBuild(ss, names, seqs, comm=comm)

    def step():
        return job.run()

    dt, info = harness.timed_steps(step, args.steps, args.warmup, dist if world > 1 else None,
                                   sync=torch.cuda.synchronize, device="cuda")
    # sharded: the ranks share one set of bp; replicas: each rank has its own
    value = harness.throughput(bp, 1 if sharded else world, args.steps, dt) / 1e6

    # dominant kernel of the last step: algorithmic bytes / HIP-event duration
    # (events recorded on the engine's own stream around each launch)
    kts = job.kernel_times()
    # (collective stages of a sharded run are timed too but are not kernels)
    kern = [k for k in kts if not k["name"].endswith("_allreduce")]
    dom = max(kern, key=lambda k: k["ms"]) if kern else None
    roofline = None
    if dom and dom["ms"] > 0:
        ach = dom["bytes"] / (dom["ms"] * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": None, "kernel": dom["name"],
                    "launches_per_step": dom["launches"],
                    "avg_launch_ms": round(dom["ms"] / dom["launches"], 4),
                    "bytes_per_launch": dom["bytes"] / dom["launches"]}
    kernels = sorted(({"name": k["name"], "ms": round(k["ms"], 4), "launches": k["launches"]}
                      for k in kts), key=lambda k: -k["ms"])

    if roofline is not None:
        roofline.update(pmc_traffic(dom["name"], args.config))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_sample)

    if rank == 0:
        line = {
            "metric": "anchored+aligned Mbp/sec at 1/2/4/8 MI355X; bit-exact anchor set vs CPU",
            "value": round(value, 3),
            "unit": "Mbp/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded Brucella-like proxy, npge_amd/synth.py)",
            "config": {"workload": job.workload_name(args.config), "bp_per_rank": bp,
                       "genomes": synth.CONFIGS[args.config][0], "anchor_size": 20,
                       "anchor_fp": 0.1, "max_anchor_fragments": 100000,
                       "parallelism": ("sharded x%d (RCCL)" % world) if sharded
                       else "replica-per-gpu x%d" % world},
            "last_step": info,
            "kernels_last_step": kernels,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(kernel, config):
    """HBM traffic per launch of `kernel` from the newest committed PMC summary
    for this config (profiles/*_<config>_pmc_traffic.json, written by
    tools/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes
    of this bench).  PMC counters cannot be read from inside this process."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "*_%s_pmc_traffic.json" % config.lower())))
    if not files:
        return {"traffic": None}
    doc = json.load(open(files[-1]))
    for name, v in doc["kernels"].items():
        if name.split("::")[-1] == "k_" + kernel:
            return {"traffic": v["traffic_bytes_per_launch"], "traffic_source": os.path.basename(files[-1]),
                    "traffic_fetch": v["fetch_bytes_per_launch"], "traffic_write": v["write_bytes_per_launch"]}
    return {"traffic": None}


def cpu_baseline(config):
    """The CPU restatement (oracle/) timed on this host on the same workload:
    single thread (reference 1-worker semantics) and, under "all_cores", with
    FragmentTG + BlocksJobs threading over the host cores this job may use (the
    reference's --workers; the Bloom pass sequential)."""
    import time
    from npge_amd import synth
    from oracle import oracle as orc
    names, seqs = synth.genome_set(config)
    bp = synth.total_bp(seqs)

    def run(workers):
        t = time.perf_counter()
        o = orc.BlockSetOracle(seqs, names, seed=1)
        o.set_workers(workers)
        o.apply("DraftPangenome")
        return time.perf_counter() - t, o.hash()

    t1, h1 = run(1)
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    workers = max(1, min(avail, int(os.environ.get("OMP_NUM_THREADS", avail)), 16))
    tn, hn = run(workers)
    if hn != h1:
        raise AssertionError("threaded oracle DraftPangenome differs from the 1-thread run")
    return {"value": round(bp / 1e6 / t1, 4), "unit": "Mbp/s", "cores": 1, "kind": "port",
            "sample": "%s synthetic set (%d bp), one full step of the same workload, oracle/ "
                      "C++ -O3, 1 thread" % (config, bp), "seconds": round(t1, 3),
            "all_cores": {"value": round(bp / 1e6 / tn, 4), "cores": workers, "seconds": round(tn, 3),
                          "threading": "FragmentTG per sequence (AnchorFinder pass 2), BlocksJobs per block (DummyAligner, FragmentsExtender, "
                                       "FixEnds, Filter); the Bloom pass and the loop's set "
                                       "operations sequential"}}

if __name__ == "__main__":
    main()
