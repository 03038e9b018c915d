#!/usr/bin/env python3
"""Headline benchmark: anchored+aligned Mbp/s on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one synthetic genome set already
resident in HBM: AnchorFinder (k=20, fp=0.1, max 100000 fragments) followed by
the block build on its anchors (DraftPangenome-equivalent).
value = input bp of all ranks / max-over-ranks wall time of the K timed steps.

Multi-GPU (torch.distributed.run, one rank per GPU), the same workload at
every N so that the per-N values compare:
  --mode replicas (default): every rank processes its own genome set of the
    config (rank-specific seed) -- independent pangenome jobs, no data-path
    collective, weak scaling; value = all ranks' bp / max-over-ranks time;
  --mode sharded: ONE genome set, the AnchorFinder windows and the aligner
    jobs split over the ranks, the exchanges on the library's own RCCL
    communicator over xGMI (npge_amd/comm.py RcclComm) -- strong scaling;
  --mode pairs (BASELINE C4's split; default config C4): every genome pair of
    the set is one DraftPangenome, the pairs split round-robin over the ranks
    and run --pair-workers at a time per GPU, RCCL only for the final gather
    of every pair's blocks (npge_amd/pairs.py) -- strong scaling over the
    fixed pair job; value = all pairs' input bp / time.
Every line also carries, each timed on its own after the headline:
"sharded" (N > 1: one set over the ranks; with --mode sharded "replicas"
instead) and "pairs" (the C4 pair-sharded job at this N), so one SCALE run
gives all three curves.  (DESIGN.md "Multi-GPU").

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
    ap.add_argument("--config", default=None,
                    help="synthetic genome set (npge_amd/synth.py); default C3 = the 17-genome ≥50x target "
                         "config (C4 with --mode pairs)")
    ap.add_argument("--mode", choices=("replicas", "sharded", "pairs"), default="replicas",
                    help="replicas (every rank its own set, weak scaling; default), sharded (one set over "
                         "the ranks, strong scaling) or pairs (C4 genome pairs over the ranks)")
    ap.add_argument("--pair-workers", type=int, default=16,
                    help="pairs: pairs run at a time per GPU (16: the host cores a GPU is allotted; profiles/r04ka_pairs_worker_sweep.jsonl)")
    ap.add_argument("--pairs", type=int, default=0, help="pairs: the first P pairs only (0 = all)")
    ap.add_argument("--no-replicas-line", action="store_true",
                    help="N > 1: skip the secondary one-set (or, with --mode sharded, replica) measurement")
    ap.add_argument("--pairs-config", default="C4", help="the secondary pairs line's config")
    ap.add_argument("--no-pairs-line", action="store_true",
                    help="skip the secondary C4 pair-sharded measurement")
    ap.add_argument("--anchor-loop", nargs="?", const="fast", default=False, choices=["fast", "full"],
                    help="each step also runs one AnchorLoopFast (fast, lua_lib.lua:741-758) or one AnchorLoop "
                         "(full, lua_lib.lua:711-737) after DraftPangenome")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL, one rank per GPU) or gloo (rehearsal: ranks may share a GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", default=None, help="synthetic config timed for cpu_baseline (default: --config)")
    ap.add_argument("--cpu-runs", type=int, default=5, help="timed CPU runs (median) after one warm-up")
    ap.add_argument("--hw-queues", type=int, default=20,
                    help="hardware queues per process (GPU_MAX_HW_QUEUES; HIP's default is 4): the pair job runs "
                         "--pair-workers streams at once; 20 queues with 16 workers: +9 %%, 24 or more: far slower "
                         "(profiles/r04ab_ab_hw_queues.txt, r04ac_pairs_workers_queues_*.jsonl); 0 leaves the "
                         "environment alone")
    ap.add_argument("--launch-check", action="store_true",
                    help="only the rank launch and rendezvous (no GPU call): prints n_gpus and the "
                         "communicator's rank count (tests/test_bench_launch.py)")
    a = ap.parse_args()
    if a.config is None:
        a.config = "C4" if a.mode == "pairs" else "C3"
    return a


def launch_ranks(args):
    """--gpus N > 1 without a launcher (no WORLD_SIZE in the environment):
    start the N ranks as child processes of torch.distributed.run, one per GPU,
    before this process makes any GPU call, and return their exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, NPGX_BENCH_LAUNCHER="bench.py")
    return subprocess.call(cmd, env=env)


def ranks_from_env(args):
    """(world, rank, local_rank) of this process; --gpus N must equal the
    launcher's WORLD_SIZE (a mismatch exits non-zero)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d: every GPU is one rank, refusing to run"
              % (args.gpus, world), file=sys.stderr, flush=True)
        sys.exit(2)
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def launcher_name():
    if os.environ.get("NPGX_BENCH_LAUNCHER"):
        return "bench.py -> torch.distributed.run"
    return "external (torch.distributed.run)" if "WORLD_SIZE" in os.environ else "none (one process)"


def launch_check(args, world, rank):
    """The rendezvous alone, with no GPU call: every rank joins the process
    group, the npgx_comm binding (host staging) all-gathers every rank's id,
    and rank 0 prints the rank counts."""
    import ctypes
    import torch.distributed as dist
    from npge_amd import pairs
    from npge_amd.comm import TorchComm
    if world > 1:
        dist.init_process_group(args.dist_backend)
        comm = TorchComm(dist, staging="cpu", copy=ctypes.memmove)
        import numpy as np
        ids, counts = pairs.gather_u64(comm, np.array([rank], dtype=np.uint64))
        assert ids.tolist() == list(range(world)) and counts == [1] * world
        comm_ranks = comm.world
    else:
        comm_ranks = 1
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "comm_ranks": comm_ranks,
                          "launcher": launcher_name(), "dist_backend": args.dist_backend}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.hw_queues > 0:  # read by the HIP runtime when it starts: before any GPU call (ranks inherit it)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))  # nothing here has touched the GPU
    world, rank, local_rank = ranks_from_env(args)
    if args.launch_check:
        launch_check(args, world, rank)
        return

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
    comm = None
    if world > 1:  # one communicator for the sharded set and the pair gather
        from npge_amd import comm as ncomm
        if args.dist_backend == "nccl":
            comm = ncomm.RcclComm(dist, local_rank)  # the library's own RCCL communicator
        else:  # gloo rehearsal: ranks may share a GPU (RCCL refuses that)
            comm = ncomm.TorchComm(dist, staging="cpu")
        ncomm.check(comm)  # every collective once, results verified, before any timing
        if comm.count() != world:
            raise SystemExit("bench.py: the communicator has %d ranks, WORLD_SIZE is %d" % (comm.count(), world))
    comm_ranks = comm.count() if comm is not None else 1
    if args.mode == "pairs":
        line = run_pairs(args, dist, world, rank, local_rank, comm, args.config, args.pairs,
                         args.steps, args.warmup, baseline=not args.no_cpu_baseline)
        if rank == 0:
            line["comm_ranks"] = comm_ranks
            line["launcher"] = launcher_name()
            print(json.dumps(line), flush=True)
        finish(dist, world, comm)
        return
    sharded = args.mode == "sharded" and world > 1
    seed = harness.rank_seed(synth.BASE_SEED, 0 if sharded else rank, args.config)
    names, seqs = synth.genome_set(args.config, seed=seed)
    bp = synth.total_bp(seqs)
    ss = _capi.SeqSet(seqs, names)          # resident in HBM before timing
    job = pipeline.BlockBuild(ss, names, seqs, comm=comm if sharded else None, anchor_loop=args.anchor_loop)

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
                    "kernel_scope": "the longest of the HIP-event-timed launches (NPGX_TIMERS=1: the aligner's "
                                    "k_align_jobs / k_align_wide); every kernel of the step is ranked in the "
                                    "rocprofv3 kernel-stats summaries under profiles/",
                    "launches_per_step": dom["launches"],
                    "avg_launch_ms": round(dom["ms"] / dom["launches"], 4),
                    "bytes_per_launch": dom["bytes"] / dom["launches"]}
    kernels = sorted(({"name": k["name"], "ms": round(k["ms"], 4), "launches": k["launches"]}
                      for k in kts), key=lambda k: -k["ms"])

    if roofline is not None:
        roofline.update(pmc_traffic(dom["name"], args.config))
    # stage accounting from one extra, untimed step with HIP events at the
    # stage boundaries (markers cost the GPU time: never in the timed region)
    stages = job.stage_timeline()
    stages["ms_per_step"] = round(dt / args.steps * 1e3, 4)
    if args.anchor_loop:  # (the stage clock splits the DraftPangenome part of the step only)
        stages["scope"] = "DraftPangenome only: the step's AnchorLoopFast is not split into stages"
    workload = job.workload_name(args.config)
    del job

    # the boundary takes host buffers: npgx_seqset_create's own timings, the
    # host to_atgcn (excluded, like the CPU side's input conversion) and the
    # upload proper (one DMA of the text + k_pack: BASELINE.md's "H2D included
    # on the GPU side"), median of 3; `value` stays HBM-resident (the task's
    # measurement contract), `pcie_inclusive` adds the upload to every step
    import statistics
    hosts, ups = [], []
    for _ in range(3):
        ss2 = _capi.SeqSet(seqs, names)
        h_ms, u_ms = ss2.timings()
        hosts.append(h_ms)
        ups.append(u_ms)
        ss2.close()
    up = statistics.median(ups) / 1e3
    step_s = dt / args.steps
    pcie = {"upload_ms": round(up * 1e3, 3), "host_to_atgcn_ms": round(statistics.median(hosts), 3),
            "value": round(harness.throughput(bp, 1 if sharded else world, 1, step_s + up) / 1e6, 3),
            "note": "upload = H2D of the text from pinned staging + k_pack, per step; host to_atgcn excluded"}

    # secondary lines, each in its own timed region after the headline's
    other = None
    if world > 1 and not args.no_replicas_line:
        if sharded:  # the same step in replica mode (every rank its own set, no collective)
            rseed = harness.rank_seed(synth.BASE_SEED, rank, args.config)
            rnames, rseqs = synth.genome_set(args.config, seed=rseed)
            rcomm = None
        else:        # one set (rank 0's seed) sharded over the ranks on the communicator
            rnames, rseqs = synth.genome_set(args.config, seed=harness.rank_seed(synth.BASE_SEED, 0, args.config))
            rcomm = comm
        rss = _capi.SeqSet(rseqs, rnames)
        rjob = pipeline.BlockBuild(rss, rnames, rseqs, comm=rcomm, anchor_loop=args.anchor_loop)
        rdt, _ = harness.timed_steps(rjob.run, args.steps, args.warmup, dist,
                                     sync=torch.cuda.synchronize, device="cuda")
        rbp = synth.total_bp(rseqs)
        other = {"value": round(harness.throughput(rbp, world if sharded else 1, args.steps, rdt) / 1e6, 3),
                 "unit": "Mbp/s", "ms_per_step": round(rdt / args.steps * 1e3, 4),
                 "scaling": "weak" if sharded else "strong",
                 "parallelism": ("replica-per-gpu x%d (independent sets, no collective)" % world) if sharded
                 else "sharded x%d (one set: AnchorFinder windows and aligner jobs over the ranks; %s)"
                      % (world, "library RCCL communicator" if args.dist_backend == "nccl" else args.dist_backend)}
        del rjob, rss
    pairs_line = None
    if not args.no_pairs_line and args.anchor_loop is False:
        # BASELINE C4's split at every N: genome pairs over the ranks, RCCL gather at the end
        pairs_line = run_pairs(args, dist, world, rank, local_rank, comm, args.pairs_config, args.pairs,
                               min(args.steps, 2), 1, baseline=not args.no_cpu_baseline, cpu_runs=3)
        if pairs_line is not None:
            pairs_line = {k: pairs_line[k] for k in ("value", "unit", "unit_note", "input_set_mbp_s",
                                                     "ms_per_step", "scaling", "config", "last_step",
                                                     "device_mem_used_gb", "roofline", "cpu_baseline")}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_sample or args.config, args.cpu_runs)
        if args.anchor_loop:  # the CPU leg times DraftPangenome only: not like-for-like
            cpu["workload"] = ("DraftPangenome only (the GPU step adds %s): no speedup ratio implied"
                               % ("AnchorLoop" if args.anchor_loop == "full" else "AnchorLoopFast"))

    if rank == 0:
        line = {
            "metric": "anchored+aligned Mbp/sec at 1/2/4/8 MI355X; bit-exact anchor set vs CPU",
            "value": round(value, 3),
            "unit": "Mbp/s",
            "n_gpus": world,
            "comm_ranks": comm_ranks,
            "launcher": launcher_name(),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded Brucella-like proxy, npge_amd/synth.py)",
            "config": {"workload": workload, "bp_per_rank": bp,
                       "genomes": synth.CONFIGS[args.config][0], "anchor_size": 20,
                       "anchor_fp": 0.1, "max_anchor_fragments": 100000,
                       "inputs": "resident in HBM before the timed region (upload: pcie_inclusive)",
                       "timers": "HIP events around the k_align_jobs launches only (NPGX_TIMERS=1: every "
                                 "event is a queue marker that costs the GPU time; per-kernel times of the "
                                 "rest: the rocprofv3 summaries in profiles/)",
                       "parallelism": ("sharded x%d (one set; %s)" % (world, "library RCCL communicator"
                                                                       if args.dist_backend == "nccl" else
                                                                       args.dist_backend)) if sharded
                       else "replica-per-gpu x%d (independent sets, no data-path collective)" % world},
            "last_step": info,
            "stage_timeline": stages,
            "kernels_last_step": kernels,
            "roofline": roofline,
            "pcie_inclusive": pcie,
            "cpu_baseline": cpu,
            ("replicas" if sharded else "sharded"): other,
            "pairs": pairs_line,
        }
        print(json.dumps(line), flush=True)
    finish(dist, world, comm)


def finish(dist, world, comm):
    import gc
    gc.collect()  # block sets hold the communicator: free them first
    if world > 1:
        if comm is not None and hasattr(comm, "close"):
            comm.close()
        dist.destroy_process_group()


def run_pairs(args, dist, world, rank, local_rank, comm, config, n_pairs, steps, warmup, baseline, cpu_runs=None):
    """The pair-sharded job (npge_amd/pairs.py, BASELINE C4's split).  One step =
    every pair of the set through DraftPangenome once (the rank's share,
    --pair-workers at a time) + the final all-gather of every pair's blocks
    over `comm`.  Returns rank 0's line (None on other ranks)."""
    import gc
    import torch
    from npge_amd import harness, pairs, synth
    names, seqs = synth.genome_set(config)
    sel = pairs.all_pairs(names)
    if n_pairs:
        sel = sel[:n_pairs]
    gdev = torch.device("cuda", local_rank) if world > 1 and args.dist_backend == "nccl" else None
    job = pairs.PairJobs(names, seqs, rank=rank, world=world, comm=comm, workers=args.pair_workers,
                         pairs=sel, device=local_rank, gather_device=gdev)
    torch.cuda.synchronize()
    dt, info = harness.timed_steps(job.run, steps, warmup, dist if world > 1 else None,
                                   sync=torch.cuda.synchronize, device="cuda")
    total = job.total_bp()
    value = total * steps / dt / 1e6          # the whole pair job over the max-over-ranks time
    set_bp = synth.total_bp(seqs)             # the genome set itself (each genome is in G - 1 pairs)
    agg = {k["name"]: k for k in job.kernel_times()}  # each pair's own times, taken right after it ran
    mem = round((lambda f: (f[1] - f[0]) / 2**30)(torch.cuda.mem_get_info()), 2)
    del job
    gc.collect()
    kern = [k for k in agg.values() if not k["name"].endswith("_allreduce")]
    dom = max(kern, key=lambda k: k["ms"]) if kern else None
    roofline = None
    if dom and dom["ms"] > 0:
        ach = dom["bytes"] / (dom["ms"] * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": None, "kernel": dom["name"],
                    "launches_per_rank_step": dom["launches"],
                    "avg_launch_ms": round(dom["ms"] / dom["launches"], 4),
                    "bytes_per_launch": dom["bytes"] / dom["launches"],
                    "note": "HIP-event kernel times of every pair of the rank, each pair's collected on its "
                            "worker right after it ran; concurrent pairs' events overlap, so this understates "
                            "the kernel's rate"}
        # HBM traffic per launch from the pair workload's own PMC passes
        # (profiles/*_<config>pairs_pmc_traffic.json, tools/round_end.sh)
        roofline.update(pmc_traffic(dom["name"], config + "pairs"))
    cpu = None
    if rank == 0 and world == 1 and baseline:
        cpu = cpu_baseline_pair(names, seqs, sel, cpu_runs or args.cpu_runs)
    if rank != 0:
        return None
    return {
        "metric": "anchored+aligned Mbp/sec at 1/2/4/8 MI355X; bit-exact anchor set vs CPU",
        "value": round(value, 3), "unit": "Mbp/s",
        "unit_note": "pair bp: every pair's two genomes count (each genome is in %d pairs); the genome "
                     "set's own rate is input_set_mbp_s" % (synth.CONFIGS[config][0] - 1),
        "input_set_mbp_s": round(set_bp * steps / dt / 1e6, 3),
        "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(dt / steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded, npge_amd/synth.py)",
        "config": {"workload": "%s pair-sharded: DraftPangenome per genome pair (%d pairs, %d bp), "
                               "final all-gather of every pair's blocks" % (config, len(sel), total),
                   "genomes": synth.CONFIGS[config][0], "pairs": len(sel), "bp_job": total,
                   "pair_workers": args.pair_workers,
                   "inputs": "every pair's sequences resident in HBM before the timed region",
                   "parallelism": "pairs round-robin over %d rank(s); %s" % (
                       world, "library RCCL communicator" if comm is not None and args.dist_backend == "nccl"
                       else (args.dist_backend if world > 1 else "no collective"))},
        "last_step": info,
        "device_mem_used_gb": mem,
        "kernels_last_step": sorted(({"name": k["name"], "ms": round(k["ms"], 4), "launches": k["launches"]}
                                     for k in agg.values()), key=lambda k: -k["ms"])[:12],
        "roofline": roofline,
        "cpu_baseline": cpu,
    }


def _oracle_pair_seconds(args):
    """One genome pair through the oracle's DraftPangenome, 1 thread (runs in
    a spawned worker process of cpu_baseline_pair's allotted-cores leg)."""
    import time
    from oracle import oracle as orc
    orc.use_native()  # the parent built it: the same -march=native library
    pn, ps = args
    o = orc.BlockSetOracle(ps, pn, seed=1)
    t = time.perf_counter()
    o.apply("DraftPangenome")
    return time.perf_counter() - t, o.hash()


def cpu_baseline_pair(names, seqs, sel, runs):
    """The oracle's DraftPangenome on genome pairs of the job (a bounded sample
    of the pair workload): one pair on one thread, median of `runs` (>= 3)
    after a warm-up; and the allotted-cores leg, as many pairs at once as the
    job has cores (OMP_NUM_THREADS), one spawned process per pair -- pairs are
    independent on the CPU too."""
    import multiprocessing as mp
    import statistics
    import time
    from concurrent.futures import ProcessPoolExecutor
    from oracle import oracle as orc
    native = orc.use_native()
    runs = max(3, runs)
    pn, ps = [names[i] for i in sel[0]], [seqs[i] for i in sel[0]]
    bp = sum(len(s) for s in ps)
    ts = [_oracle_pair_seconds((pn, ps))[0] for _ in range(runs + 1)][1:]
    t1 = statistics.median(ts)
    info = _cpu_info()
    cores = min(max(1, int(os.environ.get("OMP_NUM_THREADS", info["affinity"]))), info["affinity"], len(sel))
    batch = [([names[i] for i in idx], [seqs[i] for i in idx]) for idx in sel[:cores]]
    bbp = sum(len(s) for _, ps_ in batch for s in ps_)
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this process's GPU state
    # a worker that dies raises BrokenProcessPool here instead of hanging
    with ProcessPoolExecutor(max_workers=cores, mp_context=ctx) as pool:
        list(pool.map(_oracle_pair_seconds, batch))  # warm-up: the workers load the oracle
        t = time.perf_counter()
        list(pool.map(_oracle_pair_seconds, batch))
        tn = time.perf_counter() - t
    return {"value": round(bp / 1e6 / t1, 4), "unit": "Mbp/s", "cores": 1, "kind": "port",
            "sample": "one genome pair of the job (%s, %d bp), DraftPangenome, oracle/ C++ %s, 1 thread, "
                      "median of %d runs after 1 warm-up" % ("+".join(pn), bp,
                                                            "-O3 -march=native" if native else "-O3", runs),
            "workload": "DraftPangenome", "seconds": round(t1, 3), "runs_s": [round(x, 3) for x in ts],
            "host": info,
            "allotted_cores": {"value": round(bbp / 1e6 / tn, 4), "cores": cores, "seconds": round(tn, 3),
                               "sample": "the job's first %d pairs (%d bp) at once, one process per pair "
                                         "(1 thread each), after a warm-up pass" % (cores, bbp)}}


def pmc_traffic(kernel, config):
    """HBM traffic per launch of `kernel` from the newest committed PMC summary
    for this config (profiles/*_<config>_pmc_traffic.json, written by
    tools/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes
    of this bench).  PMC counters cannot be read from inside this process."""
    import glob
    # newest session tag: by round, then r03z < r03aa < r03ab (shorter suffixes first)
    def tag_key(f):
        tag = os.path.basename(f).split("_")[0]
        rnd = int(tag[1:3]) if tag[1:3].isdigit() else 0
        return (rnd, len(tag[3:]), tag[3:])
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "*_%s_pmc_traffic.json" % config.lower())),
                   key=tag_key)
    if not files:
        return {"traffic": None}
    doc = json.load(open(files[-1]))
    for name, v in doc["kernels"].items():
        if name.split("::")[-1].split("<")[0] == "k_" + kernel:  # (k_align_jobs<true>: the kernel's forms)
            if "active_traffic_bytes_per_launch" in v:  # launches that read something (the timed ones)
                return {"traffic": v["active_traffic_bytes_per_launch"], "traffic_source": os.path.basename(files[-1]),
                        "traffic_fetch": v["active_fetch_bytes_per_launch"],
                        "traffic_write": v["active_write_bytes_per_launch"],
                        "traffic_launches": "active (%d of %d dispatches read memory)" % (v["active_dispatches"],
                                                                                          v["dispatches"])}
            return {"traffic": v["traffic_bytes_per_launch"], "traffic_source": os.path.basename(files[-1]),
                    "traffic_fetch": v["fetch_bytes_per_launch"], "traffic_write": v["write_bytes_per_launch"]}
    return {"traffic": None}


def _cpu_info():
    """Host CPU facts for the record: nproc (the whole machine), the cores this
    job may use, and the lscpu model name."""
    import subprocess
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = os.cpu_count()
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                info["model"] = ln.split(":", 1)[1].strip()
    except Exception:  # lscpu missing: leave the model out
        pass
    return info


def cpu_baseline(config, runs=5):
    """The CPU restatement (oracle/) timed on this host on the same workload,
    built -O3 -march=native on this host (oracle/Makefile `native`): one thread
    (reference 1-worker semantics) and, under "allotted_cores", with FragmentTG +
    BlocksJobs threading (the reference's --workers; the Bloom pass sequential)
    over every core this job is allotted.  Each is the median of `runs` timed
    runs after one warm-up (steady clock), input packing excluded like the GPU
    side's upload."""
    import statistics
    import time
    from npge_amd import synth
    from oracle import oracle as orc
    native = orc.use_native()
    names, seqs = synth.genome_set(config)
    bp = synth.total_bp(seqs)

    def run(workers):
        o = orc.BlockSetOracle(seqs, names, seed=1)
        o.set_workers(workers)
        t = time.perf_counter()
        o.apply("DraftPangenome")
        dt = time.perf_counter() - t
        print("cpu_baseline: %s workers=%d %.3f s" % (config, workers, dt), file=sys.stderr, flush=True)
        return dt, o.hash()

    def median_of(workers):
        run(workers)  # warm-up
        ts, hs = [], set()
        for _ in range(runs):
            dt, h = run(workers)
            ts.append(dt)
            hs.add(h)
        if len(hs) != 1:
            raise AssertionError("oracle DraftPangenome not reproducible across runs")
        return statistics.median(ts), hs.pop(), ts

    info = _cpu_info()
    # the cores this job is allotted: the scheduler's OMP_NUM_THREADS share when
    # set (the GPU box's per-GPU CPU share), else every core in the affinity mask
    workers = max(1, int(os.environ.get("OMP_NUM_THREADS", info["affinity"])))
    workers = min(workers, info["affinity"])
    t1, h1, ts1 = median_of(1)
    tn, hn, tsn = median_of(workers)
    if hn != h1:
        raise AssertionError("threaded oracle DraftPangenome differs from the 1-thread run")
    return {"value": round(bp / 1e6 / t1, 4), "unit": "Mbp/s", "cores": 1, "kind": "port",
            "sample": "%s synthetic set (%d bp), one full DraftPangenome step, "
                      "oracle/ C++ %s, 1 thread, median of %d runs after 1 warm-up"
                      % (config, bp, "-O3 -march=native" if native else "-O3 (prebuilt)", runs),
            "workload": "DraftPangenome",
            "seconds": round(t1, 3), "runs_s": [round(x, 3) for x in ts1],
            "host": info,
            # the threads this job is allotted (OMP_NUM_THREADS, the box's per-GPU CPU share),
            # not every core of the machine (host.affinity)
            "allotted_cores": {"value": round(bp / 1e6 / tn, 4), "cores": workers, "seconds": round(tn, 3),
                          "runs_s": [round(x, 3) for x in tsn],
                          "threading": "FragmentTG per sequence (AnchorFinder pass 2), BlocksJobs per block "
                                       "(DummyAligner, FragmentsExtender, FixEnds, Filter); the Bloom pass "
                                       "and the loop's set operations sequential"}}


if __name__ == "__main__":
    main()
