#!/usr/bin/env python3
"""Banded-DP stress (BASELINE config C5's "long-sequence banded DP stress"):
GeneralAligner (npgx_dp_*) over pairs of homologous stretches of a synthetic
Burkholderia-scale genome pair (C5: 50 Mbp, 1% divergence), gap_range 63 (one
full wave, 127 diagonals).

Reports GCUPS (band cells / kernel time from HIP events on the aligner's
stream), the algorithmic-bytes rate against 8 TB/s, and the CPU restatement
timed on a bounded sample of the same pairs (1 thread).  One JSON line.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def make_pairs(n, length, d, seed):
    import numpy as np
    from npge_amd import synth
    rng = np.random.default_rng(seed)
    root = rng.integers(0, 4, n * length).astype(np.uint8)
    der = synth._mutate(rng, root, d)
    A = synth.LETTERS[root].tobytes()
    B = synth.LETTERS[der].tobytes()
    # homologous windows: the derived genome drifts by indels; re-anchor by ratio
    ratio = len(B) / len(A)
    pairs = []
    for i in range(n):
        a0 = i * length
        b0 = int(a0 * ratio)
        pairs.append((A[a0:a0 + length], B[b0:b0 + length]))
    return pairs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4096)
    ap.add_argument("--length", type=int, default=12207)  # 4096 x 12.2 kb = 50 Mbp
    ap.add_argument("--gap-range", type=int, default=63)
    ap.add_argument("--max-errors", type=int, default=-1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-pairs", type=int, default=8)
    args = ap.parse_args()

    import torch
    torch.cuda.set_device(0)
    from npge_amd import _capi
    from npge_amd.dp import GeneralAligner
    _capi.check(_capi.lib().npgx_set_device(0))
    pairs = make_pairs(args.pairs, args.length, 0.01, 20261015 + 5)
    g = GeneralAligner(gap_range=args.gap_range, max_errors=args.max_errors,
                       cut_tail=args.max_errors >= 0)
    g.align_batch(pairs[:64])  # warm-up
    ms, cells, byts, wall = [], 0, 0, []
    for _ in range(args.steps):
        t = time.perf_counter()
        g.align_batch(pairs)
        wall.append(time.perf_counter() - t)
        k = [x for x in g.kernel_times() if x["name"] == "general_align"][0]
        ms.append(k["ms"])
        cells, byts = k["units"], k["bytes"]
    kms = sorted(ms)[len(ms) // 2]
    if os.environ.get("NPGX_PROFILE") == "1":
        f, b, st = g.phase_cycles()
        print("phase cycles per step: forward %.1f traceback %.1f (per wave, steps %d)"
              % (f / st, b / st, st), file=sys.stderr)
    bp = sum(len(a) + len(b) for a, b in pairs)

    # CPU restatement on a bounded sample (1 thread)
    from oracle import oracle as orc
    cs = pairs[:args.cpu_pairs]
    t = time.perf_counter()
    ccells = 0
    for a, b in cs:
        orc.general_align(a, b, args.gap_range, args.max_errors, 1, 1, args.max_errors >= 0)
    ct = time.perf_counter() - t
    r = g.align_batch(cs)
    # cells of the sample from the engine's own count
    k = [x for x in g.kernel_times() if x["name"] == "general_align"][0]
    ccells = k["units"]

    line = {
        "metric": "GeneralAligner banded DP (gap_range %d) cell updates/s" % args.gap_range,
        "value": round(cells / (kms * 1e-3) / 1e9, 3), "unit": "GCUPS",
        "kernel_ms": round(kms, 3), "wall_ms_incl_pcie": round(sorted(wall)[len(wall) // 2] * 1e3, 3),
        "pairs": args.pairs, "length": args.length, "cells": cells,
        "bp_per_s_kernel": round(bp / (kms * 1e-3) / 1e6, 1),
        "config": {"workload": "C5-style: %d x %d nt homologous pairs, 1%% divergence, "
                               "max_errors %d" % (args.pairs, args.length, args.max_errors)},
        "roofline": {"bound": "latency (dependent anti-diagonal steps)", "achieved_GBps":
                     round(byts / (kms * 1e-3) / 1e9, 2), "peak_GBps": 8000.0,
                     "frac": round(byts / (kms * 1e-3) / 1e9 / 8000.0, 5),
                     "bytes_per_launch": byts},
        "cpu_baseline": {"value": round(ccells / ct / 1e9, 5), "unit": "GCUPS", "cores": 1,
                         "kind": "port", "sample": "%d pairs of the same set, oracle/general_aligner.cpp"
                                                   % len(cs), "seconds": round(ct, 3)},
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
