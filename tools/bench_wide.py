#!/usr/bin/env python3
"""Wide alignment problems (more than 64 rows: repeat families, consensus
anchors -> k_align_wide, one 256-thread workgroup per problem) on the GPU box:
batches of synthetic repeat families (mutated copies of an ancestor at 0.5-5 %
divergence with indels, some with unrelated tails), one npgx_align_batch per
batch, GPU time as the median of 5 runs after a warm-up; the CPU restatement
(oracle/, one thread) on the first few families of each batch for the
comparison, and every family of the CPU sample checked identical.
Usage: bench_wide.py [--cpu-families K]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np

from npge_amd import _capi  # noqa: E402
from npge_amd.aligner import BatchAligner  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from test_similar_aligner_gpu import _family  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cpu-families", type=int, default=3)
args = ap.parse_args()
_capi.check(_capi.lib().npgx_set_device(0))
CASES = [  # (families, rows, length, divergence, unrelated-tail share)
    (64, 100, 500, 0.01, 0.0),
    (64, 200, 300, 0.02, 0.0),
    (32, 300, 1000, 0.01, 0.2),
    (16, 150, 2000, 0.05, 0.0),
]
al = BatchAligner()
out = []
for fam, n, L, d, tail in CASES:
    rng = np.random.default_rng(1000 + n + L)
    jobs = [_family(rng, n, L, d, tail_unrelated=tail) for _ in range(fam)]
    res = al.align(jobs)  # warm-up
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        res = al.align(jobs)
        ts.append(time.perf_counter() - t)
    gpu = statistics.median(ts)
    kt = {}
    for k in al.kernel_times():
        kt[k["name"]] = kt.get(k["name"], 0.0) + k["ms"]
    residues = sum(len(r) for j in jobs for r in j)
    t = time.perf_counter()
    for j, job in enumerate(jobs[:args.cpu_families]):
        exp = orc.align(job, mode="align_seqs")
        assert res[j] == exp, "family %d differs from the oracle" % j
    cpu = (time.perf_counter() - t) / max(1, min(args.cpu_families, fam))
    rec = {"families": fam, "rows": n, "length": L, "divergence": d, "unrelated_tails": tail,
           "residues": residues, "gpu_ms_batch": round(gpu * 1e3, 3),
           "gpu_residues_per_s": round(residues / gpu / 1e6, 2),
           "kernel_ms": {k: round(v, 3) for k, v in kt.items()},
           "cpu_ms_per_family_1thread": round(cpu * 1e3, 1),
           "speedup_vs_cpu_family_rate": round(cpu * fam / gpu, 1),
           "checked_vs_oracle": min(args.cpu_families, fam)}
    print(json.dumps(rec), flush=True)
    out.append(rec)
