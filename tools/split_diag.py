#!/usr/bin/env python3
"""Diagnostic (GPU box): jobs whose split alignment (NPGX_ALIGN_SPLIT=<n>)
differs from the oracle -- prints the job shape and the first differing column."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
split = sys.argv[1] if len(sys.argv) > 1 else "100"
os.environ["NPGX_ALIGN_SPLIT"] = split
os.environ["NPGX_ALIGN_DEFER"] = sys.argv[2] if len(sys.argv) > 2 else "0"
os.environ["NPGX_ALIGN_DEFER_ROWS"] = sys.argv[3] if len(sys.argv) > 3 else "0"
os.environ["NPGX_SPLIT_DEBUG"] = "1"
from test_similar_aligner_gpu import _random_jobs  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from npge_amd.aligner import BatchAligner  # noqa: E402

jobs = _random_jobs(11, 40, nmax=17, lmax=1500)
got = BatchAligner().align(jobs)
bad = 0
for j, (job, g) in enumerate(zip(jobs, got)):
    exp = orc.align(job, mode="align_seqs")
    if g == exp:
        continue
    bad += 1
    L = len(exp[0]) if exp else 0
    c = next((i for i in range(min(len(g[0]), L)) if any(gr[i] != er[i] for gr, er in zip(g, exp))), None)
    print("job %d: n=%d lens=%s gpu_len=%d exp_len=%d first_diff_col=%s" % (
        j, len(job), [len(r) for r in job], len(g[0]) if g else 0, L, c))
    r0 = job[0]
    gr = g[0].replace("-", "")
    # where the GPU's row 0 text goes on after the first difference, in the input
    k = c
    pieces = []
    at = 0
    while at < len(g[0]):
        seg = g[0][at:at + 30].replace("-", "")
        pieces.append((at, r0.find(seg) if seg else -2))
        at += 30
    print("  col->input pos of 30-col pieces:", pieces[:70])
    for i, (gr_, er_) in enumerate(zip(g, exp)):
        dc = [q for q in range(min(len(gr_), len(er_))) if gr_[q] != er_[q]]
        if dc:
            print("  row %d: %d cols differ, first %s; gpu %s exp %s" % (
                i, len(dc), dc[:8], gr_[dc[0]:dc[0] + 20], er_[dc[0]:dc[0] + 20]))
    if bad <= 0:
        lo = max(0, (c or 0) - 20)
        for gr, er in zip(g, exp):
            print("  gpu", gr[lo:lo + 60])
            print("  exp", er[lo:lo + 60])
print("bad", bad, "of", len(jobs))
