#!/usr/bin/env python3
"""Diagnostic (GPU box): the test_long_flanks sequence of aligner settings in
one process; reports every job whose rows differ from the oracle."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
from test_similar_aligner_gpu import _random_jobs  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from npge_amd.aligner import BatchAligner  # noqa: E402

jobs = _random_jobs(11, 40, nmax=17, lmax=1500)
exp = [orc.align(j, mode="align_seqs") for j in jobs]
seq = [("0", "0", "0"), ("1", "0", "0"), ("1000", "0", "0"), ("1000", "4", "0"), ("8000", "4", "0"),
       ("8000", "4", "512"), ("0", "0", "100"), ("1000", "4", "64")] * 8
for d, r, s in seq:
    os.environ["NPGX_ALIGN_DEFER"] = d
    os.environ["NPGX_ALIGN_DEFER_ROWS"] = r
    os.environ["NPGX_ALIGN_SPLIT"] = s
    got = BatchAligner().align(jobs)
    bad = [(j, len(jobs[j]), len(got[j][0]) if got[j] else 0, len(exp[j][0]) if exp[j] else 0)
           for j in range(len(jobs)) if got[j] != exp[j]]
    print(d, r, s, "bad", bad, flush=True)
