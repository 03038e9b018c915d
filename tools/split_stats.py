#!/usr/bin/env python3
"""Diagnostic (GPU box): one DraftPangenome with NPGX_SPLIT_DEBUG=1 -- per split
aligner job, the sync states found, the segments that reached one, overflows
and the chain of segments (stderr)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NPGX_SPLIT_DEBUG"] = "1"
os.environ["NPGX_JOB_STATS"] = "1"
from npge_amd import _capi, synth  # noqa: E402
from npge_amd.anchor_finder import AnchorFinder  # noqa: E402
from npge_amd.blockset import BlockSetEngine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
_capi.check(_capi.lib().npgx_set_device(0))
names, seqs = synth.genome_set(cfg)
ss = _capi.SeqSet(seqs, names)
eng = BlockSetEngine(ss)
eng.apply("DraftPangenome", af=AnchorFinder())

# the longest jobs of the last batch: wall time from the first segment's start,
# and the finishing wave's phases (clock64 cycles at ~2.4 GHz)
os.environ.pop("NPGX_SPLIT_DEBUG", None)
js = eng.job_stats()
if len(js):
    import numpy as np
    o = np.argsort(-js[:, 1])[:8]
    print("cols rows wall_us fin_us ph0_us(chain) ph1_us(regions+realign) ph2_us(realing_end) regions_us nreg")
    for j in o:
        r = js[j]
        print("%6d %3d %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f %d" % (
            r[1], r[6], (r[23] - r[11]) / 100.0, r[0] / 2400.0, r[8] / 2400.0, r[9] / 2400.0, r[10] / 2400.0,
            r[22] / 2400.0, r[5]))
