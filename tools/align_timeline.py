#!/usr/bin/env python3
"""Per-launch timeline of the similar aligner during one DraftPangenome
(GPU box diagnostic): job start/end from the device's constant-rate clock
(job stats 11 / 23, wall_clock64 at 100 MHz), grouped into launches by gaps.
Shows how much of each launch is the tail after most jobs have finished."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

os.environ.setdefault("NPGX_TIMERS", "2")  # every launch timed (read at handle creation)

os.environ.setdefault("NPGX_JOB_STATS", "1")
from npge_amd import _capi, synth  # noqa: E402
from npge_amd.anchor_finder import AnchorFinder  # noqa: E402
from npge_amd.blockset import BlockSetEngine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
_capi.check(_capi.lib().npgx_set_device(0))
names, seqs = synth.genome_set(cfg)
ss = _capi.SeqSet(seqs, names)
eng = BlockSetEngine(ss)
af = AnchorFinder()
for rep in range(3):
    af.clear_used()
    eng.apply("DraftPangenome", af=af)
js = eng.job_stats()
t0, t1, cols, rows = js[:, 11], js[:, 23], js[:, 1], js[:, 6]
ok = t1 > 0
js, t0, t1, cols, rows = js[ok], t0[ok], t1[ok], cols[ok], rows[ok]
o = np.argsort(t0)
gaps = np.diff(t0[o])
cut = np.where(gaps > 2000)[0]  # > 20 us without a job start: next launch
bounds = np.concatenate([[0], cut + 1, [len(o)]])
US = 0.01  # ticks -> us at 100 MHz
tot_span = tot_busy = 0.0
print("launch jobs span_us p50_us p90_us p99_us last_job_us(cols,rows) busy_frac")
for a, b in zip(bounds[:-1], bounds[1:]):
    ids = o[a:b]
    s0 = t0[ids].min()
    ends = np.sort(t1[ids] - s0) * US
    span = ends[-1]
    dur = (t1[ids] - t0[ids]) * US
    i = ids[np.argmax(dur)]
    busy = dur.sum() / (span * 4096) if span > 0 else 0
    tot_span += span
    tot_busy += dur.sum()
    print("%3d %6d %8.1f %7.1f %7.1f %7.1f %8.1f(%d,%d) %.3f" % (
        0, len(ids), span, ends[int(0.5 * (len(ends) - 1))], ends[int(0.9 * (len(ends) - 1))],
        ends[int(0.99 * (len(ends) - 1))], dur.max(), cols[i], rows[i], busy))
print("sum of launch spans %.1f us; job-time %.1f us (x4096 slots: %.3f)" % (tot_span, tot_busy,
                                                                         tot_busy / max(tot_span * 4096, 1)))
