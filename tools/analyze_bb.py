#!/usr/bin/env python3
"""Runs DraftPangenome on a synthetic config a few times and prints the stage
timings and the aligner's per-job cost profile (GPU box diagnostic)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

os.environ.setdefault("NPGX_TIMERS", "2")  # every launch timed (read at handle creation)

os.environ.setdefault("NPGX_JOB_STATS", "1")  # per-job statistics (read at aligner creation)

from npge_amd import _capi, synth
from npge_amd.anchor_finder import AnchorFinder
from npge_amd.blockset import BlockSetEngine

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
_capi.check(_capi.lib().npgx_set_device(0))
if cfg.endswith(":pair"):  # the first genome pair of a config (the pair-sharded job's unit)
    from npge_amd import pairs as _pairs
    names, seqs = synth.genome_set(cfg.split(":")[0])
    idx = _pairs.all_pairs(names)[0]
    names, seqs = [names[i] for i in idx], [seqs[i] for i in idx]
else:
    names, seqs = synth.genome_set(cfg)
ss = _capi.SeqSet(seqs, names)
eng = BlockSetEngine(ss)
best = None
af = AnchorFinder()
for rep in range(5):
    af.clear_used()
    t = time.perf_counter()
    eng.apply("DraftPangenome", af=af)
    dt = time.perf_counter() - t
    st = eng.stats()
    staged = sum(list(st["ms_stage"].values())[:10])
    print("rep", rep, "apply wall %.2f ms, stages 0-9 %.2f ms" % (dt * 1e3, staged), file=sys.stderr)
    if best is None:
        best = dict(st, ms_stage=dict(st["ms_stage"]))
    else:
        for k, v in st["ms_stage"].items():
            best["ms_stage"][k] = min(best["ms_stage"][k], v)
st = dict(st, ms_stage_min=best["ms_stage"])
kts = eng.kernel_times()
print("aligner launches (ms):", [(k["name"][6:], round(k["ms"], 3)) for k in kts if k["name"].startswith("align")],
      file=sys.stderr)
kt = {}
for k in kts:  # last rep, summed per kernel (HIP events)
    e = kt.setdefault(k["name"], [0.0, 0])
    e[0] += k["ms"]
    e[1] += 1
kt = {n: [round(v[0], 3), v[1]] for n, v in sorted(kt.items(), key=lambda x: -x[1][0])}
print(json.dumps({"config": cfg, "wall_ms": round(dt * 1e3, 2), "stats": st, "kernels": kt}, default=str))
js = eng.job_stats()
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/jobstats_%s%s.npy" % (cfg, "_prof" if os.environ.get("NPGX_PROFILE") == "1" else ""), js)
cyc, cols, calls, shifts, gaps, regions, rows, fast = js.T[:8]
print("jobs", len(js), "total cycles %.3e" % cyc.sum(), "columns", cols.sum(), "shifts", shifts.sum(),
      "aligned calls", calls.sum(), "gaps", gaps.sum())
order = np.argsort(-cyc)
print("top jobs by cycles (cycles, cols, calls, shifts, gaps, regions, rows, fast runs, cyc/col):")
for i in order[:25]:
    print("  ", cyc[i], cols[i], calls[i], shifts[i], gaps[i], regions[i], rows[i], fast[i],
          round(cyc[i] / max(cols[i], 1), 1))
# job-stat columns (include/npge_amd.h npgx_align_job_stats): 8-10 the phases
# process_seqs / fix_bad_regions / realing_end, 11 and 23 wall-clock start and
# end (not cycles), 12-21 the profiling build's Proc counters, 22 regions
names = ["process_seqs", "fix_bad_regions", "realing_end"]
prof_names = ["fast_run", "eq/mismatch", "try_gap", "try_aligned", "vec_words", "vec_compares",
              "vec_chunks", "vec_calls", "append_end", "child_return"]
cols_ph = [8, 9, 10] + list(range(12, 22)) + [22]
all_names = names + prof_names + ["regions"]
ph = js[:, cols_ph]
tot = ph.sum(axis=0)
print("phase cycles (all jobs):", {n: "%.3e" % t for n, t in zip(all_names, tot)})
for i in order[:5]:
    print("  top job phases:", {n: int(t) for n, t in zip(all_names, ph[i])})
print("cycles per column (median, p90, p99):", np.percentile(cyc / np.maximum(cols, 1), [50, 90, 99]))
if shifts.sum():
    m = shifts > 0
    print("jobs with shifts:", m.sum(), "cycles share:", cyc[m].sum() / cyc.sum())
    # regression: cycles ~ a*cols + b*shifts
    A = np.vstack([cols, shifts, gaps, np.ones_like(cols)]).T.astype(float)
    coef = np.linalg.lstsq(A, cyc.astype(float), rcond=None)[0]
    print("fit cycles = %.1f*cols + %.1f*shifts + %.1f*gaps + %.1f" % tuple(coef))
big = cols > 20000
if big.any():
    A = np.vstack([cols[big], shifts[big], gaps[big], fast[big], np.ones(big.sum())]).T.astype(float)
    coef = np.linalg.lstsq(A, cyc[big].astype(float), rcond=None)[0]
    print("long jobs (%d): fit cycles = %.1f*cols + %.1f*shifts + %.1f*gaps + %.1f*fast + %.1f" % ((big.sum(),) + tuple(coef)))
