#!/usr/bin/env python3
"""GPU idle analysis of one DraftPangenome bench step from a rocprofv3 kernel
trace CSV: the dispatches of the last whole step (between Filter's last two
k_slice_counts), busy time vs wall span, and the largest idle gaps with the
dispatches on either side.  Usage: step_timeline.py kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
# steps end with Filter's k_slice_counts: a whole step is the dispatches after
# one k_slice_counts up to and including the next (the first is the warm-up)
ends = [i for i, e in enumerate(ev) if "k_slice_counts" in e[2]]
a, b = ends[-2] + 1, ends[-1] + 1
step = ev[a:b]
t0, t1 = step[0][0], max(e[1] for e in step)
busy, last_end = 0, t0
gaps = []
for i, (s, e, n) in enumerate(step):
    if s > last_end:
        gaps.append((s - last_end, i))
    busy += max(0, e - max(s, last_end))
    last_end = max(last_end, e)
print("step dispatches %d, span %.3f ms, busy %.3f ms (%.1f %%)" % (len(step), (t1 - t0) / 1e6, busy / 1e6,
                                                                  100.0 * busy / (t1 - t0)))
kinds = {}
for s, e, n in step:
    k = kinds.setdefault(n if n.startswith("__amd") else "kernels", [0, 0])
    k[0] += 1
    k[1] += e - s
print({k: (v[0], round(v[1] / 1e6, 3)) for k, v in kinds.items()})
gaps.sort(reverse=True)
print("largest idle gaps (us): before -> after")
for g, i in gaps[:25]:
    print("  %8.1f  %s -> %s" % (g / 1e3, step[i - 1][2][-40:], step[i][2][-40:]))
print("idle total %.3f ms in %d gaps; gaps > 20 us: %.3f ms" % (sum(g for g, _ in gaps) / 1e6, len(gaps),
                                                                 sum(g for g, _ in gaps if g > 20000) / 1e6))
