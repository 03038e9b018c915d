#!/usr/bin/env python3
"""GPU occupancy of the pair-sharded job from a rocprofv3 kernel trace CSV:
the last step (after the largest idle gap, i.e. the warm-up step's end),
wall span, time with at least one kernel running, mean kernels in flight,
and per-kernel totals.  Usage: pairs_busy.py kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
# split at the largest gap between consecutive dispatch ends/starts
last_end, best, cut = ev[0][1], 0, 0
for i in range(1, len(ev)):
    g = ev[i][0] - last_end
    if g > best:
        best, cut = g, i
    last_end = max(last_end, ev[i][1])
step = ev[cut:]
t0, t1 = step[0][0], max(e for _, e, _ in step)
pts = sorted([(s, 1) for s, _, _ in step] + [(e, -1) for _, e, _ in step])
busy, inflight, area, prev = 0, 0, 0, t0
for t, d in pts:
    if inflight > 0:
        busy += t - prev
    area += inflight * (t - prev)
    inflight += d
    prev = t
print("step from dispatch %d (gap %.1f ms before it): %d dispatches, span %.1f ms, busy %.1f ms (%.1f %%), "
      "mean in flight %.2f" % (cut, best / 1e6, len(step), (t1 - t0) / 1e6, busy / 1e6, 100.0 * busy / (t1 - t0),
                               area / max(busy, 1)))
tot = {}
for s, e, n in step:
    k = tot.setdefault(n[-48:], [0, 0])
    k[0] += 1
    k[1] += e - s
for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:15]:
    print("  %-48s %6d  %9.1f ms" % (n, c, t / 1e6))
