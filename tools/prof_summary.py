#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (sqlite .db or
kernel_stats.csv) into a short markdown table: kernel, calls, total us, avg us, %."""
import csv
import glob
import os
import re
import sqlite3
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)
    if "rocprim" in name:
        m = re.search(r"detail::(\w+?)(_impl|_config|<)", name)
        n = "rocprim::" + (m.group(1) if m else "kernel")
    return n[:80]


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4]))
                for r in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels")]
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main(src, title=""):
    paths = glob.glob(os.path.join(src, "**", "*.db"), recursive=True) + \
        glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
    if os.path.isfile(src):
        paths = [src]
    agg = {}
    for p in paths:
        for name, calls, tot, avg, pct in rows_from(p):
            k = short(name)
            a = agg.setdefault(k, [0, 0.0])
            a[0] += calls
            a[1] += tot
    total = sum(v[1] for v in agg.values()) or 1.0
    print("# rocprofv3 kernel summary %s" % title)
    print()
    print("| kernel | calls | total us | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for k, (calls, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("| %s | %d | %.1f | %.2f | %.1f |" % (k, calls, tot, tot / max(calls, 1), 100 * tot / total))


if __name__ == "__main__":
    main(sys.argv[1], " ".join(sys.argv[2:]))
