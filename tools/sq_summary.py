#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 SQ counters (one or more --pmc pass
directories with run_counter_collection.csv), and the wave-cycle split the
guide defines (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
~= WAVE_CYCLES, all in quad-cycles).

usage: sq_summary.py <pass dir> [<pass dir> ...] [--kernels substr,substr]
"""
import collections
import csv
import os
import sys


def main():
    dirs = [a for a in sys.argv[1:] if not a.startswith("--")]
    pick = None
    for a in sys.argv[1:]:
        if a.startswith("--kernels="):
            pick = a.split("=", 1)[1].split(",")
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in dirs:
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if pick and not any(p in name for p in pick):
                continue
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
    for name, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0)
        print(name)
        for k in sorted(c):
            share = " (%.1f %% of wave cycles)" % (100 * c[k] / wc) if wc and k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
            print("   %-24s %16.0f%s" % (k, c[k], share))


if __name__ == "__main__":
    main()
