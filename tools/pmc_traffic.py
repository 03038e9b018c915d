#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from rocprofv3 PMC passes
(tools/pmc_session.sh): FETCH_SIZE and WRITE_SIZE come from separate passes
(they do not fit one pass on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC
slots").  Both counters are in KiB.  FETCH_SIZE is reported as measured: the
guide's x2 correction holds for 16-B-per-lane streaming reads, and these
kernels read bytes and words (uncalibrated width), so the raw value is kept
and the correction is noted.

usage: pmc_traffic.py <dir with <tag>_FETCH_SIZE/ and <tag>_WRITE_SIZE/> <tag> <out.json>
"""
import collections
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0]
        acc[name][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return acc


def per_kernel(path, counter):
    acc = per_dispatch(path, counter)
    return {k: (len(v), sum(v.values()) / len(v)) for k, v in acc.items()}


def main():
    root, tag, out = sys.argv[1], sys.argv[2], sys.argv[3]
    f = per_kernel(os.path.join(root, tag + "_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_kernel(os.path.join(root, tag + "_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    # launches that read (next to) nothing (the device loop's re-run launch of the
    # aligner when no job overflowed: the same kernel, an empty queue) are
    # averaged separately: the "active" figures match the HIP-event-timed
    # launches bench.py prices
    fd = per_dispatch(os.path.join(root, tag + "_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    wd = per_dispatch(os.path.join(root, tag + "_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fk = f.get(k, (0, 0.0))[1] * 1024
        wk = w.get(k, (0, 0.0))[1] * 1024
        res[k] = {"dispatches": max(f.get(k, (0, 0))[0], w.get(k, (0, 0))[0]),
                  "fetch_bytes_per_launch": round(fk), "write_bytes_per_launch": round(wk),
                  "traffic_bytes_per_launch": round(fk + wk)}
        # the fetch and write passes are separate runs of the same program:
        # dispatches pair up in order
        fl = [fd[k][d] for d in sorted(fd.get(k, {}))]
        wl = [wd[k][d] for d in sorted(wd.get(k, {}))]
        if fl and len(fl) == len(wl):
            act = [(a, b) for a, b in zip(fl, wl) if a > 64]  # (KiB: an empty launch reads a few lines)
            if act and len(act) < len(fl):
                af = sum(a for a, _ in act) / len(act) * 1024
                aw = sum(b for _, b in act) / len(act) * 1024
                res[k].update({"active_dispatches": len(act), "active_fetch_bytes_per_launch": round(af),
                               "active_write_bytes_per_launch": round(aw),
                               "active_traffic_bytes_per_launch": round(af + aw)})
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-trace, "
                     "bench.py --steps 1 --warmup 1; KiB x 1024; FETCH_SIZE uncorrected (byte/word "
                     "accesses, not 16-B/lane streaming)", "kernels": res}
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"])[:12]:
        print("%-40s %6d  fetch %12d  write %12d" % (k[-40:], v["dispatches"], v["fetch_bytes_per_launch"],
                                                    v["write_bytes_per_launch"]))


if __name__ == "__main__":
    main()
