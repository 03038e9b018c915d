#!/usr/bin/env python3
"""Per-iteration aligner kernels of the last whole DraftPangenome step in a
rocprofv3 kernel trace: the iteration's aligner span (first to last aligner
kernel), its k_align_jobs and k_align_sub durations (us).
usage: align_iters.py run_kernel_trace.csv [...]"""
import csv
import sys

AL = ("k_align_jobs", "k_align_sub", "k_split_find", "k_chain_copy", "k_split_post", "k_sub_post", "k_align_finish",
      "k_scatter", "k_split_chain", "k_sub_rows", "k_plan_subs", "k_fin_copy", "k_fin_prefix", "k_retry_list",
      "k_job_rows", "k_sub_retry_list")


def iterations(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]) for r in rows)
    ends = [i for i, e in enumerate(ev) if e[2] == "k_slice_counts"]
    step = ev[ends[-2] + 1:ends[-1] + 1]
    its = []
    for s, e, n in step:
        if n == "k_dt_decode":
            its.append([])
        if its and n in AL:
            its[-1].append((s, e, n))
    out = []
    for lst in its:
        span = (lst[-1][1] - lst[0][0]) / 1e3
        out.append((round(span), [round((e - s) / 1e3) for s, e, n in lst if n == "k_align_jobs"],
                    [round((e - s) / 1e3) for s, e, n in lst if n == "k_align_sub"]))
    return out, (step[-1][1] - step[0][0]) / 1e6


if __name__ == "__main__":
    for p in sys.argv[1:]:
        its, span = iterations(p)
        print(p, "step span %.2f ms, aligner spans %.0f us" % (span, sum(x[0] for x in its)))
        for x in its:
            print("   ", x)
