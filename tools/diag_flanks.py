#!/usr/bin/env python3
"""GPU box diagnostic: aligns every FragmentsExtender flank job of a synthetic
config on the GPU aligner and with the oracle, and saves the jobs that differ
(gpurun_out/diag_flanks_<cfg>.json)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as orc
from npge_amd import synth
from npge_amd.aligner import BatchAligner

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from helpers import flank_jobs as _flank_jobs  # noqa: E402


def flank_jobs(seqs, names):
    o = orc.BlockSetOracle(seqs, names)
    af = orc.AnchorFinder()
    r = af.run(seqs, names)
    bs = r["block_start"]
    blocks = [[(int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i]), None)
               for i in range(bs[b], bs[b + 1])] for b in range(len(bs) - 1)]
    o.set_blocks(blocks)
    o.apply("RemoveNonStem").apply("DummyAligner")
    return _flank_jobs(o.blocks(), seqs)


cfg = sys.argv[1] if len(sys.argv) > 1 else "small"
names, seqs = synth.genome_set(cfg)
o = orc.BlockSetOracle(seqs, names)
af = orc.AnchorFinder()
r = af.run(seqs, names)
bs = r["block_start"]
o.set_blocks([[(int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i]), None)
               for i in range(bs[b], bs[b + 1])] for b in range(len(bs) - 1)])
o.apply("RemoveNonStem").apply("DummyAligner")
bad = []
al = BatchAligner()
for it in range(8):
    jobs = _flank_jobs(o.blocks(), seqs)
    if not jobs:
        break
    gpu = al.align(jobs)
    nb = 0
    for j, rows in enumerate(jobs):
        ref = orc.align(rows, "align_seqs")
        if ref != gpu[j]:
            nb += 1
            bad.append({"iteration": it, "rows": rows, "oracle": ref, "gpu": gpu[j]})
    print("iteration", it, "jobs", len(jobs), "max len", max(len(r) for j in jobs for r in j), "differ", nb)
    o.apply("FragmentsExtender").apply("FixEnds")
os.makedirs("gpurun_out", exist_ok=True)
bad.sort(key=lambda x: sum(len(r) for r in x["rows"]))
json.dump(bad[:10], open("gpurun_out/diag_flanks_%s.json" % cfg, "w"))
