#!/usr/bin/env python3
"""GPU box diagnostic: finds the first ExtendLoopFast iteration count at which
the engine and the oracle differ, then aligns that iteration's flank jobs on
the GPU aligner in one batch and saves the jobs that differ from the oracle."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as orc
from npge_amd import _capi, synth
from npge_amd.aligner import BatchAligner
from npge_amd.blockset import BlockSetEngine
from helpers import flank_jobs


def canon(blocks):
    return sorted(tuple(sorted(b)) for b in blocks)


cfg = sys.argv[1] if len(sys.argv) > 1 else "small"
names, seqs = synth.genome_set(cfg)
o = orc.BlockSetOracle(seqs, names)
af = orc.AnchorFinder()
r = af.run(seqs, names)
bs = r["block_start"]
o.set_blocks([[(int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i]), None)
               for i in range(bs[b], bs[b + 1])] for b in range(len(bs) - 1)])
o.apply("RemoveNonStem").apply("DummyAligner")
b0 = o.blocks()
ss = _capi.SeqSet(seqs, names)
prev = b0
for k in range(1, 11):
    eng = BlockSetEngine(ss, max_iterations=k)
    eng.set_blocks(b0).apply("ExtendLoopFast")
    ok = orc.BlockSetOracle(seqs, names, max_iterations=k)
    ok.set_blocks(b0)
    ok.apply("ExtendLoopFast")
    same = canon(eng.blocks()) == canon(ok.blocks())
    print("iterations", k, "blocks", len(ok.blocks()), "same", same, flush=True)
    if not same:
        jobs = flank_jobs(prev, seqs)
        gpu = BatchAligner().align(jobs)
        bad = [{"rows": rows, "oracle": orc.align(rows, "align_seqs"), "gpu": gpu[j]}
               for j, rows in enumerate(jobs) if orc.align(rows, "align_seqs") != gpu[j]]
        print("flank jobs", len(jobs), "differ", len(bad))
        # per-block difference
        e = canon(eng.blocks())
        c = canon(ok.blocks())
        only_e = [b for b in e if b not in set(c)]
        only_o = [b for b in c if b not in set(e)]
        print("only engine", len(only_e), "only oracle", len(only_o))
        json.dump({"bad_jobs": bad[:5], "only_engine": only_e[:3], "only_oracle": only_o[:3],
                   "prev": prev}, open("gpurun_out/diag_elf_%s.json" % cfg, "w"))
        break
    prev = ok.blocks()
