"""Regenerates tests/golden/fullsize/*.json: fingerprints (tests/helpers.py
af_digest / blocks_digest) of the CPU restatement's outputs on the C4 and C5
synthetic sets (npge_amd/synth.py, seeded), which the oracle needs minutes for
and which therefore cannot be recomputed inside a GPU test.

    python tests/golden/make_fullsize.py [C4 C5 C5sub2 loop:C4 draft:C5 ...]

Cases: <cfg> = the whole set; <cfg>subN = its first N sequences.  Each case
records AnchorFinder (defaults, two runs on one instance so the persistent
used-hash set is covered) and, where listed in DP_CASES, DraftPangenome.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as orc  # noqa: E402
from npge_amd import synth  # noqa: E402
from helpers import af_digest, blocks_digest, oracle_anchor_loop  # noqa: E402

DP_CASES = {"C3", "C4", "C5sub2"}
LOOP_CASES = {"C3", "C4"}  # DraftPangenome -> AnchorLoopFast


def case_input(case):
    cfg, _, n = case.partition("sub")
    names, seqs = synth.genome_set(cfg)
    if n:
        names, seqs = names[:int(n)], seqs[:int(n)]
    return names, seqs


def make(case):
    names, seqs = case_input(case)
    out = {"case": case, "n_seqs": len(seqs), "bp": synth.total_bp(seqs), "af": []}
    o = orc.AnchorFinder()
    for _ in range(2):
        t = time.time()
        r = o.run(seqs, names)
        out["af"].append(af_digest(r, r["used"]))
        print(case, "AnchorFinder %.1f s" % (time.time() - t), flush=True)
    if case in DP_CASES:
        t = time.time()
        b = orc.BlockSetOracle(seqs, names)
        b.set_workers(os.cpu_count() or 1)
        b.apply("DraftPangenome")
        st = b.stats()
        out["draft"] = dict(blocks_digest(b.blocks()), hash=int(b.hash()),
                            stats={k: int(v) for k, v in st.items()})
        print(case, "DraftPangenome %.1f s" % (time.time() - t), flush=True)
        if case in LOOP_CASES:
            t = time.time()
            lst = oracle_anchor_loop(b, workers=os.cpu_count() or 1)
            out["anchor_loop"] = dict(blocks_digest(b.blocks()), hash=int(b.hash()),
                                      iterations=int(lst["iterations"]))
            print(case, "AnchorLoopFast %.1f s" % (time.time() - t), flush=True)
    with open(os.path.join(HERE, "fullsize", case + ".json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def add_draft(case):
    """Only the DraftPangenome entry, into an existing fixture."""
    names, seqs = case_input(case)
    path = os.path.join(HERE, "fullsize", case + ".json")
    with open(path) as f:
        out = json.load(f)
    t = time.time()
    b = orc.BlockSetOracle(seqs, names)
    b.set_workers(os.cpu_count() or 1)
    b.apply("DraftPangenome")
    st = b.stats()
    out["draft"] = dict(blocks_digest(b.blocks()), hash=int(b.hash()),
                        stats={k: int(v) for k, v in st.items()})
    print(case, "DraftPangenome %.1f s" % (time.time() - t), flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def add_loop(case):
    """Only the AnchorLoopFast entry, into an existing fixture."""
    names, seqs = case_input(case)
    path = os.path.join(HERE, "fullsize", case + ".json")
    with open(path) as f:
        out = json.load(f)
    t = time.time()
    b = orc.BlockSetOracle(seqs, names)
    b.set_workers(os.cpu_count() or 1)
    b.apply("DraftPangenome")
    lst = oracle_anchor_loop(b, workers=os.cpu_count() or 1)
    out["anchor_loop"] = dict(blocks_digest(b.blocks()), hash=int(b.hash()),
                              iterations=int(lst["iterations"]))
    print(case, "DraftPangenome + AnchorLoopFast %.1f s" % (time.time() - t), flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    for c in sys.argv[1:] or ["C4", "C5sub2", "C5"]:
        if c.startswith("loop:"):
            add_loop(c[5:])
        elif c.startswith("draft:"):
            add_draft(c[6:])
        else:
            make(c)
