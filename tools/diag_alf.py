#!/usr/bin/env python3
"""AnchorLoopFast step by step on the engine's processors and on the oracle's
(GPU box diagnostic): prints the first step where the two block sets differ,
with the differing blocks.  Usage: diag_alf.py [config]"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
from helpers import consensus_order, oracle_anchor_blocks  # noqa: E402
from npge_amd import _capi, synth  # noqa: E402
from npge_amd.anchor_finder import AnchorFinder  # noqa: E402
from npge_amd.anchor_loop import anchor_blocks  # noqa: E402
from npge_amd.blockset import BlockSetEngine  # noqa: E402
from oracle import oracle as orc  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "rtiny"
_capi.check(_capi.lib().npgx_set_device(0))
names, seqs = synth.genome_set(cfg)


def canon(blocks):
    return sorted(tuple(sorted(b)) for b in blocks)


def compare(step, eb, ob):
    ce, co = canon(eb), canon(ob)
    if ce == co:
        print("%-22s equal (%d blocks)" % (step, len(ce)), flush=True)
        return True
    se, so = set(ce), set(co)
    print("%-22s DIFFER: engine %d blocks, oracle %d; %d only in engine, %d only in oracle" % (
        step, len(ce), len(co), len(se - so), len(so - se)), flush=True)
    for tag, only in (("engine", se - so), ("oracle", so - se)):
        for b in sorted(only)[:4]:
            print("  only in %s:" % tag)
            for f in b:
                row = f[4]
                print("    seq %d [%d, %d] ori %+d row %s" % (f[0], f[1], f[2], f[3],
                                                             None if row is None else "%d cols %s..%s" % (
                                                                 len(row), row[:40], row[-40:])))
    return False


eng = BlockSetEngine(_capi.SeqSet(seqs, names))
eng.apply("DraftPangenome", af=AnchorFinder())
o = orc.BlockSetOracle(seqs, names)
o.apply("DraftPangenome")
ok = compare("DraftPangenome", eng.blocks(), o.blocks())
for op in ("Filter", "Rest"):
    eng.apply(op)
    o.apply(op)
    ok = ok and compare(op, eng.blocks(), o.blocks())
eng.set_blocks(sorted(eng.blocks(), key=consensus_order))
o.set_blocks(sorted(o.blocks(), key=consensus_order))
ecs, ocs = eng.conseq(), o.conseq()
print("ConSeq texts equal:", ecs == ocs, len(ecs), "sequences", flush=True)
cs = ocs
css = _capi.SeqSet(cs, orc.cons_names(cs))
ce = BlockSetEngine(css, max_iterations=-1, extend_portion_x1e4=5000)
oc = orc.BlockSetOracle(cs, orc.cons_names(cs), portion_x1e4=5000, max_iterations=-1)
ea = anchor_blocks(AnchorFinder().find(css))
oa = oracle_anchor_blocks(orc.AnchorFinder().run(cs, orc.cons_names(cs)))
compare("consensus anchors", ea, oa)
ce.set_blocks(oa)
oc.set_blocks(oa)
for op in ("DummyAligner", "FragmentsExtender", "Align", "ExtendLoopFast"):
    ce.apply(op)
    oc.apply(op)
    if not compare("cons " + op, ce.blocks(), oc.blocks()):
        ce.set_blocks(oc.blocks())  # continue from the oracle's state
eng.deconseq(ce)
o.deconseq(oc)
compare("DeConSeq", eng.blocks(), o.blocks())
eng.set_blocks(o.blocks())
eng.apply("Align")
o.apply("Align")
compare("Align", eng.blocks(), o.blocks())
