#!/usr/bin/env python3
"""Diagnostic (GPU box): AnchorLoopFast step by step on the engine and the
oracle; prints the first step where the block sets differ."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from npge_amd import _capi, synth  # noqa: E402
from npge_amd.anchor_finder import AnchorFinder  # noqa: E402
from npge_amd.anchor_loop import anchor_blocks, block_order  # noqa: E402
from npge_amd.blockset import BlockSetEngine  # noqa: E402
from oracle import oracle as orc  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "tiny"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else -1


def canon(bl):
    return sorted(tuple(sorted(b)) for b in bl)


def cmp(tag, a, b):
    ca, cb = canon(a), canon(b)
    if ca == cb:
        print("%-28s same (%d blocks)" % (tag, len(ca)))
        return True
    sa, sb = set(ca), set(cb)
    print("%-28s DIFFER engine %d oracle %d: engine-only %d oracle-only %d" % (tag, len(ca), len(cb),
                                                                               len(sa - sb), len(sb - sa)))
    for x in list(sa - sb)[:3]:
        print("   engine-only", [(f[0], f[1], f[2], f[3], (f[4] or "")[:30]) for f in x])
    for x in list(sb - sa)[:3]:
        print("   oracle-only", [(f[0], f[1], f[2], f[3], (f[4] or "")[:30]) for f in x])
    return False


_capi.check(_capi.lib().npgx_set_device(0))
names, seqs = synth.genome_set(cfg)
o = orc.BlockSetOracle(seqs, names)
o.apply("DraftPangenome")
start = o.blocks()
eng = BlockSetEngine(_capi.SeqSet(seqs, names))
eng.set_blocks(start)
for step in ("Filter", "Rest"):
    eng.apply(step)
    o.apply(step)
    cmp(step, eng.blocks(), o.blocks())
eng.set_blocks(sorted(eng.blocks(), key=block_order))
o.set_blocks(sorted(o.blocks(), key=block_order))
cs_e, cs_o = eng.conseq(), o.conseq()
print("conseq same:", cs_e == cs_o, len(cs_e))
css = _capi.SeqSet(cs_e, [""] * len(cs_e))
ce = BlockSetEngine(css, max_iterations=iters)
co = orc.BlockSetOracle(cs_o, [""] * len(cs_o), portion_x1e4=5000, max_iterations=iters)
af = AnchorFinder()
ae = anchor_blocks(af.find(css))
ao = anchor_blocks(orc.AnchorFinder().run(cs_o, [""] * len(cs_o)))
cmp("AnchorFinder", ae, ao)
ce.set_blocks(ae)
co.set_blocks(ao)
for se, so in (("DummyAligner", "DummyAligner"), ("FragmentsExtender --extend-length-portion:=0.5", "FragmentsExtender"),
               ("Align", "MetaAligner"), ("ExtendLoopFast", "ExtendLoopFast")):
    ce.apply(se)
    co.apply(so)
    cmp("cons " + so, ce.blocks(), co.blocks())
print("cons iterations engine %d oracle %d" % (ce.stats()["iterations"], co.stats()["iterations"]))
n0 = len(eng.blocks())
eng.deconseq(ce)
o.deconseq(co)
cmp("DeConSeq", eng.blocks(), o.blocks())
eng.apply("Align")
o.apply("MetaAligner")
cmp("Align", eng.blocks(), o.blocks())
