"""AnchorLoopFast (src/algo/lua_lib.lua:741-756) on the HIP engine:

    Filter; Rest target=target other=target; ConSeq target=cons other=target;
    AnchorFinder target=cons; DummyAligner target=cons;
    ExtendAndAlign target=cons (FragmentsExtender --extend-length-portion:=0.5,
    Align); ExtendLoopFast target=cons; DeConSeq target=target other=cons;
    Align; Clear target=cons

AnchorFinder runs on the consensus sequences of the current blocks (and the
uncovered stretches Rest adds), the anchors are grown into aligned blocks on
those consensuses and DeConSeq maps them back onto the genomes, where they are
appended to the blocks.  The pipe's `MoveUnchanged target=null other=cons`
step drops cons blocks whose hash an earlier run of the same pipe saw; one run
(this function) has no earlier run, so it is a no-op here.  Every step is the
engine's (GPU kernels + native host code); nothing falls back to the CPU.
"""
import numpy as np

from . import _capi
from .anchor_finder import AnchorFinder
from .blockset import BlockSetEngine


def anchor_blocks(r):
    """AnchorFinder SoA result -> blocks [(seq, min, max, ori, None), ...]."""
    bs = r["block_start"]
    return [[(int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i]), None)
             for i in range(bs[b], bs[b + 1])] for b in range(len(bs) - 1)]


def block_order(b):
    """Canonical block order before ConSeq: the sorted fragment coordinates."""
    return sorted((f[0], f[1], f[2], f[3]) for f in b)


def anchor_loop_fast(eng, af=None):
    """Runs AnchorLoopFast on `eng` (a BlockSetEngine over the genomes) in
    place; returns the consensus block set's statistics (anchors found, blocks
    mapped back)."""
    af = af or AnchorFinder()
    eng.apply("Filter").apply("Rest")
    # ConSeq's sequence order feeds AnchorFinder's rank ties (equal size and
    # name -> input index); the reference's is its std::set<Block*> pointer
    # order, i.e. arbitrary: pinned here to the blocks sorted by fragments
    eng.set_blocks(sorted(eng.blocks(), key=block_order))
    cs = eng.conseq()
    css = _capi.SeqSet(cs, [""] * len(cs))  # ConSeq names = block names (empty here)
    # the pipe's ExtendLoopFast runs to convergence (set_max_iterations(-1),
    # lua_lib.lua:697-699); DraftPangenome's cap of 10 does not apply here
    cons = BlockSetEngine(css, max_iterations=-1)
    af.clear_used()
    anchors = anchor_blocks(af.find(css))
    cons.set_blocks(anchors)
    # ExtendAndAlign (lua_lib.lua:669-674), then ExtendLoopFast
    cons.apply("DummyAligner").apply("FragmentsExtender --extend-length-portion:=0.5").apply("Align")
    cons.apply("ExtendLoopFast")
    loop_iterations = cons.stats()["iterations"]
    n_cons = len(cons.blocks())
    n_before = len(eng.blocks())
    eng.deconseq(cons)
    eng.apply("Align")
    return dict(consensus_sequences=len(cs), anchors=len(anchors), cons_blocks=n_cons,
                mapped_blocks=len(eng.blocks()) - n_before, loop_iterations=loop_iterations)
