"""AnchorLoopFast (src/algo/lua_lib.lua:741-758) on the HIP engine:

    Filter; Rest target=target other=target; ConSeq target=cons other=target;
    AnchorFinder target=cons; MoveUnchanged target=null other=cons;
    DummyAligner target=cons; ExtendAndAlign target=cons (FragmentsExtender
    --extend-length-portion:=0.5, Align); ExtendLoopFast target=cons (to
    convergence); DeConSeq target=target other=cons; Align; Clear target=cons

AnchorFinder runs on the consensus sequences of the current blocks (and the
uncovered stretches Rest adds), the anchors are grown into aligned blocks on
those consensuses and DeConSeq maps them back onto the genomes, where they are
appended to the blocks.  The whole pipe is one engine call
(``npgx_blockset_apply(b, "AnchorLoopFast", af)``): the consensus sequences
get a device sequence set and an engine of their own inside the library, and
no block list crosses into Python.  Like the reference's pipe object, the
AnchorFinder handle (its used-hash set) and the engine (the MoveUnchanged
hashes) carry state from one run to the next: pass the same AnchorFinder to
repeated runs of one pipe, a fresh one for a new pipe.
"""
from .anchor_finder import AnchorFinder


def anchor_blocks(r):
    """AnchorFinder SoA result -> blocks [(seq, min, max, ori, None), ...]."""
    bs = r["block_start"]
    return [[(int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i]), None)
             for i in range(bs[b], bs[b + 1])] for b in range(len(bs) - 1)]


def block_order(b):
    """Canonical block order before ConSeq: the sorted fragment coordinates
    (the order the engine pins, for the oracle side of the tests)."""
    return sorted((f[0], f[1], f[2], f[3]) for f in b)


def anchor_loop_fast(eng, af=None):
    """Runs AnchorLoopFast on `eng` (a BlockSetEngine over the genomes) in
    place; returns the pipe's statistics (consensus sequences, anchors found,
    consensus blocks, blocks mapped back, consensus loop iterations)."""
    af = af or AnchorFinder()
    eng.apply("AnchorLoopFast", af=af)
    return dict(eng.stats()["loop"])
