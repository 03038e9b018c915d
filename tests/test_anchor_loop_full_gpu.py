"""The AnchorLoop pipe (lua_lib.lua:711-737) and the processors only it uses
-- UniqueNames, RemoveWithSameName, SplitExtendable (SplitExtendable.cpp:46-84),
ExtendLoop (lua_lib.lua:677-688) with AddingLoopBySize / SmthUnion
(TrySmth.cpp:35-178) -- on the engine vs the oracle's restatement
(oracle/npge_oracle.cpp anchor_loop): fragments and rows bit-exact, the
pipe's counts equal.  Parity is pinned to the restatement (the reference
has no fixture for these pipes) and to its conventions."""
import pytest

from oracle import oracle as orc
from npge_amd import synth

pytestmark = pytest.mark.gpu


def canon(blocks):
    return sorted(tuple(sorted(b)) for b in blocks)


def _engine(seqs, names, blocks):
    from npge_amd import _capi
    from npge_amd.blockset import BlockSetEngine
    return BlockSetEngine(_capi.SeqSet(seqs, names)).set_blocks(blocks)


@pytest.mark.parametrize("cfg", ["tiny", "rtiny", "small", "C2"])
def test_anchor_loop(cfg):
    """C2 (3 genomes, 9.9 Mbp): the oracle pipe takes about 90 s on one thread."""
    from npge_amd.anchor_finder import AnchorFinder
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    start = o.blocks()
    eng = _engine(seqs, names, start)
    eng.apply("AnchorLoop", af=AnchorFinder())
    o.set_blocks(start)
    o.apply("AnchorLoop")
    est, ost = eng.anchor_loop_stats(), o.anchor_loop_stats()
    assert est == ost
    assert ost["anchors_left"] > 0 and ost["split_blocks"] > 0
    assert canon(eng.blocks()) == canon(o.blocks())


def test_extend_loop():
    """ExtendLoop alone, from DummyAligner'd anchors."""
    from npge_amd.anchor_loop import anchor_blocks
    names, seqs = synth.genome_set("tiny")
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(anchor_blocks(orc.AnchorFinder().run(seqs, names)))
    o.apply("DummyAligner")
    start = o.blocks()
    eng = _engine(seqs, names, start)
    eng.apply("ExtendLoop")
    o.apply("ExtendLoop")
    assert len(o.blocks()) > 0
    assert eng.stats()["iterations"] == o.stats()["iterations"]
    assert canon(eng.blocks()) == canon(o.blocks())


def test_adding_loop_by_size():
    """AddingLoopBySize alone on overlapping blocks (DraftPangenome's and
    their 50-bp shifted copies): the cuts of SmthUnion, bit-exact."""
    from test_oracle_anchor_loop import overlapping_input, overlaps
    names, seqs, blocks = overlapping_input()
    eng = _engine(seqs, names, blocks)
    eng.apply("AddingLoopBySize")
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(blocks)
    o.apply("AddingLoopBySize")
    assert overlaps(o.blocks()) == 0
    assert canon(eng.blocks()) == canon(o.blocks())


def test_processor_mirror():
    """new_p('AddingLoopBySize') / new_p('ExtendLoop') of the Python mirror
    (lua_lib.lua:59-61 call shapes) over model block sets: the engine's
    blocks, through the same C ABI."""
    from test_oracle_anchor_loop import overlapping_input
    from npge_amd import script  # noqa: F401  (registers the engine processors)
    from npge_amd.model import Block, BlockSet, Fragment, Sequence
    from npge_amd.processor import new_p
    names, seqs, blocks = overlapping_input()
    sq = [Sequence(n, s) for n, s in zip(names, seqs)]
    other = BlockSet(seqs=list(sq), blocks=[Block([Fragment(sq[f[0]], f[1], f[2], f[3], f[4]) for f in b])
                                            for b in blocks])
    target = BlockSet(seqs=list(sq))
    p = new_p("AddingLoopBySize")
    p.set_bs("target", target)
    p.set_bs("other", other)
    p.run()
    got = canon([[(sq.index(f.seq), f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments]
                 for b in target.blocks])
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(blocks)
    o.apply("AddingLoopBySize")
    assert not other.blocks and got == canon(o.blocks())


def test_anchor_loop_failure_keeps_blocks(monkeypatch):
    """A failure inside AnchorLoop while the set's own blocks wait aside
    (after the first DeConSeq; NPGX_TEST_FAIL_ANCHOR_LOOP=1 injects it): the
    call reports the error and the set holds its own blocks as the pipe's
    first steps left them (Filter, then Rest: lua_lib.lua:711-737 applies the
    processors to the target one by one), not the deconseq list it was
    working on; the handle then runs the pipe again."""
    from npge_amd.anchor_finder import AnchorFinder
    names, seqs = synth.genome_set("tiny")
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    start = o.blocks()
    eng = _engine(seqs, names, start)
    monkeypatch.setenv("NPGX_TEST_FAIL_ANCHOR_LOOP", "1")
    with pytest.raises(Exception, match="injected failure"):
        eng.apply("AnchorLoop", af=AnchorFinder())
    o.set_blocks(start)
    o.apply("Filter")
    o.apply("Rest")
    mid = o.blocks()
    assert canon(eng.blocks()) == canon(mid)
    monkeypatch.delenv("NPGX_TEST_FAIL_ANCHOR_LOOP")
    eng.apply("AnchorLoop", af=AnchorFinder())
    o.apply("AnchorLoop")
    assert canon(eng.blocks()) == canon(o.blocks())
