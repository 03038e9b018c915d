"""Rest and AnchorLoopFast (lua_lib.lua:741-756) on the engine vs the same
pipe over the oracle's processors: anchors found on the consensus sequences
of the DraftPangenome blocks, grown on the consensuses and mapped back by
DeConSeq; fragments and rows bit-exact."""
import pytest

from oracle import oracle as orc
from npge_amd import synth

pytestmark = pytest.mark.gpu


def canon(blocks):
    return sorted(tuple(sorted(b)) for b in blocks)


def _engine(seqs, names, blocks=None):
    from npge_amd import _capi
    from npge_amd.blockset import BlockSetEngine
    eng = BlockSetEngine(_capi.SeqSet(seqs, names))
    if blocks is not None:
        eng.set_blocks(blocks)
    return eng


def test_rest_kats():
    """src/test/rest.cpp through the engine."""
    seqs, names = ["tGGtccgagcgGAcggcc", "tGGtccgagcggacggcc"], ["s1", "s2"]
    from npge_amd.io import to_atgcn
    seqs = [to_atgcn(s) for s in seqs]
    blocks = [[(0, 1, 2, 1, None), (1, 1, 2, 1, None)], [(0, 11, 12, 1, None)]]
    eng = _engine(seqs, names, blocks).apply("Rest")
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(blocks)
    o.apply("Rest")
    assert eng.blocks() == o.blocks()
    assert len(eng.blocks()) == 7
    assert _engine(["AAA"], ["s"], []).apply("Rest").blocks() == [[(0, 0, 2, 1, None)]]


def _oracle_loop(o):
    from helpers import oracle_anchor_loop
    return oracle_anchor_loop(o)


@pytest.mark.parametrize("cfg", ["tiny", "small"])
def test_anchor_loop_fast(cfg):
    from npge_amd.anchor_finder import AnchorFinder
    from npge_amd.anchor_loop import anchor_loop_fast
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    start = o.blocks()
    eng = _engine(seqs, names, start)
    st = anchor_loop_fast(eng, AnchorFinder())
    o.set_blocks(start)
    ost = _oracle_loop(o)
    assert st["consensus_sequences"] > len(start)
    assert st["anchors"] > 0 and st["mapped_blocks"] > 0
    assert st["loop_iterations"] == ost["iterations"]
    assert canon(eng.blocks()) == canon(o.blocks())


def test_extend_loop_to_convergence():
    """ExtendLoopFast with max_iterations -1 (the AnchorLoopFast pipe's
    set_max_iterations(-1)) runs past DraftPangenome's cap of 10 until the
    block set repeats; engine and oracle agree on blocks and iterations."""
    from npge_amd import _capi
    from npge_amd.blockset import BlockSetEngine
    from npge_amd.anchor_loop import anchor_blocks
    names, seqs = synth.genome_set("small")  # converges after 14 iterations
    anchors = anchor_blocks(orc.AnchorFinder().run(seqs, names))
    eng = BlockSetEngine(_capi.SeqSet(seqs, names), max_iterations=-1).set_blocks(anchors)
    o = orc.BlockSetOracle(seqs, names, max_iterations=-1)
    o.set_blocks(anchors)
    for se, so in (("RemoveNonStem --exact", "RemoveNonStem"), ("DummyAligner", "DummyAligner"),
                   ("ExtendLoopFast", "ExtendLoopFast")):
        eng.apply(se)
        o.apply(so)
    assert eng.stats()["iterations"] == o.stats()["iterations"] > 10
    assert canon(eng.blocks()) == canon(o.blocks())


def test_fragments_extender_portion_option():
    """The standalone FragmentsExtender defaults to extend-length-portion 0
    (FragmentsExtender.cpp:28-30); "--extend-length-portion:=0.5" is the
    ExtendAndAlign / ExtendAndFix setting."""
    names, seqs = synth.genome_set("tiny")
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    start = o.blocks()
    for opt, portion in (("", 0), (" --extend-length-portion:=0.5", 5000), (" --extend-length-portion=0.25", 2500)):
        eng = _engine(seqs, names, start).apply("FragmentsExtender" + opt)
        ref = orc.BlockSetOracle(seqs, names, portion_x1e4=portion)
        ref.set_blocks(start)
        ref.apply("FragmentsExtender")
        assert canon(eng.blocks()) == canon(ref.blocks())


def _repeat_genomes(copies, genomes=2, unit=300, seed=5, where=None):
    """Genomes of random sequence with `copies` slightly mutated copies of one
    repeat unit each (an IS-element-like family); `where` collects the copies
    as fragments (genome, first, last, ori)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    rep = rng.integers(0, 4, unit)
    names, seqs = [], []
    for g in range(genomes):
        parts = []
        for _ in range(copies):
            parts.append(rng.integers(0, 4, int(rng.integers(200, 400))))
            if where is not None:
                at = sum(len(p) for p in parts)
                where.append((g, at, at + unit - 1, 1 if len(where) % 3 else -1, None))
            r = rep.copy()
            m = rng.random(unit) < 0.01
            r[m] = (r[m] + rng.integers(1, 4, int(m.sum()))) % 4
            parts.append(r)
        s = np.concatenate(parts)
        names.append("G%02d&chr1&c" % (g + 1))
        seqs.append("".join("ATGC"[x] for x in s))
    return names, seqs


def test_more_than_64_rows():
    """A block of more than 64 fragments (a repeat family across genomes) is
    aligned by the workgroup-per-problem aligner (wide_aligner.hip):
    AnchorLoopFast (FragmentsExtender flanks and the closing Align of
    80-fragment blocks) on genomes carrying 40 copies each, and 30 copies (60
    fragments, the batched aligner), both matching the oracle."""
    from npge_amd.anchor_finder import AnchorFinder
    from npge_amd.anchor_loop import anchor_loop_fast
    for copies in (40, 30):
        names, seqs = _repeat_genomes(copies)
        eng = _engine(seqs, names, [])
        st = anchor_loop_fast(eng, AnchorFinder())
        o = orc.BlockSetOracle(seqs, names)
        o.set_blocks([])
        ost = _oracle_loop(o)
        assert st["anchors"] > 0
        assert st["loop_iterations"] == ost["iterations"]
        assert canon(eng.blocks()) == canon(o.blocks())


def test_align_more_than_64_fragments():
    """MetaAligner on a block of 80 unaligned repeat copies (mixed
    orientations, widened by random amounts) next to ordinary blocks: rows
    bit-exact vs the oracle's align_block + refine_alignment; then the whole
    Align pipe (MoveGaps / CutGaps / Filter on the 80-row block) likewise."""
    import numpy as np
    where = []
    names, seqs = _repeat_genomes(40, where=where)
    rng = np.random.default_rng(8)
    wide = [(g, max(0, a - int(rng.integers(0, 30))), min(len(seqs[g]) - 1, b + int(rng.integers(0, 30))), o, None)
            for g, a, b, o, _ in where]
    blocks = [wide, wide[:3], wide[10:75]]
    eng = _engine(seqs, names, blocks).apply("MetaAligner")
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(blocks)
    o.apply("MetaAligner")
    got = eng.blocks()
    assert got == o.blocks()
    assert max(len(b) for b in got) == 80 and any("-" in (f[4] or "") for b in got for f in b)
    eng = _engine(seqs, names, blocks).apply("Align")
    o.set_blocks(blocks)
    o.apply("Align")
    assert canon(eng.blocks()) == canon(o.blocks())
