"""Block build parity: the engine's processors (GPU aligner + host bookkeeping,
through the C ABI) vs the CPU restatement, block for block, fragment
coordinates AND gapped rows bit-exact.

Covers FragmentsExtender, FixEnds, ExtendLoopFast (MoveUnchanged,
OverlaplessUnion, Pipe convergence), Filter, DummyAligner, RemoveNonStem and the
whole DraftPangenome on seeded synthetic genome sets, plus the reference's
filter/1 and fix_ends/1 fixtures.
"""
import os

import pytest

from oracle import oracle as orc
from npge_amd import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def canon(blocks):
    return sorted(tuple(sorted(b)) for b in blocks)


def _engine(seqs, names, **kw):
    from npge_amd import _capi
    from npge_amd.blockset import BlockSetEngine
    ss = _capi.SeqSet(seqs, names)
    return ss, BlockSetEngine(ss, **kw)


def _stem_blocks(seqs, names):
    o = orc.BlockSetOracle(seqs, names)
    af = orc.AnchorFinder()
    r = af.run(seqs, names)
    bs = r["block_start"]
    blocks = [[(int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i]), None)
               for i in range(bs[b], bs[b + 1])] for b in range(len(bs) - 1)]
    o.set_blocks(blocks)
    o.apply("RemoveNonStem").apply("DummyAligner")
    return o.blocks()


@pytest.mark.parametrize("cfg", ["tiny", "small"])
def test_processors_step_by_step(cfg):
    names, seqs = synth.genome_set(cfg)
    b0 = _stem_blocks(seqs, names)
    assert b0
    ss, eng = _engine(seqs, names)
    o = orc.BlockSetOracle(seqs, names)
    # FragmentsExtender --extend-length-portion 0.5 (ExtendAndFix)
    eng.set_blocks(b0).apply("FragmentsExtender")
    o.set_blocks(b0)
    o.apply("FragmentsExtender")
    b1 = o.blocks()
    assert eng.blocks() == b1
    # FixEnds
    eng.apply("FixEnds")
    o.apply("FixEnds")
    b2 = o.blocks()
    assert canon(eng.blocks()) == canon(b2)
    # a second extension on the fixed blocks (longer flanks, gapped rows)
    eng.set_blocks(b2).apply("FragmentsExtender")
    o.set_blocks(b2)
    o.apply("FragmentsExtender")
    assert eng.blocks() == o.blocks()
    # Filter on the extended blocks
    eng.apply("Filter")
    o.apply("Filter")
    assert canon(eng.blocks()) == canon(o.blocks())


@pytest.mark.parametrize("cfg,iters", [("tiny", 10), ("small", 3), ("small", 10)])
def test_extend_loop_fast(cfg, iters):
    names, seqs = synth.genome_set(cfg)
    b0 = _stem_blocks(seqs, names)
    ss, eng = _engine(seqs, names, max_iterations=iters)
    o = orc.BlockSetOracle(seqs, names, max_iterations=iters)
    eng.set_blocks(b0).apply("ExtendLoopFast")
    o.set_blocks(b0)
    o.apply("ExtendLoopFast")
    assert eng.stats()["iterations"] == o.stats()["iterations"]
    assert canon(eng.blocks()) == canon(o.blocks())
    assert eng.hash() == o.hash()


@pytest.mark.parametrize("cfg", ["tiny", "small"])
def test_draft_pangenome(cfg):
    from npge_amd.anchor_finder import AnchorFinder
    names, seqs = synth.genome_set(cfg)
    ss, eng = _engine(seqs, names)
    eng.apply("DraftPangenome", af=AnchorFinder())
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    st, ost = eng.stats(), o.stats()
    assert st["anchor_blocks"] == ost["anchor_blocks"]
    assert st["stem_blocks"] == ost["stem_blocks"]
    assert st["iterations"] == ost["iterations"]
    assert st["aligned_residues"] == ost["aligned_residues"]
    assert canon(eng.blocks()) == canon(o.blocks())


def test_filter_and_fix_ends_fixture():
    from npge_amd import io as nio
    bs = nio.read_blockset(open(os.path.join(GOLD, "filter", "1", "in.fasta")).read())
    exp = nio.read_blockset(open(os.path.join(GOLD, "filter", "1", "out.fasta")).read())
    names = sorted({f.seq.name for b in bs.blocks for f in b.fragments})
    texts = {f.seq.name: f.row for b in bs.blocks for f in b.fragments}
    seqs = [texts[n] for n in names]
    blocks = [[(names.index(f.seq.name), f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments]
              for b in bs.blocks]
    want = sorted((f.id(), f.row) for b in exp.blocks for f in b.fragments)
    for proc, kw in (("Filter", dict(min_identity_x1e4=10000)), ("FixEnds", {})):
        ss, eng = _engine(seqs, names, **kw)
        eng.set_blocks(blocks).apply(proc)
        got = sorted(("%s_%d_%d" % (names[s], mn, mx), row) for b in eng.blocks()
                     for s, mn, mx, ori, row in b)
        assert got == want, proc


@pytest.mark.parametrize("case,opts", [("stem", ""), ("stem-exact", " --exact")])
def test_remove_non_stem_fixture(case, opts):
    """test-script/stem/1 and stem-exact/1 (RemoveNonStem, RemoveNonStem
    --exact): the fixtures hold fragments only; the sequences a&1&c, b&1&c,
    c&1&c (genomes a, b, c) are synthesised long enough for them."""
    from npge_amd.io import read_blockset
    d = os.path.join(GOLD, case, "1")
    src = read_blockset(open(os.path.join(d, "in.fasta")).read())
    exp = read_blockset(open(os.path.join(d, "out.fasta")).read())
    names = ["a&1&c", "b&1&c", "c&1&c"]
    seqs = ["A" * 40] * 3
    idx = {n: i for i, n in enumerate(names)}
    blocks = [[(idx[f.seq.name], f.min_pos, f.max_pos, f.ori, None) for f in b.fragments] for b in src.blocks]
    ss, eng = _engine(seqs, names)
    eng.set_blocks(blocks).apply("RemoveNonStem" + opts)
    got = canon([[(s, mn, mx, o) for (s, mn, mx, o, _) in b] for b in eng.blocks()])
    want = canon([[(idx[f.seq.name], f.min_pos, f.max_pos, f.ori) for f in b.fragments] for b in exp.blocks])
    assert got == want


@pytest.mark.parametrize("cfg", ["tiny", "small"])
def test_meta_aligner(cfg):
    """MetaAligner (align_block with the similar aligner + refine_alignment)
    on unaligned blocks of unequal fragments: the anchors widened by random
    amounts per fragment, single fragments, and already aligned blocks (left
    as they are)."""
    import numpy as np
    names, seqs = synth.genome_set(cfg)
    b0 = _stem_blocks(seqs, names)
    rng = np.random.default_rng(3)
    blocks = []
    for b in b0[:400]:
        nb = []
        for s, mn, mx, ori, _ in b:
            a = int(rng.integers(0, 40))
            z = int(rng.integers(0, 40))
            nb.append((s, max(0, mn - a), min(len(seqs[s]) - 1, mx + z), ori, None))
        blocks.append(nb)
    blocks += [[b[0][:4] + (None,)] for b in b0[400:420]]  # single fragments
    blocks += b0[420:440]                                   # aligned already
    ss, eng = _engine(seqs, names)
    o = orc.BlockSetOracle(seqs, names)
    eng.set_blocks(blocks).apply("MetaAligner")
    o.set_blocks(blocks)
    o.apply("MetaAligner")
    got = eng.blocks()
    assert got == o.blocks()
    assert any("-" in (f[4] or "") for b in got for f in b)


def _ou_blocks(rng, n_seqs, seq_len, n_blocks, max_len, self_overlap=False):
    blocks = []
    for _ in range(n_blocks):
        k = int(rng.integers(1, min(n_seqs, 6) + 1))
        frs = []
        for s in rng.choice(n_seqs, size=k, replace=False):
            mn = int(rng.integers(0, seq_len - max_len))
            frs.append((int(s), mn, mn + int(rng.integers(0, max_len)), int(rng.choice([-1, 1])), None))
        blocks.append(frs)
    if self_overlap is True:  # a block overlapping itself: the ordered multiset mode
        s, mn, mx, ori, _ = blocks[7][0]
        blocks[7].append((s, mn, mx + 5, -ori, None))
    elif self_overlap:  # that many, spread over the order, some reaching far (free ones included)
        for i in rng.choice(n_blocks, size=self_overlap, replace=False):
            s, mn, mx, ori, _ = blocks[i][0]
            ext = int(rng.integers(0, 2000)) if i % 3 == 0 else int(rng.integers(0, 10))
            a = max(0, mn - int(rng.integers(0, 5)))
            blocks[i].append((s, a, min(seq_len - 1, mx + ext), -ori, None))
    return blocks


def test_overlapless_union_many_sequences():
    """OverlaplessUnion over a consensus-like set: 5000 sequences, about one
    fragment each plus overlapping clusters and self-overlapping blocks
    (free_blocks' bucket-by-sequence path), against the oracle."""
    import numpy as np
    rng = np.random.default_rng(11)
    n_seqs, seq_len = 5000, 1200
    seqs = ["".join(rng.choice(list("ACGT"), size=seq_len)) for _ in range(n_seqs)]
    names = ["c%d&c&c" % i for i in range(n_seqs)]
    blocks = _ou_blocks(rng, n_seqs, seq_len, 2500, 600, 40)
    hot = [int(x) for x in rng.choice(n_seqs, size=20, replace=False)]  # clusters on a few sequences
    for _ in range(300):
        s = hot[int(rng.integers(0, len(hot)))]
        mn = int(rng.integers(0, seq_len - 200))
        blocks.append([(s, mn, mn + int(rng.integers(10, 200)), 1, None),
                       (int(rng.integers(0, n_seqs)), 5, 50, -1, None)])
    ss, eng = _engine(seqs, names)
    o = orc.BlockSetOracle(seqs, names)
    eng.set_blocks(blocks).apply("OverlaplessUnion")
    o.set_blocks(blocks)
    o.apply("OverlaplessUnion")
    want = o.blocks()
    assert eng.blocks() == want
    assert 0 < len(want) < len(blocks)


@pytest.mark.parametrize("max_len,self_overlap", [(40, False), (400, False), (3000, False), (40, True),
                                                  (40, 60), (400, 60), (3000, 60)])
def test_overlapless_union_many_blocks(max_len, self_overlap):
    """OverlaplessUnion --ou-move over 1500 blocks: sparse (most blocks in
    conflict with no other: admitted by free_blocks without the sequential
    test), dense (most rejected), long fragments past the interval-map
    threshold, one or 60 self-overlapping blocks (the ordered multiset mode,
    switched on by free and by conflicting blocks); then a second call on the
    same engine (only the touched bitmap ranges cleared in between)."""
    import numpy as np
    rng = np.random.default_rng(max_len + self_overlap)
    n_seqs, seq_len = 8, 400000
    seqs = ["".join(rng.choice(list("ACGT"), size=seq_len)) for _ in range(n_seqs)]
    names = ["g%d&c&c" % i for i in range(n_seqs)]
    blocks = _ou_blocks(rng, n_seqs, seq_len, 1500, max_len, self_overlap)
    ss, eng = _engine(seqs, names)
    o = orc.BlockSetOracle(seqs, names)
    for rnd in range(2):
        eng.set_blocks(blocks).apply("OverlaplessUnion")
        o.set_blocks(blocks)
        o.apply("OverlaplessUnion")
        want = o.blocks()
        assert eng.blocks() == want, rnd
        assert 0 < len(want) <= len(blocks)
