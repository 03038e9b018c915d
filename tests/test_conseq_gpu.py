"""ConSeq / DeConSeq on the engine (npgx_blockset_conseq: consensus kernel on
the GPU; npgx_blockset_deconseq) vs the CPU restatement: the reference's
conseq.cpp / block.cpp cases, then seeded synthetic sets (DraftPangenome
blocks -> consensus sequences -> blocks over the consensuses, unaligned and
aligned -> mapped back), fragments and rows bit-exact."""
import numpy as np
import pytest

from oracle import oracle as orc
from npge_amd import synth

pytestmark = pytest.mark.gpu

S1, S2, S3 = "-CAGGCCGG", "-CAGGCTG-", "GCTGGATG-"


def _engine(seqs, names, blocks=None):
    from npge_amd import _capi
    from npge_amd.blockset import BlockSetEngine
    ss = _capi.SeqSet(seqs, names)
    eng = BlockSetEngine(ss)
    if blocks is not None:
        eng.set_blocks(blocks)
    return eng


def _pair(seqs, names, blocks):
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(blocks)
    return _engine(seqs, names, blocks), o


def test_conseq_kats():
    """conseq.cpp:24-178 and block.cpp:73-87,490-512 through the C ABI."""
    cases = [
        ([S1, S2, S3], [[(0, 0, 7, 1, None), (1, 0, 6, 1, None), (2, 1, 7, 1, None)]], ["CAGGCCGG"]),
        ([S1, S2, S3], [[(0, 0, 7, 1, "CAGGCCGG"), (1, 0, 6, 1, "CAGGCTG-"), (2, 1, 7, 1, "CTGGATG-")]],
         ["CAGGCTGG"]),
        ([S1, S2, S3, "GCAGAGCCGG"],
         [[(0, 0, 7, 1, "-CAGGCCGG"), (1, 0, 6, 1, "-CAGGCTG-"), (2, 0, 7, 1, "GCTGGATG-")],
          [(3, 0, 9, 1, "GCAGAGCCGG")]], ["GCAGGCTGG", "GCAGAGCCGG"]),
        (["TAGTCCG-", "TGTT-CG-", "TG---CG-"],
         [[(0, 0, 6, 1, "TAGTCCG-"), (1, 0, 5, 1, "TGTT-CG-"), (2, 0, 3, 1, "TG---CG-")]], ["TGTTCCGA"]),
    ]
    for seqs, blocks, want in cases:
        names = ["s%d" % i for i in range(len(seqs))]
        eng, o = _pair(seqs, names, blocks)
        assert eng.conseq() == want == o.conseq()


def test_deconseq_kat_alignment():
    """conseq.cpp:123-178 DeConSeq_alignment: composed rows."""
    s4 = "GCAGAGCCGG"
    seqs, names = [S1, S2, S3, s4], ["s1", "s2", "s3", "s4"]
    src = _engine(seqs, names, [[(0, 0, 7, 1, "-CAGGCCGG"), (1, 0, 6, 1, "-CAGGCTG-"),
                                 (2, 0, 7, 1, "GCTGGATG-")], [(3, 0, 9, 1, s4)]])
    cs = src.conseq()
    cons = _engine(cs, ["b", "ba"], [[(0, 0, 8, 1, "GCAG-GCTGG"), (1, 0, 9, 1, "GCAGAGCCGG")]])
    tgt = _engine(seqs, names, [])
    tgt.deconseq(cons, source=src)
    (blk,) = tgt.blocks()
    assert sorted(r for *_, r in blk) == ["-CAG-GCCGG", "-CAG-GCTG-", "GCAGAGCCGG", "GCTG-GATG-"]
    # into the source itself (AnchorLoopFast: DeConSeq target=target): appended
    src.deconseq(cons)
    assert len(src.blocks()) == 3 and src.blocks()[2] == blk


def test_deconseq_keeps_empty_blocks():
    """DeConSeq inserts every new block, empty ones included
    (DeConSeq.cpp:86-99): an empty consensus block maps to an empty block in
    its place; engine and oracle agree."""
    seqs, names = [S1, S2], ["a", "b"]
    src_blocks = [[(0, 0, 7, 1, None), (1, 0, 6, 1, None)]]
    src = _engine(seqs, names, src_blocks)
    cs = src.conseq()
    cons_blocks = [[(0, 0, 3, 1, None)], [], [(0, 2, 5, -1, None), (0, 0, 1, 1, None)]]
    cons = _engine(cs, ["c"], cons_blocks)
    tgt = _engine(seqs, names, [])
    tgt.deconseq(cons, source=src)
    got = tgt.blocks()
    assert len(got) == 3 and got[1] == []
    o_src = orc.BlockSetOracle(seqs, names)
    o_src.set_blocks(src_blocks)
    o_cons = orc.BlockSetOracle(cs, ["c"])
    o_cons.set_blocks(cons_blocks)
    o_tgt = orc.BlockSetOracle(seqs, names)
    o_tgt.deconseq(o_cons, source=o_src)
    assert got == o_tgt.blocks()


def test_deconseq_mismatch_is_an_error():
    from npge_amd import _capi
    src = _engine([S1, S2], ["a", "b"], [[(0, 0, 7, 1, None), (1, 0, 6, 1, None)]])
    cons = _engine(["CAGGCCGGA"], ["c"], [[(0, 0, 2, 1, None)]])  # length differs from the block
    with pytest.raises(_capi.NpgxError):
        _engine([S1, S2], ["a", "b"], []).deconseq(cons, source=src)


def _random_cons_blocks(rng, cs, n_blocks):
    out = []
    for _ in range(n_blocks):
        k = int(rng.integers(2, 4))
        blk = []
        for _ in range(k):
            s = int(rng.integers(len(cs)))
            L = len(cs[s])
            ln = int(rng.integers(1, min(L, 160) + 1))
            a = int(rng.integers(0, L - ln + 1))
            blk.append((s, a, a + ln - 1, int(rng.choice([1, -1])), None))
        out.append(blk)
    return out


@pytest.mark.parametrize("cfg", ["tiny", "small"])
def test_conseq_deconseq_synthetic(cfg):
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    src_blocks = o.blocks()
    # plus some unaligned and single-fragment blocks
    src_blocks = src_blocks + [[b[0][:4] + (None,)] for b in src_blocks[:5]] + \
        [[f[:4] + (None,) for f in b] for b in src_blocks[5:10]]
    assert len(src_blocks) >= 15
    src, osrc = _pair(seqs, names, src_blocks)
    cs = src.conseq()
    assert cs == osrc.conseq()
    cnames = ["cons%05d" % i for i in range(len(cs))]
    rng = np.random.default_rng(7)
    cblocks = _random_cons_blocks(rng, cs, 60)
    # unaligned consensus blocks
    cons, ocons = _pair(cs, cnames, cblocks)
    tgt, otgt = _engine(seqs, names, []), orc.BlockSetOracle(seqs, names)
    tgt.deconseq(cons, source=src)
    otgt.deconseq(ocons, source=osrc)
    assert tgt.blocks() == otgt.blocks()
    # aligned consensus blocks (DummyAligner + FragmentsExtender: gapped rows)
    cons.apply("DummyAligner").apply("FragmentsExtender")
    ablocks = cons.blocks()
    assert any("-" in (f[4] or "") for b in ablocks for f in b)
    ocons.set_blocks(ablocks)
    tgt, otgt = _engine(seqs, names, []), orc.BlockSetOracle(seqs, names)
    tgt.deconseq(cons, source=src)
    otgt.deconseq(ocons, source=osrc)
    got = tgt.blocks()
    assert got == otgt.blocks()
    assert sum(len(b) for b in got) >= sum(len(b) for b in ablocks)


def test_processors_conseq_deconseq():
    """ConSeq / DeConSeq processors on the host model (AnchorLoopFast's
    ConSeq target=cons other=target ... DeConSeq target=target other=cons)."""
    import npge_amd.conseq  # noqa: F401  (registers the processors)
    from npge_amd.model import Block, BlockSet, Fragment, Sequence
    from npge_amd.processor import new_p
    ss = [Sequence("s1", "CAGGCCGG"), Sequence("s2", "CAGGCTG"), Sequence("s3", "GCTGGATG"),
          Sequence("s4", "GCAGAGCCGG")]
    b = Block([Fragment(ss[0], 0, 7, 1, "-CAGGCCGG"), Fragment(ss[1], 0, 6, 1, "-CAGGCTG-"),
               Fragment(ss[2], 0, 7, 1, "GCTGGATG-")], name="b")
    ba = Block([Fragment(ss[3], 0, 9, 1, "GCAGAGCCGG")], name="ba")
    target = BlockSet(seqs=list(ss), blocks=[b, ba])
    cons = BlockSet()
    p = new_p("ConSeq")
    p.set_bs("other", target)
    p.set_bs("target", cons)
    p.run()
    assert [(s.name, s.data) for s in cons.seqs] == [("b", "GCAGGCTGG"), ("ba", "GCAGAGCCGG")]
    assert cons.seqs[0].block is b
    cons.blocks.append(Block([Fragment(cons.seqs[0], 0, 8, 1, "GCAG-GCTGG"),
                              Fragment(cons.seqs[1], 0, 9, 1, "GCAGAGCCGG")], name="cb"))
    p = new_p("DeConSeq")
    p.set_bs("other", cons)
    p.set_bs("target", target)
    p.run()
    assert len(target.blocks) == 3
    nb = target.blocks[2]
    assert nb.name == "cb"
    assert sorted(f.row for f in nb.fragments) == ["-CAG-GCCGG", "-CAG-GCTG-", "GCAGAGCCGG", "GCTG-GATG-"]
    assert all(f.seq in ss for f in nb.fragments)
