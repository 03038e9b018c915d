"""Pins the oracle's ConSeq / DeConSeq restatement (ConSeq.cpp:37-50,
DeConSeq.cpp:27-96, Block::consensus Block.cpp:147-185, Block::slice
Block.cpp:238-289) to the reference's own unit tests: src/test/conseq.cpp
(ConSeq_main, ConSeq_alignment, DeConSeq_alignment) and the consensus cases of
src/test/block.cpp (Block_length2, Block_consensus).  CPU only."""
from oracle import oracle as orc

# CompactSequence drops '-' (to_atgcn, Sequence.cpp:151-179)
S1, S2, S3 = "-CAGGCCGG", "-CAGGCTG-", "GCTGGATG-"


def _near(a, b):
    return abs(a - b) <= 1


def _source(rows=None, f3_min=1):
    o = orc.BlockSetOracle([S1, S2, S3], ["s1", "s2", "s3"])
    f = [(0, 0, 7, 1), (1, 0, 6, 1), (2, f3_min, 7, 1)]
    o.set_blocks([[x + ((rows[i] if rows else None),) for i, x in enumerate(f)]])
    return o


def test_conseq_main():
    """conseq.cpp:24-72: unaligned block -> the longest fragment; DeConSeq of
    two unaligned consensus fragments -> one block of 6 fragments at about the
    same places (proportional slicing, convert_position.cpp:44-67)."""
    src = _source()
    assert src.conseq() == ["CAGGCCGG"]
    cons = orc.BlockSetOracle(["CAGGCCGG"], ["block1"])
    cons.set_blocks([[(0, 0, 2, 1, None), (0, 4, 6, -1, None)]])
    tgt = orc.BlockSetOracle([S1, S2, S3], ["s1", "s2", "s3"])
    tgt.deconseq(cons, source=src)
    blocks = tgt.blocks()
    assert len(blocks) == 1 and len(blocks[0]) == 6
    for seq, mn, mx, ori, row in blocks[0]:
        assert row is None
        if seq == 2:
            mn, mx = mn - 1, mx - 1
        assert ((_near(mn, 0) and _near(mx, 2) and ori == 1) or (_near(mn, 4) and _near(mx, 6) and ori == -1))
    # Block::consensus of the unaligned slice: its first longest fragment = "CAG"
    assert max(mx - mn + 1 for _, mn, mx, _, _ in blocks[0]) == 3
    assert tgt.conseq() == ["CAG"]


def test_conseq_alignment():
    """conseq.cpp:74-121: aligned block -> column consensus; unaligned
    consensus fragments map exactly through the rows."""
    src = _source(rows=["CAGGCCGG", "CAGGCTG-", "CTGGATG-"])
    assert src.conseq() == ["CAGGCTGG"]
    cons = orc.BlockSetOracle(["CAGGCTGG"], ["c"])
    cons.set_blocks([[(0, 0, 2, 1, None), (0, 4, 6, -1, None)]])
    tgt = orc.BlockSetOracle([S1, S2, S3], ["s1", "s2", "s3"])
    tgt.deconseq(cons, source=src)
    (blk,) = tgt.blocks()
    for seq, mn, mx, ori, row in blk:
        if seq == 2:
            mn, mx = mn - 1, mx - 1
        assert (mn, mx, ori) in ((0, 2, 1), (4, 6, -1))


def test_deconseq_alignment():
    """conseq.cpp:123-178: a block and a single-fragment block -> consensus
    sequences; an aligned block over both consensuses -> one block of four
    fragments with the composed rows."""
    s4 = "GCAGAGCCGG"
    src = orc.BlockSetOracle([S1, S2, S3, s4], ["s1", "s2", "s3", "s4"])
    src.set_blocks([
        [(0, 0, 7, 1, "-CAGGCCGG"), (1, 0, 6, 1, "-CAGGCTG-"), (2, 0, 7, 1, "GCTGGATG-")],
        [(3, 0, 9, 1, s4)],
    ])
    cs = src.conseq()
    assert cs == ["GCAGGCTGG", "GCAGAGCCGG"]
    cons = orc.BlockSetOracle(cs, ["b", "ba"])
    cons.set_blocks([[(0, 0, 8, 1, "GCAG-GCTGG"), (1, 0, 9, 1, "GCAGAGCCGG")]])
    tgt = orc.BlockSetOracle([S1, S2, S3, s4], ["s1", "s2", "s3", "s4"])
    tgt.deconseq(cons, source=src)
    (blk,) = tgt.blocks()
    assert len(blk) == 4
    assert sorted(r for *_, r in blk) == ["-CAG-GCCGG", "-CAG-GCTG-", "GCAGAGCCGG", "GCTG-GATG-"]


def test_block_consensus_kats():
    """block.cpp:73-87 (unaligned: the longest fragment) and block.cpp:490-512
    (aligned; ties go to the first letter in A T G C N order; a column without
    letters gives 'A')."""
    o = orc.BlockSetOracle(["CAGGACGG", "CAGGAAG-", "CTGGACG-"], ["a", "b", "c"])
    o.set_blocks([[(0, 0, 7, 1, None), (1, 0, 6, 1, None), (2, 0, 6, 1, None)]])
    assert o.conseq() == ["CAGGACGG"]
    o = orc.BlockSetOracle(["TAGTCCG-", "TGTT-CG-", "TG---CG-"], ["a", "b", "c"])
    o.set_blocks([[(0, 0, 6, 1, "TAGTCCG-"), (1, 0, 5, 1, "TGTT-CG-"), (2, 0, 3, 1, "TG---CG-")]])
    assert o.conseq()[0] in ("TGGTCCGA", "TGTTCCGA")
    assert o.conseq() == ["TGTTCCGA"]


def test_deconseq_reverse_and_single_letter():
    """Slicing at an inverted consensus fragment reverses the source rows and
    complements them; a one-letter piece of an ori -1 fragment becomes ori +1
    (Fragment::set_begin_last, Fragment.cpp:117-127)."""
    src = orc.BlockSetOracle(["AACCGGTT", "AACGGTT"], ["x", "y"])
    # y read backwards: complement of "AACGGTT" reversed = "AACCGTT"
    src.set_blocks([[(0, 0, 7, 1, "AACCGGTT"), (1, 0, 6, -1, "AACC-GTT")]])
    (c,) = src.conseq()
    assert c == "AACCGGTT"
    cons = orc.BlockSetOracle([c], ["c"])
    cons.set_blocks([[(0, 3, 5, -1, "CCG"), (0, 4, 4, 1, "G")]])
    tgt = orc.BlockSetOracle(["AACCGGTT", "AACGGTT"], ["x", "y"])
    tgt.deconseq(cons, source=src)
    (blk,) = tgt.blocks()
    # columns 5, 4, 3 of the source rows: x "GGC" -> complement "CCG"; y "G-C"
    # -> "C-G"; then column 4 alone: x 'G' (ori +1), y gap -> dropped
    assert blk == [(0, 3, 5, -1, "CCG"), (1, 2, 3, 1, "C-G"), (0, 4, 4, 1, "G")]
