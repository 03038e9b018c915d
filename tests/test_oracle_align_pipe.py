"""Pins the oracle's Align-pipe processors (MoveGaps, CutGaps,
SelfOverlapsResolver; Align.cpp:36-52) to the reference's own tests:
test-script/cut_gaps/{1,2,to_empty} and cut_gaps_strict/{1,to_empty,to_empty2}
(in.fasta -> CutGaps --cut-strict=0/1 -> out.fasta, compared by fragment ids
and rows, like meta_test.cxx's blockset hash plus the rows), src/test/cut_gaps.cpp,
src/test/move_gaps.cpp and src/test/hit.cpp."""
import os

import pytest

from oracle import oracle as orc
from npge_amd import io as nio
from npge_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load_fixture(text, **params):
    """(oracle, sequence names, blocks) of a .bs text holding sequences and blocks."""
    bs = nio.read_blockset(text)
    names = [s.name for s in bs.seqs]
    o = orc.BlockSetOracle([s.data for s in bs.seqs], names, **params)
    blocks = [[(names.index(f.seq.name), f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments]
              for b in bs.blocks]
    o.set_blocks(blocks)
    return o, names, blocks


def frag_records(blocks, names):
    """{fragment id: row} over the non-empty blocks (Fragment::id, Fragment.cpp:173-183)."""
    out = {}
    for b in blocks:
        for s, mn, mx, ori, row in b:
            a, z = (mn, mx) if ori == 1 else (mx, mn)
            if mn == mx and ori == -1:
                z = -1
            out["%s_%d_%d" % (names[s], a, z)] = row
    return out


def expected_records(text):
    return {f.id(): f.row for b in nio.read_blockset(text).blocks for f in b.fragments}


CUT_CASES = [("cut_gaps", c) for c in ("1", "2", "to_empty")] + \
            [("cut_gaps_strict", c) for c in ("1", "to_empty", "to_empty2")]


@pytest.mark.parametrize("script,case", CUT_CASES)
def test_cut_gaps_fixture(script, case):
    # script.npge: run_main('Read'); run('CutGaps', '--cut-strict=0|1'); run_main('RawWrite')
    d = os.path.join(GOLD, script, case)
    o, names, _ = load_fixture(open(os.path.join(d, "in.fasta")).read())
    o.apply("CutGapsStrict" if script == "cut_gaps_strict" else "CutGaps")
    got = frag_records(o.blocks(), names)
    assert got == expected_records(open(os.path.join(d, "out.fasta")).read())


CUT_GAPS_INPUT = """>a_0_10 block=a
AAAA---AAAA---AAA
>a_0_4 block=a
------AAAAA------
>a_0_6 block=a
-----AAAAAAA-----
>a_0_8 block=a
AAA----AAAAAA----
"""

CUT_GAPS_OUTPUT = """>a_0_4 block=a
AAAAA
>a_1_5 block=a
AAAAA
>a_3_6 block=a
-AAAA
>a_4_7 block=a
-AAAA
"""


def test_cut_gaps_kat():
    """src/test/cut_gaps.cpp:37-51 (sequence A = 18 x 'A')."""
    o, names, _ = load_fixture(">a\n" + "A" * 18 + "\n" + CUT_GAPS_INPUT)
    o.apply("CutGaps")
    blocks = o.blocks()
    assert len(blocks) == 1
    assert frag_records(blocks, names) == expected_records(CUT_GAPS_OUTPUT)


MOVE_GAPS_INPUT = """>a_0_4 block=a
A------AAAA------
>a_0_6 block=a
AA-----AAAA-----A
>a_0_8 block=a
AAA----AAAA----AA
>a_0_10 block=a
AAAA---AAAA---AAA
>a_0_3 block=a
AAAA-------------
"""

MOVE_GAPS_OUTPUT = """>a_0_10 block=a
AAAA---AAAA---AAA
>a_0_3 block=a
AAAA-------------
>a_0_4 block=a
------AAAAA------
>a_0_6 block=a
-----AAAAAAA-----
>a_0_8 block=a
AAA----AAAAAA----
"""


def test_move_gaps_kat():
    """src/test/move_gaps.cpp:42-59: max-tail 3, max-tail-to-gap 0.5."""
    o, names, _ = load_fixture(">a\n" + "A" * 18 + "\n" + MOVE_GAPS_INPUT, max_tail=3,
                               max_tail_to_gap_x1e4=5000)
    o.apply("MoveGaps")
    assert frag_records(o.blocks(), names) == expected_records(MOVE_GAPS_OUTPUT)


def test_move_gaps_default_ratio():
    """With the default max-tail-to-gap 1.0 (MAX_TAIL_TO_GAP) a 3-letter end
    tail behind a 3-column gap moves inside (3 / 3 <= 1; at 0.5 it stays, as
    in move_gaps.cpp); the 4-letter head is longer than max-tail 3."""
    rows = ">a_0_10 block=a\nAAAA---AAAA---AAA\n>a_0_10 block=b\nAAAAAAAAAAA------\n"
    o, names, _ = load_fixture(">a\n" + "A" * 18 + "\n" + rows)
    o.apply("MoveGaps")
    got = sorted(f[4] for b in o.blocks() for f in b)
    assert got == sorted(["AAAAAAAAAAA------", "AAAA---AAAAAAA---"])


def _seq_block(seq, frags):
    o = orc.BlockSetOracle([seq], ["s1"])
    o.set_blocks([[(0, a, b, ori, None) for a, b, ori in frags]])
    return o


def test_self_overlaps_kats():
    """src/test/hit.cpp:16-61."""
    s = "TGGTCCGAGCGGACGGCC"
    o = _seq_block(s, [(0, 5, 1), (5, 10, 1)]).apply("SelfOverlapsResolver")
    (b,) = o.blocks()
    assert max(mx - mn + 1 for _, mn, mx, _, _ in b) == 5  # alignment_length 6 -> 5
    o = _seq_block(s, [(0, 5, 1), (0, 5, 1)]).apply("SelfOverlapsResolver")
    assert o.blocks() == [[]]
    o = _seq_block(s, [(0, 5, 1), (0, 5, -1)]).apply("SelfOverlapsResolver")
    (b,) = o.blocks()
    assert sorted(b) == [(0, 0, 2, 1, None), (0, 3, 5, -1, None)]  # [0, 1, 2], [5, 4, 3]


def test_self_overlaps_untouched():
    """A block without self-overlaps keeps its fragments and rows."""
    o = _seq_block("ACGTACGTAC", [(0, 3, 1), (5, 8, 1)])
    before = o.blocks()
    assert o.apply("SelfOverlapsResolver").blocks() == before


@pytest.mark.parametrize("cfg", ["tiny"])
def test_align_pipe_runs(cfg):
    """Align on a DraftPangenome result with its rows dropped: every block
    comes back aligned and passes Filter (the pipe's last processor), and a
    second Align changes nothing."""
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    start = [[f[:4] + (None,) for f in b] for b in o.blocks()]
    o.set_blocks(start)
    o.apply("Align")
    got = o.blocks()
    assert got and all(f[4] is not None for b in got for f in b)
    assert all(len(b) >= 2 for b in got)
    assert o.apply("Align").blocks() == got
