"""Pins the oracle's block-set processors to the reference's own tests:
test-script/filter/1 and test-script/fix_ends/1 (same fixture,
fix_ends/1 -> ../filter/1) and src/test/filter.cpp."""
import os

import pytest

from oracle import oracle as orc
from npge_amd import io as nio

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _from_bs(path):
    bs = nio.read_blockset(open(path).read())
    return bs


def _oracle_for_fixture(path, **params):
    """Sequences are implied by the fragment records (Read of a .bs holding only
    blocks); rows are the records' texts."""
    bs = _from_bs(path)
    seqs = {}
    for b in bs.blocks:
        for f in b.fragments:
            text = f.row.replace("-", "") if f.row else ""
            if f.ori == 1:
                seqs[f.seq.name] = (f.min_pos, text)
    names = sorted(seqs)
    data = [seqs[n][1] for n in names]
    o = orc.BlockSetOracle(data, names, **params)
    blocks = [[(names.index(f.seq.name), f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments]
              for b in bs.blocks]
    o.set_blocks(blocks)
    return o, names


def _ids(blocks, names):
    out = set()
    for b in blocks:
        out.add(tuple(sorted("%s_%d_%d" % (names[s], mn if ori == 1 else mx, mx if ori == 1 else mn)
                             for s, mn, mx, ori, _ in b)))
    return out


def test_filter_fixture():
    # run('Filter', '--find-subblocks=1 --min-identity=1')
    o, names = _oracle_for_fixture(os.path.join(GOLD, "filter", "1", "in.fasta"),
                                   filter_min_identity_x1e4=10000)
    o.apply("Filter")
    exp = _from_bs(os.path.join(GOLD, "filter", "1", "out.fasta"))
    got = o.blocks()
    assert _ids(got, names) == {tuple(sorted(f.id() for f in b.fragments)) for b in exp.blocks}
    exp_rows = sorted(f.row for b in exp.blocks for f in b.fragments)
    assert sorted(f[4] for b in got for f in b) == exp_rows


def test_fix_ends_fixture():
    # run('FixEnds') on the same fixture
    o, names = _oracle_for_fixture(os.path.join(GOLD, "filter", "1", "in.fasta"))
    o.apply("FixEnds")
    exp = _from_bs(os.path.join(GOLD, "filter", "1", "out.fasta"))
    assert _ids(o.blocks(), names) == {tuple(sorted(f.id() for f in b.fragments)) for b in exp.blocks}


def _unit_block(rows, **params):
    seqs = [nio.to_atgcn(r) for r in rows]
    names = ["s%d" % i for i in range(len(rows))]
    p = dict(filter_min_fragment=0, filter_min_block=0, filter_max_block=-1,
             filter_min_identity_x1e4=0)
    p.update(params)
    o = orc.BlockSetOracle(seqs, names, **p)
    o.set_blocks([[(i, 0, len(s) - 1, 1, r) for i, (s, r) in enumerate(zip(seqs, rows))]])
    return o


def test_filter_good_blocks():
    o = _unit_block(["TAGTCCG-", "TGTT-CGT", "TG---CG-"], filter_min_fragment=2,
                    filter_frame_length=2, filter_min_block=2, filter_min_identity_x1e4=9900,
                    filter_min_end=1)
    o.apply("FindGoodSubblocks")
    gb = o.blocks()
    assert len(gb) == 1
    assert len(gb[0]) == 3 and len(gb[0][0][4]) == 2 and gb[0][0][4] == "CG"


def test_filter_good_blocks_min_end3():
    o = _unit_block(["TAGTCCG-", "TGTT-CGT", "TG---CG-"], filter_min_fragment=2,
                    filter_frame_length=2, filter_min_block=2, filter_min_identity_x1e4=9900,
                    filter_min_end=3)
    o.apply("FindGoodSubblocks")
    assert len(o.blocks()) == 0


def test_filter_good_blocks3():
    o = _unit_block(["TATTCCG-", "TGTTACGT", "TGT--CG-"], filter_min_fragment=1,
                    filter_frame_length=1, filter_min_block=2, filter_min_identity_x1e4=9900,
                    filter_min_end=1)
    o.apply("FindGoodSubblocks")
    assert len(o.blocks()) == 3


def test_filter_good_blocks4():
    o = _unit_block(["TTTTTTTTTT", "T-TTT----T"], filter_min_fragment=3, filter_frame_length=3,
                    filter_min_block=2, filter_min_identity_x1e4=6000, filter_min_end=1)
    o.apply("FindGoodSubblocks")
    assert len(o.blocks()) >= 1


def test_filter_good_blocks_expand():
    o = _unit_block(["TGTTCCG", "TATTCC-", "-ATTCCG"], filter_min_fragment=1,
                    filter_frame_length=1, filter_min_block=2, filter_min_identity_x1e4=9900,
                    filter_min_end=1)
    o.apply("FindGoodSubblocks")
    gb = o.blocks()
    assert len(gb) == 1
    assert len(gb[0]) == 3 and len(gb[0][0][4]) == 4 and gb[0][0][4] == "TTCC"


def test_filter_good_block_sizes():
    # Filter_good_block: two 1-letter fragments; min-fragment 100 -> bad, 1 -> good
    o = _unit_block(["A", "A"], filter_min_fragment=100, filter_frame_length=100,
                    filter_min_block=2)
    o.apply("Filter")
    assert len(o.blocks()) == 0
    o = _unit_block(["A", "A"], filter_min_fragment=1, filter_frame_length=1, filter_min_block=2)
    o.apply("Filter")
    assert len(o.blocks()) == 1


@pytest.mark.parametrize("cfg", ["tiny"])
def test_draft_pangenome_runs(cfg):
    from npge_amd import synth
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    st = o.stats()
    assert st["anchor_blocks"] > 0 and st["n_blocks"] > 0
    for b in o.blocks():
        L = len(b[0][4])
        for s, mn, mx, ori, row in b:
            assert len(row) == L
            text = seqs[s][mn:mx + 1]
            if ori == -1:
                text = text[::-1].translate(str.maketrans("ATGC", "TACG"))
            assert row.replace("-", "") == text


def test_oracle_workers_identical():
    """The threaded oracle (FragmentTG per sequence in AnchorFinder pass 2,
    BlocksJobs per block, BlocksJobs.cpp:38-240) gives the same blocks as the
    1-worker run: bench.py's cpu_baseline "allotted_cores" leg times the same work."""
    from npge_amd import synth
    names, seqs = synth.genome_set("tiny")
    ref = orc.BlockSetOracle(seqs, names).apply("DraftPangenome")
    for w in (2, 5):
        o = orc.BlockSetOracle(seqs, names).set_workers(w).apply("DraftPangenome")
        assert o.hash() == ref.hash()
        assert o.blocks() == ref.blocks()
        assert o.stats() == ref.stats()
