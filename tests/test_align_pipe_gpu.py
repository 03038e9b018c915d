"""The reference's Align pipe on the engine (Align.cpp:36-52): MoveGaps,
CutGaps (permissive and strict), SelfOverlapsResolver, LiteAlign and Align,
fragments and rows bit-exact vs the oracle -- on the reference's own cases
(test-script/cut_gaps*, src/test/move_gaps.cpp, src/test/hit.cpp), on random
gapped blocks, and on DraftPangenome results."""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from npge_amd import io as nio
from npge_amd import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def canon(blocks):
    return sorted(tuple(sorted(b)) for b in blocks)


def _engine(seqs, names, blocks=None, **kw):
    from npge_amd import _capi
    from npge_amd.blockset import BlockSetEngine
    eng = BlockSetEngine(_capi.SeqSet(seqs, names), **kw)
    if blocks is not None:
        eng.set_blocks(blocks)
    return eng


def _both(seqs, names, blocks, eng_kw=None, orc_kw=None):
    eng = _engine(seqs, names, blocks, **(eng_kw or {}))
    o = orc.BlockSetOracle(seqs, names, **(orc_kw or {}))
    o.set_blocks(blocks)
    return eng, o


def _fixture(path):
    bs = nio.read_blockset(open(path).read())
    names = [s.name for s in bs.seqs]
    seqs = [s.data for s in bs.seqs]
    blocks = [[(names.index(f.seq.name), f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments]
              for b in bs.blocks]
    return seqs, names, blocks


def _records(blocks, names):
    out = {}
    for b in blocks:
        for s, mn, mx, ori, row in b:
            a, z = (mn, mx) if ori == 1 else (mx, mn)
            if mn == mx and ori == -1:
                z = -1
            out["%s_%d_%d" % (names[s], a, z)] = row
    return out


@pytest.mark.parametrize("script,case", [("cut_gaps", c) for c in ("1", "2", "to_empty")] +
                         [("cut_gaps_strict", c) for c in ("1", "to_empty", "to_empty2")])
def test_cut_gaps_fixture(script, case):
    d = os.path.join(GOLD, script, case)
    seqs, names, blocks = _fixture(os.path.join(d, "in.fasta"))
    strict = script == "cut_gaps_strict"
    eng, o = _both(seqs, names, blocks)
    eng.apply("CutGaps --cut-strict=%d" % strict)
    o.apply("CutGapsStrict" if strict else "CutGaps")
    assert eng.blocks() == o.blocks()
    exp = nio.read_blockset(open(os.path.join(d, "out.fasta")).read())
    assert _records(eng.blocks(), names) == {f.id(): f.row for b in exp.blocks for f in b.fragments}


def test_move_gaps_kat():
    """src/test/move_gaps.cpp:42-59 (max-tail 3, max-tail-to-gap 0.5)."""
    rows = ["A------AAAA------", "AA-----AAAA-----A", "AAA----AAAA----AA", "AAAA---AAAA---AAA",
            "AAAA-------------"]
    want = ["------AAAAA------", "-----AAAAAAA-----", "AAA----AAAAAA----", "AAAA---AAAA---AAA",
            "AAAA-------------"]
    seqs, names = ["A" * 18], ["a"]
    blocks = [[(0, 0, len(r.replace("-", "")) - 1, 1, r) for r in rows]]
    eng = _engine(seqs, names, blocks).apply("MoveGaps --max-tail=3 --max-tail-to-gap=0.5")
    assert [f[4] for f in eng.blocks()[0]] == want


def test_self_overlaps_kats():
    """src/test/hit.cpp:16-61."""
    s = "TGGTCCGAGCGGACGGCC"
    for frags in ([(0, 5, 1), (5, 10, 1)], [(0, 5, 1), (0, 5, 1)], [(0, 5, 1), (0, 5, -1)]):
        blocks = [[(0, a, b, ori, None) for a, b, ori in frags]]
        eng, o = _both([s], ["s1"], blocks)
        eng.apply("SelfOverlapsResolver")
        o.apply("SelfOverlapsResolver")
        assert eng.blocks() == o.blocks()


def _random_gapped_blocks(rng, seqs, n_blocks, max_len=300, max_rows=9, gap_rate=0.05, overlap=False):
    """Blocks of fragments with equal-length gapped rows whose letters are the
    fragments' texts: terminal tails, inner gaps, empty-ish rows, both
    orientations; `overlap`: some blocks hold two overlapping fragments of one
    sequence."""
    comp = {"A": "T", "T": "A", "G": "C", "C": "G", "N": "N"}
    blocks = []
    for _ in range(n_blocks):
        k = int(rng.integers(1, max_rows + 1))
        frs = []
        for _ in range(k):
            s = int(rng.integers(0, len(seqs)))
            n = int(rng.integers(1, max_len))
            mn = int(rng.integers(0, len(seqs[s]) - n))
            frs.append((s, mn, mn + n - 1, int(rng.choice([-1, 1]))))
        if overlap and k >= 1 and rng.random() < 0.5:
            s, mn, mx, ori = frs[0]
            a = int(rng.integers(mn, mx + 1))
            frs.append((s, a, min(len(seqs[s]) - 1, a + int(rng.integers(1, max_len))), -ori))
        texts = []
        for s, mn, mx, ori in frs:
            t = seqs[s][mn:mx + 1]
            texts.append(t if ori == 1 else "".join(comp[c] for c in reversed(t)))
        L = max(len(t) for t in texts) + int(rng.integers(0, 40))
        rows = []
        for t in texts:
            gaps = L - len(t)
            # terminal gaps and tails, inner gaps where the random draw says so
            where = sorted(rng.integers(0, len(t) + 1, size=gaps))
            if rng.random() < 0.3:  # a short tail cut off by a gap run
                tail = int(rng.integers(1, 5))
                where = sorted([min(len(t), tail)] * gaps)
            row, j = [], 0
            for p in range(len(t) + 1):
                while j < len(where) and where[j] == p:
                    row.append("-")
                    j += 1
                if p < len(t):
                    row.append(t[p])
            rows.append("".join(row))
        blocks.append([f + (r,) for f, r in zip(frs, rows)])
    return blocks


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("proc,oproc,opts,okw", [
    ("MoveGaps", "MoveGaps", "", {}),
    ("MoveGaps --max-tail=4 --max-tail-to-gap=0.25", "MoveGaps", None,
     dict(max_tail=4, max_tail_to_gap_x1e4=2500)),
    ("MoveGaps --max-tail=70 --max-tail-to-gap=5", "MoveGaps", None, dict(max_tail=70, max_tail_to_gap_x1e4=50000)),
    ("CutGaps", "CutGaps", "", {}),
    ("CutGaps --cut-strict=1", "CutGapsStrict", "", {}),
    ("SelfOverlapsResolver", "SelfOverlapsResolver", "", {}),
])
def test_random_blocks(seed, proc, oproc, opts, okw):
    rng = np.random.default_rng(seed)
    seqs = ["".join(rng.choice(list("ACGT"), size=5000)) for _ in range(4)]
    names = ["g%d&c&c" % i for i in range(4)]
    blocks = _random_gapped_blocks(rng, seqs, 300, overlap=proc == "SelfOverlapsResolver")
    eng, o = _both(seqs, names, blocks, orc_kw=okw)
    eng.apply(proc)
    o.apply(oproc)
    assert eng.blocks() == o.blocks()


@pytest.mark.parametrize("seed", [3, 4])
@pytest.mark.parametrize("pipe", ["Align", "LiteAlign"])
def test_align_pipe_random(seed, pipe):
    """Align / LiteAlign on gapped blocks, blocks without rows and
    self-overlapping blocks (SelfOverlapsResolver cuts them, MetaAligner
    realigns them)."""
    rng = np.random.default_rng(seed)
    seqs = ["".join(rng.choice(list("ACGT"), size=4000)) for _ in range(3)]
    names = ["g%d&c&c" % i for i in range(3)]
    blocks = _random_gapped_blocks(rng, seqs, 200, max_len=250, overlap=True)
    blocks = [b if i % 3 else [f[:4] + (None,) for f in b] for i, b in enumerate(blocks)]
    eng, o = _both(seqs, names, blocks)
    eng.apply(pipe)
    o.apply(pipe)
    assert canon(eng.blocks()) == canon(o.blocks())


@pytest.mark.parametrize("cfg", ["tiny", "small"])
def test_align_pipe_on_draft(cfg):
    """Align on a DraftPangenome result whose blocks are widened by random
    amounts and lose their rows (the closing Align of AnchorLoopFast sees
    DeConSeq's blocks like these), next to the unchanged aligned blocks."""
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    b0 = o.blocks()
    rng = np.random.default_rng(7)
    blocks = []
    for i, b in enumerate(b0):
        if i % 2:
            blocks.append(b)
            continue
        nb = []
        for s, mn, mx, ori, _ in b:
            nb.append((s, max(0, mn - int(rng.integers(0, 30))), min(len(seqs[s]) - 1, mx + int(rng.integers(0, 30))),
                       ori, None))
        blocks.append(nb)
    eng, o = _both(seqs, names, blocks)
    eng.apply("Align")
    o.apply("Align")
    got = eng.blocks()
    assert canon(got) == canon(o.blocks())
    assert got and all(len(b) >= 2 for b in got)
