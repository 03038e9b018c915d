"""Parity at BASELINE.json's C4 (32 x 5 Mbp, 2 % divergence) and C5
(8 x 50 Mbp, 1 %) sizes, and AnchorLoopFast at C3 and C4.  The CPU restatement needs minutes there, so its
outputs are committed as fingerprints (tests/golden/fullsize/*.json, made by
tests/golden/make_fullsize.py; tests/helpers.py af_digest / blocks_digest):
the GPU run's SoA anchor set, Bloom parameters, counts and persistent used-hash
set over two runs on one instance must hash identically.  C5 is checked whole
and on its 2 x 50 Mbp subset, plus properties that need no oracle: every
anchor block holds >= 2 k-mer fragments with one text up to orientation and
no N."""
import json
import os

import numpy as np
import pytest

from npge_amd import synth
from helpers import af_digest, blocks_digest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "fullsize")


def _case(case):
    cfg, _, n = case.partition("sub")
    names, seqs = synth.genome_set(cfg)
    if n:
        names, seqs = names[:int(n)], seqs[:int(n)]
    with open(os.path.join(GOLD, case + ".json")) as f:
        gold = json.load(f)
    assert gold["n_seqs"] == len(seqs) and gold["bp"] == synth.total_bp(seqs)
    return names, seqs, gold


def _diff(got, want):
    return {k: (got.get(k), want[k]) for k in want if got.get(k) != want[k]}


_COMP = bytes.maketrans(b"ACGTN", b"TGCAN")


def _check_properties(r, seqs, k=20):
    bs = np.asarray(r["block_start"], dtype=np.int64)
    mn = np.asarray(r["min_pos"], dtype=np.int64)
    mx = np.asarray(r["max_pos"], dtype=np.int64)
    sq = np.asarray(r["seq"], dtype=np.int64)
    ori = np.asarray(r["ori"], dtype=np.int64)
    assert len(bs) > 1 and bs[0] == 0 and bs[-1] == len(sq)
    assert np.all(np.diff(bs) >= 2)
    assert np.all(mx - mn == k - 1) and np.all(mn >= 0)
    lens = np.array([len(s) for s in seqs])
    assert np.all(mx < lens[sq]) and np.all(np.abs(ori) == 1)
    raw = [s.encode() for s in seqs]
    for b in range(len(bs) - 1):
        texts = set()
        for i in range(bs[b], bs[b + 1]):
            t = raw[sq[i]][mn[i]:mx[i] + 1]
            if ori[i] == -1:
                t = t.translate(_COMP)[::-1]
            texts.add(t)
        assert len(texts) == 1, b
        assert b"N" not in texts.pop(), b


@pytest.mark.parametrize("case", ["C4", "C5sub2", "C5"])
def test_anchor_finder_c45(case):
    from npge_amd import _capi
    from npge_amd.anchor_finder import AnchorFinder
    names, seqs, gold = _case(case)
    ss = _capi.SeqSet(seqs, names)
    af = AnchorFinder()
    for run in range(2):
        r = af.find(ss)
        got = af_digest(r, af.used_hashes())
        assert got == gold["af"][run], (run, _diff(got, gold["af"][run]))
        if run == 0 and case == "C5":
            _check_properties(r, seqs)


@pytest.mark.parametrize("case", ["C4", "C5sub2", "C5"])
def test_draft_pangenome_c45(case):
    from npge_amd import _capi
    from npge_amd.anchor_finder import AnchorFinder
    from npge_amd.blockset import BlockSetEngine
    names, seqs, gold = _case(case)
    eng = BlockSetEngine(_capi.SeqSet(seqs, names))
    eng.apply("DraftPangenome", af=AnchorFinder())
    want = gold["draft"]
    st = eng.stats()
    for k in ("anchor_blocks", "stem_blocks", "iterations", "aligned_residues"):
        assert st[k] == want["stats"][k], k
    got = dict(blocks_digest(eng.blocks()), hash=int(eng.hash()))
    want = {k: want[k] for k in got}
    assert got == want, _diff(got, want)


@pytest.mark.parametrize("case", ["C3", "C4"])
def test_anchor_loop_fullsize(case):
    """DraftPangenome -> AnchorLoopFast (the bench's --anchor-loop workload).
    C4: on the 32 genome-long consensus sequences the pipe's ExtendLoopFast
    grows whole-genome blocks (alignments of millions of columns, split into
    segments), 18 iterations (fixture: 250 s on the CPU); C3: the 17-genome
    draft's consensus blocks.  Blocks, rows and blockset_hash equal the oracle
    pipe's."""
    from npge_amd import _capi
    from npge_amd.anchor_finder import AnchorFinder
    from npge_amd.blockset import BlockSetEngine
    names, seqs, gold = _case(case)
    eng = BlockSetEngine(_capi.SeqSet(seqs, names))
    eng.apply("DraftPangenome", af=AnchorFinder())
    eng.apply("AnchorLoopFast", af=AnchorFinder())
    want = gold["anchor_loop"]
    assert eng.stats()["loop"]["loop_iterations"] == want["iterations"]
    got = dict(blocks_digest(eng.blocks()), hash=int(eng.hash()))
    want = {k: want[k] for k in got}
    assert got == want, _diff(got, want)
