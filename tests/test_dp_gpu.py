"""GeneralAligner on the GPU (npgx_dp_*) vs the CPU restatement
(oracle/general_aligner.cpp), bit-exact on every output: first_last,
second_last, score, status and the exported alignment.  Seeded pairs with
substitutions, indels, N letters and divergent tails; gap_range 0..63 (the
band edge, one wave), max_errors -1 / 0 / small / large, cut_tail on and off,
empty inputs, and long pairs checked by size-independent properties."""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _mutate(rng, s, d):
    out = []
    for ch in s:
        x = rng.random()
        if x < d / 3:
            continue
        if x < 2 * d / 3:
            out.append(ch)
            out.append("ACGT"[rng.integers(4)])
            continue
        out.append("ACGT"[rng.integers(4)] if x < d else ch)
    return "".join(out)


def _pairs(rng, n, lo, hi):
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        alphabet = 5 if rng.random() < 0.2 else 4
        a = "".join("ACGTN"[k] for k in rng.integers(0, alphabet, L))
        b = _mutate(rng, a, float(rng.choice([0.0, 0.01, 0.05, 0.2, 0.6]))) or "G"
        if rng.random() < 0.3:
            a += "".join("ACGT"[k] for k in rng.integers(0, 4, int(rng.integers(1, 60))))
            b += "".join("ACGT"[k] for k in rng.integers(0, 4, int(rng.integers(1, 60))))
        if rng.random() < 0.5:
            a, b = b, a
        out.append((a, b))
    return out


def _check(pairs, gr, me, cut, gp=1, mm=1):
    from npge_amd.dp import GeneralAligner
    g = GeneralAligner(gap_range=gr, max_errors=me, gap_penalty=gp, mismatch_penalty=mm,
                       cut_tail=cut)
    r = g.align_batch(pairs)
    for i, (a, b) in enumerate(pairs):
        o = orc.general_align(a, b, gr, me, gp, mm, cut)
        assert r["status"][i] == o["status"], (i, a, b)
        if o["status"] != 0:
            continue
        got = (int(r["first_last"][i]), int(r["second_last"][i]), int(r["score"][i]))
        assert got == (o["first_last"], o["second_last"], o["score"]), (i, gr, me, cut)
        ops = r["ops"][r["op_off"][i]:r["op_off"][i + 1]]
        np.testing.assert_array_equal(ops, o["ops"], err_msg="pair %d" % i)
    return g


@pytest.mark.parametrize("gr", [0, 1, 2, 7, 31, 62, 63])
@pytest.mark.parametrize("me", [-1, 0, 3, 40])
def test_dp_matches_oracle(gr, me):
    rng = np.random.default_rng(1000 + 7 * gr + me)
    pairs = _pairs(rng, 120, 1, 400)
    for cut in ((False, True) if me != -1 else (False,)):
        _check(pairs, gr, me, cut)


def test_dp_penalties_and_long_pairs():
    rng = np.random.default_rng(77)
    pairs = _pairs(rng, 16, 2000, 5000)
    _check(pairs, 63, 200, True)
    _check(pairs, 20, -1, False)
    _check(_pairs(rng, 60, 1, 300), 9, 12, True, gp=2, mm=3)
    _check(_pairs(rng, 60, 1, 300), 5, 7, False, gp=0, mm=1)


def test_dp_empty_and_mixed_batch():
    pairs = [("", "ACGT"), ("ACGT", ""), ("ACGT", "ACGT"), ("A", "A"), ("N", "N")]
    g = _check(pairs, 3, 0, False)
    r = g.result()
    assert list(r["status"][:2]) == [-2, -2]


def test_dp_long_properties():
    """100 kb pairs (beyond what the oracle's full matrix holds): the exported
    ops consume exactly the aligned prefixes, the summed step costs equal the
    score, and with max_errors = -1 the path ends at the last cells."""
    from npge_amd.dp import GeneralAligner
    rng = np.random.default_rng(3)
    a = "".join("ACGT"[k] for k in rng.integers(0, 4, 100_000))
    pairs = [(a, _mutate(rng, a, 0.01)), (_mutate(rng, a, 0.02), a)]
    for me, cut in ((500, True), (-1, False)):
        g = GeneralAligner(gap_range=63, max_errors=me, cut_tail=cut)
        r = g.align_batch(pairs)
        for i, (x, y) in enumerate(pairs):
            ops = r["ops"][r["op_off"][i]:r["op_off"][i + 1]]
            ia = int(np.sum((ops == 0) | (ops == 1)))
            ib = int(np.sum((ops == 0) | (ops == 2)))
            assert (ia - 1, ib - 1) == (int(r["first_last"][i]), int(r["second_last"][i]))
            xa = np.frombuffer(x[:ia].encode(), dtype=np.uint8)
            yb = np.frombuffer(y[:ib].encode(), dtype=np.uint8)
            m = ops == 0
            pa = np.cumsum((ops == 0) | (ops == 1)) - 1
            pb = np.cumsum((ops == 0) | (ops == 2)) - 1
            mism = int(np.sum(xa[pa[m]] != yb[pb[m]]))
            cost = mism + int(np.sum(~m))
            if me == -1:
                assert (ia, ib) == (len(x), len(y))
            else:
                assert cost == int(r["score"][i]) <= me


@pytest.mark.parametrize("gr,me,cut", [(63, -1, False), (63, 400, True), (20, 150, True),
                                       (5, -1, False)])
def test_dp_c5_shaped_pairs(gr, me, cut):
    """C5-shaped pairs (BASELINE.json configs[4]: 1 % divergence, the
    synth.py mutation model with 1-10 nt indels, N runs) of 20-100 kb, bit-exact
    vs the restatement, whose band storage holds pairs of this length."""
    from npge_amd import synth
    rng = np.random.default_rng(1000 + gr)
    pairs = []
    for i in range(8):
        L = int(rng.integers(20_000, 100_001))
        root = rng.integers(0, 4, L).astype(np.uint8)
        x = synth.LETTERS[root].copy()
        y = synth.LETTERS[synth._mutate(rng, root, 0.01)].copy()
        if i % 3 == 0:
            p0 = int(rng.integers(0, L - 600))
            x[p0:p0 + int(rng.integers(50, 501))] = ord("N")
        a, b = x.tobytes().decode(), y.tobytes().decode()
        pairs.append((a, b) if i % 2 else (b, a))
    _check(pairs, gr, me, cut)
