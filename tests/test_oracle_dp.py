"""The CPU restatement of GeneralAligner (oracle/general_aligner.cpp) pinned
without a GPU.  The reference has no test of GeneralAligner, so the pins are:
  * textbook known answers: with the band covering the whole matrix and
    max_errors = -1 the score is the Levenshtein distance (unit costs, N never
    matches -- FragmentDistance.cpp:18-21), checked on literal KATs and against
    an independent textbook DP on seeded random pairs;
  * structural invariants of export_alignment: the ops consume exactly
    first[0..first_last] and second[0..second_last], and the summed step
    costs equal the reported score;
  * the stop rule: the last kept row's minimum is <= max_errors, and cut_tail
    ends on a zero-cost step.
Band limits, the stop row and tie-breaking beyond that follow
GeneralAligner.hpp:113-282 as restated ("parity unpinned")."""
import numpy as np
import pytest

from oracle import oracle as orc


def lev(a, b):
    """Textbook edit distance (Wagner-Fischer), N never equal to anything."""
    prev = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        cur = [i] + [0] * len(b)
        for j in range(1, len(b) + 1):
            s = 0 if (a[i - 1] == b[j - 1] and a[i - 1] != "N") else 1
            cur[j] = min(prev[j - 1] + s, prev[j] + 1, cur[j - 1] + 1)
        prev = cur
    return prev[-1]


def cost_of(a, b, ops, gp=1, mm=1):
    i = j = 0
    tot = 0
    for o in ops:
        if o == 0:
            tot += 0 if (a[i] == b[j] and a[i] != "N") else mm
            i += 1
            j += 1
        elif o == 1:
            tot += gp
            i += 1
        else:
            tot += gp
            j += 1
    return tot, i, j


KATS = [("ACGT", "ACGT", 0), ("AAAA", "AAA", 1), ("ACGTACGT", "TACGTACG", 2),
        ("GATTACA", "GCATGCT", 4), ("AAAAAAAA", "TTTTTTTT", 8), ("ACGTN", "ACGTN", 1),
        ("A", "T", 1), ("AC", "CA", 2), ("ACGGT", "AGT", 2)]


@pytest.mark.parametrize("a,b,d", KATS)
def test_levenshtein_kats(a, b, d):
    assert lev(a, b) == d
    r = orc.general_align(a, b, gap_range=max(len(a), len(b)), max_errors=-1)
    assert r["status"] == 0
    assert r["score"] == d
    tot, i, j = cost_of(a, b, r["ops"])
    assert (tot, i, j) == (d, len(a), len(b))
    assert (r["first_last"], r["second_last"]) == (len(a) - 1, len(b) - 1)


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


def test_random_full_band_equals_edit_distance():
    rng = np.random.default_rng(5)
    for _ in range(60):
        n = int(rng.integers(1, 80))
        a = "".join("ACGTN"[k] for k in rng.integers(0, 5 if rng.random() < 0.2 else 4, n))
        b = _mutate(rng, a, float(rng.choice([0.05, 0.2, 0.5]))) or "A"
        r = orc.general_align(a, b, gap_range=max(len(a), len(b)), max_errors=-1)
        assert r["score"] == lev(a, b)
        tot, i, j = cost_of(a, b, r["ops"])
        assert (tot, i, j) == (r["score"], len(a), len(b))


def test_stop_rule_and_cut_tail_invariants():
    rng = np.random.default_rng(11)
    for _ in range(200):
        n = int(rng.integers(5, 300))
        a = "".join("ACGT"[k] for k in rng.integers(0, 4, n))
        b = _mutate(rng, a, float(rng.choice([0.01, 0.05, 0.2])))
        if not b:
            continue
        if rng.random() < 0.3:  # a divergent tail
            a += "".join("ACGT"[k] for k in rng.integers(0, 4, 40))
            b += "".join("ACGT"[k] for k in rng.integers(0, 4, 40))
        gr = int(rng.choice([0, 1, 3, 10, 63]))
        me = int(rng.choice([0, 2, 5, 30]))
        for cut in (False, True):
            r = orc.general_align(a, b, gap_range=gr, max_errors=me, cut_tail=cut)
            assert r["status"] == 0
            tot, i, j = cost_of(a, b, r["ops"])
            assert (i - 1, j - 1) == (r["first_last"], r["second_last"])
            assert tot == r["score"]
            assert r["score"] <= me
            # every prefix of the path stays inside the band
            ii = jj = 0
            for o in r["ops"]:
                ii += o in (0, 1)
                jj += o in (0, 2)
                assert abs(ii - jj) <= gr + 1 or ii == 0 or jj == 0
            if cut and len(r["ops"]):
                last = r["ops"][-1]
                assert last == 0 and a[i - 1] == b[j - 1] and a[i - 1] != "N"


def test_empty_input_status():
    assert orc.general_align("", "ACG", 3, 0)["status"] == -2
    assert orc.general_align("ACG", "", 3, -1)["status"] == -2
