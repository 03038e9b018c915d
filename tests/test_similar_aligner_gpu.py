"""SimilarAligner / DummyAligner parity: batched HIP kernel (through the C ABI)
vs the CPU restatement of AbstractAligner::align_seqs (bit-exact rows).

Cases: the reference's own tests (src/test/similar_aligner.cpp, aligner.cpp,
test-lua/aligner-remove-gaps.lua) and seeded random families of rows built the
way FragmentsExtender flanks look: mutated copies of a common ancestor
(substitutions, indels, N runs), with homology that may end part-way, plus
unrelated rows, empty rows and single rows.
"""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

KATS = [
    ["ATTT", "ANTT", "ATTT"],
    ["ATGC", "AGC", "ATGC"],
    ["CCCATATGG", "CCATATCG"],
    ["ACCAGCTTTCGACCGCGGTGGCGATCGCGATATTAG", "ACCAGCTGGTGGCGATCGCGATATTAG",
     "ACCAGCTTTCGACCGCGGTGGCGATCGCGATATTAG"],
    ["ATG", "AG", ""],
    ["ATG", "AG"],
    ["CGAAT", "CAAAT"],
    ["GTTT", "GTTTT"],
    ["GCTATAAAGCAGCCTTCTTAGCTCACC", "ACTTGATGTGCGGCTCGGGATATTTCA",
     "CCCTCTCTGGGCAGGGCGAACATTAAA", "TTGTAATGCTATTCCATAGTGAGATGA"],
    ["AGAGCGGTTCCGGCGATTCCGTT", "AGAGCGATTCCGTT"],
    ["TTATGAGTCGAGAATATGGTGCCAAAGT", "TTATGAGTCGAGATATGGTGCCAAAGT"],
    ["AT", "A"], ["AT", "T"], ["", ""], ["A"], ["ACGT"], ["", "ACGT", ""],
]


def _aligner(kind="similar"):
    from npge_amd.aligner import BatchAligner
    return BatchAligner(kind)


def _family(rng, n, length, d, indel=0.1, tail_unrelated=0.0, nrate=0.0):
    anc = rng.integers(0, 4, length)
    rows = []
    for _ in range(n):
        out = []
        i = 0
        cut = length if rng.random() >= tail_unrelated else int(rng.integers(0, length + 1))
        while i < length:
            if i >= cut:
                out.append(int(rng.integers(0, 4)))
                i += 1
                continue
            r = rng.random()
            if r < d * (1 - indel):
                out.append((int(anc[i]) + int(rng.integers(1, 4))) % 4)
                i += 1
            elif r < d:
                k = int(rng.integers(1, 6))
                if rng.random() < 0.5:
                    out.extend(int(x) for x in rng.integers(0, 4, k))
                else:
                    i += k
            else:
                out.append(int(anc[i]))
                i += 1
        s = "".join("ATGC"[x] for x in out)
        if nrate and rng.random() < nrate and len(s) > 10:
            a = int(rng.integers(0, len(s) - 5))
            s = s[:a] + "N" * 5 + s[a + 5:]
        rows.append(s)
    return rows


def _random_jobs(seed, count, nmax=20, lmax=300):
    rng = np.random.default_rng(seed)
    jobs = []
    for _ in range(count):
        n = int(rng.integers(1, nmax + 1))
        L = int(rng.integers(0, lmax + 1))
        d = float(rng.choice([0.0, 0.005, 0.02, 0.05, 0.15, 0.4]))
        jobs.append(_family(rng, n, L, d, tail_unrelated=float(rng.choice([0.0, 0.5])),
                            nrate=float(rng.choice([0.0, 0.3]))))
    return jobs


def _check(jobs, kind="similar"):
    mode = "align_seqs" if kind == "similar" else "dummy"
    got = _aligner(kind).align(jobs)
    for j, (job, g) in enumerate(zip(jobs, got)):
        exp = orc.align(job, mode=mode)
        if g != exp:
            col = next((c for c in range(min(len(g[0]), len(exp[0]))) if any(x[c] != y[c] for x, y in zip(g, exp))),
                       None) if g and exp else None
            raise AssertionError("job %d (%d rows, lengths %s): %d columns vs %d expected, first difference at "
                                 "column %s" % (j, len(job), [len(r) for r in job], len(g[0]) if g else 0,
                                                len(exp[0]) if exp else 0, col))


def test_kats_similar():
    _check(KATS)


def test_kats_expected_rows():
    got = _aligner().align([["ATGC", "AGC", "ATGC"], ["ATG", "AG"], ["AT", "A"], ["AT", "T"]])
    assert got[0] == ["ATGC", "A-GC", "ATGC"]
    assert got[1] == ["ATG", "A-G"]
    assert got[2] == ["AT", "A-"]          # AbstractAligner::test (aligner.cpp:14-28)
    assert got[3] == ["AT", "-T"]


def test_kats_dummy():
    got = _aligner("dummy").align([["A-T-G-CATG", "ACT-GTCAT-"], ["AT", "A"], ["AT", "T"]])
    assert got[0] == ["A-TG-CATG", "ACTGTCAT-"]   # similar_aligner.cpp aligner_remove_gap_cols
    assert got[1] == ["AT", "A-"]
    assert got[2] == ["AT", "T-"]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_families(seed):
    _check(_random_jobs(seed, 150))


# NPGX_ALIGN_DEFER / NPGX_ALIGN_DEFER_ROWS (read when the aligner is created):
# the column and row counts from
# which fix_bad_regions' re-alignments leave the job's workgroup and run as
# sub-jobs of their own (0: never, 1: every alignment)
# NPGX_ALIGN_SPLIT: long jobs are cut into segments of about this many
# columns at sync states (0: never); small values put many sync states into
# every job, including the high-divergence ones where the speculation misses
@pytest.mark.parametrize("defer,rows,split", [("0", "0", "0"), ("1", "0", "0"), ("1000", "0", "0"),
                                              ("1000", "4", "0"), ("8000", "4", "0"), ("8000", "4", "512"),
                                              ("0", "0", "100"), ("1000", "4", "64")])
def test_long_flanks(defer, rows, split, monkeypatch):
    monkeypatch.setenv("NPGX_ALIGN_DEFER", defer)
    monkeypatch.setenv("NPGX_ALIGN_DEFER_ROWS", rows)  # deferred only with at least this many rows
    monkeypatch.setenv("NPGX_ALIGN_SPLIT", split)
    _check(_random_jobs(11, 40, nmax=17, lmax=1500))


@pytest.mark.parametrize("defer,rows,split", [("0", "0", "0"), ("1000", "0", "0"), ("8000", "4", "0"),
                                              ("8000", "4", "512"), ("1000", "0", "128")])
def test_very_long_rows(defer, rows, split, monkeypatch):
    """Alignments of thousands of columns with hundreds of low-similarity
    regions (the LDS region reduction and its block minima) and some rows
    unrelated from part-way."""
    monkeypatch.setenv("NPGX_ALIGN_DEFER", defer)
    monkeypatch.setenv("NPGX_ALIGN_DEFER_ROWS", rows)
    monkeypatch.setenv("NPGX_ALIGN_SPLIT", split)
    rng = np.random.default_rng(21)
    jobs = []
    for _ in range(12):
        n = int(rng.integers(2, 18))
        L = int(rng.integers(4000, 12000))
        d = float(rng.choice([0.02, 0.05, 0.1]))
        jobs.append(_family(rng, n, L, d, tail_unrelated=float(rng.choice([0.0, 0.3]))))
    _check(jobs)


@pytest.mark.parametrize("budget_mb,split", [("1", "0"), ("1", "256"), ("8", "128")])
def test_capped_slot_scratch(budget_mb, split, monkeypatch):
    """NPGX_SLOT_BUDGET_MB: per-slot word tables and stacks capped below the
    jobs' bounds (the sizing giant whole-genome alignments get).  Searches
    through unrelated tails outgrow the capped table, their jobs end as
    overflowed and re-run at the full bound on fewer slots: same result."""
    monkeypatch.setenv("NPGX_SLOT_BUDGET_MB", budget_mb)
    monkeypatch.setenv("NPGX_ALIGN_SPLIT", split)
    rng = np.random.default_rng(23)
    jobs = []
    for _ in range(10):
        n = int(rng.integers(2, 18))
        L = int(rng.integers(4000, 12000))
        jobs.append(_family(rng, n, L, 0.05, tail_unrelated=float(rng.choice([0.0, 0.5]))))
    _check(jobs)


@pytest.mark.parametrize("split", ["64", "256"])
def test_split_similar_families(split, monkeypatch):
    """Long, highly similar families (the C2/C3 flank shape: the sync states
    mostly hold) with short segments, and repeats inside the rows (a sync word
    that is not unique in its window is skipped)."""
    monkeypatch.setenv("NPGX_ALIGN_SPLIT", split)
    rng = np.random.default_rng(31)
    jobs = []
    for _ in range(16):
        n = int(rng.integers(2, 20))
        L = int(rng.integers(2000, 9000))
        jobs.append(_family(rng, n, L, float(rng.choice([0.005, 0.01, 0.02])), nrate=0.3))
    unit = "".join("ATGC"[x] for x in rng.integers(0, 4, 150))
    for _ in range(4):  # tandem repeats of a 150-mer between unique stretches
        base = _family(rng, 1, 3000, 0.0)[0]
        rows = _family(rng, int(rng.integers(3, 9)), 1, 0.0)
        jobs.append([base[:1000] + unit * 8 + base[1000:] for _ in rows])
    _check(jobs)


@pytest.mark.parametrize("twins", ["0", "1", "-1"])
@pytest.mark.parametrize("split", ["128", "384"])
def test_twins(twins, split, monkeypatch):
    """Twins (similar_aligner.hip, align_device "Twins"): every split job also
    walks its reversed rows in the same launch, and a job that turns out to be
    one bad region takes that walk as its re-alignment (NPGX_TWINS 1: always,
    0: never, -1: in launches with few tasks).  Families from nearly identical
    (a good alignment: the twin is not used) to unrelated (one bad region;
    chains that fail on missed sync states fall back), many rows and two."""
    monkeypatch.setenv("NPGX_TWINS", twins)
    monkeypatch.setenv("NPGX_ALIGN_SPLIT", split)
    rng = np.random.default_rng(41)
    jobs = []
    for d in (0.005, 0.02, 0.06, 0.15, 0.4):
        for n in (2, 5, 17):
            L = int(rng.integers(1500, 6000))
            jobs.append(_family(rng, n, L, d, tail_unrelated=float(rng.choice([0.0, 0.3]))))
    _check(jobs)


def test_wide_blocks():
    _check(_random_jobs(12, 20, nmax=64, lmax=200))


def test_unrelated_rows():
    rng = np.random.default_rng(7)
    jobs = [["".join("ATGC"[x] for x in rng.integers(0, 4, int(rng.integers(50, 400))))
             for _ in range(int(rng.integers(2, 10)))] for _ in range(30)]
    _check(jobs)


def test_dummy_random():
    _check(_random_jobs(5, 50), kind="dummy")


def test_more_than_64_rows():
    """Problems of more than 64 non-empty rows go to the workgroup-per-problem
    aligner (wide_aligner.hip): repeat-family-like mutated copies, unrelated
    tails, N runs, empty rows, next to narrow jobs in the same batch."""
    rng = np.random.default_rng(65)
    jobs = [["ACGT"] * 65, ["ACGT"] * 64 + ["ACGA"], [""] * 10 + ["AC"] * 70]
    for n, L, d in ((65, 40, 0.02), (80, 300, 0.01), (100, 200, 0.05), (130, 150, 0.15), (70, 500, 0.005),
                    (300, 120, 0.03), (66, 250, 0.4)):
        jobs.append(_family(rng, n, L, d, tail_unrelated=0.3, nrate=0.05))
    jobs.append(_family(rng, 5, 100, 0.05))  # a narrow job in the same batch
    _check(jobs)
    _check(jobs, kind="dummy")


def test_more_than_64_rows_random():
    rng = np.random.default_rng(99)
    jobs = [_family(rng, int(rng.integers(65, 200)), int(rng.integers(1, 400)),
                    float(rng.choice([0.0, 0.01, 0.05, 0.2])), tail_unrelated=float(rng.choice([0.0, 0.5])))
            for _ in range(12)]
    _check(jobs)


@pytest.mark.parametrize("cfg", ["tiny", "small"])
def test_flank_batch(cfg):
    """Every flank job of the first FragmentsExtender pass of a synthetic set,
    in ONE batch (thousands of jobs: the launch shrinks its LDS stage), equals
    the oracle's align_seqs job for job."""
    from npge_amd import synth
    from helpers import flank_jobs
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    af = orc.AnchorFinder()
    r = af.run(seqs, names)
    bs = r["block_start"]
    blocks = [[(int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i]), None)
               for i in range(bs[b], bs[b + 1])] for b in range(len(bs) - 1)]
    o.set_blocks(blocks)
    o.apply("RemoveNonStem").apply("DummyAligner")
    jobs = flank_jobs(o.blocks(), seqs)
    assert len(jobs) > 100
    from npge_amd.aligner import BatchAligner
    gpu = BatchAligner().align(jobs)
    bad = [j for j, rows in enumerate(jobs) if orc.align(rows, "align_seqs") != gpu[j]]
    assert not bad, "%d of %d jobs differ (first %d)" % (len(bad), len(jobs), bad[0])


def test_refinement_kats_kernel():
    """src/test/similar_aligner.cpp refinement_3/4/5 through k_refine
    (npgx_refine_batch)."""
    from npge_amd.aligner import refine_batch
    got = refine_batch([["CCGG", "CG-G", "CG-G", "CG-G"], ["CCGGCC", "CGG--C"],
                        ["-CCCCCC", "CCCACCC", "CCCTCCC"]])
    assert got == [["CCGG", "C-GG", "C-GG", "C-GG"], ["CCGGCC", "C-GG-C"],
                   ["CCC-CCC", "CCCACCC", "CCCTCCC"]]


@pytest.mark.parametrize("seed", [21, 22])
def test_refine_random(seed):
    """k_refine vs the oracle's refine_alignment on the similar aligner's
    output for random families, and on those alignments with random gaps
    shuffled in (many moves, pure-gap columns, long gap runs)."""
    from npge_amd.aligner import refine_batch
    rng = np.random.default_rng(seed)
    jobs = [j for j in _random_jobs(seed, 120, nmax=12, lmax=250) if j and any(j)]
    alns = [orc.align(j, mode="similar") for j in jobs]
    alns = [a for a in alns if a and a[0]]
    noisy = []
    for a in alns:
        rows = []
        for r in a:
            r = list(r)
            for _ in range(int(rng.integers(0, 6))):
                p = int(rng.integers(0, len(r)))
                q = int(rng.integers(0, len(r)))
                r[p], r[q] = r[q], r[p]  # letters and gaps trade places
            rows.append("".join(r))
        noisy.append(rows)
    for batch in (alns, noisy):
        got = refine_batch(batch)
        for a, g in zip(batch, got):
            assert g == orc.align(a, mode="refine"), a


@pytest.mark.parametrize("head", ["128", "4", "1", "0"])
def test_wide_long_restart_searches(head, monkeypatch):
    """The wide aligner's prefix search (prefix_search, wide_aligner.hip)
    against the oracle: more than 64 rows with unrelated insertions of up to
    3000 bases between shared stretches, repeats planted in the insertions,
    unrelated tails.  NPGX_WIDE_LONG_HEAD moves the switch from the shift-by-
    shift search (0: never switch)."""
    monkeypatch.setenv("NPGX_WIDE_LONG_HEAD", head)
    rng = np.random.default_rng(77)
    jobs = []
    for n in (65, 90, 130):
        for ins, rep in ((300, 0.0), (1500, 0.5), (3000, 0.0)):
            jobs.append(_restart_family(rng, n, 200, ins, repeat=rep))
    jobs.append(_family(rng, 80, 400, 0.02, tail_unrelated=0.5))
    _check(jobs)


def test_wide_unrelated_long_tails():
    """More than 64 rows whose homology ends after a short core, followed by
    unrelated tails of 20k+ bases: the wide aligner's word
    search scans ~20k shifts x 70 rows before giving up; its tables grow to
    the proven size on a retry instead of failing, and the rows match the
    oracle."""
    rng = np.random.default_rng(99)
    core = rng.integers(0, 4, 200)
    rows = []
    for _ in range(70):
        c = core.copy()
        m = rng.random(len(c)) < 0.01
        c[m] = (c[m] + 1) % 4
        tail = rng.integers(0, 4, int(rng.integers(20000, 21000)))
        rows.append("".join("ATGC"[x] for x in np.concatenate([c, tail])))
    _check([rows])


def _restart_family(rng, n, core, ins, d=0.01, repeat=0.0):
    """Rows that agree, then each carry an unrelated insertion of up to `ins`
    bases at the same place, then agree again: try_aligned searches past the
    insertions (hundreds to thousands of shifts).  With `repeat`, the
    insertions also hold copies of the next words of the shared text, so the
    search meets complete words at several shifts (first sightings, the
    highest-row rule and words.size() == 1 all decide)."""
    anc = "".join("ATGC"[x] for x in rng.integers(0, 4, 2 * core + 40))
    rows = []
    for _ in range(n):
        left = list(anc[:core])
        right = list(anc[core:])
        for part in (left, right):
            for i in range(len(part)):
                if rng.random() < d:
                    part[i] = "ATGC"[int(rng.integers(0, 4))]
        k = int(rng.integers(0, ins + 1))
        mid = "".join("ATGC"[x] for x in rng.integers(0, 4, k))
        if repeat and k > 40 and rng.random() < repeat:
            a = int(rng.integers(0, k - 20))
            mid = mid[:a] + anc[core:core + 20] + mid[a + 20:]
        rows.append("".join(left) + mid + "".join(right))
    return rows


@pytest.mark.parametrize("head,m", [("128", "512"), ("32", "512"), ("0", "512"), ("1", "64"), ("64", "2048")])
def test_long_restart_searches(head, m, monkeypatch):
    """try_aligned's prefix search (find_word_long, sa_device.hpp) against the
    oracle's find_best_word loop: unrelated insertions of up to 6000 bases
    between shared stretches, 2 to 40 rows (the vector search up to 8 rows,
    the row-parallel one above), repeats planted in the insertions, low-
    complexity inserts (many equal words), and no shared word at all.
    NPGX_LONG_HEAD / NPGX_LONG_M move the switch from the incremental search
    (0: never switch) and the first prefix."""
    monkeypatch.setenv("NPGX_LONG_HEAD", head)
    monkeypatch.setenv("NPGX_LONG_M", m)
    rng = np.random.default_rng(51)
    jobs = []
    for n in (2, 3, 5, 8, 9, 17, 40):
        for ins, rep in ((300, 0.0), (2000, 0.5), (6000, 0.0), (1500, 1.0)):
            jobs.append(_restart_family(rng, n, 300, ins, repeat=rep))
    for n in (2, 12):  # low-complexity insertions: poly-A and a dinucleotide repeat
        core = "".join("ATGC"[x] for x in rng.integers(0, 4, 400))
        jobs.append([core[:200] + "A" * int(rng.integers(100, 900)) + core[200:] for _ in range(n)])
        jobs.append([core[:200] + "AT" * int(rng.integers(50, 700)) + core[200:] for _ in range(n)])
    for n in (2, 10):  # nothing shared after the core: the search runs out
        core = "".join("ATGC"[x] for x in rng.integers(0, 4, 150))
        jobs.append([core + "".join("ATGC"[x] for x in rng.integers(0, 4, 3000)) for _ in range(n)])
    _check(jobs)
