"""The device ExtendLoopFast (npge_amd/csrc/elf_device.inc):
block table, block_hash, MoveUnchanged, flank plan, stitch, FixEnds slicing,
OverlaplessUnion and the Pipe state on the GPU.

* OverlaplessUnion@device (the loop's OverlaplessUnion on arbitrary blocks)
  against the oracle's OverlaplessUnion (OverlaplessUnion.cpp:25-80): sparse,
  dense and long-fragment sets, many sequences, equal sizes and lengths
  (the pinned tie-breaks decide), and the inputs the device hands to the
  host (blocks overlapping themselves: SetFc's multiset mode).
* ExtendLoopFast / DraftPangenome with the device loop against the host loop
  (NPGX_ELF_DEVICE=0) and the oracle: fragments, rows, stats.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from npge_amd import synth

from test_block_build_gpu import _engine, _ou_blocks, _stem_blocks, canon

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("max_len,self_overlap", [(40, False), (400, False), (3000, False), (40, True),
                                                  (400, 60)])
def test_ou_device_many_blocks(max_len, self_overlap):
    rng = np.random.default_rng(max_len + 7 * int(self_overlap))
    n_seqs, seq_len = 8, 400000
    seqs = ["".join(rng.choice(list("ACGT"), size=seq_len)) for _ in range(n_seqs)]
    names = ["g%d&c&c" % i for i in range(n_seqs)]
    blocks = _ou_blocks(rng, n_seqs, seq_len, 1500, max_len, self_overlap)
    ss, eng = _engine(seqs, names)
    o = orc.BlockSetOracle(seqs, names)
    eng.set_blocks(blocks).apply("OverlaplessUnion@device")
    o.set_blocks(blocks)
    o.apply("OverlaplessUnion")
    want = o.blocks()
    assert eng.blocks() == want
    assert 0 < len(want) <= len(blocks)


@pytest.mark.parametrize("n_chain,n_dup", [(2000, 300), (1700, 300), (1, 0), (0, 2)])
def test_ou_device_ties_and_chains(n_chain, n_dup):
    """Blocks of equal size and length (the minimum fragment, then the sorted
    fragment list, then the input order decide) in long overlap chains (the
    priority sweeps run many rounds), and blocks without fragments in range
    of nothing else; down to one block of two fragments (its fragments
    sorted all the same: with one block the block sort is skipped) and two
    equal blocks."""
    rng = np.random.default_rng(5)
    n_seqs, seq_len = 3, 200000
    seqs = ["".join(rng.choice(list("ACGT"), size=seq_len)) for _ in range(n_seqs)]
    names = ["t%d&c&c" % i for i in range(n_seqs)]
    blocks = []
    for i in range(n_chain):  # a chain along sequence 0: each block overlaps the next
        a = 50 * i
        blocks.append([(0, a, a + 60, 1, None), (1 + i % 2, a, a + 60, -1 if i % 3 else 1, None)])
    for i in range(n_dup):  # duplicates of earlier blocks' first fragments
        if n_chain:
            j = int(rng.integers(0, n_chain))
            blocks.append([blocks[j][0], (2, 150000 + 70 * i, 150000 + 70 * i + 60, 1, None)])
        else:  # two equal blocks
            blocks.append([(0, 100, 160, 1, None), (1, 500, 560, -1, None)])
    perm = rng.permutation(len(blocks))
    blocks = [blocks[int(k)] for k in perm]
    ss, eng = _engine(seqs, names)
    o = orc.BlockSetOracle(seqs, names)
    eng.set_blocks(blocks).apply("OverlaplessUnion@device")
    o.set_blocks(blocks)
    o.apply("OverlaplessUnion")
    assert eng.blocks() == o.blocks()


def test_ou_device_many_sequences():
    rng = np.random.default_rng(12)
    n_seqs, seq_len = 4000, 1200
    seqs = ["".join(rng.choice(list("ACGT"), size=seq_len)) for _ in range(n_seqs)]
    names = ["c%d&c&c" % i for i in range(n_seqs)]
    blocks = _ou_blocks(rng, n_seqs, seq_len, 2500, 600, False)
    ss, eng = _engine(seqs, names)
    o = orc.BlockSetOracle(seqs, names)
    eng.set_blocks(blocks).apply("OverlaplessUnion@device")
    o.set_blocks(blocks)
    o.apply("OverlaplessUnion")
    assert eng.blocks() == o.blocks()


def _draft(cfg, device, monkeypatch):
    from npge_amd.anchor_finder import AnchorFinder
    monkeypatch.setenv("NPGX_ELF_DEVICE", "1" if device else "0")
    monkeypatch.setenv("NPGX_ELF_CHECK", "1")  # a bad table or flank plan fails loudly instead of faulting
    names, seqs = synth.genome_set(cfg)
    ss, eng = _engine(seqs, names)
    eng.apply("DraftPangenome", af=AnchorFinder())
    st = eng.stats()
    return eng.blocks(), eng.rows_digest(), st


def test_ou_device_multi_launch_passes(monkeypatch):
    """The table passes in their many-workgroup form (tables of more than
    2048 blocks take it; NPGX_ELF_PASS_WG=0 forces it here): one launch with
    decoupled look-back over 256-block tiles."""
    monkeypatch.setenv("NPGX_ELF_PASS_WG", "0")
    rng = np.random.default_rng(31)
    n_seqs, seq_len = 6, 300000
    seqs = ["".join(rng.choice(list("ACGT"), size=seq_len)) for _ in range(n_seqs)]
    names = ["m%d&c&c" % i for i in range(n_seqs)]
    blocks = _ou_blocks(rng, n_seqs, seq_len, 1200, 400, False)
    ss, eng = _engine(seqs, names)
    o = orc.BlockSetOracle(seqs, names)
    eng.set_blocks(blocks).apply("OverlaplessUnion@device")
    o.set_blocks(blocks)
    o.apply("OverlaplessUnion")
    assert eng.blocks() == o.blocks()


@pytest.mark.parametrize("cfg,only", [("tiny", p) for p in ("plan", "stitch", "fix_ends_plan", "slice",
                                                            "ou_prep", "ou_scan", "ou_compact")]
                         + [("tiny", ""), ("rtiny", "")])
def test_draft_device_multi_launch_passes(cfg, only, monkeypatch):
    """Every table pass (or one, `only`) in its many-workgroup form: one
    launch with decoupled look-back over 256-block tiles."""
    monkeypatch.setenv("NPGX_ELF_PASS_WG", "0")
    monkeypatch.setenv("NPGX_ELF_PASS_MULTI", only)
    b_dev, d_dev, s_dev = _draft(cfg, True, monkeypatch)
    b_host, d_host, s_host = _draft(cfg, False, monkeypatch)
    assert canon(b_dev) == canon(b_host)
    assert d_dev == d_host
    assert s_dev["iterations"] == s_host["iterations"]


@pytest.mark.parametrize("cfg", ["tiny", "small", "rtiny", "rsmall"])
def test_draft_device_equals_host_loop(cfg, monkeypatch):
    b_dev, d_dev, s_dev = _draft(cfg, True, monkeypatch)
    b_host, d_host, s_host = _draft(cfg, False, monkeypatch)
    assert canon(b_dev) == canon(b_host)
    assert d_dev == d_host
    for k in ("iterations", "aligned_residues", "align_jobs", "stem_blocks"):
        assert s_dev[k] == s_host[k], k


@pytest.mark.parametrize("cfg,iters", [("tiny", 10), ("small", 2), ("rtiny", 10)])
def test_extend_loop_fast_device_vs_oracle(cfg, iters, monkeypatch):
    monkeypatch.setenv("NPGX_ELF_DEVICE", "1")
    monkeypatch.setenv("NPGX_ELF_CHECK", "1")
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


def test_extend_loop_fast_device_host_fallback(monkeypatch):
    """Blocks overlapping themselves (a fragment next to a shifted copy of
    itself on the same sequence) send the device loop's OverlaplessUnion to
    the host (SetFc's multiset mode); the result equals the host loop's and
    the oracle's."""
    names, seqs = synth.genome_set("small")
    b0 = _stem_blocks(seqs, names)
    blocks = [[f[:4] + (None,) for f in b] for b in b0]
    for i in range(0, len(blocks), 7):
        q, mn, mx, ori, _ = blocks[i][0]
        if mn > 30 and mx + 30 < len(seqs[q]):
            blocks[i].append((q, mn + 3, mx + 3, ori, None))
    res = []
    for dev in ("1", "0"):
        monkeypatch.setenv("NPGX_ELF_DEVICE", dev)
        ss, eng = _engine(seqs, names, max_iterations=4)
        eng.set_blocks(blocks).apply("DummyAligner").apply("ExtendLoopFast")
        res.append((canon(eng.blocks()), eng.rows_digest(), eng.stats()["iterations"],
                    eng.stats()["counters"]["spare"]))
    assert res[0][:3] == res[1][:3]
    assert res[0][3] > 0  # the device loop handed OverlaplessUnion to the host
    o = orc.BlockSetOracle(seqs, names, max_iterations=4)
    o.set_blocks(blocks)
    o.apply("DummyAligner")
    o.apply("ExtendLoopFast")
    assert canon(o.blocks()) == res[0][0]


def test_blockset_tune(monkeypatch):
    """npgx_blockset_tune: "long-head" (the aligner forms without the prefix
    search's call at 0) and "elf-device" change no result; unknown keys and
    values out of range are refused."""
    from npge_amd import _capi
    from npge_amd.anchor_finder import AnchorFinder
    monkeypatch.delenv("NPGX_ELF_DEVICE", raising=False)
    names, seqs = synth.genome_set("rtiny")
    res = []
    for tune in ({}, {"long-head": 0}, {"elf-device": 0}, {"long-head": 0, "elf-device": 1}):
        ss, eng = _engine(seqs, names)
        for k, v in tune.items():
            eng.tune(k, v)
        eng.apply("DraftPangenome", af=AnchorFinder())
        res.append((canon(eng.blocks()), eng.rows_digest()))
    assert all(r == res[0] for r in res[1:])
    ss, eng = _engine(seqs, names)
    for k, v in (("no-such-key", 1), ("elf-device", 2), ("long-head", -1)):
        with pytest.raises(_capi.NpgxError):
            eng.tune(k, v)


@pytest.mark.parametrize("fail_iter", [0, 1, 2])
def test_extend_loop_fast_device_failure_keeps_blocks(fail_iter, monkeypatch):
    """A failure inside the device loop (injected after iteration k's stitch:
    the first stitch wrote the other row buffer, the later ones would have
    overwritten the entry rows) leaves the set with its blocks and rows as
    they came in; the handle then runs the loop to the oracle's result."""
    from npge_amd import _capi
    monkeypatch.setenv("NPGX_ELF_DEVICE", "1")
    names, seqs = synth.genome_set("small")
    b0 = _stem_blocks(seqs, names)
    ss, eng = _engine(seqs, names, max_iterations=6)
    eng.set_blocks(b0).apply("DummyAligner")
    before, d_before = canon(eng.blocks()), eng.rows_digest()
    monkeypatch.setenv("NPGX_TEST_FAIL_ELF", str(fail_iter))
    with pytest.raises(_capi.NpgxError, match="injected"):
        eng.apply("ExtendLoopFast")
    assert canon(eng.blocks()) == before
    assert eng.rows_digest() == d_before
    monkeypatch.delenv("NPGX_TEST_FAIL_ELF")
    eng.apply("ExtendLoopFast")
    o = orc.BlockSetOracle(seqs, names, max_iterations=6)
    o.set_blocks(b0)
    o.apply("DummyAligner")
    o.apply("ExtendLoopFast")
    assert canon(eng.blocks()) == canon(o.blocks())
    assert eng.hash() == o.hash()


def _many_rows_set(n_genomes=40, length=30000, div=0.004, seed=77):
    """A family of n_genomes close copies of one root: blocks of ~n_genomes
    rows whose flanks grow with their blocks (portion 0.5)."""
    rng = np.random.default_rng(seed)
    root = rng.integers(0, 4, size=length)
    seqs = []
    for g in range(n_genomes):
        s = root.copy()
        m = rng.random(length) < div
        s[m] = (s[m] + rng.integers(1, 4, size=int(m.sum()))) % 4
        seqs.append("".join("ACGT"[c] for c in s))
    return ["f%d&c&c" % g for g in range(n_genomes)], seqs


@pytest.mark.parametrize("budget_mb", ["0", "1"])
def test_extend_loop_fast_device_async_budget(budget_mb, monkeypatch):
    """The asynchronous aligner plans every job's re-run at the proven bound
    (3 n Σlen bytes) and the stitch arena at n Σlen: past NPGX_ASYNC_BUDGET_MB
    an iteration takes the synchronous aligner instead.  Many rows and long
    flanks, budgets that force the fallback in every iteration (0) or in the
    late ones (1 MiB): the result equals the default budget's, the host
    loop's and the oracle's."""
    from npge_amd.anchor_finder import AnchorFinder
    names, seqs = _many_rows_set()
    res = []
    for dev, budget in (("1", None), ("1", budget_mb), ("0", None)):
        monkeypatch.setenv("NPGX_ELF_DEVICE", dev)
        if budget is None:
            monkeypatch.delenv("NPGX_ASYNC_BUDGET_MB", raising=False)
        else:
            monkeypatch.setenv("NPGX_ASYNC_BUDGET_MB", budget)
        ss, eng = _engine(seqs, names)
        eng.apply("DraftPangenome", af=AnchorFinder())
        st = eng.stats()
        res.append((canon(eng.blocks()), eng.rows_digest(), st["iterations"], st["device_iterations"],
                    st["device_sync_iterations"]))
    assert res[0][:3] == res[1][:3] == res[2][:3]
    assert res[0][3] > 0 and res[0][4] == 0      # the default budget: every iteration asynchronous
    assert res[1][4] > 0                         # the small budget: the synchronous fallback ran
    if budget_mb == "0":
        assert res[1][4] >= res[1][3] - 1        # (an iteration without jobs has no aligner)
    assert res[2][3] == 0
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    assert canon(o.blocks()) == res[0][0]
