"""DraftPangenome's anchors on the device (anchors_to_device, elf_device.inc):
the AnchorFinder's sorted FoundFragment keys -> groups -> RemoveNonStem
--exact -> the DummyAligner's rows -> the device ExtendLoopFast's first
table, with no host blocks in between.  Checked against the host path
(NPGX_ANCHOR_DEVICE=0: the AnchorFinder groups on the host, add_anchors,
dummy_align, the table upload) and the oracle; the AnchorFinder's own result,
statistics and used-hash set after a deferred run equal a plain run's (its
host grouping then runs when they are asked for, AnchorFinder.cpp:356-391)."""
import numpy as np
import pytest

from oracle import oracle as orc
from npge_amd import synth
from npge_amd.anchor_finder import AnchorFinder

from test_block_build_gpu import _engine, canon

pytestmark = pytest.mark.gpu


def _draft(seqs, names, anc, monkeypatch, runs=1, clear=False):
    monkeypatch.setenv("NPGX_ANCHOR_DEVICE", anc)
    ss, eng = _engine(seqs, names)
    af = AnchorFinder()
    out = []
    for _ in range(runs):
        if clear:
            af.clear_used()
        eng.apply("DraftPangenome", af=af)
        st = eng.stats()
        r = af.result()
        out.append((canon(eng.blocks()), eng.rows_digest(), st["anchor_blocks"], st["stem_blocks"],
                    st["iterations"], st["device_iterations"] > 0,
                    [r[k].tolist() for k in ("block_start", "seq", "min_pos", "max_pos", "ori")],
                    af.used_hashes().tolist()))
    return out


@pytest.mark.parametrize("cfg", ["tiny", "small", "rtiny", "rsmall"])
def test_draft_anchors_on_device_equal_host_path(cfg, monkeypatch):
    names, seqs = synth.genome_set(cfg)
    dev = _draft(seqs, names, "1", monkeypatch)
    host = _draft(seqs, names, "0", monkeypatch)
    assert dev == host
    assert dev[0][5]  # (the device loop ran)
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    assert dev[0][0] == canon(o.blocks())


def test_deferred_anchor_finder_keeps_its_used_set(monkeypatch):
    """Three runs on one AnchorFinder handle without clearing it: every run
    after the first skips the hashes the earlier ones used (the persistent
    set, AnchorFinder.cpp:30-35), so a deferred run's used hashes must reach
    the set before the next run; then with the set cleared between runs."""
    names, seqs = synth.genome_set("small")
    for clear in (False, True):
        dev = _draft(seqs, names, "1", monkeypatch, runs=3, clear=clear)
        host = _draft(seqs, names, "0", monkeypatch, runs=3, clear=clear)
        assert dev == host
        if not clear:
            assert len(dev[2][7]) > len(dev[0][7])


def test_many_genomes_take_the_host_path(monkeypatch):
    """More than 64 genomes: the stem test's set does not fit 64 bits and the
    anchors go through the host (the same result either way)."""
    rng = np.random.default_rng(4)
    root = rng.integers(0, 4, size=3000)
    seqs, names = [], []
    for g in range(66):
        s = root.copy()
        m = rng.random(s.size) < 0.002
        s[m] = (s[m] + 1) % 4
        seqs.append("".join("ACGT"[c] for c in s))
        names.append("h%d&c&c" % g)
    dev = _draft(seqs, names, "1", monkeypatch)
    host = _draft(seqs, names, "0", monkeypatch)
    assert dev == host
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    assert dev[0][0] == canon(o.blocks())
