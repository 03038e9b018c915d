"""Parity at BASELINE.json's full single-GPU sizes: the C2 (3 genomes, 9.9 Mbp)
and C3 (17 genomes, 56 Mbp) synthetic sets.  AnchorFinder's SoA anchor set and
the whole DraftPangenome (AnchorFinder -> RemoveNonStem -> DummyAligner ->
ExtendLoopFast(10) -> Filter) on the GPU engine vs the CPU restatement:
fragments and gapped rows bit-exact, the reference's blockset_hash equal.
The oracle needs about 3 s (C2) and 12 s (C3) per DraftPangenome here."""
import pytest

from oracle import oracle as orc
from npge_amd import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_anchor_finder_fullsize(cfg):
    from test_anchor_finder_gpu import _assert_same, _run_both
    names, seqs = synth.genome_set(cfg)
    (rg, ro, used), = _run_both(seqs, names)
    _assert_same(rg, ro, used)
    assert len(rg["block_start"]) > 1000


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_draft_pangenome_fullsize(cfg):
    from npge_amd import _capi
    from npge_amd.anchor_finder import AnchorFinder
    from npge_amd.blockset import BlockSetEngine
    names, seqs = synth.genome_set(cfg)
    eng = BlockSetEngine(_capi.SeqSet(seqs, names))
    eng.apply("DraftPangenome", af=AnchorFinder())
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    st, ost = eng.stats(), o.stats()
    for k in ("anchor_blocks", "stem_blocks", "iterations", "aligned_residues"):
        assert st[k] == ost[k], k
    got, want = eng.blocks(), o.blocks()
    assert sorted(tuple(sorted(b)) for b in got) == sorted(tuple(sorted(b)) for b in want)
    assert eng.hash() == o.hash()
    assert sum(len(b) for b in got) > 100
