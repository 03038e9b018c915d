"""Repeat-rich, rearranged inputs (npge_amd/synth.py REPEATS: IS-like element
families planted in the root and per genome, inversions; VERDICT r03 #7, the
reference's src/test/test_repeats.sh.in:1-30 plants repeats too).

DraftPangenome keeps only stem blocks (RemoveNonStem --exact), so the repeat
copies reach the aligner in AnchorLoopFast: the AnchorFinder on the consensus
sequences groups every copy of an element family -- anchor blocks of about
100 fragments in rsmall -- and FragmentsExtender aligns their flanks as
alignment problems of more than 64 rows (k_align_wide).  Engine vs the same
pipe over the oracle's processors, fragments and rows bit-exact; the
AnchorFinder's repeat property (every anchor block holds >= 2 fragments with
one text up to orientation) on the consensus sequences."""
import collections

import pytest

from npge_amd import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def canon(blocks):
    return sorted(tuple(sorted(b)) for b in blocks)


@pytest.mark.parametrize("cfg", ["rtiny", "rsmall"])
def test_repeats_draft_and_anchor_loop(cfg):
    from helpers import oracle_anchor_loop, rows_digest
    from npge_amd import _capi
    from npge_amd.anchor_finder import AnchorFinder
    from npge_amd.anchor_loop import anchor_loop_fast
    from npge_amd.blockset import BlockSetEngine
    names, seqs = synth.genome_set(cfg)
    eng = BlockSetEngine(_capi.SeqSet(seqs, names))
    eng.apply("DraftPangenome", af=AnchorFinder())
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    assert canon(eng.blocks()) == canon(o.blocks())
    st = anchor_loop_fast(eng, AnchorFinder())
    ost = oracle_anchor_loop(o)
    assert st["loop_iterations"] == ost["iterations"]
    ob = o.blocks()
    assert canon(eng.blocks()) == canon(ob)
    assert eng.rows_digest() == rows_digest(ob)
    if cfg == "rsmall":  # the wide path ran: alignment problems of more than 64 rows
        assert any(k["name"] == "align_wide" for k in eng.kernel_times()), "no problem of more than 64 rows"


def test_repeat_anchor_groups_on_consensus():
    """The consensus AnchorFinder of rsmall groups the element copies: blocks
    of more than 64 fragments, each of one text up to orientation."""
    from npge_amd import _capi
    from npge_amd.anchor_finder import AnchorFinder
    from npge_amd.blockset import BlockSetEngine
    names, seqs = synth.genome_set("rsmall")
    eng = BlockSetEngine(_capi.SeqSet(seqs, names))
    eng.apply("DraftPangenome", af=AnchorFinder())
    eng.apply("Filter").apply("Rest")
    cs = eng.conseq()
    css = _capi.SeqSet(cs, orc.cons_names(cs))
    af = AnchorFinder()
    r = af.find(css)
    bs = r["block_start"]
    sizes = collections.Counter(int(bs[b + 1] - bs[b]) for b in range(len(bs) - 1))
    assert max(sizes) > 64
    comp = str.maketrans("ATGC", "TACG")
    for b in range(len(bs) - 1):
        texts = set()
        for i in range(bs[b], bs[b + 1]):
            q, mn, mx, ori = int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i])
            t = cs[q][mn:mx + 1]
            texts.add(t if ori == 1 else t.translate(comp)[::-1])
        assert len(texts) == 1 and bs[b + 1] - bs[b] >= 2


def test_r3_draft_fullsize():
    """R3 (C3-shaped: 17 genomes, 56 Mbp, with the element families and
    inversions): DraftPangenome bit-exact at full size, rows by digest --
    the set whose aligner share is 7x C3's (Measurement)."""
    from helpers import rows_digest
    from npge_amd import _capi
    from npge_amd.anchor_finder import AnchorFinder
    from npge_amd.blockset import BlockSetEngine
    names, seqs = synth.genome_set("R3")
    eng = BlockSetEngine(_capi.SeqSet(seqs, names))
    eng.apply("DraftPangenome", af=AnchorFinder())
    o = orc.BlockSetOracle(seqs, names)
    o.set_workers(8)  # BlocksJobs threads: output identical for any count
    o.apply("DraftPangenome")
    ob = o.blocks()
    assert len(ob) > 1000
    assert canon([[f[:4] for f in b] for b in eng.blocks()]) == canon([[f[:4] for f in b] for b in ob])
    assert eng.rows_digest() == rows_digest(ob)
