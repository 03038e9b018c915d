"""AnchorFinder parity: HIP engine (through the C ABI) vs the CPU restatement.

Bit-exact on the SoA anchor set (block boundaries, sequence, min, max, ori in
reference order), the Bloom sizing/parameters, |H|, the FoundFragment count and
the persistent used-hash set.  Inputs: the reference's own fixtures
(test-script/anchor_finder, src/test/anchor_finder.cpp) and seeded synthetic
genome sets, including N runs, palindromes, repeats, truncation by
max-anchor-fragments, anchor-similar=false, k=32 and repeated runs on one
instance.
"""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from npge_amd import io as nio
from npge_amd import synth
from npge_amd.model import Sequence, normalized_blocks

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _gpu_af(**kw):
    from npge_amd.anchor_finder import AnchorFinder
    p = AnchorFinder(bloom_params=kw.pop("params", None))
    for k, v in kw.items():
        p.set_opt_value(k.replace("_", "-"), v)
    return p


def _run_both(seqs, names, k=20, seed=1, fp="0.1", similar=True, maxf=100000, params=None,
              repeats=1):
    from npge_amd import _capi
    ss = _capi.SeqSet(seqs, names)
    g = _gpu_af(anchor_size=k, bloom_seed=seed, anchor_fp=fp, anchor_similar=similar,
                max_anchor_fragments=maxf, params=params)
    fp_x = int(round(float(fp) * 10000))
    o = orc.AnchorFinder(anchor_size=k, anchor_fp_x1e4=fp_x, anchor_similar=similar,
                         max_anchor_fragments=maxf, seed=seed, params=params)
    out = []
    for _ in range(repeats):
        rg = g.find(ss)
        ro = o.run(seqs, names)
        out.append((rg, ro, g.used_hashes()))
    return out


def _assert_same(rg, ro, used_g=None):
    assert rg["members"] == ro["members"]
    assert rg["bits"] == ro["bits"]
    assert rg["hashes"] == ro["hashes"]
    assert list(rg["params"]) == list(ro["params"])
    assert rg["n_collected"] == ro["n_collected"]
    assert rg["n_found_frags"] == ro["n_found_frags"]
    for key in ("block_start", "seq", "min_pos", "max_pos", "ori"):
        np.testing.assert_array_equal(np.asarray(rg[key], dtype=np.int64),
                                      np.asarray(ro[key], dtype=np.int64), err_msg=key)
    if used_g is not None:
        np.testing.assert_array_equal(used_g, ro["used"])


@pytest.mark.parametrize("case", ["1", "bug-n-in-init-frame", "complement-no-inverse",
                                  "inverse", "inverse-no-complement"])
@pytest.mark.parametrize("seed", [1, 7])
def test_script_fixtures(case, seed):
    d = os.path.join(GOLD, "anchor_finder", case)
    recs = list(nio.read_fasta(open(os.path.join(d, "in.fasta")).read()))
    exp = nio.read_blockset(open(os.path.join(d, "out.fasta")).read())
    names = [n for n, _, _ in recs]
    seqs = [nio.to_atgcn(r) for _, _, r in recs]
    (rg, ro, used), = _run_both(seqs, names, k=20, seed=seed)
    _assert_same(rg, ro, used)
    from helpers import af_blocks_from_result
    got = af_blocks_from_result(rg, [Sequence(n, s) for n, s in zip(names, seqs)])
    assert normalized_blocks(got) == normalized_blocks(exp.blocks)


@pytest.mark.parametrize("seqs,k", [(["tgGTCCGagCGGACggcc"], 5), (["tgGTNCGagCGNACggcc"], 5),
                                    (["GTNCGATAnnnGTNCGATA"], 5), (["ATGCAT"], 6),
                                    (["GAAAGAAA"], 3), (["GAAAGAAA", "GAAAGAAA"], 3),
                                    (["A" * 50, "T" * 40, "ACGT" * 30], 4), ([""], 5),
                                    (["ACG"], 5)])
def test_unit_cases(seqs, k):
    seqs = [orc.to_atgcn(s) for s in seqs]
    names = ["s%d" % i for i in range(len(seqs))]
    for seed in (1, 2, 3):
        (rg, ro, used), = _run_both(seqs, names, k=k, seed=seed)
        _assert_same(rg, ro, used)


@pytest.mark.parametrize("config", ["tiny", "small"])
@pytest.mark.parametrize("k,similar,maxf,fp", [(20, True, 100000, "0.1"), (15, False, 100000, "0.1"),
                                               (20, True, 500, "0.1"), (32, True, 100000, "0.01"),
                                               (11, True, 100000, "0.3")])
def test_synthetic(config, k, similar, maxf, fp):
    names, seqs = synth.genome_set(config)
    (rg, ro, used), = _run_both(seqs, names, k=k, similar=similar, maxf=maxf, fp=fp)
    _assert_same(rg, ro, used)


def test_repeated_runs_used_hashes():
    names, seqs = synth.genome_set("tiny")
    for rg, ro, used in _run_both(seqs, names, k=20, maxf=300, repeats=4):
        _assert_same(rg, ro, used)


def test_explicit_params():
    names, seqs = synth.genome_set("tiny")
    (rg, ro, used), = _run_both(seqs, names, params=[12345, 67890, 4242424242, 7])
    _assert_same(rg, ro, used)


def test_consensus_naming_and_ties():
    # single "genome" -> consensus sizing (AnchorFinder.cpp:90-92); equal-size
    # sequences ranked by name (pinned tie-break)
    rng = np.random.default_rng(5)
    base = "".join("ATGC"[i] for i in rng.integers(0, 4, 3000))
    seqs = [base, base[::-1], base[100:] + base[:100], base]
    names = ["c3", "c1", "c2", "c0"]
    (rg, ro, used), = _run_both(seqs, names, k=12)
    _assert_same(rg, ro, used)


@pytest.mark.parametrize("epochs", [1, 2, 3, 7, 40])
def test_bloom_epochs_same_result(epochs):
    """The epoch-filtered Bloom pass (bit array of the earlier epochs skipping
    atomics and first[] reads) gives the reference's result for any epoch
    split, including epochs that cut a sequence and the repeated-run used set."""
    from npge_amd import _capi
    names, seqs = synth.genome_set("small")
    ss = _capi.SeqSet(seqs, names)
    g = _gpu_af(anchor_size=20, bloom_seed=3, max_anchor_fragments=20000)
    g.set_opt_value("bloom-epochs", epochs)
    o = orc.AnchorFinder(anchor_size=20, anchor_fp_x1e4=1000, anchor_similar=True,
                         max_anchor_fragments=20000, seed=3)
    for _ in range(2):
        rg = g.find(ss)
        ro = o.run(seqs, names)
        _assert_same(rg, ro, g.used_hashes())
