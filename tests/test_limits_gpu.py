"""The engine's size limits are refused loudly (NPGX_ERR_RANGE / ARG), never
wrapped or cut short, and the largest allowed values still match the oracle:
AnchorFinder's 32-bit window orders (at most 2^32 - 2 bases per run; the
refusal exercised through NPGX_AF_MAX_BASES, which lowers the limit),
aligned-check <= 16 (48-bit word keys), GeneralAligner gap_range <= 63 (one
wave per pair)."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def test_aligned_check_edge():
    from npge_amd import _capi
    from npge_amd.aligner import BatchAligner
    from test_similar_aligner_gpu import _random_jobs
    jobs = _random_jobs(11, 60, nmax=8, lmax=200)
    got = BatchAligner(aligned_check=16).align(jobs)
    for job, g in zip(jobs, got):
        assert g == orc.align(job, mode="align_seqs", params=(1, 2, 16, 100, 9000))
    with pytest.raises(_capi.NpgxError):
        BatchAligner(aligned_check=17)


def test_gap_range_edge():
    from npge_amd import _capi
    from npge_amd.dp import GeneralAligner
    rng = np.random.default_rng(5)
    a = "".join("ACGT"[k] for k in rng.integers(0, 4, 300))
    b = a[:100] + a[160:]
    r = GeneralAligner(gap_range=63, max_errors=-1).align_batch([(a, b)])
    o = orc.general_align(a, b, 63, -1)
    assert int(r["score"][0]) == o["score"]
    with pytest.raises(_capi.NpgxError):
        GeneralAligner(gap_range=64, max_errors=-1).align_batch([(a, b)])


def test_anchor_finder_order_limit():
    """A run over more bases than the 32-bit orders hold fails with
    NPGX_ERR_RANGE (limit lowered to 10 kb for the test; a fresh process
    because the library reads the variable once)."""
    code = textwrap.dedent('''
        import os, sys
        os.environ["NPGX_AF_MAX_BASES"] = "10000"
        sys.path.insert(0, ".")
        from npge_amd import _capi
        from npge_amd.anchor_finder import AnchorFinder
        import numpy as np
        rng = np.random.default_rng(1)
        seqs = ["".join("ACGT"[k] for k in rng.integers(0, 4, n)) for n in (6000, 3000)]
        ss = _capi.SeqSet(seqs, ["a&c&c", "b&c&c"])
        AnchorFinder().find(ss)  # 9000 bases: allowed
        ss2 = _capi.SeqSet(seqs + seqs[:1], ["a&c&c", "b&c&c", "c&c&c"])
        try:
            AnchorFinder().find(ss2)
        except _capi.NpgxError as e:
            assert "2^32" in str(e), e
            print("refused")
        ''')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=root)
    assert out.returncode == 0, out.stderr
    assert "refused" in out.stdout
