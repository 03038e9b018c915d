"""The pair-sharded job as bench.py runs it: 16 pairs at a
time on 20 hardware queues per process (bench.py --pair-workers 16
--hw-queues 20).  GPU_MAX_HW_QUEUES is read when HIP initialises, so the run
is a child process that sets it before its first GPU call; the child
compares the 16-worker run with a 1-worker run of the same 32 C4 pairs
(fragment records, blockset hashes, rows digests) and two pairs against the
CPU restatement, rows included."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
from npge_amd import _capi, pairs, synth
_capi.check(_capi.lib().npgx_set_device(0))
from test_pairs_gpu import _oracle_pair, _canon, rows_digest
names, seqs = synth.genome_set("C4")
sample = pairs.all_pairs(names)[:32]
one = pairs.PairJobs(names, seqs, workers=1, pairs=sample)
many = pairs.PairJobs(names, seqs, workers=16, pairs=sample)
i1, i16 = one.run(), many.run()
assert i1["aligned_residues"] == i16["aligned_residues"] > 0
r1, r16 = one.local_records(), many.local_records()
assert np.array_equal(r1[0], r16[0]) and np.array_equal(r1[1], r16[1])
d1, d16 = one.row_digests(), many.row_digests()
assert d1 == d16 and len(set(d16.values())) == len(sample)
for k in (3, 29):
    o = _oracle_pair(names, seqs, sample[k])
    ob = o.blocks()
    eng = many.jobs[k][2].eng
    assert eng.hash() == o.hash()
    assert eng.rows_digest() == rows_digest(ob)
    assert _canon(eng.blocks(), rows=True) == _canon(ob, rows=True)
print("OK", len(sample), "pairs", i16["aligned_residues"], "residues")
"""


def test_pairs_16_workers_20_queues():
    env = dict(os.environ, GPU_MAX_HW_QUEUES="20", HSA_ENABLE_IPC_MODE_LEGACY="0")
    code = CHILD.replace("ROOT", repr(ROOT))
    p = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert p.stdout.strip().splitlines()[-1].startswith("OK 32 pairs")
