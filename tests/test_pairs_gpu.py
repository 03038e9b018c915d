"""Pair-sharded block build (npge_amd/pairs.py, BASELINE C4's split) on the
GPU: every genome pair's DraftPangenome, run several pairs at a time on their
own host threads and streams, equals the CPU restatement's DraftPangenome on
that pair (blockset hash, fragment coordinates AND gapped rows: the rows
themselves and the device rows digest the gather carries); the 12-worker
concurrent run (shared aligner scratch) equals the one-at-a-time run row for
row; and the pair jobs split over 2 gloo ranks on the box's GPU gather to the
one-rank records on every rank."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from npge_amd import pairs, synth
from helpers import rows_digest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_pair(names, seqs, idx):
    from oracle import oracle as orc
    o = orc.BlockSetOracle([seqs[i] for i in idx], [names[i] for i in idx])
    o.apply("DraftPangenome")
    return o


def _canon(blocks, rows=False):
    return sorted(tuple(sorted(f if rows else f[:4] for f in b)) for b in blocks)


@pytest.mark.parametrize("workers", [1, 3])
def test_pairs_equal_oracle(workers):
    names, seqs = synth.genome_set("small")      # 5 genomes -> 10 pairs
    job = pairs.PairJobs(names, seqs, workers=workers)
    assert len(job.pairs) == 10
    info = job.run()
    assert info["gathered_pairs"] == 10          # one rank: its records are the whole job
    assert info["stem_blocks"] > 0 and info["aligned_residues"] > 0
    digests = job.row_digests()
    for p, _, bb in job.jobs:
        o = _oracle_pair(names, seqs, job.pairs[p])
        ob = o.blocks()
        assert bb.eng.hash() == o.hash(), "pair %d" % p
        assert _canon(bb.eng.blocks(), rows=True) == _canon(ob, rows=True), "pair %d" % p
        # the gathered summary's device digest is the oracle rows' digest
        assert digests[p] == bb.eng.rows_digest() == rows_digest(ob), "pair %d" % p


def test_pairs_concurrent_equal_sequential_c4():
    names, seqs = synth.genome_set("C4")
    sample = pairs.all_pairs(names)[:24]         # 2 x 5 Mbp each, 2 % divergence
    a = pairs.PairJobs(names, seqs, workers=1, pairs=sample)
    b = pairs.PairJobs(names, seqs, workers=12, pairs=sample)  # the bench's 12 workers, shared scratch
    ia, ib = a.run(), b.run()
    assert ia["aligned_residues"] == ib["aligned_residues"] > 0
    ra, rb = a.local_records(), b.local_records()
    # coordinates, blockset hashes and rows digests of every pair
    assert np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1], rb[1])
    assert a.row_digests() == b.row_digests() and len(set(a.row_digests().values())) == len(sample)
    # a second pass over the same resident pairs does the identical work
    b.run()
    assert np.array_equal(b.local_records()[0], ra[0]) and b.row_digests() == a.row_digests()
    # two C4 pairs against the CPU restatement, rows included
    for k in (0, 13):
        o = _oracle_pair(names, seqs, sample[k])
        ob = o.blocks()
        eng = b.jobs[k][2].eng
        assert eng.hash() == o.hash()
        assert eng.rows_digest() == rows_digest(ob)
        assert _canon(eng.blocks(), rows=True) == _canon(ob, rows=True)


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from npge_amd import _capi
    from npge_amd.comm import TorchComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _capi.check(_capi.lib().npgx_set_device(0))
    names, seqs = synth.genome_set("small")
    comm = TorchComm(dist, staging="cpu")
    job = pairs.PairJobs(names, seqs, rank=rank, world=world, comm=comm, workers=2)
    info = job.run()
    out[rank] = (job.records, job.summary, info["pairs_rank"])
    dist.barrier()
    dist.destroy_process_group()


def test_pairs_sharded_gather_equals_single():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    names, seqs = synth.genome_set("small")
    one = pairs.PairJobs(names, seqs, workers=2)
    one.run()
    frs, sums = one.local_records()
    want_f = pairs.unpack_fragments(frs)
    want_h = {int(r[0] >> 32): (int(r[1]), int(r[2])) for r in sums.reshape(-1, pairs.SUMMARY_WORDS).tolist()}
    assert out[0][2] + out[1][2] == 10
    for r in range(world):
        rec, summ, _ = out[r]
        assert pairs.unpack_fragments(rec) == want_f
        assert {int(r[0] >> 32): (int(r[1]), int(r[2]))
                for r in summ.reshape(-1, pairs.SUMMARY_WORDS).tolist()} == want_h
