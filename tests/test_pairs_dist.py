"""Host side of the pair-sharded block build (npge_amd/pairs.py) on CPU: the
pair list and its round-robin assignment (every pair on exactly one rank),
the fragment record packing, and the final gather over an npgx_comm with
world sizes 2 and 3 over gloo (host buffers and ctypes.memmove stand in for
device buffers, as the library's callbacks see them): every rank ends with
the records of all ranks in rank order, ragged and empty shares included."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from npge_amd import pairs, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_pairs_and_assignment():
    names, _ = synth.genome_set("tiny")          # 3 genomes x 2 chromosomes
    g = pairs.genomes_of(names)
    assert list(g.values()) == [[0, 1], [2, 3], [4, 5]]
    ps = pairs.all_pairs(names)
    assert ps == [(0, 1, 2, 3), (0, 1, 4, 5), (2, 3, 4, 5)]
    c4 = ["G%02d&chr1&c" % (i + 1) for i in range(32)]
    assert len(pairs.all_pairs(c4)) == 32 * 31 // 2
    for world in (1, 2, 3, 8):
        got = sorted(p for r in range(world) for p in pairs.assign(496, r, world))
        assert got == list(range(496))
        sizes = [len(pairs.assign(496, r, world)) for r in range(world)]
        assert max(sizes) - min(sizes) <= 1


def _blocks(rng, nb, nseq):
    bs = np.zeros(nb + 1, dtype=np.int64)
    np.cumsum(rng.integers(1, 5, nb), out=bs[1:])
    nf = int(bs[-1])
    seq = rng.integers(0, nseq, nf).astype(np.int32)
    mn = rng.integers(0, 5_000_000, nf).astype(np.int64)
    mx = mn + rng.integers(0, 20000, nf)
    ori = np.where(rng.random(nf) < 0.5, 1, -1).astype(np.int8)
    return bs, seq, mn, mx, ori


def test_record_round_trip():
    rng = np.random.default_rng(3)
    bs, seq, mn, mx, ori = _blocks(rng, 300, 2047)   # up to 2047 sequences in a pair
    rec = pairs.pack_fragments(495, bs, seq, mn, mx, ori)
    assert rec.dtype == np.uint64 and len(rec) == 2 * int(bs[-1])
    got = pairs.unpack_fragments(rec)[495]
    want = [[(int(seq[i]), int(mn[i]), int(mx[i]), int(ori[i])) for i in range(bs[b], bs[b + 1])]
            for b in range(300)]
    assert got == want
    assert len(pairs.pack_fragments(7, np.zeros(1, dtype=np.int64), seq[:0], mn[:0], mx[:0], ori[:0])) == 0


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from npge_amd.comm import TorchComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = TorchComm(dist, staging="cpu", copy=ctypes.memmove)
    recs = []
    for p in pairs.assign(10, rank, world):
        if p == 4:                       # a pair with no blocks
            continue
        recs.append(pairs.pack_fragments(p, *_blocks(np.random.default_rng(p), 5 + p, 3)))
    mine = np.concatenate(recs) if recs else np.zeros(0, dtype=np.uint64)
    got, counts = pairs.gather_u64(c, mine)
    out[rank] = (got, counts)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_over_gloo(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    want = {p: pairs.unpack_fragments(pairs.pack_fragments(p, *_blocks(np.random.default_rng(p), 5 + p, 3)))[p]
            for p in range(10) if p != 4}
    for r in range(world):
        got, counts = out[r]
        assert len(got) == sum(counts)
        assert np.array_equal(got, out[0][0])
        assert pairs.unpack_fragments(got) == want


def test_pair_cpu_baseline_record(monkeypatch):
    """bench.py's CPU leg for the pair job: the oracle's DraftPangenome on one
    pair, timed (no GPU), median of >= 3 runs; and the allotted-cores leg, as
    many pairs at once as cores in spawned processes.  The record names its
    samples and cores."""
    import bench
    names, seqs = synth.genome_set("tiny")
    sel = pairs.all_pairs(names)
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    r = bench.cpu_baseline_pair(names, seqs, sel, 1)
    assert r["value"] > 0 and r["cores"] == 1 and r["kind"] == "port" and len(r["runs_s"]) == 3
    assert "G01" in r["sample"] and "G02" in r["sample"] and r["workload"] == "DraftPangenome"
    a = r["allotted_cores"]
    assert a["value"] > 0 and a["cores"] == min(2, len(sel))
