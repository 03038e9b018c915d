"""The collective adapter of the sharded AnchorFinder (npge_amd/comm.py) with
world_size 2 and 3 over gloo on CPU: the npgx_comm callbacks are invoked through
their C function pointers exactly as the library calls them (host buffers and
ctypes.memmove stand in for device buffers and npgx_memcpy), and the exact
sharding's host arithmetic (chunk ranges, sign-flipped MIN) is checked against
the single-rank answer."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flip(a):
    return (a.astype(np.uint32) ^ np.uint32(0x80000000)).view(np.int32)


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from npge_amd.comm import NPGX_OP_MIN, NPGX_OP_SUM, TorchComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = TorchComm(dist, staging="cpu", copy=ctypes.memmove)
    s = c.struct
    assert (s.rank, s.world) == (rank, world)
    rng = np.random.default_rng(100 + rank)

    # first-setter MIN over ranks of uint32 orders (0xFFFFFFFF = unset), through
    # the order-preserving int32 flip the library applies around the call
    first = rng.integers(0, 2**32, 1000, dtype=np.uint64).astype(np.uint32)
    first[rank::3] = 0xFFFFFFFF
    buf = _flip(first).copy()
    assert s.allreduce_i32(None, buf.ctypes.data, len(buf), NPGX_OP_MIN) == 0
    got_min = (buf.view(np.uint32) ^ np.uint32(0x80000000)).astype(np.uint32)

    cnt = np.arange(50, dtype=np.int32) * (rank + 1)
    assert s.allreduce_i32(None, cnt.ctypes.data, len(cnt), NPGX_OP_SUM) == 0

    allv = (ctypes.c_int64 * world)()
    n_local = [0, 7, 3][rank]                 # ragged, one rank empty
    assert s.allgather_i64(None, n_local, allv) == 0
    counts = [allv[r] for r in range(world)]
    src = np.arange(n_local, dtype=np.uint64) + np.uint64(1000 * rank + (1 << 63))
    dst = np.zeros(max(1, sum(counts)), dtype=np.uint64)
    assert s.allgatherv_u64(None, src.ctypes.data if n_local else 0, allv, dst.ctypes.data) == 0
    out[rank] = (first, got_min, cnt, counts, dst[:sum(counts)])
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_comm_callbacks_gloo(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    firsts = [out[r][0] for r in range(world)]
    want_min = np.minimum.reduce(firsts)
    want_cnt = np.arange(50, dtype=np.int32) * sum(r + 1 for r in range(world))
    counts = [[0, 7, 3][r] for r in range(world)]
    want_cat = np.concatenate([np.arange(n, dtype=np.uint64) + np.uint64(1000 * r + (1 << 63))
                               for r, n in enumerate(counts)])
    for r in range(world):
        _, got_min, cnt, cs, cat = out[r]
        np.testing.assert_array_equal(got_min, want_min)
        np.testing.assert_array_equal(cnt, want_cnt)
        assert cs == counts
        np.testing.assert_array_equal(cat, want_cat)


def test_chunk_ranges_cover_once():
    """The library splits chunks [n*r/W, n*(r+1)/W): every chunk exactly once."""
    for n in (0, 1, 5, 1000, 38671):
        for W in (1, 2, 3, 8):
            seen = []
            for r in range(W):
                seen.extend(range(n * r // W, n * (r + 1) // W))
            assert seen == list(range(n))
