"""The library's own RCCL communicator (npgx_rccl_comm_create, csrc/comm_rccl.hip)
on the box's one GPU: a world of one rank (RCCL refuses two ranks on one
GPU; the multi-rank paths are the same calls), every collective checked by
npgx_comm_check, and the TorchComm callbacks over gloo through the same
check with two ranks."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code, world=1):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29650 + world), WORLD_SIZE=str(world))
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-c", textwrap.dedent(code)], cwd=ROOT, env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    return [o for o, _ in outs]


def test_rccl_world_one():
    out = _run('''
        import sys
        sys.path.insert(0, ".")
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from npge_amd import _capi, comm
        _capi.check(_capi.lib().npgx_set_device(0))
        c = comm.RcclComm(dist, 0)
        comm.check(c)
        c.close()
        print("ok")
    ''')
    assert out[0].strip().endswith("ok")


def test_torch_comm_check_gloo_two_ranks():
    """TorchComm (gloo, host staging, the library's device buffers copied
    through npgx_memcpy) through npgx_comm_check on two ranks sharing the GPU."""
    out = _run('''
        import sys
        sys.path.insert(0, ".")
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from npge_amd import _capi, comm
        _capi.check(_capi.lib().npgx_set_device(0))
        c = comm.TorchComm(dist, staging="cpu")
        comm.check(c)
        print("ok")
    ''', world=2)
    assert all(o.strip().endswith("ok") for o in out)


def test_rccl_world_one_pair_gather():
    """The pair-sharded job's final gather through the library's RCCL
    communicator with device exchange buffers (the driver's N > 1 path):
    at world size 1 the gathered records equal the rank's own."""
    out = _run('''
        import sys
        sys.path.insert(0, ".")
        import numpy as np
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from npge_amd import _capi, comm, pairs, synth
        _capi.check(_capi.lib().npgx_set_device(0))
        c = comm.RcclComm(dist, 0)
        names, seqs = synth.genome_set("tiny")
        job = pairs.PairJobs(names, seqs, comm=c, workers=2, gather_device=torch.device("cuda", 0))
        info = job.run()
        frs, sums = job.local_records()
        assert info["gathered_pairs"] == 3 and len(frs) > 0
        assert np.array_equal(job.records, frs) and np.array_equal(job.summary, sums)
        del job
        c.close()
        print("ok")
    ''')
    assert out[0].strip().endswith("ok")
