"""bench.py's multi-rank paths on the GPU box's one GPU: two ranks launched by
torch.distributed.run with the gloo backend (rehearsal of the driver's RCCL
runs; ranks share the GPU), replicas, sharded and pairs modes.  Checks the
JSON contract fields, that the sharded line reports one set's bp, and the
secondary lines (one set sharded / replicas, the pair-sharded job)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["replicas", "sharded", "pairs"])
def test_bench_two_ranks_gloo(mode):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--steps", "1", "--warmup", "1", "--config", "small", "--mode", mode,
           "--dist-backend", "gloo", "--no-cpu-baseline", "--pairs-config", "small", "--pair-workers", "2"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["value"] > 0
    if mode == "pairs":  # 10 pairs of the 5-genome set over 2 ranks, all gathered on rank 0
        assert d["scaling"] == "strong" and d["config"]["pairs"] == 10
        assert d["last_step"]["gathered_pairs"] == 10 and d["last_step"]["pairs_rank"] == 5
        assert abs(d["value"] - d["config"]["bp_job"] / (d["ms_per_step"] / 1e3) / 1e6) / d["value"] < 1e-3
        return
    assert d["pairs"]["value"] > 0 and d["pairs"]["last_step"]["gathered_pairs"] == 10
    bp = d["config"]["bp_per_rank"]
    ranks = 1 if mode == "sharded" else 2
    assert abs(d["value"] - bp * ranks / (d["ms_per_step"] / 1e3) / 1e6) / d["value"] < 1e-3
    assert d["scaling"] == ("strong" if mode == "sharded" else "weak")
    if mode == "sharded":  # the secondary replica-mode measurement of the same step
        assert d["replicas"]["value"] > 0 and d["replicas"]["scaling"] == "weak"
    else:                  # the secondary one-set sharded measurement
        assert d["sharded"]["value"] > 0 and d["sharded"]["scaling"] == "strong"


def test_bench_gpus_two_self_launched():
    """--gpus 2 with no launcher: bench.py starts the two ranks itself."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1", "--config", "small",
           "--dist-backend", "gloo", "--no-cpu-baseline", "--no-pairs-line", "--no-replicas-line"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["comm_ranks"] == 2 and d["launcher"].startswith("bench.py")
    assert abs(d["value"] - d["config"]["bp_per_rank"] * 2 / (d["ms_per_step"] / 1e3) / 1e6) / d["value"] < 1e-3
