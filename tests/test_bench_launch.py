"""bench.py's rank launch on CPU (no GPU call): `--gpus N` without a launcher
starts N ranks itself (torch.distributed.run children, before any GPU call in
the parent), every rank joins the process group and the npgx_comm binding
sees N ranks; a --gpus / WORLD_SIZE mismatch exits non-zero."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _line(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout + out.stderr[-2000:]
    return json.loads(lines[0])


def test_gpus_two_launches_two_ranks():
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--config", "tiny",
           "--no-cpu-baseline", "--launch-check"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=_env())
    assert out.returncode == 0, out.stderr[-2000:]
    d = _line(out)
    assert d["n_gpus"] == 2 and d["comm_ranks"] == 2
    assert d["launcher"].startswith("bench.py")


def test_gpus_one_stays_one_process():
    cmd = [sys.executable, "bench.py", "--gpus", "1", "--launch-check"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=120, env=_env())
    assert out.returncode == 0, out.stderr[-2000:]
    d = _line(out)
    assert d["n_gpus"] == 1 and d["comm_ranks"] == 1


def test_world_size_mismatch_exits_nonzero():
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--launch-check"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=120,
                         env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert out.returncode != 0
    assert "WORLD_SIZE" in out.stderr
