"""The opt-in buffer cache (NPGX_BUF_CACHE=1, seqset.hip buf_alloc / buf_free):
freed device and pinned buffers are reused by size class after one device
synchronisation, reused device buffers zeroed.  The setting is read once per
process, so the check runs in a child: the smoke pipeline (DraftPangenome on
the GPU, bit-exact against the oracle) three times in one process, the later
runs on buffers the earlier ones freed."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_smoke_with_buffer_cache():
    env = dict(os.environ, NPGX_BUF_CACHE="1")
    code = "import __graft_entry__ as g\nfor _ in range(3): g.smoke()\n"
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count("smoke ok") == 3, r.stdout[-2000:]
