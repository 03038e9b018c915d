"""The bench line's stage accounting (bench.py "stage_timeline"): the GPU
timeline of one extra, untimed DraftPangenome step split at its stage
boundaries by HIP events (npgx_blockset_tune "stage-clock").  On the recorded
round-6 lines the stages must sum to within 10 % of the line's ms_per_step
and name the aligner, not the hash, as the largest stage; the host-side
stage wall times of the device loop are enqueue times and are reported apart
(last_step.ms_stage_host)."""
import glob
import json
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (DraftPangenome lines: with --anchor-loop the clock splits the DraftPangenome
# part only, and the line says so in stage_timeline.scope)
LINES = sorted(p for p in glob.glob(os.path.join(REPO, "profiles", "r06*_bench_C[23]*.json")) if "_alf" not in p)


def _line(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


@pytest.mark.parametrize("path", LINES, ids=[os.path.basename(p) for p in LINES])
def test_recorded_stages_sum_to_the_step(path):
    d = _line(path)
    st = d["stage_timeline"]
    total = sum(st["ms"].values())
    assert abs(total - st["sum_ms"]) < 0.01 * max(total, 1.0)
    assert abs(total - d["ms_per_step"]) <= 0.10 * d["ms_per_step"], (total, d["ms_per_step"])
    assert st["largest"] == "align" == max(st["ms"], key=st["ms"].get)
    ls = d["last_step"]
    assert "ms_stage" not in ls and "ms_stage_host" in ls
    if ls.get("device_loop"):
        assert "ms_align_wall" not in ls  # (enqueue time only in the device loop)


def test_some_line_is_recorded():
    assert LINES, "no round-6 C2/C3 bench line under profiles/"
