#!/bin/bash
# round 6: the device loop reads the aligner's kernel timers once after the
# loop instead of after every iteration (libnpge_amd_alt.so: every
# iteration): the loop's tests and the bench's kernel times, A/B at C3 / C2
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06x
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py tests/test_bench_gpu.py tests/test_fullsize_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C2; do
  step "timers once (new) vs each iteration (alt), $cfg"
  timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 3 --config $cfg --steps 10 --no-pairs-line > $O/ab_timers_$cfg.txt 2>&1 || { tail -5 $O/ab_timers_$cfg.txt; exit 1; }
  cut -c1-150 $O/ab_timers_$cfg.txt
done
python - <<'PY'
import json
d = json.loads(open("gpurun_out/ab_new.log").read().strip().splitlines()[-1])
print("kernels_last_step", d.get("kernels_last_step"), "roofline avg_launch_ms", (d.get("roofline") or {}).get("avg_launch_ms"))
PY
step done
