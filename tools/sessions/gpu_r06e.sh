#!/bin/bash
# round 6: the prefix search's first prefixes in the LDS word table, the
# OverlaplessUnion admission without rounds for conflict-free chunks; where
# the unsplit twins' time goes (kernel traces with and without them)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06e
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_elf_device_gpu.py tests/test_repeats_gpu.py tests/test_fullsize_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in C3 R3; do
  step "ab long lds $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06e NPGX_LONG_LDS 0 1 --config $cfg --steps 10 --warmup 3 || exit 1
done
cd /tmp
for tw in 0 3; do
  step "rocprof C3 utwins $tw"
  NPGX_UTWINS=$tw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_tw$tw -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3_tw$tw.log 2>&1 || { tail -5 $O/prof_c3_tw$tw.log; exit 1; }
done
step done
