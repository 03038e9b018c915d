#!/bin/bash
# round 6: chain copies with their row loads batched; twins within 512
# tasks; the table passes' single-workgroup switch point (NPGX_ELF_PASS_WG)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06g
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_fullsize_gpu.py tests/test_repeats_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in C3 C2; do
  step "ab pass wg $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06g NPGX_ELF_PASS_WG 2048 256 --config $cfg --steps 10 --warmup 3 || exit 1
done
cd /tmp
step "rocprof C3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
python3 $R/tools/align_iters.py $O/prof_c3/run_kernel_trace.csv
step done
