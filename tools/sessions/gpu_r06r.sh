#!/bin/bash
# round 6: the table passes with batched fragment loads (OverlaplessUnion's
# small-table kernels and the AnchorFinder tallies reverted: r06q); parity,
# C3 / C2 benches, membership-table slots per hash A/B (NPGX_AF_TABLE_SLOTS),
# a C3 kernel trace
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06r
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py tests/test_fullsize_gpu.py tests/test_block_build_gpu.py tests/test_anchor_device_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C2 C3 C2; do
  step "bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['stage_timeline']['ms'])"
done
step "af table slots A/B C3"
timeout -k 10 600 tools/gpu_ab_env.sh r06r NPGX_AF_TABLE_SLOTS 4 8 --config C3 --steps 10 --warmup 3 || exit 1
step "rocprof C3"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python $R/bench.py --config C3 --steps 5 --warmup 2 --no-cpu-baseline --no-pairs-line > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
cd $R
step done
