#!/bin/bash
# round 6: the pair line's drop (1493 -> 1399-1445 Mbp/s): 4 vs 8 waves per
# sync-state search, alternating builds; the OverlaplessUnion admission with
# 4 positions a thread and the small-table sorts in one launch (C2 / C3
# parity and time, NPGX_OU_SMALL A/B)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06p
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest ou"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py tests/test_fullsize_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C2; do
  step "ou small A/B $cfg"
  timeout -k 10 600 tools/gpu_ab_env.sh r06p NPGX_OU_SMALL 0 1 --config $cfg --steps 10 --warmup 3 || exit 1
done
step "pairs sw4 vs sw8"
timeout -k 10 1000 tools/ab_bench.sh libnpge_amd_sw4.so 2 --mode pairs --config C4 > $O/ab_pairs_sw4.txt 2>&1 || { tail -5 $O/ab_pairs_sw4.txt; exit 1; }
cat $O/ab_pairs_sw4.txt | cut -c1-200
for cfg in C2 C3; do
  step "bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['stage_timeline']['ms'])"
done
step done
