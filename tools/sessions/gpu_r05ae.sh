#!/bin/bash
# round 5: failed sub-jobs re-run whole at their proven bound -- aligner / repeats / device-loop /
# anchor-loop parity, R3 re-run count, R3 / R3+ALF / C3 / C5 lines
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ae
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 1100 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_repeats_gpu.py tests/test_elf_device_gpu.py tests/test_anchor_loop_gpu.py tests/test_fullsize_c45_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step "r3 retries"
NPGX_ELF_DEVICE=0 NPGX_RETRY_DEBUG=1 timeout -k 10 300 python bench.py --config R3 --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/r3_retry.log 2> $O/r3_retry.err || { tail -5 $O/r3_retry.err; exit 1; }
echo "retried: $(grep -c 'retry job' $O/r3_retry.err)"; grep "retry job" $O/r3_retry.err | head -5
for v in "R3:" "R3:--anchor-loop" "C3:" "C5:"; do
  cfg=${v%%:*}; ex=${v#*:}
  step "bench $cfg $ex"
  timeout -k 10 400 python bench.py --config $cfg $ex --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}${ex}.log 2>&1 || { tail -5 $O/bench_${cfg}${ex}.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_${cfg}${ex}.log').read().strip().splitlines()[-1]); print('$cfg $ex', d['ms_per_step'], [(k['name'], round(k['ms'], 1)) for k in d.get('kernels_last_step', [])])"
done
step done
