#!/bin/bash
# round 5: overflowed bad-region sub-jobs re-run at once in a proven-bound room (instead of their
# whole job at attempt 1): aligner / repeat / device-loop parity, R3 retry reasons and step time
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05p
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_repeats_gpu.py tests/test_elf_device_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step "r3 retry reasons"
NPGX_ELF_DEVICE=0 NPGX_RETRY_DEBUG=1 timeout -k 10 300 python bench.py --config R3 --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/r3_retry.log 2> $O/r3_retry.err || { tail -5 $O/r3_retry.err; exit 1; }
echo "retried: $(grep -c 'retry job' $O/r3_retry.err)"; grep "retry job" $O/r3_retry.err | head
for cfg in R3 C3 C5; do
  step "bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$cfg', d['ms_per_step'], [(k['name'], round(k['ms'], 2)) for k in d.get('kernels_last_step', [])])"
done
step done
