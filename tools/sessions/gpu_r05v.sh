#!/bin/bash
# round 5: the table passes in one launch (decoupled look-back) -- parity with every step
# synchronised, then C3 / C2 with the look-back form against the count / rocPRIM scan / fill form
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05v
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest_elf
NPGX_ELF_SYNC=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_elf_device_gpu.py > $O/pytest_elf.log 2>&1 || { tail -30 $O/pytest_elf.log; exit 1; }
tail -1 $O/pytest_elf.log
for v in lb:0 scan:1; do
  IFS=: read tag sc <<< "$v"
  for cfg in C3 C2; do
    step "$tag $cfg"
    NPGX_ELF_PASS_SCAN=$sc timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_${tag}_$cfg.log 2>&1 || { tail -5 $O/bench_${tag}_$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${tag}_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$tag $cfg', d['ms_per_step'], 'host', s['ms_host_bookkeeping'])"
  done
done
step done
