#!/bin/bash
# round 5: the device ExtendLoopFast after the r05b fault (small: > 8192 blocks, the multi-launch
# table passes): its tests with every step synchronised and the host-side table / flank-plan check,
# then C3 / R3 / C2 bench lines of the host loop, the device loop and the round-4 fast_run order
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05e
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest_elf
NPGX_ELF_SYNC=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py > $O/pytest_elf.log 2>&1 || { tail -40 $O/pytest_elf.log; exit 1; }
tail -3 $O/pytest_elf.log
for v in host:0:libnpge_amd.so dev:1:libnpge_amd.so fr1:0:libnpge_amd_fr1.so; do
  IFS=: read tag dev lib <<< "$v"
  for cfg in C3 R3 C2; do
    step "bench $tag $cfg"
    NPGX_ELF_DEVICE=$dev NPGX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_${tag}_$cfg.log 2>&1 || { tail -5 $O/bench_${tag}_$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${tag}_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$tag $cfg', d['ms_per_step'], 'align', s['ms_stage']['align_batch'], 'host', s['ms_host_bookkeeping'], 'af', s['ms_stage']['anchor_finder'])"
  done
done
step done
