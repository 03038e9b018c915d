#!/bin/bash
# round 5: device loop with the wave block_hash, the piece-list stitch and the wave fragment sort:
# parity (synchronised, checked), C3 / C2 / R3 lines host vs device, a device-loop C3 trace; prefix
# search switch point (NPGX_LONG_HEAD 64 / 128) at C3 / R3
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r05h
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest_elf
NPGX_ELF_SYNC=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py > $O/pytest_elf.log 2>&1 || { tail -30 $O/pytest_elf.log; exit 1; }
tail -1 $O/pytest_elf.log
for v in dev:1 host:0; do
  IFS=: read tag dev <<< "$v"
  for cfg in C3 C2 R3; do
    step "bench $tag $cfg"
    NPGX_ELF_DEVICE=$dev timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_${tag}_$cfg.log 2>&1 || { tail -5 $O/bench_${tag}_$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${tag}_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$tag $cfg', d['ms_per_step'], 'align', s['ms_stage']['align_batch'], 'host', s['ms_host_bookkeeping'], 'af', s['ms_stage']['anchor_finder'])"
  done
done
step "rocprof dev"
cd /tmp
NPGX_ELF_DEVICE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dev -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_dev.log 2>&1 || { tail -5 $O/prof_dev.log; exit 1; }
cd $R
python tools/step_timeline.py $O/prof_dev/run_kernel_trace.csv > $O/step_timeline_dev.txt 2>&1; head -3 $O/step_timeline_dev.txt
for lh in 64 128; do
  for cfg in C3 R3; do
    step "bench lh$lh $cfg"
    NPGX_LONG_HEAD=$lh NPGX_ELF_DEVICE=0 timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_lh${lh}_$cfg.log 2>&1 || { tail -5 $O/bench_lh${lh}_$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_lh${lh}_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('lh$lh $cfg', d['ms_per_step'], 'align', s['ms_stage']['align_batch'])"
  done
done
step done
