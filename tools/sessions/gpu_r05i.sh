#!/bin/bash
# round 5: the whole GPU suite with the device ExtendLoopFast on by default (its tables checked on
# the host every iteration), then the prefix-search switch point and the single-workgroup pass
# threshold at C3 / R3 / C2
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05i
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest_gpu
NPGX_ELF_CHECK=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
b() {  # tag cfg env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_${tag}_$cfg.log 2>&1 || { tail -5 $O/bench_${tag}_$cfg.log; return 1; }
  python -c "import json; d=json.loads(open('$O/bench_${tag}_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$tag $cfg', d['ms_per_step'], 'align', s['ms_stage']['align_batch'], 'host', s['ms_host_bookkeeping'])"
}
for lh in 64 96 128 192 256; do
  for cfg in C3 R3; do
    step "lh$lh $cfg"; b lh$lh $cfg NPGX_LONG_HEAD=$lh || exit 1
  done
done
for pw in 0 2048; do
  for cfg in C3 C2; do
    step "pw$pw $cfg"; b pw$pw $cfg NPGX_LONG_HEAD=128 NPGX_ELF_PASS_WG=$pw || exit 1
  done
done
step done
