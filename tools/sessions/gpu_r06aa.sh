#!/bin/bash
# round 6: Bloom epoch count with one launch an epoch (AnchorFinder alone,
# C3 / C5: automatic (24) vs 16 / 32 / 48 / 64), and the pair job on the
# device loop again (NPGX_PAIR_TUNING elf-device 1 vs the default host loop)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06aa
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "epoch sweep"
timeout -k 10 600 python tools/af_epoch_sweep.py C3,C5 0,16,32,48,64 4 > $O/epochs.txt 2>&1 || { tail -5 $O/epochs.txt; exit 1; }
cut -c1-120 $O/epochs.txt
for rep in 1 2; do
  for v in '{"long-head": 0, "elf-device": 0}' '{"long-head": 0, "elf-device": 1}'; do
    step "pairs $v"
    NPGX_PAIR_TUNING="$v" timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$rep.log 2>&1 || { tail -5 $O/pairs_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/pairs_$rep.log').read().strip().splitlines()[-1]); print('pairs', d['value'], d['ms_per_step'])"
  done
done
step done
