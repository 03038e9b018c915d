#!/bin/bash
# A/B: hardware queues per process (GPU_MAX_HW_QUEUES, the box default 4)
# for the pair job (16 worker threads, one stream each) and the C3 line
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04ab
mkdir -p $O
for q in 4 16 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --mode pairs --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_q$q.log 2>&1 || { tail -5 $O/pairs_q$q.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_q$q.log').read().strip().splitlines()[-1]); print('pairs queues $q', d['value'], d['ms_per_step'], d['last_step'].get('host_cores_busy'))"
done
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/c3_q$q.log 2>&1 || { tail -5 $O/c3_q$q.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/c3_q$q.log').read().strip().splitlines()[-1]); print('C3 queues $q', d['value'], d['ms_per_step'])"
done
