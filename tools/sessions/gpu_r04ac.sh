#!/bin/bash
# pair workers x hardware queues sweep (the pair job, one GPU)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04ac
mkdir -p $O
for wq in ${SWEEP:-16:16 20:20 24:24 16:32 24:32}; do
  w=${wq%%:*}; q=${wq##*:}
  timeout -k 10 300 python bench.py --mode pairs --pair-workers $w --hw-queues $q --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_w${w}_q$q.log 2>&1 || { tail -5 $O/pairs_w${w}_q$q.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_w${w}_q$q.log').read().strip().splitlines()[-1]); print('pairs workers $w queues $q', d['value'], d['ms_per_step'], d['last_step'].get('host_cores_busy'))"
done
