#!/bin/bash
# AnchorLoop bench after the SmthUnion fixes (C2, C3) + host profile C2
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04q
mkdir -p $O
for cfg in C2 C3; do
  echo "== bench $cfg full $(date +%T)"
  timeout -k 10 400 python bench.py --config $cfg --anchor-loop full --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/bench_${cfg}_full.log 2>&1 || { tail -5 $O/bench_${cfg}_full.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_${cfg}_full.log').read().strip().splitlines()[-1]); l=d['last_step'].get('anchor_loop'); print(d['value'], d['ms_per_step'], json.dumps({k: v for k, v in (l or {}).items() if not isinstance(v, dict)}))"
done
echo "== hostprof C2 full $(date +%T)"
NPGX_PROFILE=1 timeout -k 10 300 python tools/host_profile.py C2 2 full > $O/host_C2_full.txt 2>&1 || { tail -5 $O/host_C2_full.txt; exit 1; }
head -30 $O/host_C2_full.txt
