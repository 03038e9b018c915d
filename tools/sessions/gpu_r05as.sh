#!/bin/bash
# round 5: the C3 line with this session's library against the one built from
# 59477e8 (before the geometric buffer growth and the wide aligner changes),
# alternating on one box
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05as
mkdir -p $O
for v in new1 old1 new2 old2 new3 old3; do
  echo "== $v $(date +%T)"
  if [ ${v%?} = old ]; then export NPGX_LIB=libnpge_amd_r05old.so; else unset NPGX_LIB; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/c3_$v.log 2>&1 || { tail -5 $O/c3_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/c3_$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value'])"
done
unset NPGX_LIB
echo "== done $(date +%T)"
