# C3 bench over (NPGX_ALIGN_DEFER, NPGX_ALIGN_SPLIT) pairs, twice each
set -o pipefail
mkdir -p gpurun_out/dsw
for rep in 1 2; do
for cfg in 8000:384 1000:384 500:384 300:384 500:256 1000:256; do
  d=${cfg%:*}; sp=${cfg#*:}
  NPGX_ALIGN_DEFER=$d NPGX_ALIGN_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dsw/c3_${d}_${sp}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/dsw/c3_${d}_${sp}_$rep.json').read().strip().splitlines()[-1]); k={x['name']:x['ms'] for x in d['kernels_last_step']}; print('$d $sp $rep', d['ms_per_step'], d['last_step']['ms_align_wall'], round(k.get('align_jobs',0),2), round(k.get('align_sub',0),2))"
done
done
