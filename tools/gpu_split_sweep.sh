# C3 (and C5 once) at several segment lengths (NPGX_ALIGN_SPLIT), alternating twice
set -o pipefail
mkdir -p gpurun_out/sw
for rep in 1 2; do
for sp in ${SPS:-384 256 192}; do
  NPGX_ALIGN_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pairs-line > gpurun_out/sw/c3_${sp}_$rep.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw/c3_${sp}_$rep.json').read().strip().splitlines()[-1]); print('C3', $sp, $rep, d['ms_per_step'], d['last_step']['ms_align_wall'])"
done
done
for sp in ${SPS:-384 256 192}; do
  NPGX_ALIGN_SPLIT=$sp timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > gpurun_out/sw/c5_${sp}.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw/c5_${sp}.json').read().strip().splitlines()[-1]); print('C5', $sp, d['ms_per_step'], d['last_step']['ms_align_wall'])"
done
