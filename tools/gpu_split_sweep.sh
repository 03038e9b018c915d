# C3 bench at several segment lengths (NPGX_ALIGN_SPLIT), alternating twice
set -o pipefail
mkdir -p gpurun_out/sw
for rep in 1 2; do
for sp in 384 256 192 128; do
  NPGX_ALIGN_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sw/c3_${sp}_$rep.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw/c3_${sp}_$rep.json').read().strip().splitlines()[-1]); print($sp, $rep, d['ms_per_step'], d['last_step']['ms_align_wall'])"
done
done
