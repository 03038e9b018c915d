# stream_wait A/B: pairs (64 C4 pairs, 12 workers) and C3, new build vs NPGX_LIB=libnpge_amd_prev.so
set -o pipefail
mkdir -p gpurun_out/wab
for i in 1 2; do
  for v in new prev; do
    unset NPGX_LIB; [ $v = prev ] && export NPGX_LIB=libnpge_amd_prev.so
    timeout -k 10 300 python -u bench.py --mode pairs --pairs 64 --pair-workers 12 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wab/p_$v.json 2> gpurun_out/wab/p_$v.err || { tail -20 gpurun_out/wab/p_$v.err; exit 1; }
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pairs-line > gpurun_out/wab/c3_$v.json 2> gpurun_out/wab/c3_$v.err || { tail -20 gpurun_out/wab/c3_$v.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/wab/p_$v.json'));l=d['last_step'];c=json.load(open('gpurun_out/wab/c3_$v.json'))
print('$v', 'pairs', d['value'], d['ms_per_step'], 'cores', l['host_cores_busy'], 'align', l['mean_pair_ms_align'], 'host', l['mean_pair_ms_host'], '| C3', c['ms_per_step'])"
  done
done
