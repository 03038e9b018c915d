# GPU_MAX_HW_QUEUES 4 (default) vs 16: the C4 pair job (496 pairs, 12 workers) and C3, alternating
set -o pipefail
mkdir -p gpurun_out/hq
for i in 1 2; do for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --mode pairs --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/hq/p$q.json 2> gpurun_out/hq/p$q.err || { tail -5 gpurun_out/hq/p$q.err; exit 1; }
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pairs-line > gpurun_out/hq/c$q.json 2> gpurun_out/hq/c$q.err || { tail -5 gpurun_out/hq/c$q.err; exit 1; }
  python -c "
import json;p=json.load(open('gpurun_out/hq/p$q.json'));c=json.load(open('gpurun_out/hq/c$q.json'))
print('q', $q, 'pairs', p['value'], p['ms_per_step'], '| C3', c['ms_per_step'])"
done; done
