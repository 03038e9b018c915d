# pair-sharded mode: --pair-workers x GPU_MAX_HW_QUEUES sweep on a C4 pair sample (no tests)
set -o pipefail
mkdir -p gpurun_out/pairsq
for q in ${QS:-4 8 16}; do for w in ${WS:-8 16}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --mode pairs --pairs ${NP:-64} --pair-workers $w --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/pairsq/q${q}w$w.json 2> gpurun_out/pairsq/q${q}w$w.err || { tail -20 gpurun_out/pairsq/q${q}w$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/pairsq/q${q}w$w.json'));print('q', $q, 'w', $w, d['value'], d['ms_per_step'], d['device_mem_used_gb'])"
done; done
