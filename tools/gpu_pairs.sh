# pair-sharded mode: parity tests, then a --pair-workers sweep on a C4 pair sample
set -o pipefail
mkdir -p gpurun_out/pairs
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_pairs_gpu.py > gpurun_out/pairs/tests.log 2>&1 || { tail -30 gpurun_out/pairs/tests.log; exit 1; }
tail -3 gpurun_out/pairs/tests.log
for w in ${WS:-1 2 4 8}; do
  timeout -k 10 300 python -u bench.py --mode pairs --pairs ${NP:-32} --pair-workers $w --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/pairs/w$w.json 2> gpurun_out/pairs/w$w.err || { tail -20 gpurun_out/pairs/w$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/pairs/w$w.json'));print($w, d['value'], d['ms_per_step'], d['device_mem_used_gb'], d['last_step'])"
done
