# pairs/bench/RCCL tests, then the default bench line (C3 headline + C4 pair job at N=1)
set -o pipefail
mkdir -p gpurun_out/pf
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_pairs_gpu.py tests/test_comm_rccl_gpu.py tests/test_bench_gpu.py > gpurun_out/pf/tests.log 2>&1 || { tail -40 gpurun_out/pf/tests.log; exit 1; }
tail -3 gpurun_out/pf/tests.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/pf/bench.json 2> gpurun_out/pf/bench.err || { tail -30 gpurun_out/pf/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/pf/bench.json'));print(d['value'], d['ms_per_step']);print(d['pairs'])"
