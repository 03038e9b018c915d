set -o pipefail
mkdir -p gpurun_out/af
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_anchor_finder_gpu.py tests/test_af_sharded_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_c45_gpu.py -k "anchor_finder or sharded" > gpurun_out/af/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/af/c3.json 2>gpurun_out/af/c3.err && \
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/af/c3_FETCH_SIZE -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/af/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/af/c3_WRITE_SIZE -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/af/pmc2.log 2>&1
rc=$?
tail -2 $GRAFT_REPO_ROOT/gpurun_out/af/tests.log
echo exit $rc
