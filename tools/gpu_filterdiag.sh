set -o pipefail
mkdir -p gpurun_out/fd
NPGX_FILTER_DEBUG=1 timeout -k 10 300 python -u bench.py --config ${1:-C5} --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/fd/out.json 2> gpurun_out/fd/err.txt
echo exit $?
