set -o pipefail
mkdir -p gpurun_out/pd
NPGX_PREP_DEBUG=1 timeout -k 10 300 python -u bench.py --config ${1:-C2} --steps 1 --warmup 2 --no-cpu-baseline > gpurun_out/pd/out.json 2> gpurun_out/pd/err.txt
echo exit $?
