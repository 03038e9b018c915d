set -o pipefail
mkdir -p gpurun_out/sd
timeout -k 10 300 python -u tools/split_stats.py C3 > gpurun_out/sd/c3.out 2> gpurun_out/sd/c3.err
echo exit $?
