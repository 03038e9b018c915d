set -o pipefail
mkdir -p gpurun_out/hp
timeout -k 10 500 python -u tools/host_profile.py ${1:-C5} ${2:-2} > gpurun_out/hp/out_${1:-C5}.txt 2>&1
echo exit $?
