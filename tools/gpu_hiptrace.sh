# HIP API time per call kind over a short bench run (default C2)
set -o pipefail
mkdir -p gpurun_out/ht
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d gpurun_out/ht/${1:-C2} -o run -- python -u bench.py --config ${1:-C2} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ht/b_${1:-C2}.log 2>&1
echo exit $?
