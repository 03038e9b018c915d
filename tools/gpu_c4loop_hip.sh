# HIP API time split of one C4 DraftPangenome -> AnchorLoopFast step
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --hip-trace --stats --output-format csv -d gpurun_out/hip -o run -- python -u bench.py --config C4 --anchor-loop --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/b_c4hip.log 2>&1
echo exit $?
find gpurun_out/hip -name "*stats*"
