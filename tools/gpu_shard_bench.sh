# sharded-mode rehearsal on one GPU (gloo, 2 ranks share the card) + 1-GPU C4 DraftPangenome reference
set -o pipefail
mkdir -p gpurun_out/sb
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --config C4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sb/c4_1.json 2> gpurun_out/sb/c4_1.err && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --mode sharded --dist-backend gloo --config C4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sb/c4_s2.json 2> gpurun_out/sb/c4_s2.err
rc=$?
tail -3 gpurun_out/sb/c4_s2.err
echo exit $rc
