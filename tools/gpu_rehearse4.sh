# 4-rank rehearsal of the driver's default multi-GPU bench line on the box's one GPU (gloo:
# ranks share the GPU), small configs so that it finishes in seconds
set -o pipefail
mkdir -p gpurun_out/reh
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 4 --steps 2 --warmup 1 --config small --pairs-config small --pair-workers 2 --dist-backend gloo --no-cpu-baseline \
  > gpurun_out/reh/b4.json 2> gpurun_out/reh/b4.err || { tail -30 gpurun_out/reh/b4.err; exit 1; }
python -c "
import json;d=json.loads([l for l in open('gpurun_out/reh/b4.json') if l.startswith('{')][-1])
print(d['n_gpus'], d['value'], d['scaling'], d['config']['parallelism']); print('sharded', d['sharded']['value'], d['sharded']['parallelism']); print('pairs', d['pairs']['value'], d['pairs']['last_step']['pairs_rank'], d['pairs']['last_step']['gathered_pairs'])"
