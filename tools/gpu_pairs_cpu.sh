# pair mode: host cores busy vs worker count (64 C4 pairs), and nproc / cgroup quota
set -o pipefail
mkdir -p gpurun_out/pc
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc
for w in ${WS:-1 6 12}; do
  timeout -k 10 300 python -u bench.py --mode pairs --pairs 64 --pair-workers $w --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/pc/w$w.json 2> gpurun_out/pc/w$w.err || { tail -20 gpurun_out/pc/w$w.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/pc/w$w.json'));l=d['last_step']
print('w', $w, d['value'], d['ms_per_step'], 'cores_busy', l['host_cores_busy'], 'align', l['mean_pair_ms_align'], 'host', l['mean_pair_ms_host'])"
done
