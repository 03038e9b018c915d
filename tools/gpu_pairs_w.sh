# pair-mode per-pair stage times at several worker counts (64 C4 pairs)
set -o pipefail
mkdir -p gpurun_out/pw
for w in ${WS:-1 4 12}; do
  timeout -k 10 300 python -u bench.py --mode pairs --pairs ${NP:-64} --pair-workers $w --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/pw/w$w.json 2> gpurun_out/pw/w$w.err || { tail -20 gpurun_out/pw/w$w.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/pw/w$w.json'));l=d['last_step']
print('w', $w, d['value'], d['ms_per_step'], 'align', l['mean_pair_ms_align'], 'host', l['mean_pair_ms_host']); print(l['mean_pair_ms'])"
done
