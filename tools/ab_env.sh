#!/bin/bash
# A/B timing of one library build with and without an environment switch
# (diagnostic):  tools/ab_env.sh VAR=VALUE [rounds] [extra bench args]
# alternates bench.py runs without ("base") and with ("env") the variable.
KV=$1; N=${2:-3}; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in base env; do
    if [ $v = env ]; then export "$KV"; else unset "${KV%%=*}"; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_%s.log" % sys.argv[1]).read().strip().splitlines()[-1])
s = d["last_step"]["ms_stage"]
print(sys.argv[1], d["ms_per_step"], " ".join("%s=%.2f" % (k[:8], v) for k, v in s.items()), flush=True)
PY
  done
done
