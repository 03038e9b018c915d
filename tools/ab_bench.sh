#!/bin/bash
# A/B timing of two builds of the library on one box (diagnostic):
#   tools/ab_bench.sh <alt .so in npge_amd/> [rounds] [extra bench args]
# alternates bench.py runs with the default library and NPGX_LIB=<alt>.
ALT=$1; N=${2:-3}; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in new alt; do
    if [ $v = alt ]; then export NPGX_LIB=$ALT; else unset NPGX_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_%s.log" % sys.argv[1]).read().strip().splitlines()[-1])
ls = d["last_step"]
s = (d.get("stage_timeline") or {}).get("ms") or ls.get("ms_stage_host") or ls.get("mean_pair_ms") or {}
al = d["last_step"].get("anchor_loop") or {}
extra = ""
if al:
    extra = " | loop " + " ".join("%s=%.2f" % (k[:8], v) for k, v in al["ms_loop"].items()) + " | loop ou=%.2f admit=%.2f" % (
        al["ms_stage"]["overlapless_union"], al["ms_stage"]["ou_admit"])
print(sys.argv[1], d["ms_per_step"], " ".join("%s=%.2f" % (k[:8], v) for k, v in s.items()) + extra, flush=True)
PY
  done
done
