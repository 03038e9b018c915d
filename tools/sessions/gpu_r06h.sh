#!/bin/bash
# round 6: the pair job's latency vs throughput -- one worker (a pair alone
# on the GPU) against the default 16, and the profiling build's per-job
# phases of one C4 pair (2-row jobs)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06h
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for w in 1 4 16; do
  step "pairs workers $w"
  timeout -k 10 400 python bench.py --mode pairs --config C4 --pairs 32 --pair-workers $w --steps 1 --warmup 1 --no-cpu-baseline > $O/pairs_w$w.log 2>&1 || { tail -5 $O/pairs_w$w.log; exit 1; }
  python - $O/pairs_w$w.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ls = d["last_step"]
print("workers", ls["workers"], "ms/step %.1f" % d["ms_per_step"], "value %.1f" % d["value"], "host cores %.2f" % ls["host_cores_busy"],
      "pair ms", {k: v for k, v in ls["mean_pair_ms"].items() if v > 0.5}, "host", ls["mean_pair_ms_host"])
PY
done
step "analyze prof C4 pair"
NPGX_ELF_DEVICE=0 NPGX_PROFILE=1 NPGX_JOB_STATS=1 timeout -k 10 300 python tools/analyze_bb.py C4:pair > $O/analyze_pair_prof.txt 2>&1 || { tail -5 $O/analyze_pair_prof.txt; exit 1; }
grep -E "phase cycles|fit cycles|cycles per column|^jobs" $O/analyze_pair_prof.txt
mv gpurun_out/jobstats_C4:pair_prof.npy $O/jobstats_pair_prof.npy || true
step done
