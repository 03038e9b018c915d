#!/bin/bash
# A/B of an environment switch on one box (run via gpurun from the repo root):
#   tools/gpu_ab_env.sh TAG VAR VALUE_A VALUE_B [bench args...]
# alternates bench.py runs A B A B with VAR set to each value (no CPU
# baseline, no pairs line) and prints ms_per_step of each.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=$1; VAR=$2; VA=$3; VB=$4
shift 4
SFX=$(echo "$*" | tr -c 'A-Za-z0-9' '_' | cut -c1-40)
O=$R/gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  for v in "$VA" "$VB"; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-pairs-line "$@" > $O/ab_${VAR}_${v}_${SFX}_$rep.log 2>&1 || { tail -5 $O/ab_${VAR}_${v}_${SFX}_$rep.log; exit 1; }
    python - "$O/ab_${VAR}_${v}_${SFX}_$rep.log" "$VAR=$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ls = d["last_step"]
if d.get("stage_timeline"):
    st = d["stage_timeline"]["ms"]
    print("%-14s ms/step %.3f value %.1f align %.3f af %.3f ou %.3f fix_ends %.3f plan %.3f" % (
        sys.argv[2], d["ms_per_step"], d["value"], st["align"], st["anchor_finder"], st["overlapless_union"],
        st["fix_ends"], st["elf_plan"]))
elif "ms_stage" in ls:
    st = ls["ms_stage"]
    print("%-14s ms/step %.3f value %.1f align %.3f (kernel wait %.3f) host %.3f" % (
        sys.argv[2], d["ms_per_step"], d["value"], st["align_batch"], st["align_kernel_wait"],
        ls["ms_host_bookkeeping"]))
else:  # the pair job
    print("%-14s ms/step %.3f value %.1f pair host %.3f align %.3f" % (
        sys.argv[2], d["ms_per_step"], d["value"], ls["mean_pair_ms_host"], ls["mean_pair_ms_align"]))
PY
  done
done
