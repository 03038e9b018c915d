#!/bin/bash
# full GPU suite + smoke + default bench, the C3 kernel trace and step
# timeline, the AF epoch sweep and the pair worker sweep
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${1:-r04ka}
tools/round_end.sh $TAG tests || exit 1
O=$R/gpurun_out/$TAG
echo "== rocprof C3 $(date +%T)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
cd $R
python tools/step_timeline.py $O/prof_c3/run_kernel_trace.csv > $O/c3_step_timeline.txt 2>&1
head -14 $O/c3_step_timeline.txt
echo "== af epochs C3 $(date +%T)"
timeout -k 10 300 python tools/af_epoch_sweep.py C3 0,4,8,12,16,24 6 > $O/af_epochs_c3.txt 2>&1 || { tail -5 $O/af_epochs_c3.txt; exit 1; }
cat $O/af_epochs_c3.txt
for w in 12 16 20; do
  echo "== pairs workers $w $(date +%T)"
  timeout -k 10 300 python bench.py --mode pairs --pair-workers $w --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_w$w.log 2>&1 || { tail -5 $O/pairs_w$w.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/pairs_w$w.log').read().strip().splitlines()[-1]); print('workers $w', d['value'], d['ms_per_step'], d['last_step']['host_cores_busy'], d['last_step']['mean_pair_ms_host'])"
done
