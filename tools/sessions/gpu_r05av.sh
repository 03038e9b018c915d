#!/bin/bash
# round 5: the buffer cache (freed device / pinned buffers reused by size
# class): the full GPU suite with it on, then C3 / C3 + AnchorLoopFast / the
# pair job with it on and off (NPGX_BUF_CACHE=0)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05av
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for v in on off on2 off2; do
  if [ ${v%2} = off ]; then export NPGX_BUF_CACHE=0; else unset NPGX_BUF_CACHE; fi
  step "C3 $v"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/c3_$v.log 2>&1 || { tail -5 $O/c3_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/c3_$v.log').read().strip().splitlines()[-1]); print('C3 $v', d['ms_per_step'], d['value'])"
  step "C3 alf $v"
  timeout -k 10 300 python bench.py --config C3 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/c3alf_$v.log 2>&1 || { tail -5 $O/c3alf_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/c3alf_$v.log').read().strip().splitlines()[-1]); print('C3 alf $v', d['ms_per_step'], d['value'])"
done
for v in on off; do
  if [ $v = off ]; then export NPGX_BUF_CACHE=0; else unset NPGX_BUF_CACHE; fi
  step "pairs $v"
  timeout -k 10 400 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$v.log 2>&1 || { tail -5 $O/pairs_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_$v.log').read().strip().splitlines()[-1]); print('pairs $v', d['ms_per_step'], d['value'])"
done
unset NPGX_BUF_CACHE
step done
