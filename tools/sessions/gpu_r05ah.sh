#!/bin/bash
# round 5: try_aligned's row-parallel search in groups of J shifts a step (4 groups; libnpge_amd_g1.so:
# one group, the round-4 step) -- aligner / repeat / device-loop / block-build parity, C3 / R3 / C5 / C2
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ah
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 1100 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_repeats_gpu.py tests/test_elf_device_gpu.py tests/test_block_build_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in g4:libnpge_amd.so g1:libnpge_amd_g1.so; do
    IFS=: read tag lib <<< "$v"
    for cfg in C3 R3 C5 C2; do
      step "$tag $cfg $rep"
      NPGX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-pairs-line > $O/bench_${tag}_${cfg}_$rep.log 2>&1 || { tail -5 $O/bench_${tag}_${cfg}_$rep.log; exit 1; }
      python -c "import json; d=json.loads(open('$O/bench_${tag}_${cfg}_$rep.log').read().strip().splitlines()[-1]); print('$tag $cfg', d['ms_per_step'])"
    done
  done
done
step done
