#!/bin/bash
# round 6: k_dt_hash_w copies each sequence name 16 loads ahead of its LDS
# stores (libnpge_amd_alt.so: a load and a store per byte): the loop's tests,
# A/B at C3 / C2 and the kernel's time in a C3 trace
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06ad
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step "pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_elf_device_gpu.py tests/test_fullsize_gpu.py tests/test_block_build_gpu.py tests/test_repeats_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in C3 C2; do
  step "name copy A/B $cfg"
  timeout -k 10 600 tools/ab_bench.sh libnpge_amd_alt.so 2 --config $cfg --steps 10 --no-pairs-line > $O/ab_$cfg.txt 2>&1 || { tail -5 $O/ab_$cfg.txt; exit 1; }
  cut -c1-150 $O/ab_$cfg.txt
done
step "rocprof C3"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
cd $R
grep -i "hash_w" $O/prof_c3/run_kernel_stats.csv | cut -c1-200
step done
