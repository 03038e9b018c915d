#!/bin/bash
# round 5: aligner kernels in two forms (with / without the prefix search's call), overflowed
# sub-jobs re-run in place, npgx_blockset_tune and the pair workers' tuning: parity, R3 retries,
# C3 / R3 / C5 lines, the pair job under three tunings
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05q
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_similar_aligner_gpu.py tests/test_repeats_gpu.py tests/test_elf_device_gpu.py tests/test_pairs_gpu.py tests/test_pairs_bench_concurrency_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step "r3 retry reasons"
NPGX_ELF_DEVICE=0 NPGX_RETRY_DEBUG=1 timeout -k 10 300 python bench.py --config R3 --steps 1 --warmup 0 --no-cpu-baseline --no-pairs-line > $O/r3_retry.log 2> $O/r3_retry.err || { tail -5 $O/r3_retry.err; exit 1; }
echo "retried: $(grep -c 'retry job' $O/r3_retry.err)"; grep "retry job" $O/r3_retry.err | head
for cfg in C3 R3 C5; do
  step "bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-pairs-line > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$cfg.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$cfg', d['ms_per_step'], [(k['name'], round(k['ms'], 2)) for k in d.get('kernels_last_step', [])])"
done
for v in 'default:' 'lh0dev:{"long-head":0,"elf-device":1}' 'lh128host:{"long-head":128,"elf-device":0}'; do
  tag=${v%%:*}; tun=${v#*:}
  step "pairs $tag"
  if [ -n "$tun" ]; then export NPGX_PAIR_TUNING="$tun"; else unset NPGX_PAIR_TUNING; fi
  timeout -k 10 500 python bench.py --mode pairs --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/pairs_$tag.log 2>&1 || { tail -5 $O/pairs_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pairs_$tag.log').read().strip().splitlines()[-1]); s=d['last_step']; print('$tag', d['value'], d['ms_per_step'], 'af', s['mean_pair_ms']['anchor_finder'], 'align', s['mean_pair_ms_align'], 'host', s['mean_pair_ms_host'])"
done
step done
