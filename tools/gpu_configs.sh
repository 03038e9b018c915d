# one bench line per BASELINE config beyond C3 (C2, C4, C4 + AnchorLoopFast, C5), no CPU leg
set -o pipefail
mkdir -p gpurun_out/cfg
for c in C2 C4 C5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cfg/$c.json 2> gpurun_out/cfg/$c.err || { echo fail $c; exit 1; }
done
timeout -k 10 400 python -u bench.py --config C4 --anchor-loop --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/C4_loop.json 2> gpurun_out/cfg/C4_loop.err
echo exit $?
