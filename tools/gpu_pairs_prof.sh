# rocprofv3 kernel trace of the pair-sharded job (64 C4 pairs), GPU occupancy of its last step
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/pp
mkdir -p $O
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --mode pairs --pairs ${NP:-64} --pair-workers ${W:-12} --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/pairs_busy.py $f | tee $O/busy.txt
