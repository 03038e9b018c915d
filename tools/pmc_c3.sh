set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r01v9c3; mkdir -p $O; cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== $c $(date +%T)"
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/c3_$c -o run -- python3 $R/bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3_$c.log 2>&1 || { tail -5 $O/c3_$c.log; exit 1; }
done
echo done
