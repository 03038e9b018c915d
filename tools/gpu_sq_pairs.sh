# SQ issue/wait counters of the aligner on the pair workload (8 C4 pairs, one worker) and on C3
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/sq; mkdir -p $O; cd /tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pairs -o run -- python3 $R/bench.py --mode pairs --pairs 8 --pair-workers 1 --steps 1 --warmup 1 --no-cpu-baseline > $O/pairs.log 2>&1 || { tail -5 $O/pairs.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/c3 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pairs-line > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
cd $R
python3 - <<'PY'
import csv, collections
for tag in ("pairs", "c3"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open("gpurun_out/sq/%s/run_counter_collection.csv" % tag)):
        n = r["Kernel_Name"].split("(")[0].split("::")[-1]
        if n in ("k_align_jobs", "k_align_sub", "k_fix_ends", "k_bloom_first_f"):
            acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
    for n, c in acc.items():
        wc = c["SQ_WAVE_CYCLES"] or 1
        print(tag, n, "waves %d  wait %.2f  inst-stall %.2f  active %.2f  | per wave: valu %.0f lds %.0f salu %.0f cycles %.0f" % (
            c["SQ_WAVES"], c["SQ_WAIT_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc,
            c["SQ_INSTS_VALU"] / max(c["SQ_WAVES"], 1), c["SQ_INSTS_LDS"] / max(c["SQ_WAVES"], 1),
            c["SQ_INSTS_SALU"] / max(c["SQ_WAVES"], 1), 4 * wc / max(c["SQ_WAVES"], 1)))
PY
