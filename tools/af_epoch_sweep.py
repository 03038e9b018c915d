#!/usr/bin/env python3
"""AnchorFinder time vs the number of Bloom epochs (GPU box diagnostic);
0 = the automatic choice.  Usage: af_epoch_sweep.py [C2,C3] [0,1,2,...] [reps]"""
import sys, time, os
sys.path.insert(0, os.getcwd())
from npge_amd import _capi, synth
from npge_amd.anchor_finder import AnchorFinder
_capi.check(_capi.lib().npgx_set_device(0))
CFGS = sys.argv[1].split(",") if len(sys.argv) > 1 else ["C2", "C3"]
EPOCHS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 3, 4, 6, 8, 12, 16, 32]
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 6
for cfg in CFGS:
    names, seqs = synth.genome_set(cfg)
    ss = _capi.SeqSet(seqs, names)
    for ep in EPOCHS:
        af = AnchorFinder()
        af.set_opt_value("bloom-epochs", ep)
        best = 1e9
        for rep in range(REPS):
            af.clear_used()
            t = time.perf_counter(); af.find(ss); dt = time.perf_counter() - t
            best = min(best, dt)
        agg = {}
        for k in af.kernel_times():  # the last run's kernels (NPGX_TIMERS=2: all of them)
            agg[k["name"]] = agg.get(k["name"], 0.0) + k["ms"]
        top = sorted(agg.items(), key=lambda kv: -kv[1])[:5]
        print(cfg, "epochs", ep, "af %.2f ms" % (best * 1e3),
              " ".join("%s %.2f" % (n, v) for n, v in top), flush=True)
