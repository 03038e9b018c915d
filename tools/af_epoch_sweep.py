#!/usr/bin/env python3
"""AnchorFinder time vs the number of Bloom epochs (GPU box diagnostic);
0 = the automatic choice (about one epoch per 2 M windows)."""
import sys, time, os
sys.path.insert(0, os.getcwd())
from npge_amd import _capi, synth
from npge_amd.anchor_finder import AnchorFinder
_capi.check(_capi.lib().npgx_set_device(0))
for cfg in ("C2", "C3"):
    names, seqs = synth.genome_set(cfg)
    ss = _capi.SeqSet(seqs, names)
    for ep in (0, 1, 2, 3, 4, 6, 8, 12, 16, 32):
        af = AnchorFinder()
        af.set_opt_value("bloom-epochs", ep)
        best = 1e9
        for rep in range(6):
            af.clear_used()
            t = time.perf_counter(); af.find(ss); dt = time.perf_counter() - t
            best = min(best, dt)
        print(cfg, "epochs", ep, "af %.2f ms" % (best * 1e3), flush=True)
