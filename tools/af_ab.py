#!/usr/bin/env python3
"""AnchorFinder wall time per config (GPU box diagnostic, A/B with NPGX_LIB)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from npge_amd import _capi, synth  # noqa: E402
from npge_amd.anchor_finder import AnchorFinder  # noqa: E402

_capi.check(_capi.lib().npgx_set_device(0))
tag = os.environ.get("NPGX_LIB", "default")
for cfg in sys.argv[1:] or ["C2", "C3", "C4"]:
    names, seqs = synth.genome_set(cfg)
    ss = _capi.SeqSet(seqs, names)
    af = AnchorFinder()
    best = 1e9
    for rep in range(5):
        af.clear_used()
        t = time.perf_counter()
        af.find(ss)
        best = min(best, time.perf_counter() - t)
    print(tag, cfg, "af %.2f ms" % (best * 1e3), flush=True)
