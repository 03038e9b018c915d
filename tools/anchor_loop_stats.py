#!/usr/bin/env python3
"""DraftPangenome then one AnchorLoopFast on synthetic sets (GPU box
diagnostic): consensus sequences, anchors on them, blocks mapped back, time."""
import sys, os
sys.path.insert(0, os.getcwd())
from npge_amd import _capi, synth
from npge_amd.blockset import BlockSetEngine
from npge_amd.anchor_finder import AnchorFinder
from npge_amd.anchor_loop import anchor_loop_fast
import time
_capi.check(_capi.lib().npgx_set_device(0))
for cfg in (sys.argv[1:] or ["tiny", "small", "C2"]):
    names, seqs = synth.genome_set(cfg)
    ss = _capi.SeqSet(seqs, names)
    eng = BlockSetEngine(ss)
    af = AnchorFinder()
    eng.apply("DraftPangenome", af=af)
    nb = len(eng.blocks())
    t = time.perf_counter()
    st = anchor_loop_fast(eng, AnchorFinder())
    print(cfg, "draft blocks", nb, st, "%.1f ms" % ((time.perf_counter() - t) * 1e3), flush=True)
