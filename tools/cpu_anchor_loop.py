#!/usr/bin/env python3
"""CPU leg for the AnchorLoop line (GPU box host): the oracle's AnchorLoop
(oracle/npge_oracle.cpp anchor_loop, one thread, -O3 -march=native) after
its DraftPangenome on the same synthetic set, timed alone; prints one JSON
line.  usage: cpu_anchor_loop.py [config]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from npge_amd import synth  # noqa: E402
from oracle import oracle as orc  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
native = orc.use_native()
names, seqs = synth.genome_set(cfg)
o = orc.BlockSetOracle(seqs, names)
o.apply("DraftPangenome")
t = time.perf_counter()
o.apply("AnchorLoop")
dt = time.perf_counter() - t
bp = synth.total_bp(seqs)
print(json.dumps({"config": cfg, "workload": "AnchorLoop after DraftPangenome (AnchorLoop timed)",
                  "seconds": round(dt, 3), "mbp_s": round(bp / 1e6 / dt, 4), "cores": 1, "kind": "port",
                  "build": "-O3 -march=native" if native else "-O3", "blocks": len(o.blocks()),
                  "counts": o.anchor_loop_stats()}))
