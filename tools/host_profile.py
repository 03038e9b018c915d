#!/usr/bin/env python3
"""Host-side sampling profile of the block build (diagnostic; GPU box):
SIGPROF sampling inside libnpge_amd.so (npge_amd/csrc/host_sampler.cpp)
during a few DraftPangenome steps; prints the hottest library functions.
usage: host_profile.py [config] [steps] [alf|full]  (alf: DraftPangenome ->
AnchorLoopFast; full: DraftPangenome -> AnchorLoop)"""
import collections
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from npge_amd import _capi, pipeline, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
L = _capi.lib()
_capi.check(L.npgx_set_device(0))
if cfg.endswith(":pair"):  # the first genome pair of a config (the pair-sharded job's unit)
    from npge_amd import pairs as _pairs
    names, seqs = synth.genome_set(cfg.split(":")[0])
    idx = _pairs.all_pairs(names)[0]
    names, seqs = [names[i] for i in idx], [seqs[i] for i in idx]
else:
    names, seqs = synth.genome_set(cfg)
ss = _capi.SeqSet(seqs, names)
loop = sys.argv[3] if len(sys.argv) > 3 else ""
job = pipeline.BlockBuild(ss, names, seqs, anchor_loop={"alf": "fast", "full": "full"}.get(loop, False))
job.run()
out = os.path.abspath("gpurun_out/host_prof_%s.txt" % cfg.replace(":", "_"))
os.makedirs(os.path.dirname(out), exist_ok=True)
L.npgx_diag_prof_start(4000)
for _ in range(steps):
    job.run()
L.npgx_diag_prof_stop(out.encode())
syms = []
for line in subprocess.check_output(["nm", "-C", "--defined-only", "-n", _capi.LIB_PATH]).decode().splitlines():
    parts = line.split(None, 2)
    if len(parts) == 3 and parts[1].lower() in "tw":
        syms.append((int(parts[0], 16), parts[2]))
import bisect
addrs = [a for a, _ in syms]
agg = collections.Counter()
callers = collections.Counter()
total = 0
for line in open(out):
    if line.startswith("#"):
        total = int(line.split()[-1])
        continue
    if line.startswith("caller "):
        _, c0, c1, n = line.split()
        def sym(o):
            i = bisect.bisect_right(addrs, int(o, 16)) - 1
            return syms[i][1][:60] if i >= 0 and int(o, 16) else "-"
        callers["%s  <-  %s" % (sym(c0), sym(c1))] += int(n)
        continue
    if line.startswith("lib "):
        parts = line.split()
        agg["[" + os.path.basename(" ".join(parts[1:-1])) + "]"] += int(parts[-1])
        continue
    off, n = line.split()
    i = bisect.bisect_right(addrs, int(off, 16)) - 1
    agg[syms[i][1][:110] if i >= 0 else "?"] += int(n)
print("samples", total)
for name, n in agg.most_common(45):
    print("%6.2f%%  %s" % (100.0 * n / max(total, 1), name))
print("\noutside the library, by calling library function (first %d samples):" % min(total, 65536))
for name, n in callers.most_common(40):
    print("%6.2f%%  %s" % (100.0 * n / max(total, 1), name))
