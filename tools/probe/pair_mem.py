"""Device memory of one C4 pair's objects (mem_get_info deltas): sequence set,
AnchorFinder handle, block set (own aligner), a second block set borrowing it."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from npge_amd import _capi, synth, pairs
from npge_amd.pipeline import BlockBuild

def used():
    torch.cuda.synchronize()
    f, t = torch.cuda.mem_get_info()
    return (t - f) / 2**20

names, seqs = synth.genome_set("C4")
ps = pairs.all_pairs(names)[:3]
m0 = used()
jobs = []
for k, idx in enumerate(ps):
    pn, pq = [names[i] for i in idx], [seqs[i] for i in idx]
    a = used()
    ss = _capi.SeqSet(pq, pn)
    b = used()
    bb = BlockBuild(ss, pn, pq, lender=jobs[0][1] if jobs else None)
    c = used()
    bb.run()
    d = used()
    bb.af.clear_used()
    e = used()
    jobs.append((ss, bb))
    print("pair %d: seqset %.0f MiB, create %.0f MiB, run +%.0f MiB" % (k, b - a, c - b, d - c), flush=True)
    for dv in ("", ):
        pass
print("total %.0f MiB" % (used() - m0))
