"""Block-build driver used by bench.py and smoke(): one step = DraftPangenome on
a device-resident genome set (AnchorFinder -> RemoveNonStem --exact ->
DummyAligner -> ExtendLoopFast(10) -> Filter, src/algo/lua_lib.lua:1569-1621).
"""
from .anchor_finder import AnchorFinder
from .blockset import BlockSetEngine

STAGES = ["AnchorFinder", "RemoveNonStem", "DummyAligner", "ExtendLoopFast(10)", "Filter"]


class BlockBuild:
    def __init__(self, seqset, names, seqs, seed=1, comm=None):
        self.ss = seqset
        self.seed = seed
        self.eng = BlockSetEngine(seqset)
        if comm is not None:  # one genome set sharded over the ranks of comm
            self.eng.set_comm(comm)
        self.af = AnchorFinder()
        self.af.set_opt_value("bloom-seed", self.seed)

    def workload_name(self, config):
        return "%s DraftPangenome: %s" % (config, " -> ".join(STAGES))

    def run(self):
        # one AnchorFinder handle (device buffers kept); its used-hash set is
        # cleared so that every step does identical work
        self.af.clear_used()
        self.eng.apply("DraftPangenome", af=self.af)
        st = self.eng.stats()
        return {"anchor_blocks": int(st["anchor_blocks"]), "stem_blocks": int(st["stem_blocks"]),
                "iterations": int(st["iterations"]), "aligned_residues": int(st["aligned_residues"]),
                "align_jobs": int(st["align_jobs"]), "ms_align_wall": round(st["ms_align"], 3),
                "ms_host_bookkeeping": round(st["ms_host"], 3), "ms_stage": st["ms_stage"],
                "counters": st["counters"]}

    def kernel_times(self):
        """Per-kernel totals of the last step: name -> (ms, bytes, launches)."""
        agg = {}
        for k in self.af.kernel_times() + self.eng.kernel_times():
            a = agg.setdefault(k["name"], {"name": k["name"], "ms": 0.0, "bytes": 0.0, "launches": 0})
            a["ms"] += k["ms"]
            a["bytes"] += k["bytes"]
            a["launches"] += 1
        return list(agg.values())
