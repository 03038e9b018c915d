"""Block-build driver used by bench.py and smoke(): one step = DraftPangenome on
a device-resident genome set (AnchorFinder -> RemoveNonStem --exact ->
DummyAligner -> ExtendLoopFast(10) -> Filter, src/algo/lua_lib.lua:1569-1621),
optionally followed by one AnchorLoopFast (lua_lib.lua:741-758) or one
AnchorLoop (lua_lib.lua:711-737), the pipes the real pipeline grows blocks
with where the exact stem anchors are too few (C4: 32 genomes at 2 %
divergence).
"""
from .anchor_finder import AnchorFinder
from .blockset import BlockSetEngine

STAGES = ["AnchorFinder", "RemoveNonStem", "DummyAligner", "ExtendLoopFast(10)", "Filter"]


class BlockBuild:
    def __init__(self, seqset, names, seqs, seed=1, comm=None, anchor_loop=False, lender=None):
        self.ss = seqset
        self.seed = seed
        # anchor_loop: False, True / "fast" (AnchorLoopFast) or "full" (AnchorLoop)
        self.loop_pipe = {True: "AnchorLoopFast", "fast": "AnchorLoopFast", "full": "AnchorLoop"}.get(anchor_loop)
        self.anchor_loop = self.loop_pipe is not None
        self.loop_af = AnchorFinder() if self.anchor_loop else None
        # lender: a BlockBuild whose aligner this one borrows (never run together)
        self.eng = BlockSetEngine(seqset, lender=lender.eng if lender is not None else None)
        if comm is not None:  # one genome set sharded over the ranks of comm
            self.eng.set_comm(comm)
        # the AnchorFinder handle: its own, or the lender's (its window layout is
        # rebuilt when the sequence set changes, its used set cleared per run)
        self.af = lender.af if lender is not None else AnchorFinder()
        self.af.set_opt_value("bloom-seed", self.seed)

    def workload_name(self, config):
        return "%s DraftPangenome: %s%s" % (config, " -> ".join(STAGES),
                                            " -> " + self.loop_pipe if self.anchor_loop else "")

    def run(self):
        # one AnchorFinder handle (device buffers kept); its used-hash set is
        # cleared so that every step does identical work
        self.af.clear_used()
        self.eng.apply("DraftPangenome", af=self.af)
        st = self.eng.stats()
        loop = None
        if self.anchor_loop:  # a fresh pipe each step: its AnchorFinder's used set cleared
            draft_kt = self.eng.kernel_times()
            self.loop_af.clear_used()
            self.eng.reset_loop()
            self.eng.apply(self.loop_pipe, af=self.loop_af)
            lst = self.eng.stats()
            if self.loop_pipe == "AnchorLoopFast":
                counts = lst["loop"]
            else:
                counts = dict(self.eng.anchor_loop_stats(), adding_loop_rounds=lst["counters"]["spare"])
                lst["ms_loop"] = dict(zip(["filter_to_anchor_finder", "dummy_to_remove_with_same_name",
                                           "split_extendable", "deconseq_1", "extend_loop_cons",
                                           "extend_loop_deconseq", "deconseq_2", "align"],
                                          lst["ms_loop"].values()))
            loop = dict(counts, pipe=self.loop_pipe, ms_host=round(lst["ms_host"], 3),
                        ms_align=round(lst["ms_align"], 3), ms_loop=lst["ms_loop"], ms_stage=lst["ms_stage"])
            self._extra_kt = draft_kt + self.loop_af.kernel_times()
        else:
            self._extra_kt = []
        out = {"anchor_blocks": int(st["anchor_blocks"]), "stem_blocks": int(st["stem_blocks"]),
               "iterations": int(st["iterations"]), "aligned_residues": int(st["aligned_residues"]),
               "align_jobs": int(st["align_jobs"]), "device_loop": st["device_iterations"] > 0,
               "ms_host_bookkeeping": round(st["ms_host"], 3), "ms_stage_host": st["ms_stage"],
               "counters": st["counters"], "anchor_loop": loop}
        if not out["device_loop"]:  # (the device loop's is the aligner's enqueue time: see stage_timeline)
            out["ms_align_wall"] = round(st["ms_align"], 3)
        return out

    def stage_timeline(self):
        """One extra DraftPangenome with the engine's stage clock on (HIP events
        at the stage boundaries on its stream; each costs the GPU a few
        microseconds, so callers run it outside any timed region): the step's
        GPU timeline by stage, which sums to the step's span, and the wall
        time of that step."""
        import time
        self.eng.tune("stage-clock", 1)
        try:
            self.af.clear_used()
            t = time.perf_counter()
            self.eng.apply("DraftPangenome", af=self.af)
            wall = (time.perf_counter() - t) * 1e3
        finally:
            self.eng.tune("stage-clock", 0)
        ms = self.eng.stats()["ms_gpu"]
        return {"ms": ms, "sum_ms": round(sum(ms.values()), 3), "step_wall_ms": round(wall, 3),
                "largest": max(ms, key=ms.get),
                "source": "HIP events at the stage boundaries of one extra untimed DraftPangenome step "
                          "(npgx_blockset_tune stage-clock; intervals include the idle time the host leaves)"}

    def kernel_times(self):
        """Per-kernel totals of the last step: name -> (ms, bytes, launches)."""
        agg = {}
        for k in self.af.kernel_times() + self.eng.kernel_times() + getattr(self, "_extra_kt", []):
            a = agg.setdefault(k["name"], {"name": k["name"], "ms": 0.0, "bytes": 0.0, "launches": 0})
            a["ms"] += k["ms"]
            a["bytes"] += k["bytes"]
            a["launches"] += 1
        return list(agg.values())
