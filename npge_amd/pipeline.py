"""Block-build driver for the benchmark and the smoke test.

Round-1 state: the step is AnchorFinder on the device-resident genome set; the
DraftPangenome block build after it (RemoveNonStem -> DummyAligner ->
ExtendLoopFast -> Filter, src/algo/lua_lib.lua:1569-1621) is added stage by
stage as its kernels reach parity (DESIGN.md "Status").
"""
import time

from .anchor_finder import AnchorFinder


class BlockBuild:
    def __init__(self, seqset, names, seqs, seed=1):
        self.ss = seqset
        self.names = names
        self.af = AnchorFinder()
        self.af.set_opt_value("bloom-seed", seed)
        self.stages = ["AnchorFinder"]

    def workload_name(self, config):
        return "%s: %s" % (config, " -> ".join(self.stages))

    def run(self):
        # a fresh instance per step keeps every step identical (no used hashes)
        self.af = AnchorFinder()
        r = self.af.find(self.ss)
        return {"anchor_blocks": int(len(r["block_start"]) - 1),
                "anchor_fragments": int(len(r["seq"])), "collected": int(r["n_collected"]),
                "found_fragments": int(r["n_found_frags"])}

    def kernel_times(self):
        return self.af.kernel_times()


def cpu_reference_step(orc, names, seqs, seed=1):
    """Seconds for the same step on the CPU restatement (1 worker)."""
    af = orc.AnchorFinder(seed=seed)
    t = time.perf_counter()
    af.run(seqs, names)
    return time.perf_counter() - t
