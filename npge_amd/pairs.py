"""Pair-sharded block build: the north star's multi-GPU split for BASELINE
config C4 ("32 genomes x 5 Mbp, 2 % divergence, pair-sharded across
8 x MI355X with RCCL gather"; DESIGN.md "Multi-GPU").

The unit is a genome pair.  Every pair (i < j) of the set's genomes is one
independent DraftPangenome (lua_lib.lua:1569-1621) over the two genomes'
sequences -- the same call the reference's `npge` runs on a two-genome input,
so each pair's blocks are bit-exact with the CPU path on that pair
(tests/test_pairs_gpu.py against oracle/).  Pairs go to ranks round-robin in
pair order (all pairs of a config have about the same size); on its GPU a
rank runs `workers` pairs at a time, each worker on its own host thread with
its own aligner (device scratch and HIP stream), which the block sets of the
worker's pairs borrow in turn (npgx_blockset_create_sharing); every pair has
its own sequence set, block set and AnchorFinder handle.  The latency-bound
iterations of one pair overlap the other workers' pairs.
The data path has no collective until the end: every rank's anchored+aligned
blocks -- fragment coordinates per pair -- are all-gathered once over the
communicator (RCCL over xGMI on the GPU box: the library's own npgx_comm), so
every rank ends with the whole job's block sets.

Host-side pieces (pair list, assignment, record packing, the gather over an
npgx_comm) use no GPU call and are tested on CPU with gloo
(tests/test_pairs_dist.py).
"""
import ctypes
import itertools
import os
import threading
import time

import numpy as np

# record layout of one fragment (2 x u64):
#   w0 = pair << 44 | block << 12 | local_seq << 1 | (ori > 0)
#   w1 = min << 32 | max
PAIR_BITS, BLOCK_BITS, SEQ_BITS = 20, 32, 11
# per-pair summary record (SUMMARY_WORDS x u64): (pair << 32 | n_blocks),
# blockset hash (coordinates, block_hash.cpp:112-130), rows digest (every
# gapped row bound to its fragment, npgx_blockset_rows_digest) -- the gather
# carries the gap columns' fingerprint beside the coordinates
SUMMARY_WORDS = 3


def genomes_of(names):
    """Genome of each sequence by its name (Sequence::genome, Sequence.cpp:193-202:
    the part before the first '&'), in first-seen order -> {genome: [seq index]}."""
    out = {}
    for i, n in enumerate(names):
        out.setdefault(n.split("&", 1)[0], []).append(i)
    return out


def all_pairs(names):
    """Every pair (i < j) of the set's genomes, in order: [(seq indices of the pair)]."""
    g = list(genomes_of(names).values())
    return [tuple(g[a] + g[b]) for a, b in itertools.combinations(range(len(g)), 2)]


def assign(n_pairs, rank, world):
    """Pair indices of `rank`: round-robin in pair order."""
    return list(range(rank, n_pairs, world))


def pack_fragments(pair, bs, seq, mn, mx, ori):
    """Fragment records of one pair's block set (npgx_blockset_copy arrays)."""
    nb = len(bs) - 1
    nf = int(bs[-1]) if nb >= 0 else 0
    if nf == 0:
        return np.zeros(0, dtype=np.uint64)
    assert pair < (1 << PAIR_BITS) and nb < (1 << BLOCK_BITS)
    assert int(seq[:nf].max()) < (1 << SEQ_BITS) and int(mx[:nf].max()) < (1 << 32)
    blk = np.repeat(np.arange(nb, dtype=np.uint64), np.diff(bs).astype(np.int64))
    w0 = ((np.uint64(pair) << np.uint64(44)) | (blk << np.uint64(12))
          | (seq[:nf].astype(np.uint64) << np.uint64(1)) | (ori[:nf] > 0).astype(np.uint64))
    w1 = (mn[:nf].astype(np.uint64) << np.uint64(32)) | mx[:nf].astype(np.uint64)
    return np.stack([w0, w1], axis=1).reshape(-1)


def unpack_fragments(rec):
    """-> {pair: [[(local_seq, min, max, ori), ...] per block]} (blocks in their order)."""
    r = rec.reshape(-1, 2)
    out = {}
    for w0, w1 in r.tolist():
        p, b = w0 >> 44, (w0 >> 12) & ((1 << BLOCK_BITS) - 1)
        blocks = out.setdefault(p, [])
        while len(blocks) <= b:
            blocks.append([])
        blocks[b].append(((w0 >> 1) & ((1 << SEQ_BITS) - 1), w1 >> 32, w1 & 0xffffffff, 1 if w0 & 1 else -1))
    return out


def _struct(comm):
    from .comm import NpgxComm, TorchComm
    if isinstance(comm, TorchComm):
        return comm.struct
    return ctypes.cast(comm.pointer(), ctypes.POINTER(NpgxComm)).contents


def gather_u64(comm, arr, device=None):
    """All-gather of a variable-length u64 array over an npgx_comm (rank
    order): allgather_i64 of the counts, then one allgatherv_u64.  device: a
    torch device for the exchange buffers (RCCL needs device memory); None
    passes host arrays (gloo TorchComm with host staging, CPU tests)."""
    c = _struct(comm)
    world = c.world
    counts = (ctypes.c_int64 * world)()
    if c.allgather_i64(c.user, int(len(arr)), counts) != 0:
        raise RuntimeError("allgather_i64 failed")
    tot = sum(counts)
    if tot == 0:
        return np.zeros(0, dtype=np.uint64), list(counts)
    arr = np.ascontiguousarray(arr, dtype=np.uint64)
    if device is None:
        src = arr if len(arr) else np.zeros(1, dtype=np.uint64)
        dst = np.zeros(tot, dtype=np.uint64)
        rc = c.allgatherv_u64(c.user, src.ctypes.data, counts, dst.ctypes.data)
        out = dst
    else:
        import torch
        src = torch.from_numpy(arr.view(np.int64) if len(arr) else np.zeros(1, dtype=np.int64)).to(device)
        dst = torch.empty(tot, dtype=torch.int64, device=device)
        torch.cuda.synchronize(device)
        rc = c.allgatherv_u64(c.user, src.data_ptr(), counts, dst.data_ptr())
        out = dst.cpu().numpy().view(np.uint64)
    if rc != 0:
        raise RuntimeError("allgatherv_u64 failed")
    return out, list(counts)


# npgx_blockset_tune settings of the pair workers (results do not change).
# Many concurrent streams: the aligner kernels without the prefix search's call
# (its scratch throttled them by a fifth, gpurun_out r05n / profiles), and
# ExtendLoopFast on the host, whose bookkeeping spreads over the workers' cores
# while the device loop's many small kernels queue behind the other workers'
PAIR_TUNING = {"long-head": 0, "elf-device": 0}


def pair_tuning():
    """PAIR_TUNING, or the JSON object in NPGX_PAIR_TUNING (A/B runs)."""
    import json
    e = os.environ.get("NPGX_PAIR_TUNING")
    return dict(json.loads(e)) if e else dict(PAIR_TUNING)


class PairJobs:
    """The rank's share of the pair-sharded job: its pairs resident in HBM (one
    sequence set + block set + AnchorFinder handle per pair, made before any
    timing), run `workers` at a time; run() = one pass over the rank's pairs
    plus the final gather."""

    def __init__(self, names, seqs, rank=0, world=1, comm=None, workers=4, pairs=None, device=0,
                 gather_device=None, tuning=None):
        from . import _capi
        from .pipeline import BlockBuild
        self.pairs = all_pairs(names) if pairs is None else list(pairs)
        self.mine = assign(len(self.pairs), rank, world)
        self.comm = comm
        self.workers = max(1, int(workers))
        self.device = device
        self.gather_device = gather_device
        self.pair_bp = [sum(len(seqs[i]) for i in self.pairs[p]) for p in range(len(self.pairs))]
        # worker w runs the rank's pairs owner[k] == w one after another, all on
        # the aligner and AnchorFinder handle of its first pair
        # (npgx_blockset_create_sharing): device memory is one aligner's
        # scratch per worker, not per pair.  One mapping decides both the
        # lender and the schedule (_run_pairs asserts it).
        self.owner = [k % self.workers for k in range(len(self.mine))]
        self.jobs = []
        first = {}
        for k, p in enumerate(self.mine):
            idx = self.pairs[p]
            pn, ps = [names[i] for i in idx], [seqs[i] for i in idx]
            ss = _capi.SeqSet(ps, pn)
            w = self.owner[k]
            lender = self.jobs[first[w]][2] if w in first else None
            first.setdefault(w, k)
            bb = BlockBuild(ss, pn, ps, lender=lender)
            if lender is None:  # the worker's aligner (shared by its pairs) and the mode its pairs inherit
                for key, value in (pair_tuning() if tuning is None else tuning).items():
                    bb.eng.tune(key, value)
            self.jobs.append((p, ss, bb))
        self.ktimes = [None] * len(self.jobs)
        self.records = None
        self.summary = None

    def total_bp(self):
        """Input bp of the whole job (all ranks' pairs)."""
        return sum(self.pair_bp)

    def rank_bp(self):
        return sum(self.pair_bp[p] for p, _, _ in self.jobs)

    def _run_pairs(self):
        from . import _capi
        infos = [None] * len(self.jobs)
        recs = self._recs = [None] * len(self.jobs)
        errors = []

        def worker(w):
            try:
                _capi.check(_capi.lib().npgx_set_device(self.device))
                for k in [k for k in range(len(self.jobs)) if self.owner[k] == w]:
                    if errors:
                        return
                    infos[k] = self.jobs[k][2].run()
                    # this pair's own kernel times: the handles it borrowed are
                    # reused by the worker's next pair
                    self.ktimes[k] = self.jobs[k][2].kernel_times()
                    recs[k] = self._records(k)  # packed on the worker, overlapping the others' pairs
            except Exception as e:  # re-raised on the calling thread
                errors.append(e)

        n = min(self.workers, len(self.jobs))
        if n <= 1:
            worker(0)
        else:
            ts = [threading.Thread(target=worker, args=(w,)) for w in range(n)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        if errors:
            raise errors[0]
        return infos

    def _records(self, k):
        """(fragment records, summary record) of the rank's k-th pair."""
        p, _, job = self.jobs[k]
        bs, seq, mn, mx, ori = job.eng.fragments()
        return (pack_fragments(p, bs, seq, mn, mx, ori),
                np.array([(p << 32) | (len(bs) - 1), job.eng.hash(), job.eng.rows_digest()], dtype=np.uint64))

    def local_records(self):
        recs = [self._records(k) for k in range(len(self.jobs))]
        return self._cat(recs)

    @staticmethod
    def _cat(recs):
        cat = (lambda a: np.concatenate(a) if a else np.zeros(0, dtype=np.uint64))
        return cat([r[0] for r in recs]), cat([r[1] for r in recs])

    def run(self):
        import resource
        r0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        infos = self._run_pairs()
        t1 = time.perf_counter()
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        # host cores kept busy while the pairs ran (user + system CPU time / wall)
        cores_busy = ((r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)) / max(t1 - t0, 1e-9)
        frs, sums = self._cat(self._recs)
        if self.comm is not None:  # the one collective: the final anchored-block gather
            frs, _ = gather_u64(self.comm, frs, self.gather_device)
            sums, _ = gather_u64(self.comm, sums, self.gather_device)
        self.records, self.summary = frs, sums
        t2 = time.perf_counter()
        done = [i for i in infos if i is not None]
        return {"pairs": len(self.pairs), "pairs_rank": len(self.jobs), "workers": self.workers,
                "ms_pairs": round((t1 - t0) * 1e3, 3), "ms_gather": round((t2 - t1) * 1e3, 3),
                "host_cores_busy": round(cores_busy, 2),
                "gathered_fragments": int(len(frs) // 2), "gathered_pairs": int(len(sums) // SUMMARY_WORDS),
                "stem_blocks": int(sum(i["stem_blocks"] for i in done)),
                "aligned_residues": int(sum(i["aligned_residues"] for i in done)),
                "align_jobs": int(sum(i["align_jobs"] for i in done)),
                # one pair's engine timings, averaged (wall clock of its own thread)
                "mean_pair_ms": {k: round(sum(i["ms_stage_host"][k] for i in done) / max(len(done), 1), 3)
                                 for k in (done[0]["ms_stage_host"] if done else {})},
                "mean_pair_ms_align": round(sum(i.get("ms_align_wall", 0.0) for i in done) / max(len(done), 1), 3),
                "mean_pair_ms_host": round(sum(i["ms_host_bookkeeping"] for i in done) / max(len(done), 1), 3)}

    def hashes(self):
        """{pair: blockset hash} of the gathered summaries (after run())."""
        s = self.summary.reshape(-1, SUMMARY_WORDS)
        return {int(r[0] >> 32): int(r[1]) for r in s.tolist()}

    def row_digests(self):
        """{pair: rows digest} of the gathered summaries (after run())."""
        s = self.summary.reshape(-1, SUMMARY_WORDS)
        return {int(r[0] >> 32): int(r[2]) for r in s.tolist()}

    def kernel_times(self):
        """Per-kernel totals over the rank's pairs of the last run(), each pair's
        times collected on its worker right after that pair ran."""
        agg = {}
        for kts in self.ktimes:
            for k in kts or []:
                a = agg.setdefault(k["name"], {"name": k["name"], "ms": 0.0, "bytes": 0.0, "launches": 0})
                a["ms"] += k["ms"]
                a["bytes"] += k["bytes"]
                a["launches"] += k["launches"]
        return list(agg.values())
