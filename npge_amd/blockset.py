"""Block-set processors on the engine (npgx_blockset_*).

Mirrors the reference's BlockSet + per-block processors of the block build:
RemoveNonStem, DummyAligner, MetaAligner, FragmentsExtender, FixEnds,
OverlaplessUnion, ExtendLoopFast, Filter, MoveGaps, CutGaps,
SelfOverlapsResolver, the Align / LiteAlign pipes (Align.cpp:17-52), Rest,
AnchorLoopFast and the DraftPangenome driver (lua_lib.lua:1569-1621).
Alignment work goes to the HIP aligner in one batch per processor pass.
"""
import ctypes

import numpy as np

from . import _capi


class BbOptions(ctypes.Structure):
    _fields_ = [("extend_length", ctypes.c_int32), ("max_iterations", ctypes.c_int32),
                ("extend_portion_x1e4", ctypes.c_int64), ("min_fragment", ctypes.c_int32),
                ("frame_length", ctypes.c_int32), ("min_end", ctypes.c_int32),
                ("min_block", ctypes.c_int32), ("max_block", ctypes.c_int32),
                ("find_subblocks", ctypes.c_int32), ("min_identity_x1e4", ctypes.c_int64),
                ("align", _capi.AlignOptions), ("max_tail", ctypes.c_int32),
                ("max_tail_to_gap_x1e4", ctypes.c_int64)]


class BbStats(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int64), ("aligned_residues", ctypes.c_int64),
                ("align_jobs", ctypes.c_int64), ("anchor_blocks", ctypes.c_int64),
                ("stem_blocks", ctypes.c_int64), ("ms_align", ctypes.c_double),
                ("ms_host", ctypes.c_double), ("ms_stage", ctypes.c_double * 16),
                ("counters", ctypes.c_int64 * 8), ("loop", ctypes.c_int64 * 8),
                ("ms_loop", ctypes.c_double * 8), ("ms_gpu", ctypes.c_double * 12),
                ("device_iterations", ctypes.c_int64), ("device_sync_iterations", ctypes.c_int64)]

STAGE_NAMES = ["anchor_finder", "stem_dummy", "move_unchanged", "flank_gather", "align_batch",
               "stitch", "fix_ends", "overlapless_union", "blockset_hash", "filter",
               "align_host_prep", "device_wait", "fix_ends_device", "fix_ends_slice",
               "ou_order", "ou_admit"]
# npgx_bb_stats.ms_gpu: DraftPangenome's GPU timeline by stage ("stage-clock" tuning)
GPU_STAGE_NAMES = ["anchor_finder", "stem_dummy", "elf_upload", "elf_plan", "flank_decode", "align", "stitch",
                   "fix_ends", "overlapless_union", "elf_download", "filter", "extend_loop_host"]
JOB_STATS = 24  # NPGX_JOB_STATS
COUNTER_NAMES = ["blocks_after_extend", "filter_whole", "filter_slices", "blocks_after_filter",
                 "ou_in", "ou_rejected", "hashes", "spare"]
# AnchorLoop's npgx_bb_stats.loop (the oracle's orc_bs_anchor_loop_stats, same order)
ANCHOR_LOOP_NAMES = ["cons_seqs", "cons_anchors", "anchors_left", "split_blocks", "cons_blocks", "dec_blocks",
                     "cons_iterations", "dec_iterations"]
LOOP_NAMES = ["consensus_sequences", "anchors", "cons_blocks", "mapped_blocks", "loop_iterations",
              "unchanged_dropped"]
LOOP_STAGE_NAMES = ["filter_rest", "conseq", "anchor_finder", "move_unchanged_dummy", "extend_and_align",
                    "extend_loop_fast", "deconseq", "align"]


def _bind(L):
    if getattr(L, "_bb_bound", False):
        return L
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    P = ctypes.POINTER
    L.npgx_bb_default_options.argtypes = [P(BbOptions)]
    L.npgx_bb_default_options.restype = None
    L.npgx_blockset_create.argtypes = [vp, P(BbOptions), P(vp)]
    L.npgx_blockset_create_sharing.argtypes = [vp, P(BbOptions), vp, P(vp)]
    L.npgx_blockset_set_blocks.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp]
    L.npgx_blockset_add_anchors.argtypes = [vp, vp]
    L.npgx_blockset_set_comm.argtypes = [vp, vp]
    L.npgx_blockset_apply.argtypes = [vp, ctypes.c_char_p, vp]
    L.npgx_blockset_counts.argtypes = [vp, P(i64), P(i64), P(i64)]
    L.npgx_blockset_copy.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp]
    L.npgx_blockset_hash.argtypes = [vp, P(ctypes.c_uint64)]
    L.npgx_blockset_rows_digest.argtypes = [vp, P(ctypes.c_uint64)]
    L.npgx_blockset_conseq.argtypes = [vp, vp, vp, P(i64), P(i64)]
    L.npgx_blockset_deconseq.argtypes = [vp, vp, vp]
    L.npgx_blockset_stats.argtypes = [vp, P(BbStats)]
    L.npgx_blockset_kernel_times.argtypes = [vp, P(_capi.KernelTime), ctypes.c_int32,
                                             P(ctypes.c_int32)]
    L.npgx_blockset_job_stats.argtypes = [vp, vp, i64, P(i64)]
    L.npgx_blockset_reset_loop.argtypes = [vp]
    L.npgx_blockset_free.argtypes = [vp]
    L.npgx_blockset_free.restype = None
    L._bb_bound = True
    return L


ALIGN_KEYS = ("mismatch_check", "gap_check", "aligned_check", "align_min_length",
              "align_min_identity_x1e4")


def default_options(**kw):
    L = _bind(_capi.lib())
    o = BbOptions()
    L.npgx_bb_default_options(ctypes.byref(o))
    for k, v in kw.items():
        if k in ALIGN_KEYS:
            setattr(o.align, k.replace("align_", ""), v)
        else:
            setattr(o, k, v)
    return o


class BlockSetEngine:
    """One npgx_blockset over a device sequence set."""

    def __init__(self, seqset, options=None, lender=None, **kw):
        """lender: another engine whose aligner this one borrows
        (npgx_blockset_create_sharing): never run the two at the same time."""
        L = _bind(_capi.lib())
        self.ss = seqset
        o = options or default_options(**kw)
        h = ctypes.c_void_p()
        if lender is None:
            _capi.check(L.npgx_blockset_create(seqset.handle, ctypes.byref(o), ctypes.byref(h)))
        else:
            _capi.check(L.npgx_blockset_create_sharing(seqset.handle, ctypes.byref(o), lender._h,
                                                       ctypes.byref(h)))
        self._lender = lender  # freed after this engine
        self._h = h

    def set_comm(self, comm):
        """Shards DraftPangenome / FragmentsExtender over comm's ranks
        (npge_amd.comm.TorchComm); None returns to one GPU."""
        self._comm = comm  # the library keeps a pointer to comm.struct
        _capi.check(_capi.lib().npgx_blockset_set_comm(self._h, comm.pointer() if comm else None))
        return self

    def set_blocks(self, blocks):
        """blocks: list of lists of (seq_index, min, max, ori, row_or_None)."""
        L = _capi.lib()
        frs = [f for b in blocks for f in b]
        bs = np.zeros(len(blocks) + 1, dtype=np.int64)
        np.cumsum([len(b) for b in blocks], out=bs[1:])
        seq = np.array([f[0] for f in frs] or [0], dtype=np.int32)
        mn = np.array([f[1] for f in frs] or [0], dtype=np.int64)
        mx = np.array([f[2] for f in frs] or [0], dtype=np.int64)
        ori = np.array([f[3] for f in frs] or [1], dtype=np.int8)
        has_rows = any(f[4] is not None for f in frs)
        if has_rows:  # per block: rows for every fragment, or none (zero-length rows)
            rows = "".join(f[4] or "" for f in frs).encode()
            ro = np.zeros(len(frs) + 1, dtype=np.int64)
            np.cumsum([len(f[4] or "") for f in frs], out=ro[1:])
            buf = ctypes.create_string_buffer(rows, max(len(rows), 1))
            _capi.check(L.npgx_blockset_set_blocks(self._h, len(blocks), _capi.ptr(bs), _capi.ptr(seq),
                                                   _capi.ptr(mn), _capi.ptr(mx), _capi.ptr(ori),
                                                   _capi.ptr(ro), ctypes.cast(buf, ctypes.c_void_p)))
        else:
            _capi.check(L.npgx_blockset_set_blocks(self._h, len(blocks), _capi.ptr(bs), _capi.ptr(seq),
                                                   _capi.ptr(mn), _capi.ptr(mx), _capi.ptr(ori),
                                                   None, None))
        return self

    def apply(self, processor, af=None):
        L = _capi.lib()
        afh = af._handle() if af is not None else None
        _capi.check(L.npgx_blockset_apply(self._h, processor.encode(), afh))
        return self

    def reset_loop(self):
        """Forget AnchorLoopFast's MoveUnchanged hashes (a fresh pipe)."""
        _capi.check(_capi.lib().npgx_blockset_reset_loop(self._h))
        return self

    def blocks(self):
        L = _capi.lib()
        nb, nf, rb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _capi.check(L.npgx_blockset_counts(self._h, ctypes.byref(nb), ctypes.byref(nf), ctypes.byref(rb)))
        n = max(nf.value, 1)
        bs = np.zeros(nb.value + 1, dtype=np.int64)
        seq = np.zeros(n, dtype=np.int32)
        mn = np.zeros(n, dtype=np.int64)
        mx = np.zeros(n, dtype=np.int64)
        ori = np.zeros(n, dtype=np.int8)
        ro = np.zeros(n + 1, dtype=np.int64)
        rows = ctypes.create_string_buffer(max(rb.value, 1))
        _capi.check(L.npgx_blockset_copy(self._h, _capi.ptr(bs), _capi.ptr(seq), _capi.ptr(mn),
                                         _capi.ptr(mx), _capi.ptr(ori), _capi.ptr(ro),
                                         ctypes.cast(rows, ctypes.c_void_p)))
        raw = rows.raw
        out = []
        for b in range(nb.value):
            blk = []
            for i in range(bs[b], bs[b + 1]):
                row = raw[ro[i]:ro[i + 1]].decode() if ro[i + 1] > ro[i] else None
                blk.append((int(seq[i]), int(mn[i]), int(mx[i]), int(ori[i]), row))
            out.append(blk)
        return out

    def fragments(self):
        """Fragment coordinates without rows (no row download): numpy arrays
        (block_start[nb + 1], seq, min, max, ori) in block order."""
        L = _capi.lib()
        nb, nf, rb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _capi.check(L.npgx_blockset_counts(self._h, ctypes.byref(nb), ctypes.byref(nf), ctypes.byref(rb)))
        n = max(nf.value, 1)
        bs = np.zeros(nb.value + 1, dtype=np.int64)
        seq = np.zeros(n, dtype=np.int32)
        mn = np.zeros(n, dtype=np.int64)
        mx = np.zeros(n, dtype=np.int64)
        ori = np.zeros(n, dtype=np.int8)
        _capi.check(L.npgx_blockset_copy(self._h, _capi.ptr(bs), _capi.ptr(seq), _capi.ptr(mn),
                                         _capi.ptr(mx), _capi.ptr(ori), None, None))
        return bs, seq[:nf.value], mn[:nf.value], mx[:nf.value], ori[:nf.value]

    def conseq(self):
        """ConSeq (ConSeq.cpp:37-50): the text of the sequence each block
        becomes, in block order (consensus of aligned blocks on the GPU)."""
        L = _bind(_capi.lib())
        nb, tot = ctypes.c_int64(), ctypes.c_int64()
        _capi.check(L.npgx_blockset_conseq(self._h, None, None, ctypes.byref(nb), ctypes.byref(tot)))
        buf = ctypes.create_string_buffer(max(tot.value, 1))
        off = np.zeros(nb.value + 1, dtype=np.int64)
        _capi.check(L.npgx_blockset_conseq(self._h, ctypes.cast(buf, ctypes.c_void_p), _capi.ptr(off),
                                           ctypes.byref(nb), ctypes.byref(tot)))
        raw = buf.raw
        return [raw[off[i]:off[i + 1]].decode() for i in range(nb.value)]

    def deconseq(self, cons, source=None):
        """DeConSeq (DeConSeq.cpp:48-96): the blocks of `cons` (an engine over
        the sequences conseq() made of `source`'s blocks, sequence i = block i)
        mapped back onto source's sequences and appended to this engine's
        blocks; source defaults to this engine."""
        L = _bind(_capi.lib())
        src = self if source is None else source
        _capi.check(L.npgx_blockset_deconseq(self._h, src._h, cons._h))
        return self

    def tune(self, key, value):
        """npgx_blockset_tune: "long-head" (the aligner's incremental shifts
        before the prefix search; 0 = never, the low-scratch kernels) or
        "elf-device" (1 / 0 / -1: ExtendLoopFast on the device / host /
        default) or "stage-clock" (1: DraftPangenome fills stats()["ms_gpu"],
        its GPU timeline by stage).  Results do not change."""
        _capi.check(_capi.lib().npgx_blockset_tune(self._h, key.encode(), ctypes.c_int64(int(value))))
        return self

    def hash(self):
        h = ctypes.c_uint64()
        _capi.check(_capi.lib().npgx_blockset_hash(self._h, ctypes.byref(h)))
        return h.value

    def rows_digest(self):
        """npgx_blockset_rows_digest: a device-computed 64-bit digest of every
        gapped row bound to its fragment (tests/helpers.py restates it)."""
        h = ctypes.c_uint64()
        _capi.check(_capi.lib().npgx_blockset_rows_digest(self._h, ctypes.byref(h)))
        return h.value

    def stats(self):
        st = BbStats()
        _capi.check(_capi.lib().npgx_blockset_stats(self._h, ctypes.byref(st)))
        d = {k: getattr(st, k) for k, _ in BbStats._fields_
             if k not in ("ms_stage", "counters", "loop", "ms_loop", "ms_gpu")}
        d["ms_gpu"] = {n: round(st.ms_gpu[i], 3) for i, n in enumerate(GPU_STAGE_NAMES)}
        d["ms_stage"] = {n: round(st.ms_stage[i], 3) for i, n in enumerate(STAGE_NAMES)}
        d["counters"] = {n: int(st.counters[i]) for i, n in enumerate(COUNTER_NAMES)}
        d["loop"] = {n: int(st.loop[i]) for i, n in enumerate(LOOP_NAMES)}
        d["ms_loop"] = {n: round(st.ms_loop[i], 3) for i, n in enumerate(LOOP_STAGE_NAMES)}
        d["loop_raw"] = [int(x) for x in st.loop]  # per pipe: AnchorLoopFast's LOOP_NAMES or AnchorLoop's
        return d

    def anchor_loop_stats(self):
        """Counts of the last AnchorLoop (include/npge_amd.h, npgx_bb_stats.loop)."""
        return dict(zip(ANCHOR_LOOP_NAMES, self.stats()["loop_raw"]))

    def job_stats(self):
        """(n_jobs, NPGX_JOB_STATS) int64 per alignment job of the last apply
        (layout in include/npge_amd.h, npgx_align_job_stats)."""
        L = _capi.lib()
        n = ctypes.c_int64()
        _capi.check(L.npgx_blockset_job_stats(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros((max(n.value, 1), JOB_STATS), dtype=np.int64)
        _capi.check(L.npgx_blockset_job_stats(self._h, _capi.ptr(out), n.value, ctypes.byref(n)))
        return out[:n.value]

    def kernel_times(self):
        return _capi.kernel_times(_capi.lib().npgx_blockset_kernel_times, self._h)

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            try:
                _capi.lib().npgx_blockset_free(self._h)
            except Exception:
                pass
            self._h = None
