"""ctypes front-end of the CPU restatement (oracle/npge_oracle.cpp).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, ``__graft_entry__.smoke()`` and
the ``cpu_baseline`` leg of bench.py, as the parity checker.  The product
package ``npge_amd`` never imports this module.

Parity is pinned against the reference's own known-answer tests
(src/test/hash.cpp, bloom_filter.cpp, anchor_finder.cpp, similar_aligner.cpp,
aligner.cpp and test-script/anchor_finder/*) -- see tests/test_oracle_kat.py.
The reference itself cannot be built here (Boost/Lua/luabind absent), so there
is no oracle/_ref build ("Oracle").
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def use_native():
    """Selects a copy of the restatement built -O3 -march=native on THIS host
    (bench.py's cpu_baseline leg, timed on the GPU box's own cores).  The build
    goes to the temp directory under a name keyed by the sources and the host's
    CPU flags, so a library built on another machine is never picked up.  Must
    be called before the first lib().  Returns False (prebuilt library kept)
    when no compiler is available."""
    global _LIB_PATH
    import hashlib
    import tempfile
    if _lib is not None:
        return _LIB_PATH.endswith("_native.so")
    srcs = ["npge_oracle.cpp", "general_aligner.cpp"]
    h = hashlib.sha1()
    for f in srcs + ["log_score.inc"]:
        h.update(open(os.path.join(_HERE, f), "rb").read())
    try:
        h.update(open("/proc/cpuinfo", "rb").read().split(b"\n\n")[0])
    except OSError:
        pass
    out = os.path.join(tempfile.gettempdir(), "npgx_oracle_%s_native.so" % h.hexdigest()[:16])
    if not os.path.exists(out):
        tmp = out + ".%d.tmp" % os.getpid()
        try:
            subprocess.check_call(["g++", "-O3", "-march=native", "-std=c++17", "-fPIC", "-shared",
                                   "-pthread", "-o", tmp] + [os.path.join(_HERE, f) for f in srcs])
        except (OSError, subprocess.CalledProcessError):
            return False
        os.replace(tmp, out)
    _LIB_PATH = out
    return True


def lib():
    global _lib
    if _lib is None:
        if _LIB_PATH.endswith("liboracle.so") and (not os.path.exists(_LIB_PATH) or any(
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, f))
            for f in ("npge_oracle.cpp", "general_aligner.cpp")
        )):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64, i64, i32, u32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32
        vp = ctypes.c_void_p
        L.orc_glibc_rand.argtypes = [u32, ctypes.c_int, vp]
        L.orc_make_hash.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.orc_make_hash.restype = u64
        L.orc_reuse_hash.argtypes = [u64, ctypes.c_int, ctypes.c_char, ctypes.c_char, ctypes.c_int]
        L.orc_reuse_hash.restype = u64
        L.orc_complement_hash.argtypes = [u64, ctypes.c_int]
        L.orc_complement_hash.restype = u64
        L.orc_optimal_bits.argtypes = [u64, ctypes.c_double]
        L.orc_optimal_bits.restype = i64
        L.orc_optimal_hashes.argtypes = [u64, u64]
        L.orc_optimal_hashes.restype = ctypes.c_int
        L.orc_weight_factor.argtypes = [i64]
        L.orc_weight_factor.restype = ctypes.c_int
        L.orc_to_atgcn.argtypes = [ctypes.c_char_p, i64, vp]
        L.orc_to_atgcn.restype = i64
        L.orc_af_create.argtypes = [ctypes.c_int, i64, ctypes.c_int, i64, u32]
        L.orc_af_create.restype = vp
        L.orc_af_set_params.argtypes = [vp, vp, ctypes.c_int]
        L.orc_af_free.argtypes = [vp]
        L.orc_af_run.argtypes = [vp, ctypes.c_int, vp, vp, vp]
        L.orc_af_run.restype = ctypes.c_int
        L.orc_af_stats.argtypes = [vp, vp]
        L.orc_af_params.argtypes = [vp, vp]
        L.orc_af_fragments.argtypes = [vp, vp, vp, vp, vp, vp]
        L.orc_af_used.argtypes = [vp, vp]
        L.orc_align.argtypes = [ctypes.c_int, ctypes.c_char_p, vp, vp, ctypes.c_int, vp, i64,
                                ctypes.POINTER(i64), ctypes.POINTER(i64)]
        L.orc_align.restype = ctypes.c_int
        P32 = ctypes.POINTER(ctypes.c_int)
        L.orc_ga_align.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, P32, P32, P32, vp, P32]
        L.orc_ga_align.restype = ctypes.c_int
        L.orc_good_slices.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      vp, ctypes.c_int]
        L.orc_good_slices.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def glibc_rand(seed, n):
    out = np.zeros(n, dtype=np.int32)
    lib().orc_glibc_rand(seed, n, _ptr(out))
    return [int(x) for x in out]


def make_hash(s, ori=1, start=None, length=None):
    """make_hash(start, length, ori) of make_hash.hpp:67-78 on string s."""
    b = s.encode() if isinstance(s, str) else s
    buf = ctypes.create_string_buffer(b, len(b))
    start = 0 if start is None else start
    length = len(b) - start if length is None else length
    addr = ctypes.addressof(buf) + start
    return lib().orc_make_hash(ctypes.cast(addr, ctypes.c_char_p), length, ori)


def reuse_hash(h, length, rm, ad, forward=True):
    return lib().orc_reuse_hash(h, length, rm.encode(), ad.encode(), int(forward))


def complement_hash(h, k):
    return lib().orc_complement_hash(h, k)


def optimal_bits(members, p):
    return lib().orc_optimal_bits(members, p)


def optimal_hashes(members, bits):
    return lib().orc_optimal_hashes(members, bits)


def good_slices(scores, frame_length, end_length, min_identity, min_length):
    """goodSlices (goodSlices.cpp:247-255) over column scores: [(start, stop)]."""
    L = lib()
    sc = np.ascontiguousarray(scores, dtype=np.int32)
    cap = len(sc) + 1
    out = np.zeros(2 * cap, dtype=np.int64)
    n = L.orc_good_slices(_ptr(sc), len(sc), frame_length, end_length, min_identity, min_length, _ptr(out), cap)
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]


def weight_factor(min_identity_x1e4):
    return lib().orc_weight_factor(min_identity_x1e4)


def general_align(a, b, gap_range, max_errors, gap_penalty=1, mismatch_penalty=1,
                  cut_tail=False):
    """GeneralAligner align (+ cut_tail) + export_alignment on nucleotide
    contents (oracle/general_aligner.cpp).  Returns dict(first_last,
    second_last, score, ops) with ops 0 = MATCH, 1 = ROW_INC (letter of the
    first sequence only), 2 = COL_INC (second only); {"status": -1} for the reference's
    "row and column are not last" exception, {"status": -2} for an empty input."""
    ab = a.encode() if isinstance(a, str) else a
    bb = b.encode() if isinstance(b, str) else b
    ops = np.zeros(len(ab) + len(bb) + 1, dtype=np.int8)
    fl, sl, sc, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = lib().orc_ga_align(ab, len(ab), bb, len(bb), gap_range, max_errors, gap_penalty,
                            mismatch_penalty, int(cut_tail), ctypes.byref(fl), ctypes.byref(sl),
                            ctypes.byref(sc), _ptr(ops), ctypes.byref(n))
    if rc != 0:
        return {"status": rc}
    return dict(status=0, first_last=fl.value, second_last=sl.value, score=sc.value, ops=ops[:n.value].copy())


def ops_to_rows(a, b, ops):
    """Gapped rows of an exported alignment (pairs of positions, -1 = gap)."""
    ra, rb, i, j = [], [], 0, 0
    for o in ops:
        if o in (0, 1):
            ra.append(a[i])
            i += 1
        else:
            ra.append("-")
        if o in (0, 2):
            rb.append(b[j])
            j += 1
        else:
            rb.append("-")
    return "".join(ra), "".join(rb)


def to_atgcn(s):
    b = s.encode() if isinstance(s, str) else s
    out = ctypes.create_string_buffer(max(len(b), 1))
    n = lib().orc_to_atgcn(b, len(b), ctypes.cast(out, ctypes.c_void_p))
    return out.raw[:n].decode()


class AnchorFinder:
    """Sequential restatement of AnchorFinder (AnchorFinder.cpp:37-406).

    The instance keeps used hashes across run() calls like the reference's
    ``AnchorFinderImpl::used_hashes_``.
    """

    def __init__(self, anchor_size=20, anchor_fp_x1e4=1000, anchor_similar=True,
                 max_anchor_fragments=100000, seed=1, params=None):
        L = lib()
        self._h = L.orc_af_create(anchor_size, anchor_fp_x1e4, int(anchor_similar),
                                  max_anchor_fragments, seed)
        if params is not None:
            p = np.asarray(params, dtype=np.uint64)
            L.orc_af_set_params(self._h, _ptr(p), len(p))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_af_free(self._h)
            self._h = None

    def run(self, seqs, names):
        """seqs: list of str/bytes; names: list of str.  Returns a dict with the
        SoA anchor set in reference order (block, then fragment order)."""
        L = lib()
        n = len(seqs)
        bufs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
        arr = (ctypes.c_char_p * n)(*bufs)
        lens = np.array([len(b) for b in bufs], dtype=np.int64)
        nm = (ctypes.c_char_p * n)(*[x.encode() for x in names])
        rc = L.orc_af_run(self._h, n, ctypes.cast(arr, ctypes.c_void_p), _ptr(lens),
                          ctypes.cast(nm, ctypes.c_void_p))
        if rc != 0:
            raise RuntimeError("oracle AnchorFinder failed: %d" % rc)
        st = np.zeros(8, dtype=np.int64)
        L.orc_af_stats(self._h, _ptr(st))
        nb, nf, nu = int(st[5]), int(st[6]), int(st[7])
        seq = np.zeros(nf, dtype=np.int32)
        mn = np.zeros(nf, dtype=np.int64)
        mx = np.zeros(nf, dtype=np.int64)
        ori = np.zeros(nf, dtype=np.int32)
        bs = np.zeros(nb + 1, dtype=np.int64)
        L.orc_af_fragments(self._h, _ptr(seq), _ptr(mn), _ptr(mx), _ptr(ori), _ptr(bs))
        params = np.zeros(int(st[2]), dtype=np.uint64)
        L.orc_af_params(self._h, _ptr(params))
        used = np.zeros(nu, dtype=np.uint64)
        L.orc_af_used(self._h, _ptr(used))
        return dict(seq=seq, min_pos=mn, max_pos=mx, ori=ori, block_start=bs,
                    members=int(st[0]), bits=int(st[1]), hashes=int(st[2]),
                    n_collected=int(st[3]), n_found_frags=int(st[4]),
                    params=params, used=used)


DEFAULT_SA = (1, 2, 10, 100, 9000)  # MISMATCH_CHECK, GAP_CHECK, ALIGNED_CHECK, MIN_LENGTH, MIN_IDENTITY


def align(rows, mode="similar", params=DEFAULT_SA, return_past_end=False):
    """mode: 'similar' = SimilarAligner::similar_aligner; 'align_seqs' =
    AbstractAligner::align_seqs(similar); 'dummy' = align_seqs(DummyAligner);
    'similar+refine'; 'refine' = refine_alignment only."""
    m = {"similar": 0, "align_seqs": 1, "dummy": 2, "similar+refine": 3, "refine": 4,
         "align_block": 5}[mode]
    L = lib()
    bufs = [r.encode() if isinstance(r, str) else bytes(r) for r in rows]
    cat = b"".join(bufs)
    lens = np.array([len(b) for b in bufs], dtype=np.int64)
    prm = np.array(params, dtype=np.int32)
    cap = max(1, 4 * (sum(len(b) for b in bufs) + 16) * max(1, len(rows)))
    out_len = ctypes.c_int64(0)
    pe = ctypes.c_int64(0)
    while True:
        out = np.zeros(cap, dtype=np.uint8)
        rc = L.orc_align(len(rows), cat, _ptr(lens), _ptr(prm), m, _ptr(out), cap,
                         ctypes.byref(out_len), ctypes.byref(pe))
        if rc == -1:
            cap = out_len.value * len(rows) + 1
            continue
        if rc != 0:
            raise RuntimeError("oracle align failed: %d" % rc)
        break
    Ln = out_len.value
    res = [out[i * Ln:(i + 1) * Ln].tobytes().decode() for i in range(len(rows))]
    return (res, pe.value) if return_past_end else res


# ---------------------------------------------------------------- block sets
PIPELINE_DEFAULTS = dict(
    extend_length=100, portion_x1e4=0, fix_min_fragment=100, fix_min_identity_x1e4=9000,
    max_iterations=10, filter_min_fragment=100, filter_min_block=2, filter_frame_length=100,
    filter_min_end=10, filter_min_identity_x1e4=9000, filter_find_subblocks=1, do_filter=1,
    mismatch_check=1, gap_check=2, aligned_check=10, min_length=100, min_identity_x1e4=9000,
    anchor_size=20, anchor_fp_x1e4=1000, max_anchor_fragments=100000, seed=1,
    filter_max_block=-1)
_PKEYS = list(PIPELINE_DEFAULTS)

OPS = {"FragmentsExtender": 0, "FixEnds": 1, "Filter": 2, "ExtendLoopFast": 3, "DummyAligner": 4,
       "RemoveNonStem": 5, "DraftPangenome": 6, "MetaAligner": 7, "FindGoodSubblocks": 8,
       "Rest": 9, "OverlaplessUnion": 10, "MoveGaps": 11, "CutGaps": 12, "CutGapsStrict": 13,
       "SelfOverlapsResolver": 14, "Align": 15, "LiteAlign": 16, "AnchorLoop": 17, "ExtendLoop": 18,
       "AddingLoopBySize": 19}


def _bs_lib():
    L = lib()
    if not getattr(L, "_bs_bound", False):
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.orc_bs_create.argtypes = [ctypes.c_int, vp, vp, vp, vp]
        L.orc_bs_create.restype = vp
        L.orc_bs_free.argtypes = [vp]
        L.orc_bs_set_blocks.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp]
        L.orc_bs_apply.argtypes = [vp, ctypes.c_int]
        L.orc_bs_apply.restype = ctypes.c_int
        L.orc_bs_set_workers.argtypes = [vp, ctypes.c_int]
        L.orc_bs_counts.argtypes = [vp, vp]
        L.orc_bs_copy.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.orc_bs_hash.argtypes = [vp]
        L.orc_bs_hash.restype = ctypes.c_uint64
        L.orc_bs_conseq.argtypes = [vp, vp, vp]
        L.orc_bs_conseq.restype = i64
        L.orc_bs_deconseq.argtypes = [vp, vp, vp]
        L.orc_bs_deconseq.restype = ctypes.c_int
        L.orc_bs_set_gap_opts.argtypes = [vp, ctypes.c_int, i64]
        L.orc_bs_anchor_loop_stats.argtypes = [vp, vp]
        L._bs_bound = True
    return L


class BlockSetOracle:
    """Oracle block set: sequences + blocks, with the hot-path processors
    (FragmentsExtender, FixEnds, Filter, ExtendLoopFast, DummyAligner,
    RemoveNonStem, DraftPangenome, MetaAligner, Rest, OverlaplessUnion,
    MoveGaps, CutGaps (permissive / strict), SelfOverlapsResolver, the
    Align / LiteAlign pipes, ExtendLoop, AddingLoopBySize and AnchorLoop)."""

    def __init__(self, seqs, names, max_tail=3, max_tail_to_gap_x1e4=10000, **params):
        L = _bs_lib()
        p = dict(PIPELINE_DEFAULTS)
        p.update(params)
        prm = np.array([p[k] for k in _PKEYS], dtype=np.int64)
        n = len(seqs)
        bufs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
        arr = (ctypes.c_char_p * max(n, 1))(*bufs)
        lens = np.array([len(b) for b in bufs] or [0], dtype=np.int64)
        nm = (ctypes.c_char_p * max(n, 1))(*[x.encode() for x in names])
        self._h = L.orc_bs_create(n, ctypes.cast(arr, ctypes.c_void_p), _ptr(lens),
                                  ctypes.cast(nm, ctypes.c_void_p), _ptr(prm))
        # MoveGaps max-tail / max-tail-to-gap (MAX_TAIL 3, MAX_TAIL_TO_GAP 1.0)
        L.orc_bs_set_gap_opts(self._h, int(max_tail), int(max_tail_to_gap_x1e4))

    def __del__(self):
        if getattr(self, "_h", None):
            _bs_lib().orc_bs_free(self._h)
            self._h = None

    def set_blocks(self, blocks):
        """blocks: list of lists of (seq_index, min, max, ori, row_or_None)."""
        frs = [f for b in blocks for f in b]
        bs = np.zeros(len(blocks) + 1, dtype=np.int64)
        np.cumsum([len(b) for b in blocks], out=bs[1:])
        seq = np.array([f[0] for f in frs] or [0], dtype=np.int32)
        mn = np.array([f[1] for f in frs] or [0], dtype=np.int64)
        mx = np.array([f[2] for f in frs] or [0], dtype=np.int64)
        ori = np.array([f[3] for f in frs] or [0], dtype=np.int32)
        rows = [(f[4] or "") for f in frs]
        rl = np.array([len(f[4]) if f[4] is not None else -1 for f in frs] or [0], dtype=np.int64)
        ro = np.zeros(max(len(frs), 1), dtype=np.int64)
        if frs:
            ro[1:len(frs)] = np.cumsum([len(r) for r in rows])[:-1]
        data = "".join(rows).encode() or b"\0"
        _bs_lib().orc_bs_set_blocks(self._h, len(blocks), _ptr(bs), _ptr(seq), _ptr(mn), _ptr(mx),
                                    _ptr(ori), _ptr(ro), _ptr(rl), data)

    def set_workers(self, workers):
        """BlocksJobs worker threads for DraftPangenome / ExtendLoopFast's
        per-block stages (BlocksJobs.cpp:38-240); output identical for any count."""
        _bs_lib().orc_bs_set_workers(self._h, int(workers))
        return self

    def apply(self, op):
        rc = _bs_lib().orc_bs_apply(self._h, OPS[op])
        if rc != 0:
            raise RuntimeError("oracle op %s failed" % op)
        return self

    def stats(self):
        c = np.zeros(7, dtype=np.int64)
        _bs_lib().orc_bs_counts(self._h, _ptr(c))
        return dict(n_blocks=int(c[0]), n_fragments=int(c[1]), iterations=int(c[3]),
                    aligned_residues=int(c[4]), anchor_blocks=int(c[5]), stem_blocks=int(c[6]))

    def blocks(self):
        L = _bs_lib()
        c = np.zeros(7, dtype=np.int64)
        L.orc_bs_counts(self._h, _ptr(c))
        nb, nf, rbytes = int(c[0]), int(c[1]), int(c[2])
        bs = np.zeros(nb + 1, dtype=np.int64)
        seq = np.zeros(max(nf, 1), dtype=np.int32)
        mn = np.zeros(max(nf, 1), dtype=np.int64)
        mx = np.zeros(max(nf, 1), dtype=np.int64)
        ori = np.zeros(max(nf, 1), dtype=np.int32)
        ro = np.zeros(max(nf, 1), dtype=np.int64)
        rl = np.zeros(max(nf, 1), dtype=np.int64)
        rows = ctypes.create_string_buffer(max(rbytes, 1))
        L.orc_bs_copy(self._h, _ptr(bs), _ptr(seq), _ptr(mn), _ptr(mx), _ptr(ori), _ptr(ro), _ptr(rl),
                      ctypes.cast(rows, ctypes.c_void_p))
        raw = rows.raw
        out = []
        for b in range(nb):
            blk = []
            for i in range(bs[b], bs[b + 1]):
                row = raw[ro[i]:ro[i] + rl[i]].decode() if rl[i] >= 0 else None
                blk.append((int(seq[i]), int(mn[i]), int(mx[i]), int(ori[i]), row))
            out.append(blk)
        return out

    def hash(self):
        return _bs_lib().orc_bs_hash(self._h)

    def anchor_loop_stats(self):
        """Counts of the last AnchorLoop (orc_bs_anchor_loop_stats)."""
        c = np.zeros(8, dtype=np.int64)
        _bs_lib().orc_bs_anchor_loop_stats(self._h, _ptr(c))
        keys = ("cons_seqs", "cons_anchors", "anchors_left", "split_blocks", "cons_blocks", "dec_blocks",
                "cons_iterations", "dec_iterations")
        return dict(zip(keys, (int(x) for x in c)))

    def conseq(self):
        """ConSeq (ConSeq.cpp:37-50): the sequence text each block becomes."""
        L = _bs_lib()
        n = len(self.blocks())
        tot = L.orc_bs_conseq(self._h, None, None)
        buf = ctypes.create_string_buffer(max(tot, 1))
        off = np.zeros(n + 1, dtype=np.int64)
        L.orc_bs_conseq(self._h, ctypes.cast(buf, ctypes.c_void_p), _ptr(off))
        raw = buf.raw
        return [raw[off[i]:off[i + 1]].decode() for i in range(n)]

    def deconseq(self, cons, source=None):
        """DeConSeq (DeConSeq.cpp:48-96): blocks of `cons` (an oracle over the
        sequences conseq() made from `source`'s blocks, sequence i = block i)
        mapped back and appended to this set's blocks."""
        src = self if source is None else source
        rc = _bs_lib().orc_bs_deconseq(self._h, src._h, cons._h)
        if rc != 0:
            raise RuntimeError("oracle DeConSeq failed (%d)" % rc)
        return self


def anchor_blocks(r):
    """AnchorFinder SoA result -> blocks [(seq, min, max, ori, None), ...] in
    result order (AnchorFinder.cpp:364-390)."""
    bs = r["block_start"]
    return [[(int(r["seq"][i]), int(r["min_pos"][i]), int(r["max_pos"][i]), int(r["ori"][i]), None)
             for i in range(bs[b], bs[b + 1])] for b in range(len(bs) - 1)]


def consensus_order(b):
    """The block order ConSeq sees (ConSeq.cpp:37-50 walks the block set):
    the reference's is the std::set<Block*> pointer order (BlockSet.hpp:30,
    arbitrary run to run); pinned here to the sorted fragment coordinates."""
    return sorted((f[0], f[1], f[2], f[3]) for f in b)


# the name of a new Block (Block.cpp:29-34), which ConSeq gives every
# consensus sequence of these pipes (Sequence.cpp:318-320)
NULL_BLOCK_NAME = "00000000"


def cons_names(cs):
    """Names of the consensus sequences ConSeq makes: each block's name, the
    null name for every block these pipes build."""
    return [NULL_BLOCK_NAME] * len(cs)


def anchor_loop_fast(o, workers=1):
    """AnchorLoopFast (src/algo/lua_lib.lua:741-758) over this restatement's
    processors, on BlockSetOracle `o` holding the current blocks:
      Filter; Rest target=target other=target;
      ConSeq target=cons other=target (blocks in consensus_order);
      AnchorFinder target=cons; MoveUnchanged target=null other=cons (a fresh
      pipe: nothing seen yet, nothing dropped); DummyAligner target=cons;
      ExtendAndAlign target=cons (FragmentsExtender --extend-length-portion:=0.5,
      then Align, Align.cpp:36-52); ExtendLoopFast target=cons (its
      set_max_iterations(-1), lua_lib.lua:697-699);
      DeConSeq target=target other=cons (DeConSeq.cpp:51-83); Align.
    Returns the consensus set's stats (its ExtendLoopFast iterations)."""
    o.apply("Filter")
    o.apply("Rest")
    o.set_blocks(sorted(o.blocks(), key=consensus_order))
    cs = o.conseq()
    oc = BlockSetOracle(cs, cons_names(cs), portion_x1e4=5000, max_iterations=-1)
    if workers > 1:
        oc.set_workers(workers)
    oc.set_blocks(anchor_blocks(AnchorFinder().run(cs, cons_names(cs))))
    for op in ("DummyAligner", "FragmentsExtender", "Align"):
        oc.apply(op)
    it0 = oc.stats()["iterations"]
    oc.apply("ExtendLoopFast")
    st = oc.stats()
    st["iterations"] -= it0
    o.deconseq(oc)
    o.apply("Align")
    return st
