"""ctypes binding of the C ABI in include/npge_amd.h (libnpge_amd.so).

The library is the product: there is no CPU fallback.  Loading fails loudly
when the in-tree .so is missing; creating a handle fails loudly when no GPU is
visible (NPGX_ERR_NODEV).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# NPGX_PROFILE=1 selects the diagnostic build with aligner cycle counters
LIB_PATH = os.path.join(_HERE, "libnpge_amd_prof.so" if os.environ.get("NPGX_PROFILE") == "1"
                        else "libnpge_amd.so")
# NPGX_LIB=<file in npge_amd/>: an alternate build of the same library (A/B timing)
if os.environ.get("NPGX_LIB"):
    LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ["NPGX_LIB"]))

NPGX_OK = 0
ERRORS = {-1: "NPGX_ERR_ARG", -2: "NPGX_ERR_HIP", -3: "NPGX_ERR_NODEV", -4: "NPGX_ERR_RANGE",
          -5: "NPGX_ERR_STATE"}


class NpgxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (ERRORS.get(code, "?"), code, msg))
        self.code = code


class KernelTime(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("ms", ctypes.c_double), ("bytes", ctypes.c_double),
                ("units", ctypes.c_int64)]


class AfOptions(ctypes.Structure):
    _fields_ = [("anchor_size", ctypes.c_int32), ("anchor_similar", ctypes.c_int32),
                ("anchor_fp_x1e4", ctypes.c_int64), ("max_anchor_fragments", ctypes.c_int64),
                ("bloom_seed", ctypes.c_uint32), ("n_bloom_params", ctypes.c_int32),
                ("bloom_params", ctypes.POINTER(ctypes.c_uint64)),
                ("bloom_epochs", ctypes.c_int32), ("pad0", ctypes.c_int32)]


class AfStats(ctypes.Structure):
    _fields_ = [("members", ctypes.c_int64), ("bloom_bits", ctypes.c_int64),
                ("bloom_hashes", ctypes.c_int32), ("pad0", ctypes.c_int32),
                ("bloom_params", ctypes.c_uint64 * 32), ("n_windows", ctypes.c_int64),
                ("n_collected_raw", ctypes.c_int64), ("n_collected", ctypes.c_int64),
                ("n_found_frags", ctypes.c_int64), ("n_kept_groups", ctypes.c_int64),
                ("n_blocks", ctypes.c_int64), ("n_fragments", ctypes.c_int64),
                ("n_used", ctypes.c_int64)]


class AlignOptions(ctypes.Structure):
    _fields_ = [("mismatch_check", ctypes.c_int32), ("gap_check", ctypes.c_int32),
                ("aligned_check", ctypes.c_int32), ("min_length", ctypes.c_int32),
                ("min_identity_x1e4", ctypes.c_int64), ("aligner_type", ctypes.c_int32),
                ("refine", ctypes.c_int32)]


_lib = None


def lib():
    """Loads libnpge_amd.so (building it first when the sources are newer and a
    hipcc is available).  Raises if it cannot be loaded."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        try:
            from . import build as _b
            _b.build(profile=LIB_PATH.endswith("_prof.so"))
        except Exception as e:  # pragma: no cover - surfaced below
            raise ImportError("npge_amd: HIP library %s missing and could not be built: %s"
                              % (LIB_PATH, e))
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32
    P = ctypes.POINTER
    L.npgx_last_error.restype = ctypes.c_char_p
    L.npgx_version.restype = ctypes.c_char_p
    L.npgx_device_count.argtypes = [P(i32)]
    L.npgx_set_device.argtypes = [i32]
    L.npgx_seqset_create.argtypes = [vp, vp, vp, i32, P(vp)]
    L.npgx_seqset_count.argtypes = [vp, P(i32)]
    L.npgx_seqset_size.argtypes = [vp, i32, P(i64)]
    L.npgx_seqset_rank.argtypes = [vp, i32, P(i32)]
    L.npgx_seqset_text.argtypes = [vp, i32, i64, i64, ctypes.c_char_p]
    L.npgx_seqset_device_bytes.argtypes = [vp, P(i64)]
    L.npgx_seqset_timings.argtypes = [vp, P(ctypes.c_double), P(ctypes.c_double)]
    L.npgx_seqset_free.argtypes = [vp]
    L.npgx_seqset_free.restype = None
    L.npgx_af_default_options.argtypes = [P(AfOptions)]
    L.npgx_af_default_options.restype = None
    L.npgx_af_create.argtypes = [P(AfOptions), P(vp)]
    L.npgx_af_run.argtypes = [vp, vp]
    L.npgx_af_stats_get.argtypes = [vp, P(AfStats)]
    L.npgx_af_result_counts.argtypes = [vp, P(i64), P(i64)]
    L.npgx_af_result_copy.argtypes = [vp, vp, vp, vp, vp, vp]
    L.npgx_af_used_hashes.argtypes = [vp, vp, i64, P(i64)]
    L.npgx_af_clear_used.argtypes = [vp]
    L.npgx_af_kernel_times.argtypes = [vp, P(KernelTime), i32, P(i32)]
    L.npgx_af_free.argtypes = [vp]
    L.npgx_af_free.restype = None
    L.npgx_af_run_sharded.argtypes = [vp, vp, vp]
    L.npgx_memcpy.argtypes = [vp, vp, i64]
    if hasattr(L, "npgx_aligner_create"):
        L.npgx_align_default_options.argtypes = [P(AlignOptions)]
        L.npgx_align_default_options.restype = None
        L.npgx_aligner_create.argtypes = [P(AlignOptions), P(vp)]
        L.npgx_align_batch.argtypes = [vp, vp, vp, vp, i32]
        L.npgx_align_result_sizes.argtypes = [vp, P(i64)]
        L.npgx_align_result_copy.argtypes = [vp, vp, vp, vp]
        L.npgx_align_kernel_times.argtypes = [vp, P(KernelTime), i32, P(i32)]
        L.npgx_aligner_free.argtypes = [vp]
        L.npgx_aligner_free.restype = None
    _lib = L
    return L


def check(rc):
    if rc != NPGX_OK:
        raise NpgxError(rc, lib().npgx_last_error().decode(errors="replace"))


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def device_count():
    n = ctypes.c_int32(0)
    check(lib().npgx_device_count(ctypes.byref(n)))
    return n.value


def kernel_times(fn, handle, cap=None):
    """Every kernel-time record of the handle's last call (sized by a first
    query unless `cap` is given)."""
    n = ctypes.c_int32(0)
    if cap is None:
        check(fn(handle, None, 0, ctypes.byref(n)))
        cap = max(n.value, 1)
    arr = (KernelTime * cap)()
    check(fn(handle, arr, cap, ctypes.byref(n)))
    return [dict(name=arr[i].name.decode(), ms=arr[i].ms, bytes=arr[i].bytes, units=arr[i].units)
            for i in range(min(n.value, cap))]


class SeqSet:
    """Device-resident packed sequences (npgx_seqset_*)."""

    def __init__(self, seqs, names=None):
        L = lib()
        n = len(seqs)
        bufs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
        self._keep = bufs
        arr = (ctypes.c_char_p * max(n, 1))(*bufs)
        lens = np.array([len(b) for b in bufs] or [0], dtype=np.int64)
        names = names if names is not None else [""] * n
        nb = [x.encode() for x in names]
        nm = (ctypes.c_char_p * max(n, 1))(*nb)
        h = ctypes.c_void_p()
        check(L.npgx_seqset_create(ctypes.cast(arr, ctypes.c_void_p), ptr(lens),
                                   ctypes.cast(nm, ctypes.c_void_p), n, ctypes.byref(h)))
        self._h = h
        self.n = n
        self._keep = None

    @property
    def handle(self):
        return self._h

    def size(self, i):
        v = ctypes.c_int64()
        check(lib().npgx_seqset_size(self._h, i, ctypes.byref(v)))
        return v.value

    def timings(self):
        """(host to_atgcn ms, upload ms = H2D + k_pack) of the creation."""
        a, b = ctypes.c_double(), ctypes.c_double()
        check(lib().npgx_seqset_timings(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def rank(self, i):
        v = ctypes.c_int32()
        check(lib().npgx_seqset_rank(self._h, i, ctypes.byref(v)))
        return v.value

    def text(self, i, start=0, length=None):
        if length is None:
            length = self.size(i) - start
        buf = ctypes.create_string_buffer(max(length, 1))
        check(lib().npgx_seqset_text(self._h, i, start, length, buf))
        return buf.raw[:length].decode()

    def device_bytes(self):
        v = ctypes.c_int64()
        check(lib().npgx_seqset_device_bytes(self._h, ctypes.byref(v)))
        return v.value

    def close(self):
        if getattr(self, "_h", None):
            lib().npgx_seqset_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
