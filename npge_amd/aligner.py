"""Aligner processors on the HIP engine.

``align_batch`` is the batched form of AbstractAligner::align_seqs
(src/algo/AbstractAligner.cpp:104-143) with aligner-type "similar"
(SimilarAligner, SimilarAligner.cpp:487-501) or "dummy" (DummyAligner.cpp:18-26),
the registry point MetaAligner dispatches on (MetaAligner.cpp:22-84).
"""
import ctypes

import numpy as np

from . import _capi
from .processor import Decimal, Processor, register

ALIGNER_TYPES = {"similar": 0, "dummy": 1}


def refine_batch(alignments):
    """refine_alignment (refine_alignment.cpp:182-190) of each alignment (a
    list of equal-length gapped rows) on the GPU (npgx_refine_batch)."""
    L = _capi.lib()
    if not getattr(L, "_refine_bound", False):
        vp = ctypes.c_void_p
        L.npgx_refine_batch.argtypes = [vp, vp, vp, ctypes.c_int32, vp, vp]
        L._refine_bound = True
    rows = [r for a in alignments for r in a]
    data = "".join(rows).encode()
    off = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum([len(r) for r in rows], out=off[1:])
    jstart = np.zeros(len(alignments) + 1, dtype=np.int32)
    np.cumsum([len(a) for a in alignments], out=jstart[1:])
    buf = ctypes.create_string_buffer(data, max(len(data), 1))
    out = ctypes.create_string_buffer(max(len(data), 1))
    lens = np.zeros(max(len(alignments), 1), dtype=np.int32)
    _capi.check(L.npgx_refine_batch(ctypes.cast(buf, ctypes.c_void_p), _capi.ptr(off), _capi.ptr(jstart),
                                    len(alignments), ctypes.cast(out, ctypes.c_void_p), _capi.ptr(lens)))
    raw = out.raw
    res, k = [], 0
    for j, a in enumerate(alignments):
        res.append([raw[off[k + i]:off[k + i] + lens[j]].decode() for i in range(len(a))])
        k += len(a)
    return res


class BatchAligner:
    """One npgx_aligner handle (one HIP stream)."""

    def __init__(self, aligner_type="similar", mismatch_check=1, gap_check=2, aligned_check=10,
                 min_length=100, min_identity="0.9"):
        L = _capi.lib()
        o = _capi.AlignOptions()
        L.npgx_align_default_options(ctypes.byref(o))
        o.mismatch_check, o.gap_check, o.aligned_check = mismatch_check, gap_check, aligned_check
        o.min_length = min_length
        o.min_identity_x1e4 = Decimal(min_identity).impl
        o.aligner_type = ALIGNER_TYPES[aligner_type]
        h = ctypes.c_void_p()
        _capi.check(L.npgx_aligner_create(ctypes.byref(o), ctypes.byref(h)))
        self._h = h

    def align(self, jobs):
        """jobs: list of lists of row strings.  Returns the aligned rows."""
        L = _capi.lib()
        rows = [r for job in jobs for r in job]
        data = "".join(rows).encode()
        off = np.zeros(len(rows) + 1, dtype=np.int64)
        np.cumsum([len(r) for r in rows], out=off[1:])
        jstart = np.zeros(len(jobs) + 1, dtype=np.int32)
        np.cumsum([len(j) for j in jobs], out=jstart[1:])
        buf = ctypes.create_string_buffer(data, max(len(data), 1))
        _capi.check(L.npgx_align_batch(self._h, ctypes.cast(buf, ctypes.c_void_p), _capi.ptr(off),
                                       _capi.ptr(jstart), len(jobs)))
        tot = ctypes.c_int64()
        _capi.check(L.npgx_align_result_sizes(self._h, ctypes.byref(tot)))
        out = ctypes.create_string_buffer(max(tot.value, 1))
        ooff = np.zeros(len(rows) + 1, dtype=np.int64)
        jl = np.zeros(len(jobs), dtype=np.int64)
        _capi.check(L.npgx_align_result_copy(self._h, ctypes.cast(out, ctypes.c_void_p),
                                             _capi.ptr(ooff), _capi.ptr(jl)))
        raw = out.raw
        res, k = [], 0
        for job in jobs:
            res.append([raw[ooff[k + i]:ooff[k + i + 1]].decode() for i in range(len(job))])
            k += len(job)
        return res

    def kernel_times(self):
        return _capi.kernel_times(_capi.lib().npgx_align_kernel_times, self._h)

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            try:
                _capi.lib().npgx_aligner_free(self._h)
            except Exception:
                pass
            self._h = None
