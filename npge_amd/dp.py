"""GeneralAligner on the GPU (npgx_dp_*, include/npge_amd.h): batched banded
min-cost Needleman-Wunsch with a gap frame and the max_errors stop rule
(src/util/GeneralAligner.hpp:28-414) on nucleotide contents.

Mirrors the reference class's setters (set_gap_range :68, set_max_errors :82,
set_gap_penalty :92) and its align -> cut_tail -> export_alignment sequence,
for a batch of independent pairs per call.  Fails loudly without the HIP
library or a GPU; there is no CPU path.
"""
import ctypes

import numpy as np

from . import _capi

MATCH, ROW_INC, COL_INC = 0, 1, 2
BAD_VALUE = 1000000


class DpOptions(ctypes.Structure):
    _fields_ = [("gap_range", ctypes.c_int32), ("max_errors", ctypes.c_int32),
                ("gap_penalty", ctypes.c_int32), ("mismatch_penalty", ctypes.c_int32),
                ("cut_tail", ctypes.c_int32)]


def _bind(L):
    if getattr(L, "_dp_bound", False):
        return L
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    P = ctypes.POINTER
    L.npgx_dp_default_options.argtypes = [P(DpOptions)]
    L.npgx_dp_default_options.restype = None
    L.npgx_dp_create.argtypes = [P(DpOptions), P(vp)]
    L.npgx_dp_align_batch.argtypes = [vp, vp, vp, vp, vp, i32]
    L.npgx_dp_result_counts.argtypes = [vp, P(i64), P(i64)]
    L.npgx_dp_result_copy.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.npgx_dp_kernel_times.argtypes = [vp, P(_capi.KernelTime), i32, P(i32)]
    L.npgx_dp_phase_cycles.argtypes = [vp, P(i64), P(i64), P(i64)]
    L.npgx_dp_free.argtypes = [vp]
    L.npgx_dp_free.restype = None
    L._dp_bound = True
    return L


class GeneralAligner:
    def __init__(self, gap_range=1, max_errors=0, gap_penalty=1, mismatch_penalty=1,
                 cut_tail=False):
        self.opt = dict(gap_range=gap_range, max_errors=max_errors, gap_penalty=gap_penalty,
                        mismatch_penalty=mismatch_penalty, cut_tail=int(bool(cut_tail)))
        self._h = None
        self._key = None

    # GeneralAligner setters
    def set_gap_range(self, v):
        self.opt["gap_range"] = v

    def set_max_errors(self, v):
        self.opt["max_errors"] = v

    def set_gap_penalty(self, v):
        self.opt["gap_penalty"] = v

    def _handle(self):
        L = _bind(_capi.lib())
        key = tuple(sorted(self.opt.items()))
        if self._h is not None and key == self._key:
            return self._h
        self.close()
        o = DpOptions()
        L.npgx_dp_default_options(ctypes.byref(o))
        for k, v in self.opt.items():
            setattr(o, k, v)
        h = ctypes.c_void_p()
        _capi.check(L.npgx_dp_create(ctypes.byref(o), ctypes.byref(h)))
        self._h, self._key = h, key
        return h

    def align_batch(self, pairs):
        """pairs: list of (first, second) str/bytes.  Returns a dict of numpy
        arrays first_last, second_last, score, status, op_off and ops (see
        include/npge_amd.h)."""
        L = _bind(_capi.lib())
        h = self._handle()
        A = [p[0].encode() if isinstance(p[0], str) else p[0] for p in pairs]
        B = [p[1].encode() if isinstance(p[1], str) else p[1] for p in pairs]
        ao = np.zeros(len(A) + 1, dtype=np.int64)
        bo = np.zeros(len(B) + 1, dtype=np.int64)
        np.cumsum([len(x) for x in A], out=ao[1:])
        np.cumsum([len(x) for x in B], out=bo[1:])
        abuf = ctypes.create_string_buffer(b"".join(A), max(1, int(ao[-1])))
        bbuf = ctypes.create_string_buffer(b"".join(B), max(1, int(bo[-1])))
        _capi.check(L.npgx_dp_align_batch(h, ctypes.cast(abuf, ctypes.c_void_p), _capi.ptr(ao),
                                          ctypes.cast(bbuf, ctypes.c_void_p), _capi.ptr(bo), len(A)))
        return self.result()

    def result(self):
        L = _bind(_capi.lib())
        n, t = ctypes.c_int64(), ctypes.c_int64()
        _capi.check(L.npgx_dp_result_counts(self._h, ctypes.byref(n), ctypes.byref(t)))
        m = max(n.value, 1)
        fl, sl, sc, st = (np.zeros(m, dtype=np.int32) for _ in range(4))
        off = np.zeros(n.value + 1, dtype=np.int64)
        ops = np.zeros(max(t.value, 1), dtype=np.int8)
        _capi.check(L.npgx_dp_result_copy(self._h, _capi.ptr(fl), _capi.ptr(sl), _capi.ptr(sc),
                                          _capi.ptr(st), _capi.ptr(off), _capi.ptr(ops)))
        k = n.value
        return dict(first_last=fl[:k], second_last=sl[:k], score=sc[:k], status=st[:k], op_off=off,
                    ops=ops[:t.value])

    def kernel_times(self):
        return _capi.kernel_times(_bind(_capi.lib()).npgx_dp_kernel_times, self._h)

    def phase_cycles(self):
        """(forward, traceback, steps) summed over the batch's waves; needs the
        diagnostic library (NPGX_PROFILE=1)."""
        f, b, s = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _capi.check(_bind(_capi.lib()).npgx_dp_phase_cycles(self._h, ctypes.byref(f), ctypes.byref(b),
                                                             ctypes.byref(s)))
        return f.value, b.value, s.value

    def close(self):
        if self._h is not None:
            try:
                _capi.lib().npgx_dp_free(self._h)
            except Exception:
                pass
            self._h = None

    def __del__(self):
        self.close()
