"""AnchorFinder processor on the HIP engine (src/algo/AnchorFinder.cpp:37-406).

Options and rules are the reference's (AnchorFinder.cpp:37-53); the Bloom
hash parameters come from ``bloom-seed`` (glibc rand after srand(seed)) or an
explicit ``bloom_params`` vector instead of the reference's time seed
(BloomFilter.cpp:55-63, DESIGN.md "Determinism").  One instance keeps one
``npgx_af`` handle, so used hashes persist across runs of the same instance
exactly like ``AnchorFinderImpl::used_hashes_``.
"""
import ctypes

import numpy as np

from . import _capi
from .model import Block, Fragment
from .processor import Decimal, Processor, register


def seqset_for(bs):
    """Device sequence set of a BlockSet, cached on the BlockSet while its
    sequence list is unchanged."""
    key = tuple((id(s), len(s.data)) for s in bs.seqs)
    cached = getattr(bs, "_npgx_seqset", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    ss = _capi.SeqSet([s.data for s in bs.seqs], [s.name for s in bs.seqs])
    bs._npgx_seqset = (key, ss)
    return ss


@register
class AnchorFinder(Processor):
    name = "AnchorFinder"

    def __init__(self, bloom_params=None):
        super().__init__()
        self.add_gopt("anchor-size", "anchor size", "ANCHOR_SIZE")
        self.add_gopt("anchor-fp", "Probability of false positive in Bloom filter "
                      "(first step of AnchorFinder)", "ANCHOR_FP", Decimal)
        self.add_opt("anchor-similar", "If neighbour anchors are skipped", True)
        self.add_gopt("max-anchor-fragments", "Maximum number of anchors fragments to return",
                      "MAX_ANCHOR_FRAGMENTS")
        self.add_opt("bloom-seed", "glibc srand() seed of the Bloom hash parameters", 1)
        self.add_opt("bloom-epochs", "epochs of the one-GPU Bloom pass (0 = automatic, 1 = single pass)", 0)
        self.add_opt_rule("anchor-size > 0", lambda p: p.opt_value("anchor-size") > 0)
        self.add_opt_rule("anchor-size <= 32", lambda p: p.opt_value("anchor-size") <= 32)
        self.bloom_params = bloom_params
        self._h = None
        self._h_key = None
        self.stats = None

    def _handle(self):
        L = _capi.lib()
        key = (self.opt_value("anchor-size"), self.opt_value("anchor-fp").impl,
               bool(self.opt_value("anchor-similar")), self.opt_value("max-anchor-fragments"),
               self.opt_value("bloom-seed"), tuple(self.bloom_params or ()), self.opt_value("bloom-epochs"))
        if self._h is not None and key == self._h_key:
            return self._h
        if self._h is not None:
            L.npgx_af_free(self._h)
            self._h = None
        o = _capi.AfOptions()
        L.npgx_af_default_options(ctypes.byref(o))
        o.anchor_size, o.anchor_fp_x1e4, o.anchor_similar = key[0], key[1], int(key[2])
        o.max_anchor_fragments, o.bloom_seed = key[3], key[4] & 0xFFFFFFFF
        o.bloom_epochs = key[6]
        if self.bloom_params:
            arr = (ctypes.c_uint64 * len(self.bloom_params))(*self.bloom_params)
            o.n_bloom_params = len(self.bloom_params)
            o.bloom_params = ctypes.cast(arr, ctypes.POINTER(ctypes.c_uint64))
        h = ctypes.c_void_p()
        _capi.check(L.npgx_af_create(ctypes.byref(o), ctypes.byref(h)))
        self._h, self._h_key = h, key
        return h

    def find(self, seqset):
        """Runs the engine on a device sequence set; returns the SoA result."""
        L = _capi.lib()
        h = self._handle()
        _capi.check(L.npgx_af_run(h, seqset.handle))
        return self.result()

    def find_sharded(self, seqset, comm):
        """Exactly sharded run over the ranks of `comm` (npge_amd.comm.TorchComm):
        this rank scans its window range; the result on every rank equals
        find() on one GPU."""
        L = _capi.lib()
        h = self._handle()
        rc = L.npgx_af_run_sharded(h, seqset.handle, comm.pointer())
        if rc != 0 and comm.errors:
            raise _capi.NpgxError(rc, "; ".join(comm.errors))
        _capi.check(rc)
        return self.result()

    def result(self):
        L = _capi.lib()
        h = self._h
        nb, nf = ctypes.c_int64(), ctypes.c_int64()
        _capi.check(L.npgx_af_result_counts(h, ctypes.byref(nb), ctypes.byref(nf)))
        bs = np.zeros(nb.value + 1, dtype=np.int64)
        seq = np.zeros(nf.value, dtype=np.int32)
        mn = np.zeros(nf.value, dtype=np.int64)
        mx = np.zeros(nf.value, dtype=np.int64)
        ori = np.zeros(nf.value, dtype=np.int8)
        _capi.check(L.npgx_af_result_copy(h, _capi.ptr(bs), _capi.ptr(seq), _capi.ptr(mn),
                                          _capi.ptr(mx), _capi.ptr(ori)))
        st = _capi.AfStats()
        _capi.check(L.npgx_af_stats_get(h, ctypes.byref(st)))
        self.stats = st
        return dict(block_start=bs, seq=seq, min_pos=mn, max_pos=mx, ori=ori.astype(np.int32),
                    members=st.members, bits=st.bloom_bits, hashes=st.bloom_hashes,
                    params=np.array(st.bloom_params[:st.bloom_hashes], dtype=np.uint64),
                    n_collected=st.n_collected, n_found_frags=st.n_found_frags,
                    n_windows=st.n_windows)

    def used_hashes(self):
        L = _capi.lib()
        n = ctypes.c_int64()
        _capi.check(L.npgx_af_used_hashes(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint64)
        _capi.check(L.npgx_af_used_hashes(self._h, _capi.ptr(out), n.value, ctypes.byref(n)))
        return out

    def clear_used(self):
        """Forgets the used hashes (a fresh AnchorFinder without new device buffers)."""
        if self._h is not None:
            _capi.check(_capi.lib().npgx_af_clear_used(self._h))

    def kernel_times(self):
        return _capi.kernel_times(_capi.lib().npgx_af_kernel_times, self._h)

    def run_impl(self):
        """AnchorFinder::run_impl: anchors of target's sequences become new
        blocks of target (AnchorFinder.cpp:373-378)."""
        bs = self.block_set()
        ss = seqset_for(bs)
        r = self.find(ss)
        b = r["block_start"]
        for i in range(len(b) - 1):
            frs = [Fragment(bs.seqs[int(r["seq"][j])], int(r["min_pos"][j]), int(r["max_pos"][j]),
                            int(r["ori"][j])) for j in range(b[i], b[i + 1])]
            bs.blocks.append(Block(frs))

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            try:
                _capi.lib().npgx_af_free(self._h)
            except Exception:
                pass
            self._h = None
