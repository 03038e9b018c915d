"""The collectives of the exactly-sharded AnchorFinder and block build
(``npgx_comm``, include/npge_amd.h; SURVEY.md §8e, DESIGN.md "Multi-GPU").

``RcclComm``: the library's own RCCL communicator (npgx_rccl_comm_create) --
the collectives run natively on its stream over xGMI; Python only hands the
unique id from rank 0 to the others (one object broadcast at start-up).

``TorchComm``: the same callbacks bound to torch.distributed -- gloo for the
CPU tests and the one-GPU rehearsal of several ranks (RCCL refuses two ranks
on one GPU).

One process per GPU.  With the ``nccl`` backend (RCCL over xGMI on MI355X) the
staging tensors live on the rank's GPU and every exchange is a device-to-device
copy plus one RCCL collective; with ``gloo`` (tests, CPU rehearsal) they live
in host memory.  The library calls these with its stream idle and expects the
data in place when the callback returns, so every callback synchronises.

The copy primitive is ``npgx_memcpy`` (hipMemcpyDefault); tests on machines
without a GPU pass ``copy=ctypes.memmove`` and host pointers.
"""
import ctypes

NPGX_OP_SUM = 0
NPGX_OP_MIN = 1

_ALLREDUCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                              ctypes.c_int32)
_ALLGATHER_I64 = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                  ctypes.POINTER(ctypes.c_int64))
_ALLGATHERV = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p)


class NpgxComm(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int32), ("world", ctypes.c_int32), ("user", ctypes.c_void_p),
                ("allreduce_i32", _ALLREDUCE), ("allgather_i64", _ALLGATHER_I64),
                ("allgatherv_u64", _ALLGATHERV)]


class TorchComm:
    """npgx_comm over a torch.distributed process group.

    staging: torch device of the exchange tensors ("cuda" for RCCL, "cpu" for
    gloo).  copy(dst, src, nbytes): raw-pointer copy between library buffers and
    the staging tensors (default npgx_memcpy)."""

    def __init__(self, dist, staging="cuda", copy=None, group=None):
        import torch
        self.torch = torch
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.staging = staging
        if copy is None:
            from . import _capi
            L = _capi.lib()

            def copy(dst, src, n):
                _capi.check(L.npgx_memcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), n))
        self.copy = copy
        self.errors = []
        self._cbs = (_ALLREDUCE(self._allreduce_i32), _ALLGATHER_I64(self._allgather_i64),
                     _ALLGATHERV(self._allgatherv_u64))
        self.struct = NpgxComm(self.rank, self.world, None, *self._cbs)

    # -- helpers
    def _sync(self):
        if self.staging != "cpu":
            self.torch.cuda.synchronize()

    def _guard(self, f, *a):
        try:
            self._sync()
            f(*a)
            self._sync()
            return 0
        except Exception as e:  # surfaced by the library as a failed collective
            self.errors.append(repr(e))
            return -1

    # -- callbacks
    def _allreduce_i32(self, _user, dev, n, op):
        def run():
            if n == 0:
                return
            t = self.torch.empty(n, dtype=self.torch.int32, device=self.staging)
            self._sync()
            self.copy(t.data_ptr(), dev, n * 4)
            rop = self.dist.ReduceOp.MIN if op == NPGX_OP_MIN else self.dist.ReduceOp.SUM
            self.dist.all_reduce(t, op=rop, group=self.group)
            self._sync()
            self.copy(dev, t.data_ptr(), n * 4)
        return self._guard(run)

    def _allgather_i64(self, _user, value, out):
        def run():
            t = self.torch.tensor([value], dtype=self.torch.int64, device=self.staging)
            parts = [self.torch.empty_like(t) for _ in range(self.world)]
            self.dist.all_gather(parts, t, group=self.group)
            for r in range(self.world):
                out[r] = int(parts[r].item())
        return self._guard(run)

    def _allgatherv_u64(self, _user, dev_in, counts, dev_out):
        def run():
            cnt = [int(counts[r]) for r in range(self.world)]
            mx = max(cnt)
            if mx == 0:
                return
            t = self.torch.zeros(mx, dtype=self.torch.int64, device=self.staging)
            self._sync()
            if cnt[self.rank]:
                self.copy(t.data_ptr(), dev_in, cnt[self.rank] * 8)
            parts = self.torch.empty(self.world * mx, dtype=self.torch.int64, device=self.staging)
            self.dist.all_gather_into_tensor(parts, t, group=self.group)
            self._sync()
            off = 0
            base = parts.data_ptr()
            for r in range(self.world):
                if cnt[r]:
                    self.copy(dev_out + off * 8, base + r * mx * 8, cnt[r] * 8)
                off += cnt[r]
        return self._guard(run)

    def pointer(self):
        return ctypes.byref(self.struct)

    def count(self):
        """The process group's rank count."""
        return self.dist.get_world_size(self.group)


class RcclComm:
    """npgx_comm owned by the library: RCCL over xGMI, one process per GPU.

    dist: an initialised torch.distributed (any backend) used once, to send
    rank 0's RCCL unique id to every rank."""

    def __init__(self, dist, device, group=None):
        from . import _capi
        L = _capi.lib()
        if not getattr(L, "_rccl_bound", False):
            vp = ctypes.c_void_p
            L.npgx_rccl_unique_id.argtypes = [vp]
            L.npgx_rccl_comm_create.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                ctypes.POINTER(vp)]
            L.npgx_rccl_comm_free.argtypes = [vp]
            L.npgx_rccl_comm_free.restype = None
            L.npgx_rccl_comm_count.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)]
            L._rccl_bound = True
        self._L = L
        self.errors = []
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        idbuf = ctypes.create_string_buffer(128)
        if self.rank == 0:
            _capi.check(L.npgx_rccl_unique_id(ctypes.cast(idbuf, ctypes.c_void_p)))
        obj = [idbuf.raw]
        dist.broadcast_object_list(obj, src=0, group=group)
        idbuf = ctypes.create_string_buffer(obj[0], 128)
        h = ctypes.c_void_p()
        _capi.check(L.npgx_rccl_comm_create(ctypes.cast(idbuf, ctypes.c_void_p), self.rank, self.world,
                                            int(device), ctypes.byref(h)))
        self._h = h

    def pointer(self):
        return self._h

    def count(self):
        """The rank count RCCL reports for this communicator (ncclCommCount)."""
        from . import _capi
        n = ctypes.c_int32()
        _capi.check(self._L.npgx_rccl_comm_count(self._h, ctypes.byref(n)))
        return n.value

    def close(self):
        if getattr(self, "_h", None):
            self._L.npgx_rccl_comm_free(self._h)
            self._h = None


def check(comm):
    """npgx_comm_check: every collective of `comm` on small device buffers,
    results verified (collective: call on every rank)."""
    from . import _capi
    L = _capi.lib()
    L.npgx_comm_check.argtypes = [ctypes.c_void_p]
    _capi.check(L.npgx_comm_check(comm.pointer()))
