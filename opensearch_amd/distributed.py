"""Multi-GPU exact k-NN: shards ↔ GPUs, one process per GPU, RCCL all-gather of per-shard top-k.

Mapping onto the reference:
  * Index shards are OpenSearch's data partitioning (IndexMetadata.java:265-268); the coordinator
    fans a query out to one copy of every shard (AbstractSearchAsyncAction.java:262-268) and merges
    the shard results by score (SearchPhaseController.java:224-246).
  * Here shard s lives on rank `shard_owner(s)` (contiguous blocks, so a GPU owns 8/G shards of an
    8-shard index).  Each rank scans its shards in one launch and produces per-shard top-k lists of
    8-byte hit keys; ONE all-gather exchanges them and the coordinator reduce runs on the device
    straight over the gathered image.
  * The product path is libosknn's own: `DeviceComm` wraps an `osk_comm` (RCCL inside the library,
    ncclCommInitRank / ncclCommInitAll) and `ShardSearchMerge` calls `osk_shards_search_merge_device`
    (scan + ncclAllGather + merge_coord, one C-ABI call per step) — what a Java host would bind.
    torch.distributed only carries the communicator id at start-up (any backend, gloo included).
  * `ShardExchange` is the same exchange written over `torch.distributed.all_gather_into_tensor`: the
    CPU (gloo) tests of the gather/merge logic and the N > 1 rehearsal on one GPU (several ranks per
    card, which RCCL refuses) use it; for host tensors it reduces in the library's host reduce.
The exchange is k·B·8 bytes per shard — latency-bound, microseconds next to a millisecond scan.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, lib, ptr


DEFAULT_DEVICE_LIMITS = (1, 100, 8)   # osk_comm_set_device_limits' defaults (include/osknn.h)


class DeviceComm:
    """An RCCL communicator owned by libosknn (`osk_comm`, include/osknn.h)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)
        r, w, n = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib().osk_comm_info(self._h, C.byref(r), C.byref(w), C.byref(n)))
        self.rank, self.world, self.n_local = r.value, w.value, n.value

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * _lib.OSK_COMM_ID_BYTES)()
        check(lib().osk_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def init_rank(cls, device: int, rank: int, world: int, uid: bytes) -> "DeviceComm":
        """One process per GPU (ncclCommInitRank; blocks until every rank has joined)."""
        buf = (C.c_uint8 * _lib.OSK_COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib().osk_comm_init_rank(device, rank, world, buf, C.byref(h)))
        return cls(h.value)

    @classmethod
    def init_all(cls, devices) -> "DeviceComm":
        """One process driving several GPUs (ncclCommInitAll): local device i is rank i."""
        d = np.asarray(devices, np.int32)
        h = C.c_void_p()
        check(lib().osk_comm_init_all(ptr(d), len(d), C.byref(h)))
        return cls(h.value)

    @classmethod
    def init_loopback(cls, device: int, rank: int, world: int, name: str, slot_bytes: int = 1 << 22) -> "DeviceComm":
        """Testing build only (inside `_lib.testing()`): `world` processes that may share one GPU, the
        all-gather through the POSIX shared-memory segment `name` ("/..."), so the world > 1 exchange
        runs on a one-GPU box."""
        raw = name.encode() + b"\0"
        if len(raw) > _lib.OSK_COMM_ID_BYTES or not name.startswith("/"):
            raise ValueError("loopback name: '/...' of at most 127 bytes")
        buf = (C.c_uint8 * _lib.OSK_COMM_ID_BYTES).from_buffer_copy(raw.ljust(_lib.OSK_COMM_ID_BYTES, b"\0"))
        h = C.c_void_p()
        check(lib().osk_comm_init_loopback(device, rank, world, buf, slot_bytes, C.byref(h)))
        return cls(h.value)

    @classmethod
    def init_all_loopback(cls, devices) -> "DeviceComm":
        """Testing build only (inside `_lib.testing()`): init_all's one-process communicator whose grouped
        all-gather is replaced by device copies, so `devices` may repeat (n local "devices" on one GPU)."""
        d = np.asarray(devices, np.int32)
        h = C.c_void_p()
        check(lib().osk_comm_init_all_loopback(ptr(d), len(d), C.byref(h)))
        return cls(h.value)

    def status(self) -> tuple[int, list[int]]:
        """(return code of osk_comm_status, [flag, rank 0's call number, differing rank, its call number]).
        Synchronise the calls' streams first."""
        info = (C.c_int64 * 4)()
        rc = lib().osk_comm_status(self._h, info)
        return rc, list(info)

    def set_device_limits(self, max_queries: int, max_k: int, max_shards_per_rank: int) -> None:
        """The device entry's exchange limits (osk_comm_set_device_limits): at world > 1 every
        osk_shards_search_merge_device call all-gathers a block of this fixed size, so ranks whose calls
        differ get count −1 instead of an all-gather of mismatched counts.  Same values on every rank."""
        check(lib().osk_comm_set_device_limits(self._h, max_queries, max_k, max_shards_per_rank))
        self._limits = (max_queries, max_k, max_shards_per_rank)

    @property
    def device_limits(self) -> tuple[int, int, int]:
        """(max queries, max k, max shards per rank) of the device entry's exchange block."""
        return getattr(self, "_limits", DEFAULT_DEVICE_LIMITS)

    def fits_device_limits(self, nq: int, k: int, shards_per_rank: int) -> bool:
        mq, mk, ms = self.device_limits
        return nq <= mq and k <= mk and shards_per_rank <= ms

    @classmethod
    def from_process_group(cls, device: int, group=None, device_limits: tuple[int, int, int] | None = None
                           ) -> "DeviceComm":
        """Rank 0 makes the id; torch.distributed (any backend) hands it to the other ranks.  device_limits
        (max queries, max k, max shards per rank), when given, are set right after init — pass the same
        values on every rank."""
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        comm = cls.init_rank(device, rank, world, obj[0])
        if device_limits is not None:
            comm.set_device_limits(*device_limits)
        return comm

    @property
    def handle(self):
        return self._h

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor, stream: int | None = None) -> None:
        check(lib().osk_comm_all_gather(self._h, send.data_ptr(), recv.data_ptr(),
                                        send.numel() * send.element_size(), stream))

    def close(self):
        if self._h.value:
            check(lib().osk_comm_release(self._h))
            self._h = C.c_void_p()


class ShardSearchMerge:
    """One rank's whole multi-GPU query step through the C-ABI (osk_shards_search_merge_device): scan of
    the rank's shards, ONE ncclAllGather of the per-shard top-k lists inside libosknn, coordinator
    TopDocs.merge on the device.  Outputs (scores, docs, shard index, count, total hits, max score)
    are preallocated and overwritten by the next call."""

    def __init__(self, comm: DeviceComm, view, shards_per_rank: int, nq: int, k: int, from_: int, size: int,
                 device: int, check_limits: bool = True):
        self.comm, self.view, self.spr = comm, view, shards_per_rank
        self.nq, self.k, self.from_, self.size = nq, k, from_, size
        # at world > 1 the exchange block must hold this call's shape (osk_comm_set_device_limits).  Checked here,
        # before any collective: a call beyond the limits would be refused on every rank (count −1, communicator
        # poisoned).  The limits are never raised implicitly — a rank that raised them alone would all-gather a
        # block of another size than its peers (undefined under RCCL: a hang).
        if check_limits and comm.world > 1 and not comm.fits_device_limits(nq, k, shards_per_rank):
            raise ValueError(f"ShardSearchMerge(nq={nq}, k={k}, shards_per_rank={shards_per_rank}) exceeds the "
                             f"communicator's device limits {comm.device_limits}: call "
                             f"comm.set_device_limits(...) with the same values on every rank first")
        dev = torch.device("cuda", device)
        self.out = (torch.empty((nq, size), dtype=torch.float32, device=dev),
                    torch.empty((nq, size), dtype=torch.int32, device=dev),
                    torch.empty((nq, size), dtype=torch.int32, device=dev),
                    torch.empty(nq, dtype=torch.int32, device=dev),
                    torch.empty(nq, dtype=torch.int64, device=dev),
                    torch.empty(nq, dtype=torch.float32, device=dev))

    def __call__(self, d_queries: int, stream: int, d_accept: int | None = None):
        sc, dc, sh, cnt, tot, mx = self.out
        check(lib().osk_shards_search_merge_device(self.comm.handle, self.view, d_queries, self.nq, self.k, d_accept,
                                                   self.spr, self.from_, self.size, sc.data_ptr(), dc.data_ptr(),
                                                   sh.data_ptr(), cnt.data_ptr(), tot.data_ptr(), mx.data_ptr(),
                                                   stream))
        return self.out


def shards_search_merge(comm: DeviceComm, views, queries: np.ndarray, k: int, from_: int, size: int, accept=None):
    """Host-buffer multi-GPU query (osk_shards_search_merge): views[i] lives on the communicator's local
    device i; accept = None or one bool mask (or None) per segment of every view, in view order.
    Returns (scores[nq,size], docs, shard_index, count[nq], total_hits[nq], max_score[nq])."""
    q = np.ascontiguousarray(queries)
    nq = q.shape[0]
    out = (np.empty((nq, size), np.float32), np.empty((nq, size), np.int32), np.empty((nq, size), np.int32),
           np.empty(nq, np.int32), np.empty(nq, np.int64), np.empty(nq, np.float32))
    hv = (C.c_void_p * len(views))(*[v.handle if hasattr(v, "handle") else v for v in views])
    acc_arr, keep = None, []
    if accept is not None:
        from .lucene import bits_from_bool
        ptrs = []
        for a in accept:
            if a is None:
                ptrs.append(None)
            else:
                keep.append(bits_from_bool(a))
                ptrs.append(keep[-1].ctypes.data)
        acc_arr = (C.c_void_p * len(ptrs))(*ptrs)
    check(lib().osk_shards_search_merge(comm.handle, hv, len(views), ptr(q), nq, k, acc_arr, from_, size,
                                        *[ptr(o) for o in out]))
    return out


def shard_owner(shard: int, n_shards: int, world: int) -> int:
    """Rank that holds `shard` (contiguous blocks of shards per rank)."""
    return shard * world // n_shards


def owned_shards(rank: int, n_shards: int, world: int) -> list[int]:
    return [s for s in range(n_shards) if shard_owner(s, n_shards, world) == rank]


def max_shards_per_rank(n_shards: int, world: int) -> int:
    return max(len(owned_shards(r, n_shards, world)) for r in range(world))


class ShardExchange:
    """The exchange step and the coordinator reduce of one rank, for a fixed (batch, k, from, size).

    keys [nq, s_pad, k] int64 (uint64 hit-key bit patterns, best first, zero-padded) of this rank's
    shards → ONE all-gather (RCCL over xGMI on the node, gloo in CPU tests) into a preallocated
    rank-major buffer [world·nq, s_pad, k] → the coordinator reduce straight over that image
    (device: osk_merge_device_ranked; host tensors: libosknn's host reduce).  A list's hit count is
    its number of non-zero keys, so counts are not exchanged.  The outputs (scores, docs, shard
    index, count, total hits, max score) are preallocated and overwritten by the next call."""

    def __init__(self, world: int, s_pad: int, nq: int, k: int, from_: int, size: int,
                 global_shard_index: torch.Tensor, device: int | None = None, group=None):
        self.world, self.s_pad, self.nq, self.k = world, s_pad, nq, k
        self.from_, self.size, self.group = from_, size, group
        self.device = device
        dev = torch.device("cuda", device) if device is not None else torch.device("cpu")
        self.gathered = torch.empty((world * nq, s_pad, k), dtype=torch.int64, device=dev)
        self.si = global_shard_index.to(device=dev, dtype=torch.int32).contiguous()
        self.out = (torch.empty((nq, size), dtype=torch.float32, device=dev),
                    torch.empty((nq, size), dtype=torch.int32, device=dev),
                    torch.empty((nq, size), dtype=torch.int32, device=dev),
                    torch.empty(nq, dtype=torch.int32, device=dev),
                    torch.empty(nq, dtype=torch.int64, device=dev),
                    torch.empty(nq, dtype=torch.float32, device=dev))

    def gather(self, keys: torch.Tensor) -> torch.Tensor:
        if self.world == 1:   # nothing to exchange
            return keys
        dist.all_gather_into_tensor(self.gathered, keys, group=self.group)
        return self.gathered

    def reduce(self, gathered: torch.Tensor, stream: int | None = None):
        nq, sl, k = self.nq, self.s_pad, self.k
        if gathered.is_cuda:
            sc, dc, sh, cnt, tot, mx = self.out
            check(lib().osk_merge_device_ranked(self.device, gathered.data_ptr(), self.world, sl,
                                                self.si.data_ptr(), nq, k, self.from_, self.size, sc.data_ptr(),
                                                dc.data_ptr(), sh.data_ptr(), cnt.data_ptr(), tot.data_ptr(),
                                                mx.data_ptr(), stream))
            return self.out
        kk = gathered.numpy().view(np.uint64).reshape(self.world, nq, sl, k)
        si = self.si.numpy()
        S = self.world * sl
        for q in range(nq):
            lists = np.ascontiguousarray(kk[:, q].reshape(S, k))
            counts = np.count_nonzero(lists, axis=1).astype(np.int32)
            sc = np.empty((S, k), np.float32)
            dc = np.empty((S, k), np.int32)
            check(lib().osk_decode_keys(ptr(lists), lists.size, ptr(sc), ptr(dc)))
            c32, t64, m32 = C.c_int32(), C.c_int64(), C.c_float()
            os_ = np.empty(self.size, np.float32)
            od = np.empty(self.size, np.int32)
            osh = np.empty(self.size, np.int32)
            check(lib().osk_topdocs_merge(S, ptr(counts), ptr(sc), ptr(dc), k, ptr(si), None, self.from_, self.size,
                                          ptr(os_), ptr(od), ptr(osh), C.byref(c32), C.byref(t64), C.byref(m32)))
            self.out[0][q] = torch.from_numpy(os_)
            self.out[1][q] = torch.from_numpy(od)
            self.out[2][q] = torch.from_numpy(osh)
            self.out[3][q], self.out[4][q], self.out[5][q] = c32.value, t64.value, m32.value
        return self.out

    def __call__(self, keys: torch.Tensor, stream: int | None = None):
        return self.reduce(self.gather(keys), stream)


class LocalShards:
    """The shards a rank owns, staged on its GPU as one osk_view (one synthetic segment per shard,
    shard s = global rows [s·rows_per_shard, (s+1)·rows_per_shard) as local docs 0..n−1)."""

    def __init__(self, rank: int, world: int, n_shards: int, rows_per_shard: int, dim: int,
                 similarity: int, encoding: int, seed: int, dist_kind: int, device: int):
        self.rank, self.world, self.n_shards = rank, world, n_shards
        self.device = device
        self.shards = owned_shards(rank, n_shards, world)
        self.s_pad = max_shards_per_rank(n_shards, world)
        self.segs = []
        for s in self.shards:
            h = C.c_void_p()
            check(lib().osk_seg_synth(device, rows_per_shard, dim, encoding, similarity, seed, dist_kind,
                                      s * rows_per_shard, C.byref(h)))
            self.segs.append(h.value)
        self.extra_views = []
        self.view = self._new_view()
        # global shardIndex of every gathered slot: rank r's slot j ↔ owned_shards(r)[j]; pad slots (a rank
        # owning fewer shards) get INT32_MAX — their lists are all-zero keys, so they never contribute a hit
        gi = []
        for r in range(world):
            own = owned_shards(r, n_shards, world)
            gi += own + [2**31 - 1] * (self.s_pad - len(own))
        self.global_shard_index = torch.tensor(gi, dtype=torch.int32)

    def _new_view(self) -> C.c_void_p:
        arr = (C.c_void_p * len(self.segs))(*self.segs)
        seg_shard = np.arange(len(self.segs), dtype=np.int32)
        seg_base = np.zeros(len(self.segs), np.int32)
        sidx = np.asarray(self.shards, np.int32)
        v = C.c_void_p()
        check(lib().osk_view_create(arr, len(self.segs), ptr(seg_shard), ptr(seg_base), len(self.segs),
                                    ptr(sidx), C.byref(v)))
        return v

    def add_view(self) -> C.c_void_p:
        """Another view over the same staged segments (its own workspace; the segments are shared and
        retained): one per search thread, so searches issued on different streams run concurrently on
        the device instead of waiting for each other's workspace."""
        v = self._new_view()
        self.extra_views.append(v)
        return v

    def search(self, d_queries: int, nq: int, k: int, keys: torch.Tensor, counts: torch.Tensor,
               stream: int | None) -> None:
        """Per-shard top-k of this rank's shards into keys [nq, s_pad, k] / counts [nq, s_pad].
        `stream` must be the handle of the torch stream the caller's tensors are used on, and not the
        null stream (handle 0 = the library's own non-blocking stream, unordered with torch's work)."""
        if not stream:
            raise ValueError("pass a non-default torch stream handle (torch.cuda.Stream().cuda_stream)")
        sl = len(self.segs)
        if sl == self.s_pad:
            check(lib().osk_view_search_device(self.view, d_queries, nq, k, None, keys.data_ptr(),
                                               counts.data_ptr(), None, stream))
            return
        tk = torch.empty((nq, sl, k), dtype=torch.int64, device=keys.device)
        tc = torch.empty((nq, sl), dtype=torch.int32, device=keys.device)
        check(lib().osk_view_search_device(self.view, d_queries, nq, k, None, tk.data_ptr(), tc.data_ptr(),
                                           None, stream))
        keys.zero_()
        counts.zero_()
        keys[:, :sl].copy_(tk)
        counts[:, :sl].copy_(tc)

    def close(self):
        for v in self.extra_views:
            lib().osk_view_release(v)
        self.extra_views = []
        if self.view:
            lib().osk_view_release(self.view)
            self.view = C.c_void_p()
        for h in self.segs:
            lib().osk_seg_release(C.c_void_p(h))
        self.segs = []
