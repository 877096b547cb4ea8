"""Multi-GPU exact k-NN: shards ↔ GPUs, one process per GPU, RCCL all-gather of per-shard top-k.

Mapping onto the reference:
  * Index shards are OpenSearch's data partitioning (IndexMetadata.java:265-268); the coordinator
    fans a query out to one copy of every shard (AbstractSearchAsyncAction.java:262-268) and merges
    the shard results by score (SearchPhaseController.java:224-246).
  * Here shard s lives on rank `shard_owner(s)` (contiguous blocks, so a GPU owns 8/G shards of an
    8-shard index).  Each rank scans its shards in one launch and produces per-shard top-k lists of
    8-byte hit keys; `torch.distributed.all_gather_into_tensor` (backend "nccl" = RCCL over xGMI on
    the MI355X node, "gloo" in CPU tests) exchanges them; the coordinator reduce then runs on the
    device (`osk_merge_device`) or, for host tensors, in the library's host reduce.
The exchange is k·B·8 bytes per shard — latency-bound, microseconds next to a millisecond scan.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, lib, ptr


def shard_owner(shard: int, n_shards: int, world: int) -> int:
    """Rank that holds `shard` (contiguous blocks of shards per rank)."""
    return shard * world // n_shards


def owned_shards(rank: int, n_shards: int, world: int) -> list[int]:
    return [s for s in range(n_shards) if shard_owner(s, n_shards, world) == rank]


def max_shards_per_rank(n_shards: int, world: int) -> int:
    return max(len(owned_shards(r, n_shards, world)) for r in range(world))


def gather_shard_topk(keys: torch.Tensor, counts: torch.Tensor, world: int, group=None):
    """keys [nq, S_l, k] int64 (uint64 bit pattern), counts [nq, S_l] int32 on every rank (S_l padded
    to the same value everywhere) → gathered keys [nq, world·S_l, k], counts [nq, world·S_l]."""
    nq, sl, k = keys.shape
    if world == 1:   # nothing to exchange
        return keys, counts
    # concatenated along dim 0 (the layout both RCCL and gloo accept), viewed as [world, nq, …]
    gk = torch.empty((world * nq, sl, k), dtype=keys.dtype, device=keys.device)
    gc = torch.empty((world * nq, sl), dtype=counts.dtype, device=counts.device)
    dist.all_gather_into_tensor(gk, keys.contiguous(), group=group)
    dist.all_gather_into_tensor(gc, counts.contiguous(), group=group)
    gk = gk.view(world, nq, sl, k)
    gc = gc.view(world, nq, sl)
    return (gk.permute(1, 0, 2, 3).reshape(nq, world * sl, k).contiguous(),
            gc.permute(1, 0, 2).reshape(nq, world * sl).contiguous())


def merge_gathered(keys: torch.Tensor, counts: torch.Tensor, shard_index: torch.Tensor, k: int,
                   from_: int, size: int, device: int = 0, stream: int | None = None):
    """Coordinator reduce over gathered per-shard lists → (scores, docs, shard_index, count,
    total_hits, max_score) tensors.  Device tensors: osk_merge_device on the GPU.  Host tensors:
    the library's host reduce (osk_topdocs_merge) per query."""
    nq, S, _ = keys.shape
    if keys.is_cuda:
        dev = keys.device
        scores = torch.empty((nq, size), dtype=torch.float32, device=dev)
        docs = torch.empty((nq, size), dtype=torch.int32, device=dev)
        shard = torch.empty((nq, size), dtype=torch.int32, device=dev)
        count = torch.empty(nq, dtype=torch.int32, device=dev)
        total = torch.empty(nq, dtype=torch.int64, device=dev)
        mx = torch.empty(nq, dtype=torch.float32, device=dev)
        si = shard_index.to(device=dev, dtype=torch.int32).contiguous()
        check(lib().osk_merge_device(device, keys.data_ptr(), counts.data_ptr(), si.data_ptr(), nq, S, k,
                                     from_, size, scores.data_ptr(), docs.data_ptr(), shard.data_ptr(),
                                     count.data_ptr(), total.data_ptr(), mx.data_ptr(), stream))
        return scores, docs, shard, count, total, mx
    kk = keys.numpy().view(np.uint64)
    cc = counts.numpy().astype(np.int32)
    si = shard_index.numpy().astype(np.int32)
    scores = np.empty((nq, size), np.float32)
    docs = np.empty((nq, size), np.int32)
    shard = np.empty((nq, size), np.int32)
    count = np.empty(nq, np.int32)
    total = np.empty(nq, np.int64)
    mx = np.empty(nq, np.float32)
    for q in range(nq):
        sc = np.empty((S, k), np.float32)
        dc = np.empty((S, k), np.int32)
        kq = np.ascontiguousarray(kk[q])
        check(lib().osk_decode_keys(ptr(kq), kq.size, ptr(sc), ptr(dc)))
        cq = np.ascontiguousarray(cc[q])
        c32, t64, m32 = C.c_int32(), C.c_int64(), C.c_float()
        os_ = np.empty(size, np.float32)
        od = np.empty(size, np.int32)
        osh = np.empty(size, np.int32)
        check(lib().osk_topdocs_merge(S, ptr(cq), ptr(sc), ptr(dc), k, ptr(si), None, from_, size, ptr(os_),
                                      ptr(od), ptr(osh), C.byref(c32), C.byref(t64), C.byref(m32)))
        scores[q], docs[q], shard[q] = os_, od, osh
        count[q], total[q], mx[q] = c32.value, t64.value, m32.value
    t = torch.from_numpy
    return t(scores), t(docs), t(shard), t(count), t(total), t(mx)


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
        arr = (C.c_void_p * len(self.segs))(*self.segs)
        seg_shard = np.arange(len(self.segs), dtype=np.int32)
        seg_base = np.zeros(len(self.segs), np.int32)
        sidx = np.asarray(self.shards, np.int32)
        self.view = C.c_void_p()
        check(lib().osk_view_create(arr, len(self.segs), ptr(seg_shard), ptr(seg_base), len(self.segs),
                                    ptr(sidx), C.byref(self.view)))
        # global shardIndex of every gathered slot: rank r's slot j ↔ owned_shards(r)[j] (pads → −1)
        gi = []
        for r in range(world):
            own = owned_shards(r, n_shards, world)
            gi += own + [2**31 - 1] * (self.s_pad - len(own))
        self.global_shard_index = torch.tensor(gi, dtype=torch.int32)

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
        if self.view:
            lib().osk_view_release(self.view)
            self.view = C.c_void_p()
        for h in self.segs:
            lib().osk_seg_release(C.c_void_p(h))
        self.segs = []
