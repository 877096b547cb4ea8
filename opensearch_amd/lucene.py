"""Host-side mirror of the Lucene / OpenSearch interfaces on the exact k-NN path.

The reference (OpenSearch 3.3.0) runs this path inside lucene-core 10.3.0 ([L], un-vendored):
`KnnFloatVectorQuery` / `KnnByteVectorQuery` are rewritten per leaf by `AbstractKnnVectorQuery`,
each leaf calls `KnnVectorsReader.search(field, target, KnnCollector, AcceptDocs)`, and the per-leaf
`TopDocs` are combined with `TopDocs.merge`.  OpenSearch drives the rewrite from
`ContextIndexSearcher.rewrite` (server/src/main/java/org/opensearch/search/internal/
ContextIndexSearcher.java:203-218) and merges shards with `TopDocs.merge(from, size, …)` in
`SearchPhaseController.mergeTopDocs` (server/src/main/java/org/opensearch/action/search/
SearchPhaseController.java:224-246).

This module keeps those names and argument meanings so the tests read like the reference's own.
Every search call goes through libosknn's C-ABI (HIP kernels on a gfx950 device); merges of host
lists go through the library's host reduce (`osk_topdocs_merge`).  There is no CPU search fallback.
"""
from __future__ import annotations

import ctypes as C
import enum
import math
import threading
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import check, lib, ptr


class VectorSimilarityFunction(enum.IntEnum):
    """[L] org.apache.lucene.index.VectorSimilarityFunction (ordinal order)."""
    EUCLIDEAN = 0
    DOT_PRODUCT = 1
    COSINE = 2
    MAXIMUM_INNER_PRODUCT = 3


class VectorEncoding(enum.IntEnum):
    """[L] org.apache.lucene.index.VectorEncoding."""
    FLOAT32 = 0
    BYTE = 1


class Relation(enum.Enum):
    EQUAL_TO = 0
    GREATER_THAN_OR_EQUAL_TO = 1


@dataclass
class TotalHits:
    value: int
    relation: Relation = Relation.EQUAL_TO


@dataclass
class ScoreDoc:
    """[L] ScoreDoc: doc, score, shardIndex (−1 until SearchPhaseController.setShardIndex)."""
    doc: int
    score: float
    shard_index: int = -1


@dataclass
class TopDocs:
    total_hits: TotalHits
    score_docs: list[ScoreDoc] = field(default_factory=list)

    @staticmethod
    def merge(start: int, size: int, shard_hits: Sequence["TopDocs"]) -> "TopDocs":
        """[L] TopDocs.merge(start, topN, shardHits): score desc, then shardIndex asc, then doc asc.

        Hits carry their own shardIndex (set by SearchPhaseController.setShardIndex,
        SearchPhaseController.java:248-253; −1 inside a shard's per-leaf merge).  Runs in libosknn's
        host reduce (osk_topdocs_merge).  totalHits = Σ, relation GTE if any input is GTE.
        """
        n = len(shard_hits)
        stride = max([len(t.score_docs) for t in shard_hits] + [1])
        counts = np.zeros(max(n, 1), np.int32)
        scores = np.zeros((max(n, 1), stride), np.float32)
        docs = np.zeros((max(n, 1), stride), np.int32)
        hsi = np.zeros((max(n, 1), stride), np.int32)
        for s, td in enumerate(shard_hits):
            counts[s] = len(td.score_docs)
            for i, sd in enumerate(td.score_docs):
                scores[s, i] = sd.score
                docs[s, i] = sd.doc
                hsi[s, i] = sd.shard_index
        out_s = np.empty(max(size, 1), np.float32)
        out_d = np.empty(max(size, 1), np.int32)
        out_sh = np.empty(max(size, 1), np.int32)
        cnt = C.c_int32()
        tot = C.c_int64()
        mx = C.c_float()
        check(lib().osk_topdocs_merge(n, ptr(counts), ptr(scores), ptr(docs), stride, None, ptr(hsi),
                                      start, size, ptr(out_s), ptr(out_d), ptr(out_sh), C.byref(cnt),
                                      C.byref(tot), C.byref(mx)))
        total = sum(t.total_hits.value for t in shard_hits)
        rel = (Relation.GREATER_THAN_OR_EQUAL_TO
               if any(t.total_hits.relation == Relation.GREATER_THAN_OR_EQUAL_TO for t in shard_hits)
               else Relation.EQUAL_TO)
        hits = [ScoreDoc(int(out_d[i]), float(out_s[i]), int(out_sh[i])) for i in range(cnt.value)]
        return TopDocs(TotalHits(total, rel), hits)


# ------------------------------------------------------------------------------------------------
# accept bits ([L] AcceptDocs = liveDocs ∩ filter, a Bits over the leaf's maxDoc)
# ------------------------------------------------------------------------------------------------
def bits_from_bool(mask: np.ndarray) -> np.ndarray:
    """bool[max_doc] → uint64[ceil(max_doc/64)], LSB-first (the C-ABI's accept-bitset format)."""
    mask = np.asarray(mask, dtype=bool)
    nbytes = (len(mask) + 63) // 64 * 8
    packed = np.packbits(mask, bitorder="little")
    buf = np.zeros(max(nbytes, 8), np.uint8)
    buf[: len(packed)] = packed
    return buf.view(np.uint64)[: max(1, (len(mask) + 63) // 64)].copy()


def _as_query_array(target, encoding: VectorEncoding, dim: int) -> np.ndarray:
    dt = np.float32 if encoding == VectorEncoding.FLOAT32 else np.int8
    q = np.ascontiguousarray(np.asarray(target, dtype=dt))
    if q.ndim == 1:
        q = q[None, :]
    if q.shape[1] != dim:
        raise ValueError(f"vector dimension {q.shape[1]} does not match field dimension {dim}")
    return q


# ------------------------------------------------------------------------------------------------
# KnnVectorsReader over HBM
# ------------------------------------------------------------------------------------------------
class GpuFlatVectorsReader:
    """[L] KnnVectorsReader for one segment's flat vector field, staged once into HBM.

    Mirrors the reader a `KnnVectorsFormat.fieldsReader(SegmentReadState)` would return: built when
    the segment opens (S/index/engine/InternalEngine.java:584-589), `search()` answers
    `LeafReader.searchNearestVectors` (4-arg signature evidenced at
    S/index/engine/TranslogLeafReader.java:379-386), `close()` frees the HBM copy.
    """

    def __init__(self, field: str, vectors, similarity: VectorSimilarityFunction,
                 encoding: VectorEncoding = VectorEncoding.FLOAT32, ord_to_doc=None,
                 max_doc: int | None = None, device: int = 0, _handle: int | None = None,
                 _dim: int | None = None, _n: int | None = None):
        self.field = field
        self.similarity = VectorSimilarityFunction(similarity)
        self.encoding = VectorEncoding(encoding)
        self.device = device
        self._h = C.c_void_p(None)
        if _handle is not None:
            self._h = C.c_void_p(_handle)
            self.dim, self.size = int(_dim), int(_n)
            self.ord_to_doc = None
            self.max_doc = int(max_doc if max_doc is not None else _n)
            return
        dt = np.float32 if self.encoding == VectorEncoding.FLOAT32 else np.int8
        rows = np.ascontiguousarray(np.asarray(vectors, dtype=dt))
        if rows.ndim != 2:
            raise ValueError("vectors must be [n, dim]")
        self.size, self.dim = rows.shape
        o2d = None
        if ord_to_doc is not None:
            o2d = np.ascontiguousarray(np.asarray(ord_to_doc, dtype=np.int32))
            if len(o2d) != self.size:
                raise ValueError("ord_to_doc length != number of vectors")
        self.ord_to_doc = o2d
        self.max_doc = int(max_doc if max_doc is not None else (int(o2d[-1]) + 1 if o2d is not None and len(o2d) else self.size))
        check(lib().osk_seg_stage(device, ptr(rows), self.size, self.dim, int(self.encoding),
                                  int(self.similarity), ptr(o2d), self.max_doc, C.byref(self._h)))

    @classmethod
    def synthetic(cls, field: str, n: int, dim: int, similarity, encoding=VectorEncoding.FLOAT32,
                  seed: int = 42, dist: int = _lib.DIST_NORMALISH_UNIT, row0: int = 0, device: int = 0):
        """A dense segment generated on the device by the counter-based generator (bench/tests)."""
        h = C.c_void_p(None)
        check(lib().osk_seg_synth(device, n, dim, int(encoding), int(similarity), seed, dist, row0,
                                  C.byref(h)))
        return cls(field, None, similarity, encoding, device=device, _handle=h.value, _dim=dim, _n=n)

    @classmethod
    def from_files(cls, field: str, directory: str, segment: str, segment_id: bytes, max_doc: int,
                   field_number: int, suffix: str = "", device: int = 0):
        """The reader a `KnnVectorsFormat.fieldsReader(SegmentReadState)` builds when the segment opens:
        the field's entry parsed from `segment.vemf`, its `.vec` slice staged into HBM
        (flatfiles.stage_field → osk_seg_stage_file)."""
        import os
        from . import flatfiles as FF
        base = segment + (f"_{suffix}" if suffix else "")
        vec, vemf = os.path.join(directory, base + ".vec"), os.path.join(directory, base + ".vemf")
        FF.check_data_file(vec, segment_id, suffix)
        entries = {e.number: e for e in FF.read_meta(vemf, segment_id, suffix)}
        if field_number not in entries:
            raise ValueError(f"field {field_number} has no vectors in {vemf}")
        e = entries[field_number]
        h = FF.stage_field(vec, e, max_doc, device)
        r = cls(field, None, VectorSimilarityFunction(e.similarity), VectorEncoding(e.encoding), max_doc=max_doc,
                device=device, _handle=h, _dim=e.dim, _n=e.size)
        return r

    @property
    def handle(self) -> int:
        if not self._h.value:
            raise RuntimeError("reader is closed")
        return self._h.value

    def search_batch(self, targets, k: int, accept_bits: np.ndarray | None = None):
        """Exact top-k for a batch of targets: (scores[nq,k], docs[nq,k], counts[nq], visited[nq])."""
        q = _as_query_array(targets, self.encoding, self.dim)
        nq = q.shape[0]
        scores = np.empty((nq, k), np.float32)
        docs = np.empty((nq, k), np.int32)
        counts = np.empty(nq, np.int32)
        visited = np.empty(nq, np.int64)
        ab = None if accept_bits is None else np.ascontiguousarray(accept_bits, dtype=np.uint64)
        check(lib().osk_seg_search(self.handle, ptr(q), nq, k, ptr(ab), ptr(scores), ptr(docs),
                                   ptr(counts), ptr(visited)))
        return scores, docs, counts, visited

    def search(self, field: str, target, k: int, accept_docs: np.ndarray | None = None) -> TopDocs:
        """[L] KnnVectorsReader.search(field, target, KnnCollector(k), AcceptDocs) → the collector's
        topDocs(): segment-local docs, score desc / doc asc, totalHits = visited (EQUAL_TO)."""
        if field != self.field:
            raise ValueError(f"unknown field {field!r}")
        ab = None if accept_docs is None else bits_from_bool(accept_docs)
        s, d, c, v = self.search_batch(target, k, ab)
        hits = [ScoreDoc(int(d[0, i]), float(s[0, i])) for i in range(int(c[0]))]
        return TopDocs(TotalHits(int(v[0])), hits)

    def close(self) -> None:
        if self._h.value:
            _GpuKnnVectorQuery._reader_closed(self)   # the reader-closed listener: drop views over it
            check(lib().osk_seg_release(self._h))
            self._h = C.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class LeafReaderContext:
    """[L] LeafReaderContext: one segment of a shard; docBase offsets its docs in the shard."""
    ord: int
    doc_base: int
    reader: GpuFlatVectorsReader
    live_docs: np.ndarray | None = None   # bool[max_doc], None = no deletions

    @property
    def max_doc(self) -> int:
        return self.reader.max_doc


class _KnnVectorQuery:
    encoding = VectorEncoding.FLOAT32

    def __init__(self, field: str, target, k: int, filter=None):
        if k < 1:
            raise ValueError("k must be at least 1")
        self.field = field
        self.target = target
        self.k = k
        self.filter = filter          # callable(leaf) -> bool[max_doc], or None

    def _accept(self, leaf: LeafReaderContext):
        acc = leaf.live_docs
        if self.filter is not None:
            f = np.asarray(self.filter(leaf), dtype=bool)
            acc = f if acc is None else (acc & f)
        return acc

    def rewrite(self, leaves: Iterable[LeafReaderContext]) -> TopDocs:
        """[L] AbstractKnnVectorQuery.rewrite: per-leaf top-k (docBase added), then
        TopDocs.merge(k, perLeafResults).  The result is what DocAndScoreQuery then matches."""
        per_leaf = []
        for leaf in leaves:
            td = leaf.reader.search(self.field, self.target, self.k, self._accept(leaf))
            for sd in td.score_docs:
                sd.doc += leaf.doc_base
            per_leaf.append(td)
        if not per_leaf:
            return TopDocs(TotalHits(0), [])
        merged = TopDocs.merge(0, self.k, per_leaf)
        # TopDocs.merge's totalHits is Σ visited; the rewritten query matches len(hits) docs
        return merged


class KnnFloatVectorQuery(_KnnVectorQuery):
    """[L] KnnFloatVectorQuery(field, float[] target, k, filter).

    Its rewrite is Lucene's per-leaf route: one KnnVectorsReader.search per leaf, run as per-leaf tasks
    on the index_searcher pool under concurrent segment search (S/search/DefaultSearchContext.java:257-267).
    Real Lucene also never calls the reader for a filtered leaf whose accepted docs number ≤ k: it runs
    exactSearch on the CPU over FloatVectorValues.scorer (Panama order, within 1e-5 of the device but not
    bit-identical).  GpuKnnFloatVectorQuery below is the plugin's query that routes both onto the device."""
    encoding = VectorEncoding.FLOAT32


class KnnByteVectorQuery(_KnnVectorQuery):
    """[L] KnnByteVectorQuery(field, byte[] target, k, filter)."""
    encoding = VectorEncoding.BYTE


class _GpuKnnVectorQuery:
    """The plugin's k-NN query (`GpuKnnFloatVectorQuery extends KnnFloatVectorQuery`):

    * rewrite: ONE device call per shard — osk_view_search over a view of all the shard's leaves, cached
      per point-in-time reader (the leaves' readers and docBases), with each leaf's AcceptDocs
      (liveDocs ∩ filter) pushed down as a bitset — instead of one KnnVectorsReader.search per leaf.
      The device merges the leaves ([L] TopDocs.merge(k, perLeaf): score desc, doc asc) in the same call;
    * every filtered leaf goes to the device whatever its cost, so Lucene's `cost ≤ k` CPU exactSearch
      branch never runs; `exact_search` (the override of [L] AbstractKnnVectorQuery.exactSearch) serves a
      caller that still asks for a per-leaf exact search, on the device.
    Results are identical to the per-leaf route (every device path is exact in the device order).

    The view cache is keyed by the point-in-time leaf set and evicted by the reader-closed listener: when a
    segment's reader closes (a refresh or merge dropped it), every cached view over it is released, so a
    view never pins the HBM of segments no searcher can reach.  Creation is under a lock, so concurrent
    rewrites of one leaf set share one view."""
    _views: dict = {}          # leaf-set key → _CachedView
    _views_lock = threading.Lock()

    class _CachedView:
        """A cached view and its users: rewrites in flight hold a use, and an evicted view closes when the
        last of them finishes (never under a search)."""
        __slots__ = ("view", "users", "evicted")

        def __init__(self, view):
            self.view, self.users, self.evicted = view, 0, False

    def _acquire_view(self, leaves: Sequence[LeafReaderContext]) -> "_GpuKnnVectorQuery._CachedView":
        key = tuple((id(lf.reader), lf.reader.handle, lf.doc_base) for lf in leaves)
        C_ = _GpuKnnVectorQuery
        with C_._views_lock:
            e = C_._views.get(key)
            if e is None:
                e = C_._CachedView(DeviceShardSet([list(leaves)], [0]))
                C_._views[key] = e
            e.users += 1
            return e

    @staticmethod
    def _release_view(e: "_GpuKnnVectorQuery._CachedView") -> None:
        with _GpuKnnVectorQuery._views_lock:
            e.users -= 1
            close = e.evicted and e.users == 0
        if close:
            e.view.close()

    @staticmethod
    def _evict(entries) -> None:
        """Evicted entries (already out of the cache): close the idle ones now, the busy ones on release."""
        with _GpuKnnVectorQuery._views_lock:
            idle = []
            for e in entries:
                e.evicted = True
                if e.users == 0:
                    idle.append(e)
        for e in idle:
            e.view.close()

    # (the cache is the base class's: subclasses' classmethods must not rebind it on themselves)
    @staticmethod
    def _reader_closed(reader) -> None:
        C_ = _GpuKnnVectorQuery
        with C_._views_lock:
            gone = [k for k in C_._views if any(rid == id(reader) for rid, _, _ in k)]
            entries = [C_._views.pop(k) for k in gone]
        C_._evict(entries)

    @staticmethod
    def cached_views() -> int:
        with _GpuKnnVectorQuery._views_lock:
            return len(_GpuKnnVectorQuery._views)

    @staticmethod
    def release_views() -> None:
        """Drop every cached view (the segments stay with their readers; a view in use closes when its
        search finishes)."""
        C_ = _GpuKnnVectorQuery
        with C_._views_lock:
            entries = list(C_._views.values())
            C_._views.clear()
        C_._evict(entries)

    def rewrite(self, leaves: Iterable[LeafReaderContext]) -> TopDocs:
        leaves = [lf for lf in leaves if lf.reader.field == self.field]
        if not leaves:
            return TopDocs(TotalHits(0), [])
        e = self._acquire_view(leaves)
        try:
            accept = [self._accept(lf) for lf in leaves]
            if all(a is None for a in accept):
                accept = None
            s, d, _, c, _, _ = e.view.search(self.target, self.k, 0, self.k, accept=accept)
        finally:
            self._release_view(e)
        n = int(c[0])
        return TopDocs(TotalHits(n), [ScoreDoc(int(d[0, i]), float(s[0, i])) for i in range(n)])

    def exact_search(self, leaf: LeafReaderContext, accept: np.ndarray | None) -> TopDocs:
        """[L] AbstractKnnVectorQuery.exactSearch(context, acceptIterator, timeout) on the device."""
        td = leaf.reader.search(self.field, self.target, self.k, accept)
        for sd in td.score_docs:
            sd.doc += leaf.doc_base
        return td


class GpuKnnFloatVectorQuery(_GpuKnnVectorQuery, KnnFloatVectorQuery):
    encoding = VectorEncoding.FLOAT32


class GpuKnnByteVectorQuery(_GpuKnnVectorQuery, KnnByteVectorQuery):
    encoding = VectorEncoding.BYTE


def shard_query_phase(query: _KnnVectorQuery, leaves: Sequence[LeafReaderContext], from_: int,
                      size: int) -> TopDocs:
    """The shard's query phase for a k-NN query: rewrite (ContextIndexSearcher.java:203-218), then
    a TopScoreDocCollector over the DocAndScoreQuery with numDocs = min(from+size, …)
    (S/search/query/TopDocsCollectorContext.java:866-891).  totalHits = number of k-NN hits."""
    rewritten = query.rewrite(leaves)
    hits = rewritten.score_docs[: from_ + size]
    return TopDocs(TotalHits(len(rewritten.score_docs)), [ScoreDoc(h.doc, h.score) for h in hits])


# ------------------------------------------------------------------------------------------------
# Several shards' leaves on one device: one launch scans them all, per-shard top-k on the device,
# then the coordinator merge on the device (SearchPhaseController.mergeTopDocs semantics).
# ------------------------------------------------------------------------------------------------
class DeviceShardSet:
    """The leaves of `n_shards` shards resident on one GPU (an `osk_view`)."""

    def __init__(self, shard_leaves: Sequence[Sequence[LeafReaderContext]],
                 shard_index: Sequence[int] | None = None):
        segs, seg_shard, seg_base = [], [], []
        for s, leaves in enumerate(shard_leaves):
            for leaf in leaves:
                segs.append(leaf.reader.handle)
                seg_shard.append(s)
                seg_base.append(leaf.doc_base)
        if not segs:
            raise ValueError("no segments")
        self.leaves = [lf for leaves in shard_leaves for lf in leaves]
        self.n_shards = len(shard_leaves)
        self.shard_index = np.asarray(shard_index if shard_index is not None else range(self.n_shards), np.int32)
        self._segs = (C.c_void_p * len(segs))(*segs)
        ss = np.asarray(seg_shard, np.int32)
        sb = np.asarray(seg_base, np.int32)
        self._h = C.c_void_p(None)
        check(lib().osk_view_create(self._segs, len(segs), ptr(ss), ptr(sb), self.n_shards,
                                    ptr(self.shard_index), C.byref(self._h)))
        r0 = self.leaves[0].reader
        self.dim, self.encoding = r0.dim, r0.encoding

    @property
    def handle(self) -> int:
        return self._h.value

    def search(self, targets, k: int, from_: int = 0, size: int = 10, accept=None):
        """Batch search + coordinator merge.  Returns per query (scores[size], docs[size],
        shard_index[size], count, total_hits, max_score) as arrays."""
        q = _as_query_array(targets, self.encoding, self.dim)
        nq = q.shape[0]
        scores = np.empty((nq, size), np.float32)
        docs = np.empty((nq, size), np.int32)
        shard = np.empty((nq, size), np.int32)
        count = np.empty(nq, np.int32)
        total = np.empty(nq, np.int64)
        mx = np.empty(nq, np.float32)
        acc_arr = None
        keep = []
        if accept is not None:
            ptrs = []
            for leaf, a in zip(self.leaves, accept):
                if a is None:
                    ptrs.append(None)
                else:
                    b = bits_from_bool(a)
                    keep.append(b)
                    ptrs.append(b.ctypes.data)
            acc_arr = (C.c_void_p * len(ptrs))(*ptrs)
        check(lib().osk_view_search(self.handle, ptr(q), nq, k, from_, size, acc_arr, ptr(scores),
                                    ptr(docs), ptr(shard), ptr(count), ptr(total), ptr(mx)))
        return scores, docs, shard, count, total, mx

    def stats(self) -> tuple[int, int]:
        """(searches that took the batched MFMA path, queries recomputed after a failed certificate)."""
        a, b = C.c_int64(), C.c_int64()
        check(lib().osk_view_stats(self.handle, C.byref(a), C.byref(b)))
        return a.value, b.value

    def counter(self, name: str) -> int:
        """A named counter of the view (osk_view_counter): "sq8_calls", "sq8_fallback_queries",
        "sq8_rescored_rows", "mfma_calls", "mfma_fallback_queries"."""
        v = C.c_int64()
        check(lib().osk_view_counter(self.handle, name.encode(), C.byref(v)))
        return v.value

    def close(self):
        if self._h.value:
            check(lib().osk_view_release(self._h))
            self._h = C.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def decode_keys(keys: np.ndarray):
    """uint64 hit keys → (scores f32, docs i32); key 0 → (−inf, INT32_MAX)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    s = np.empty(keys.shape, np.float32)
    d = np.empty(keys.shape, np.int32)
    check(lib().osk_decode_keys(ptr(keys), keys.size, ptr(s), ptr(d)))
    return s, d


def synth_host(row0: int, n: int, dim: int, seed: int, dist: int) -> np.ndarray:
    """The host twin of the device generator (libosknn osk_synth_host)."""
    out = np.empty((n, dim), np.int8 if dist == _lib.DIST_INT8 else np.float32)
    check(lib().osk_synth_host(ptr(out), row0, n, dim, seed, dist))
    return out
