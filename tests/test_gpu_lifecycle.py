"""Segment lifecycle on the GPU: staging from Lucene99 flat vector files and NRT refresh churn.

A segment's vectors reach HBM from its `.vec` slice (mmap → pinned ring → HBM, osk_seg_stage_file),
located by its `.vemf` entry (opensearch_amd/flatfiles.py — the published Lucene99FlatVectorsFormat
layout restated; parity unpinned, no Lucene jar).  Results must be bit-identical to staging the same
rows from memory.  Refreshes (S/index/engine/InternalEngine.java:584-589) open new segments and merge
old ones away while searches run on the previous reader's view: a segment closed by its reader stays
valid until no view holds it (refcounts), and every searcher sees exactly its own point-in-time set.
"""
import numpy as np
import pytest

from opensearch_amd import flatfiles as FF, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SID = bytes(range(100, 116))
COS = LU.VectorSimilarityFunction.COSINE
L2 = LU.VectorSimilarityFunction.EUCLIDEAN


def same(a, b):
    for x, y in zip(a, b):
        x, y = np.asarray(x), np.asarray(y)
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (x, y)


def test_stage_from_files_equals_stage_from_memory(tmp_path):
    rng = np.random.default_rng(1)
    max_doc = 90000
    dense = O.synth(0, max_doc, 768, 400, 3)
    docs = np.sort(rng.choice(max_doc, 30000, replace=False)).astype(np.int32)
    sparse = O.synth(0, len(docs), 100, 401, 1)
    bvec = O.synth(0, 5000, 64, 402, 4)
    bdocs = np.sort(rng.choice(max_doc, 5000, replace=False)).astype(np.int32)
    FF.write_segment(str(tmp_path), "_a", SID, max_doc, [(1, dense, int(COS), None), (4, sparse, int(L2), docs),
                                                         (6, bvec, 1, bdocs)], suffix="Lucene99_0")
    cases = [(1, dense, COS, None, LU.VectorEncoding.FLOAT32), (4, sparse, L2, docs, LU.VectorEncoding.FLOAT32),
             (6, bvec, LU.VectorSimilarityFunction.DOT_PRODUCT, bdocs, LU.VectorEncoding.BYTE)]
    for number, rows, sim, o2d, enc in cases:
        rf = LU.GpuFlatVectorsReader.from_files("f", str(tmp_path), "_a", SID, max_doc, number, "Lucene99_0")
        rm = LU.GpuFlatVectorsReader("f", rows, sim, enc, ord_to_doc=o2d, max_doc=max_doc)
        try:
            assert (rf.dim, rf.size, rf.similarity, rf.encoding) == (rows.shape[1], len(rows), sim, enc)
            q = (O.synth(0, 3, rows.shape[1], 403, 4) if enc == LU.VectorEncoding.BYTE
                 else O.synth(0, 3, rows.shape[1], 403, 3))
            acc = O.bits_from_bool(rng.random(max_doc) < 0.3)
            for k in (10, 100):
                same(rf.search_batch(q, k), rm.search_batch(q, k))
                same(rf.search_batch(q, k, acc), rm.search_batch(q, k, acc))
            s, d, c, _ = rf.search_batch(q[:1], 10, acc)
            _, od, _ = O.exact_search(rows, q[0], 10, int(sim), ord_to_doc=o2d, accept_bits=acc)
            assert np.array_equal(d[0, : c[0]], od)
        finally:
            rf.close()
            rm.close()


def test_stage_file_errors_are_codes(tmp_path):
    import ctypes as C
    from opensearch_amd import _lib
    FF.write_segment(str(tmp_path), "_b", SID, 100, [(0, np.ones((100, 8), np.float32), 1, None)])
    e = FF.read_meta(str(tmp_path / "_b.vemf"), SID)[0]
    h = C.c_void_p()
    rc = _lib.lib().osk_seg_stage_file(0, str(tmp_path / "missing.vec").encode(), e.data_offset, 100, 8, 0, 1, None,
                                       100, C.byref(h))
    assert rc == _lib.OSK_ERR_INVALID and b"cannot open" in _lib.lib().osk_last_error()
    rc = _lib.lib().osk_seg_stage_file(0, str(tmp_path / "_b.vec").encode(), e.data_offset, 1000, 8, 0, 1, None,
                                       1000, C.byref(h))
    assert rc == _lib.OSK_ERR_INVALID and b"shorter" in _lib.lib().osk_last_error()


def test_nrt_refresh_churn_with_merges(tmp_path):
    """Four refreshes: each flushes a new segment and, from the third on, merges the two oldest into
    one.  The previous refresh's view keeps answering (its segments closed by their readers) until
    released; every view's answer equals the oracle over its own point-in-time segment set."""
    rng = np.random.default_rng(7)
    dim = 128
    q = O.synth(0, 2, dim, 500, 3)
    live = []        # (name, rows, reader) of the current point-in-time
    views = []       # (view, [rows of its segments]) not yet released
    gen = 0

    def flush(rows):
        nonlocal gen
        name = f"_{gen}"
        gen += 1
        FF.write_segment(str(tmp_path), name, SID, len(rows), [(0, rows, int(COS), None)])
        return name, rows, LU.GpuFlatVectorsReader.from_files("v", str(tmp_path), name, SID, len(rows), 0)

    def check(view, segs):
        out = view.search(q, 10, 0, 10)
        for i in range(len(q)):
            lists, base = [], 0
            for rows in segs:
                sc, dc, _ = O.exact_search(rows, q[i], 10, int(COS))
                lists.append((sc, dc + base))
                base += len(rows)
            es, ed, _, _, _ = O.topdocs_merge(lists, 0, 10)
            assert np.array_equal(out[1][i, : out[3][i]], ed)
            assert np.array_equal(out[0][i, : out[3][i]].view(np.uint32), es.view(np.uint32))

    for step in range(4):
        live.append(flush(O.synth(0, int(rng.integers(3000, 9000)), dim, 600 + step, 3)))
        if len(live) >= 3:   # merge the two oldest segments into a new one; their readers close
            (n0, r0, h0), (n1, r1, h1) = live[0], live[1]
            merged = flush(np.concatenate([r0, r1]))
            h0.close()
            h1.close()
            live = [merged] + live[2:]
        leaves, base = [], 0
        for _, rows, rd in live:
            leaves.append(LU.LeafReaderContext(len(leaves), base, rd))
            base += len(rows)
        v = LU.DeviceShardSet([leaves], [0])
        views.append((v, [rows for _, rows, _ in live]))
        for view, segs in views:   # the old searchers still answer over their own segments
            check(view, segs)
        if len(views) > 2:          # the oldest searcher is released (its refcounts drop)
            old, _ = views.pop(0)
            old.close()
    for v, _ in views:
        v.close()
    for _, _, rd in live:
        rd.close()
