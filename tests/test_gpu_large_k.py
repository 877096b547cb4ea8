"""GPU parity of the select path: exact top-k for k beyond the wave lists, up to OSK_MAX_K = 10000
(index.max_result_window, S/index/IndexSettings.java:223-226).

osk_select.hip materialises one record per row — the int8 prefilter's certified [lb, ub] score
bounds (float32 fields, prefilter on) or the exact 64-bit hit key (prefilter off, byte vectors, and
any bounds-mode query whose candidates overflow) — radix-selects the k-th largest per shard, collects
every row that can reach the top k, re-scores them exactly and sorts.  The coordinator merges lists of
any length by ranking every hit with binary searches (merge_rank).  Everything is compared against the
oracle's [L] exactSearch (HitQueue: strict >, ties → lower doc) in the device summation order (docs
AND score bits) and its TopDocs.merge (score desc, shardIndex asc, doc asc).
"""
import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIMS = [LU.VectorSimilarityFunction(s) for s in range(4)]
COS = LU.VectorSimilarityFunction.COSINE


def corpus(n, dim, sim, seed, byte=False):
    if byte:
        return O.synth(0, n, dim, seed, 4)
    return O.synth(0, n, dim, seed, {0: 1, 1: 3, 2: 3, 3: 2}[int(sim)])


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def with_sq8(on, fn):
    _lib.tune("sq8", 1 if on else 0)
    try:
        return fn()
    finally:
        _lib.tune("sq8", 1)


def check_reader(r, rows, queries, k, sim, accept=None, ord_to_doc=None):
    s, d, c, v = r.search_batch(queries, k, accept)
    for i in range(len(queries)):
        os_, od, ov = O.exact_search(rows, queries[i], k, int(sim), ord_to_doc=ord_to_doc, accept_bits=accept)
        assert c[i] == len(od), (c[i], len(od))
        assert np.array_equal(d[i, : c[i]], od), (i, np.nonzero(d[i, : c[i]] != od)[0][:5])
        assert np.array_equal(bits(s[i, : c[i]]), bits(os_))
        assert v[i] == ov
        assert np.all(np.isneginf(s[i, c[i]:])) and np.all(d[i, c[i]:] == 2**31 - 1)
    return s, d, c, v


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
@pytest.mark.parametrize("k", [13, 50, 64, 100, 700])
@pytest.mark.parametrize("sq8", [1, 0], ids=["bounds", "exact"])
def test_select_f32_equals_oracle(sim, k, sq8):
    rows = corpus(30000, 192, sim, 300 + k)
    queries = corpus(2, 192, sim, 301)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        with_sq8(sq8, lambda: check_reader(r, rows, queries, k, sim))
    finally:
        r.close()


@pytest.mark.parametrize("k", [50, 100])
@pytest.mark.parametrize("dim", [3, 100, 768])
def test_select_k50_k100_dims(k, dim):
    """The verdict's bar: parity at k = 50 / 100 (the prefilter serves k ≤ 12; 13 … 10000 is the select path)."""
    rows = corpus(20000, dim, COS, 310 + dim)
    queries = corpus(3, dim, COS, 311)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    try:
        check_reader(r, rows, queries, k, COS)
    finally:
        r.close()


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
@pytest.mark.parametrize("k", [65, 100, 1000])
def test_select_byte_vectors(sim, k):
    rows = corpus(25000, 96, sim, 320, byte=True)
    queries = corpus(2, 96, sim, 321, byte=True)
    r = LU.GpuFlatVectorsReader("v", rows, sim, LU.VectorEncoding.BYTE)
    try:
        check_reader(r, rows, queries, k, sim)
    finally:
        r.close()


def test_select_k_beyond_rows_and_max_k():
    rows = corpus(3000, 64, COS, 330)
    queries = corpus(2, 64, COS, 331)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    try:
        for k in (2999, 3000, 3001, _lib.OSK_MAX_K):
            for sq8 in (1, 0):
                with_sq8(sq8, lambda: check_reader(r, rows, queries, k, COS))
        with pytest.raises(_lib.OskError):
            r.search_batch(queries, _lib.OSK_MAX_K + 1)
    finally:
        r.close()


@pytest.mark.parametrize("selectivity", [0.001, 0.05, 0.5])
def test_select_filters_and_sparse_docs(selectivity):
    rng = np.random.default_rng(int(selectivity * 1000))
    n, max_doc = 30000, 70000
    rows = corpus(n, 256, COS, 340)
    queries = corpus(2, 256, COS, 341)
    docs = np.sort(rng.choice(max_doc, n, replace=False)).astype(np.int32)
    dense = LU.GpuFlatVectorsReader("v", rows, COS)
    sparse = LU.GpuFlatVectorsReader("v", rows, COS, ord_to_doc=docs, max_doc=max_doc)
    try:
        acc = O.bits_from_bool(rng.random(n) < selectivity)
        live = O.bits_from_bool(rng.random(max_doc) < max(selectivity, 0.05))
        for sq8 in (1, 0):
            with_sq8(sq8, lambda: check_reader(dense, rows, queries, 100, COS, accept=acc))
            with_sq8(sq8, lambda: check_reader(sparse, rows, queries, 100, COS, accept=live, ord_to_doc=docs))
    finally:
        dense.close()
        sparse.close()


def test_select_ties_lower_doc_wins():
    """Every vector repeated 5×: exact ties at the k-th score broken by the lower doc, both modes."""
    base = corpus(600, 48, COS, 350)
    rows = np.concatenate([base] * 5)
    queries = np.concatenate([base[:2], corpus(1, 48, COS, 351)])
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    try:
        for k in (97, 100, 1501):
            for sq8 in (1, 0):
                with_sq8(sq8, lambda: check_reader(r, rows, queries, k, COS))
        const = np.ones((5000, 16), np.float32)
        rc = LU.GpuFlatVectorsReader("v", const, LU.VectorSimilarityFunction.EUCLIDEAN)
        try:
            for sq8 in (1, 0):
                s, d, c, _ = with_sq8(sq8, lambda: rc.search_batch(np.ones((1, 16), np.float32), 300))
                assert c[0] == 300 and np.array_equal(d[0], np.arange(300))
        finally:
            rc.close()
    finally:
        r.close()


def test_select_many_candidates_beyond_lds():
    """Rows so alike that the int8 bounds cannot tell them apart: every row of the shard is a candidate
    (40000 > the 16384 keys an LDS sort holds), so the top k is radix-selected in global memory — the
    result must equal the exact mode's."""
    rng = np.random.default_rng(360)
    rows = (np.ones((40000, 32), np.float32) + rng.standard_normal((40000, 32)).astype(np.float32) * 1e-4)
    queries = np.ones((2, 32), np.float32)
    r = LU.GpuFlatVectorsReader("v", rows, LU.VectorSimilarityFunction.DOT_PRODUCT)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    try:
        for k in (100, 5000):
            got = ds.search(queries, k, 0, k)
            want = with_sq8(0, lambda: ds.search(queries, k, 0, k))
            for a, b in zip(got, want):
                assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
            check_reader(r, rows, queries, k, LU.VectorSimilarityFunction.DOT_PRODUCT)
    finally:
        ds.close()
        r.close()


@pytest.mark.parametrize("k,from_,size", [(100, 0, 100), (1000, 100, 900), (2000, 0, 2000), (30, 5, 20)])
def test_select_multi_shard_large_merge(k, from_, size):
    """5 shards × min(k, from+size) > 4096 hits: the coordinator reduce ranks by binary search (merge_rank)."""
    sim = LU.VectorSimilarityFunction.DOT_PRODUCT
    sizes = [9000, 3000, 7000, 1, 6000, 5000]
    segs = [corpus(n, 128, sim, 370 + i) for i, n in enumerate(sizes)]
    shard_of = [0, 0, 1, 2, 3, 4]
    si = [3, 0, 4, 1, 2]
    leaves = [[] for _ in range(5)]
    readers, bases = [], [0] * 5
    for rows, s in zip(segs, shard_of):
        rd = LU.GpuFlatVectorsReader("v", rows, sim)
        readers.append(rd)
        leaves[s].append(LU.LeafReaderContext(len(leaves[s]), bases[s], rd))
        bases[s] += len(rows)
    ds = LU.DeviceShardSet(leaves, si)
    queries = corpus(2, 128, sim, 380)
    try:
        for sq8 in (1, 0):
            out = with_sq8(sq8, lambda: ds.search(queries, k, from_, size))
            s_, d_, sh_, c_, t_, m_ = out
            for i in range(len(queries)):
                per_shard = [[] for _ in range(5)]
                for li, (rows, s) in enumerate(zip(segs, shard_of)):
                    sc, dc, _ = O.exact_search(rows, queries[i], k, int(sim))
                    base = sum(len(segs[j]) for j in range(li) if shard_of[j] == s)
                    per_shard[s].append((sc, dc + base))
                lists = []
                for ps in per_shard:
                    ms, md, _, _, _ = O.topdocs_merge(ps, 0, k)
                    lists.append((ms[: from_ + size], md[: from_ + size]))
                es, ed, esh, et, em = O.topdocs_merge(lists, from_, size, si)
                assert c_[i] == len(ed)
                assert np.array_equal(d_[i, : c_[i]], ed) and np.array_equal(sh_[i, : c_[i]], esh)
                assert np.array_equal(bits(s_[i, : c_[i]]), bits(es))
                assert t_[i] == sum(min(k, sum(len(segs[j]) for j in range(6) if shard_of[j] == s)) for s in range(5))
    finally:
        ds.close()
        for r in readers:
            r.close()


@pytest.mark.parametrize("writer", [0, 1, 2, 3])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_select_bounds_writer_variants(writer, sim):
    """Every bounds writer (row groups in flight, Java or fp32 COSINE bound transform) gives the exact
    answer.  (Zero vectors cannot reach a COSINE field: Lucene rejects them at index and query time.)"""
    rows = corpus(20000, 192, sim, 390)
    queries = corpus(2, 192, sim, 391)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    _lib.tune("sel_writer", writer)
    try:
        check_reader(r, rows, queries, 100, sim)
    finally:
        _lib.tune("sel_writer", 2)
        r.close()
