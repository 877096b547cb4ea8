"""GPU parity of the certified int8 prefilter (osk_sq8.hip).

The prefilter is the default path for float32 searches below the MFMA batch threshold with k ≤ 12.
It must return exactly what the fp32 streaming scan returns — the same docs, the same score bits,
the same tie order — which the oracle's ORDER_DEVICE restatement pins.  These tests compare the
two paths (tune "sq8" 1 vs 0) and the oracle over similarities, ragged dims, batch sizes, k,
filters, sparse doc maps, multi-segment multi-shard views, heavy ties and adversarial data where
the certificate cannot exclude a whole tile and the settle re-scans that tile exactly instead.
Every test runs five times: batches scanned by the wide int8 MFMA kernel (sq8_wide, 256 queries per launch),
by the int8 MFMA kernel (sq8_mfma, tune "sq8_mfma_min"
2, the default) with 32 and with 16 queries per launch (rows ≤ 256 dims streamed by the LDS-DMA ring,
the default), with 32 queries and register row loads ("sq8_mfma_ring" 0), and by the VALU kernel
(sq8_scan, "sq8_mfma_min" 0), the last also with its single-query launches at 8 row groups in flight per wave
("sq8_scan_deep" 1).
"""
import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIMS = [LU.VectorSimilarityFunction(s) for s in range(4)]
COS = LU.VectorSimilarityFunction.COSINE


SCAN_DEEP_DEFAULT = 0


@pytest.fixture(autouse=True, params=["mfma32", "mfma16", "mfma32reg", "valu", "valudeep", "wide"])
def scan_kernel(request):
    """The int8 scan kernel of batched prefilter searches (single queries always take sq8_scan):
    sq8_mfma with 32 or 16 queries per launch (LDS-DMA ring), with register row loads, sq8_scan, or the
    wide kernel (osk_sq8w.hip, 256 queries per launch; unfiltered batches of rows ≤ 256 dims, the others
    fall back to sq8_mfma)."""
    _lib.tune("sq8_mfma_min", 0 if request.param in ("valu", "valudeep") else 2)
    _lib.tune("sq8_scan_deep", 1 if request.param == "valudeep" else 0)
    _lib.tune("sq8_mfma_queries", 16 if request.param == "mfma16" else 32)
    _lib.tune("sq8_mfma_ring", 0 if request.param == "mfma32reg" else -1)
    _lib.tune("sq8_wide_min", 2 if request.param == "wide" else 0)
    _lib.tune("sq8_wide_force", 1 if request.param == "wide" else 0)
    yield request.param
    _lib.tune("sq8_scan_deep", SCAN_DEEP_DEFAULT)
    _lib.tune("sq8_mfma_min", 2)
    _lib.tune("sq8_mfma_queries", 32)
    _lib.tune("sq8_mfma_ring", -1)
    _lib.tune("sq8_wide_min", 64)
    _lib.tune("sq8_wide_force", 0)


def corpus(n, dim, sim, seed):
    dist = {0: 1, 1: 3, 2: 3, 3: 2}[int(sim)]
    return O.synth(0, n, dim, seed, dist)


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def with_tune(key, value, fn):
    _lib.tune(key, value)
    try:
        return fn()
    finally:
        _lib.tune(key, {"sq8": 1, "sq8_force_fallback": 0}[key])


def view_of(rows_list, sim, shard_of=None, shard_index=None):
    """One DeviceShardSet over the given segments (segment i → shard shard_of[i])."""
    shard_of = shard_of or [0] * len(rows_list)
    n_shards = max(shard_of) + 1
    shard_leaves = [[] for _ in range(n_shards)]
    readers = []
    bases = [0] * n_shards
    for rows, s in zip(rows_list, shard_of):
        r = LU.GpuFlatVectorsReader("v", rows, sim)
        readers.append(r)
        shard_leaves[s].append(LU.LeafReaderContext(len(shard_leaves[s]), bases[s], r))
        bases[s] += len(rows)
    return LU.DeviceShardSet(shard_leaves, shard_index), readers


def close_all(ds, readers):
    ds.close()
    for r in readers:
        r.close()


def assert_same(a, b):
    for x, y in zip(a, b):
        x, y = np.asarray(x), np.asarray(y)
        if x.dtype == np.float32:
            assert np.array_equal(bits(x), bits(y)), (x, y)
        else:
            assert np.array_equal(x, y), (x, y)


@pytest.mark.parametrize("dim", [1, 3, 17, 64, 96, 100, 128, 384, 768, 1000, 2048, 4096])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_prefilter_equals_exact_scan_and_oracle(dim, sim):
    n = 3000 + dim % 11
    rows = corpus(n, dim, sim, 3)
    queries = corpus(5, dim, sim, 4)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        on = r.search_batch(queries, 10)
        off = with_tune("sq8", 0, lambda: r.search_batch(queries, 10))
        assert_same(on, off)
        s, d, c, v = on
        for i in range(len(queries)):
            os_, od, ov = O.exact_search(rows, queries[i], 10, int(sim))
            assert np.array_equal(d[i, : c[i]], od) and np.array_equal(bits(s[i, : c[i]]), bits(os_))
            assert v[i] == ov == n
    finally:
        r.close()


@pytest.mark.parametrize("nq", [1, 2, 3, 5, 8, 9, 15, 17, 32, 40])
@pytest.mark.parametrize("k", [1, 7, 10, 12, 16])
def test_prefilter_batches_and_k(nq, k):
    sim = COS
    rows = corpus(20000, 768, sim, 5)
    queries = corpus(nq, 768, sim, 6)
    ds, readers = view_of([rows[:9000], rows[9000:15000], rows[15000:]], sim, [0, 1, 1])
    try:
        on = ds.search(queries, k, 0, k)
        off = with_tune("sq8", 0, lambda: ds.search(queries, k, 0, k))
        assert_same(on, off)
        # the prefilter serves k ≤ 12 (its tile lists hold 16 rows); k = 16 takes the fp32 scan
        assert (ds.counter("sq8_calls") >= 1) == (k <= 12)
        # a tile whose 16-entry list overflowed past the certificate is re-scanned exactly inside the
        # settle (correct either way); here (20 tiles of ~1000 rows) a minority of tiles per query
        assert ds.counter("sq8_exact_tiles") <= 5 * nq
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_prefilter_certifies_without_fallback_on_random_data(sim):
    """On well-spread data every query is certified and only a few rows per shard are re-scored."""
    rows = corpus(60000, 256, sim, 7)
    queries = corpus(8, 256, sim, 8)
    ds, readers = view_of([rows[i * 15000:(i + 1) * 15000] for i in range(4)], sim, [0, 1, 2, 3])
    try:
        ds.search(queries, 10, 0, 10)
        assert ds.counter("sq8_fallback_queries") == 0
        rescored = ds.counter("sq8_rescored_rows")
        assert 8 * 4 * 10 <= rescored <= 8 * 4 * 2000, rescored
    finally:
        close_all(ds, readers)


def test_forced_exact_tiles_is_exact():
    """Every list re-scanned exactly inside the settle (the testing build's sq8_force_fallback knob)."""
    sim = LU.VectorSimilarityFunction.EUCLIDEAN
    rows = corpus(12000, 128, sim, 9)
    queries = corpus(11, 128, sim, 10)
    with _lib.testing():
        ds, readers = view_of([rows[:5000], rows[5000:]], sim, [0, 1], [1, 0])
        try:
            off = with_tune("sq8", 0, lambda: ds.search(queries, 10, 0, 10))
            forced = with_tune("sq8_force_fallback", 1, lambda: ds.search(queries, 10, 0, 10))
            assert_same(forced, off)
            assert ds.counter("sq8_fallback_queries") == len(queries)
            on = ds.search(queries, 10, 0, 10)
            assert_same(on, off)
            assert ds.counter("sq8_fallback_queries") == len(queries)
        finally:
            close_all(ds, readers)


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_prefilter_heavy_ties(sim):
    """Every vector 3×, queries equal to rows: exact ties broken by lower doc, certified or not."""
    base = corpus(700, 96, sim, 11)
    rows = np.concatenate([base, base[::-1], base])
    queries = np.concatenate([base[:3], corpus(3, 96, sim, 12)])
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        on = r.search_batch(queries, 12)
        off = with_tune("sq8", 0, lambda: r.search_batch(queries, 12))
        assert_same(on, off)
        for i in range(len(queries)):
            os_, od, _ = O.exact_search(rows, queries[i], 12, int(sim))
            assert np.array_equal(on[1][i], od)
    finally:
        r.close()


def test_prefilter_constant_and_zero_rows():
    for sim in [LU.VectorSimilarityFunction.EUCLIDEAN, LU.VectorSimilarityFunction.DOT_PRODUCT,
                LU.VectorSimilarityFunction.MAXIMUM_INNER_PRODUCT]:
        rows = np.ones((900, 40), np.float32)
        rows[100:200] = 0.0
        q = np.stack([np.ones(40, np.float32), np.zeros(40, np.float32)])
        r = LU.GpuFlatVectorsReader("v", rows, sim)
        try:
            assert_same(r.search_batch(q, 10), with_tune("sq8", 0, lambda: r.search_batch(q, 10)))
        finally:
            r.close()


def test_prefilter_adversarial_dynamic_range():
    """One huge component per row makes the int8 copy nearly useless: the bound is wide, many rows
    qualify, and the result must still be exact (certified with many candidates, or the fallback)."""
    rng = np.random.default_rng(13)
    rows = rng.standard_normal((5000, 64)).astype(np.float32) * 1e-3
    rows[:, 0] = 1000.0
    queries = rng.standard_normal((4, 64)).astype(np.float32)
    for sim in SIMS:
        r = LU.GpuFlatVectorsReader("v", rows, sim)
        try:
            assert_same(r.search_batch(queries, 10), with_tune("sq8", 0, lambda: r.search_batch(queries, 10)))
        finally:
            r.close()


@pytest.mark.parametrize("selectivity", [0.0, 0.002, 0.01, 0.1, 0.5, 1.0])
def test_prefilter_with_filters_and_sparse_docs(selectivity):
    sim = COS
    rng = np.random.default_rng(int(selectivity * 1000) + 1)
    n = 8000
    rows = corpus(n, 768, sim, 14)
    queries = corpus(3, 768, sim, 15)
    dense = LU.GpuFlatVectorsReader("v", rows, sim)
    docs = np.sort(rng.choice(20000, n, replace=False)).astype(np.int32)
    sparse = LU.GpuFlatVectorsReader("v", rows, sim, ord_to_doc=docs, max_doc=20000)
    try:
        acc = O.bits_from_bool(rng.random(n) < selectivity)
        on = dense.search_batch(queries, 10, acc)
        assert_same(on, with_tune("sq8", 0, lambda: dense.search_batch(queries, 10, acc)))
        live = O.bits_from_bool(rng.random(20000) < max(selectivity, 0.05))
        on = sparse.search_batch(queries, 10, live)
        assert_same(on, with_tune("sq8", 0, lambda: sparse.search_batch(queries, 10, live)))
        for i in range(len(queries)):
            os_, od, ov = O.exact_search(rows, queries[i], 10, int(sim), ord_to_doc=docs, accept_bits=live)
            assert np.array_equal(on[1][i, : on[2][i]], od) and on[3][i] == ov
    finally:
        dense.close()
        sparse.close()


def test_prefilter_multi_shard_from_size():
    sim = LU.VectorSimilarityFunction.DOT_PRODUCT
    segs = [corpus(n, 128, sim, 20 + i) for i, n in enumerate([3000, 1, 2500, 64, 4000])]
    ds, readers = view_of(segs, sim, [0, 0, 1, 2, 2], [2, 0, 1])
    queries = corpus(6, 128, sim, 30)
    try:
        for k, f, sz in [(10, 0, 10), (10, 5, 5), (16, 3, 13), (4, 0, 4)]:
            assert_same(ds.search(queries, k, f, sz), with_tune("sq8", 0, lambda: ds.search(queries, k, f, sz)))
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("scan_kernel", ["mfma32"], indirect=True)   # (one scan-kernel variant only)
@pytest.mark.parametrize("slots", [2, 4])
@pytest.mark.parametrize("dim,sim", [(17, COS), (96, LU.VectorSimilarityFunction.DOT_PRODUCT),
                                     (128, LU.VectorSimilarityFunction.EUCLIDEAN),
                                     (256, LU.VectorSimilarityFunction.MAXIMUM_INNER_PRODUCT)])
def test_mfma_ring_depths(slots, dim, sim, scan_kernel):
    """The LDS-DMA ring at every depth: ragged segment sizes (partial 16-row groups at wave ends),
    several segments and shards, a sparse field without a filter; equal to the fp32 scan and the oracle."""
    sizes = [5000, 1237, 16, 3, 777]
    segs = [corpus(n, dim, sim, 700 + i) for i, n in enumerate(sizes)]
    queries = corpus(33, dim, sim, 710)
    ds, readers = view_of(segs, sim, shard_of=[0, 0, 1, 2, 2])
    rng = np.random.default_rng(5)
    docs = np.sort(rng.choice(9000, 4000, replace=False)).astype(np.int32)
    sp_rows = corpus(4000, dim, sim, 720)
    sparse = LU.GpuFlatVectorsReader("v", sp_rows, sim, ord_to_doc=docs, max_doc=9000)
    _lib.tune("sq8_mfma_ring", slots)
    try:
        got = ds.search(queries, 10, 0, 10)
        want = with_tune("sq8", 0, lambda: ds.search(queries, 10, 0, 10))
        assert_same(got, want)
        s, d, c, _ = sparse.search_batch(queries, 10)
        for i in range(0, len(queries), 8):
            os_, od, _ = O.exact_search(sp_rows, queries[i], 10, int(sim), ord_to_doc=docs)
            assert np.array_equal(d[i, : c[i]], od) and np.array_equal(bits(s[i, : c[i]]), bits(os_))
    finally:
        _lib.tune("sq8_mfma_ring", -1)
        ds.close()
        for r in readers:
            r.close()
        sparse.close()
