"""GPU parity of the batched MFMA path (batch ≥ 16, k ≤ 12): bf16×3 candidates + exact re-score +
certificate.  It must return exactly what the streaming scan returns (same docs, same score bits) —
which the oracle's ORDER_DEVICE restatement pins — including when certificates fail and the exact
fallback runs."""
import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIMS = [LU.VectorSimilarityFunction(s) for s in range(4)]


def corpus(n, dim, sim, seed):
    dist = {0: 1, 1: 3, 2: 3, 3: 2}[int(sim)]
    return O.synth(0, n, dim, seed, dist)


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(autouse=True)
def bf16x3_from_16():
    """Batches ≥ 16 take the bf16×3 path in this module (the library default: from batch 96 when its
    256-query blocks are cheaper than the int8 prefilter, tune sq8_cost_pct)."""
    _lib.tune("mfma_min_batch", 16)
    _lib.tune("sq8_cost_pct", 100000)
    yield
    _lib.tune("mfma_min_batch", 96)
    _lib.tune("sq8_cost_pct", 100)


def streaming(ds_or_reader, fn):
    _lib.tune("mfma_min_batch", 0)
    try:
        return fn()
    finally:
        _lib.tune("mfma_min_batch", 16)


@pytest.mark.parametrize("dim", [16, 96, 128, 768, 1000])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_batched_equals_streaming_and_oracle(dim, sim):
    n = 5000 + dim
    rows = corpus(n, dim, sim, 7)
    queries = corpus(40, dim, sim, 8)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        s, d, c, v = r.search_batch(queries, 10)
        s2, d2, c2, v2 = streaming(r, lambda: r.search_batch(queries, 10))
        assert np.array_equal(d, d2) and np.array_equal(bits(s), bits(s2)) and np.array_equal(c, c2)
        assert np.array_equal(v, v2)
        for i in [0, 17, 39]:
            os_, od, _ = O.exact_search(rows, queries[i], 10, int(sim))
            assert np.array_equal(d[i], od) and np.array_equal(bits(s[i]), bits(os_))
    finally:
        r.close()


@pytest.mark.parametrize("nq", [16, 255, 256, 257, 600])
def test_batched_query_counts(nq):
    sim = LU.VectorSimilarityFunction.COSINE
    rows = corpus(20000, 128, sim, 11)
    queries = corpus(nq, 128, sim, 12)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        for k in [1, 10, 12]:
            s, d, c, _ = r.search_batch(queries, k)
            s2, d2, c2, _ = streaming(r, lambda: r.search_batch(queries, k))
            assert np.array_equal(d, d2) and np.array_equal(bits(s), bits(s2))
    finally:
        r.close()


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_certificate_holds_on_random_data(sim):
    """On non-degenerate data the bf16×3 candidates + certificate must settle every query without
    the exact fallback (otherwise the batched path is correct but pointless)."""
    dim = 128
    rows = corpus(30000, dim, sim, 21)
    queries = corpus(64, dim, sim, 22)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]])
    try:
        out = ds.search(queries, 10, 0, 10)
        calls, fb = ds.stats()
        assert calls == 1 and fb == 0, (calls, fb)
        for i in [0, 63]:
            os_, od, _ = O.exact_search(rows, queries[i], 10, int(sim))
            assert np.array_equal(out[1][i], od) and np.array_equal(bits(out[0][i]), bits(os_))
    finally:
        ds.close()
        r.close()


def test_batched_certificate_fallback_on_ties():
    """Every row identical → all scores tie → the certificate cannot hold → exact fallback."""
    sim = LU.VectorSimilarityFunction.DOT_PRODUCT
    base = corpus(1, 64, sim, 3)
    rows = np.repeat(base, 3000, axis=0)
    rows[1234] = corpus(1, 64, sim, 4)[0]
    queries = corpus(20, 64, sim, 5)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]])
    try:
        sc, dc, sh, cnt, tot, mx = ds.search(queries, 10, 0, 10)
        calls, fb = ds.stats()
        assert calls >= 1 and fb >= 1
        for i in range(len(queries)):
            os_, od, _ = O.exact_search(rows, queries[i], 10, int(sim))
            assert np.array_equal(dc[i], od) and np.array_equal(bits(sc[i]), bits(os_))
    finally:
        ds.close()
        r.close()


def test_batched_multi_shard_filters_sparse():
    sim = LU.VectorSimilarityFunction.EUCLIDEAN
    dim = 100
    rng = np.random.default_rng(9)
    specs = [[3000, 129], [4097], [1, 2000, 700]]
    shard_leaves, rows_of = [], {}
    seed = 40
    for segs in specs:
        leaves, base = [], 0
        for i, n in enumerate(segs):
            rows = corpus(n, dim, sim, seed)
            seed += 1
            o2d = np.sort(rng.choice(3 * n, n, replace=False)).astype(np.int32)
            reader = LU.GpuFlatVectorsReader("v", rows, sim, ord_to_doc=o2d, max_doc=3 * n)
            live = rng.random(3 * n) < 0.6
            leaves.append(LU.LeafReaderContext(i, base, reader, live))
            rows_of[id(leaves[-1])] = (rows, o2d)
            base += 3 * n
        shard_leaves.append(leaves)
    ds = LU.DeviceShardSet(shard_leaves, [1, 2, 0])
    queries = corpus(64, dim, sim, 99)
    acc = [lf.live_docs for lf in ds.leaves]
    try:
        out_b = ds.search(queries, 10, 2, 12, accept=acc)
        out_s = streaming(ds, lambda: ds.search(queries, 10, 2, 12, accept=acc))
        for a, b in zip(out_b, out_s):
            assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
        assert ds.stats()[0] >= 1
        # spot-check one query end to end against the oracle
        qi = 5
        shard_hits = []
        for leaves in shard_leaves:
            per_leaf = []
            for lf in leaves:
                rows, o2d = rows_of[id(lf)]
                os_, od, _ = O.exact_search(rows, queries[qi], 10, int(sim), ord_to_doc=o2d,
                                            accept_bits=O.bits_from_bool(lf.live_docs))
                per_leaf.append((os_, od + lf.doc_base))
            ms, md, _, _, _ = O.topdocs_merge(per_leaf, 0, 10, [0] * len(per_leaf))
            shard_hits.append((ms, md))
        es, ed, esh, etot, _ = O.topdocs_merge(shard_hits, 2, 12, [1, 2, 0])
        n = len(ed)
        assert np.array_equal(out_b[1][qi, :n], ed) and np.array_equal(out_b[2][qi, :n], esh)
        assert out_b[4][qi] == etot
    finally:
        ds.close()
        for leaves in shard_leaves:
            for lf in leaves:
                lf.reader.close()


@pytest.mark.parametrize("offset", [0.0, 1000.0, -3.0e4])
def test_batched_euclidean_threshold_bound_magnitudes(offset):
    """EUCLIDEAN's candidate pass filters accumulators with a dot-product bound derived from the
    running threshold (2d ≥ |x|² + |q|² − (1/t − 1), loosened).  Large |x|² (offset rows), scores near
    1 (queries that are perturbed rows) and far-away queries must all keep every true candidate: the
    batched answers equal the streaming scan's and the oracle's, and the certificate holds."""
    sim = LU.VectorSimilarityFunction.EUCLIDEAN
    dim = 128
    rows = corpus(40000, dim, sim, 31) + np.float32(offset)
    rng = np.random.default_rng(5)
    near = rows[rng.choice(len(rows), 24, replace=False)] + rng.normal(0, 0.05, (24, dim)).astype(np.float32)
    far = corpus(24, dim, sim, 32) + np.float32(offset)
    queries = np.ascontiguousarray(np.concatenate([near, far]), np.float32)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        s, d, c, v = r.search_batch(queries, 10)
        s2, d2, c2, v2 = streaming(r, lambda: r.search_batch(queries, 10))
        assert np.array_equal(d, d2) and np.array_equal(bits(s), bits(s2))
        for i in [0, 11, 23, 24, 47]:
            os_, od, _ = O.exact_search(rows, queries[i], 10, int(sim))
            assert np.array_equal(d[i], od) and np.array_equal(bits(s[i]), bits(os_))
    finally:
        r.close()
