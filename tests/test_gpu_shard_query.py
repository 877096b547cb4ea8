"""The plugin's query routes Lucene-shaped k-NN searches onto the device design.

`GpuKnnFloatVectorQuery.rewrite` (the Python mirror of INTEGRATION.md §3's Java query) makes ONE
osk_view_search per shard over a view of every leaf — instead of one KnnVectorsReader.search per leaf
([L] AbstractKnnVectorQuery.rewrite, per-leaf tasks under concurrent segment search,
S/search/DefaultSearchContext.java:257-267) — and sends every filtered leaf to the device, including
the leaves whose accepted docs number ≤ k, which Lucene's own query would score on the CPU
(exactSearch).  On a 20-segment shard with deletions and a filter that leaves some leaves with ≤ k or
zero accepted docs, the one-call route, the per-leaf route and the oracle (per-leaf exactSearch +
TopDocs.merge(k, perLeaf), S/search/internal/ContextIndexSearcher.java:203-218) agree on docs and
score bits.
"""
import numpy as np
import pytest

from opensearch_amd import lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

COS = LU.VectorSimilarityFunction.COSINE
DIM, K = 96, 10


@pytest.fixture(scope="module")
def shard():
    rng = np.random.default_rng(11)
    sizes = [int(x) for x in rng.integers(200, 3000, size=20)]
    rows = [O.synth(0, n, DIM, 900 + i, 3) for i, n in enumerate(sizes)]
    readers = [LU.GpuFlatVectorsReader("v", r, COS) for r in rows]
    base, leaves = 0, []
    for i, (r, n) in enumerate(zip(readers, sizes)):
        live = None if i % 3 else rng.random(n) > 0.1          # deletions on every third leaf
        leaves.append(LU.LeafReaderContext(i, base, r, live))
        base += n
    # a filter that leaves leaf 4 with 3 accepted docs (≤ k: Lucene's CPU exactSearch branch), leaf 7
    # with none, leaf 9 with exactly k, and the others a 30 % sample
    masks = {}
    for lf, n in zip(leaves, sizes):
        m = rng.random(n) < 0.3
        if lf.ord in (4, 9):
            m[:] = False
            m[rng.choice(n, 3 if lf.ord == 4 else K, replace=False)] = True
        if lf.ord == 7:
            m[:] = False
        masks[lf.ord] = m
    yield leaves, rows, masks
    LU.GpuKnnFloatVectorQuery.release_views()
    for r in readers:
        r.close()


def oracle(leaves, rows, q, accept_of):
    lists = []
    for lf, r in zip(leaves, rows):
        acc = accept_of(lf)
        ab = None if acc is None else O.bits_from_bool(acc)
        sc, dc, _ = O.exact_search(r, q, K, int(COS), accept_bits=ab)
        lists.append((sc, dc + lf.doc_base))
    es, ed, _, _, _ = O.topdocs_merge(lists, 0, K, list(range(len(lists))))
    return es, ed


def hits(td):
    return (np.array([h.score for h in td.score_docs], np.float32).view(np.uint32),
            np.array([h.doc for h in td.score_docs], np.int32))


@pytest.mark.parametrize("filtered", [False, True])
def test_one_call_per_shard_equals_per_leaf_and_oracle(shard, filtered):
    leaves, rows, masks = shard
    filt = (lambda lf: masks[lf.ord]) if filtered else None
    for qi in range(4):
        q = O.synth(0, 1, DIM, 950 + qi, 3)[0]
        gq = LU.GpuKnnFloatVectorQuery("v", q, K, filt)
        e = gq._acquire_view(leaves)
        view = e.view
        calls = view.counter("sq8_calls") + view.counter("select_calls")
        one = gq.rewrite(leaves)
        assert view.counter("sq8_calls") + view.counter("select_calls") == calls + 1   # one device search per shard
        gq._release_view(e)
        per_leaf = LU.KnnFloatVectorQuery("v", q, K, filt).rewrite(leaves)
        es, ed = oracle(leaves, rows, q, gq._accept)
        for td in (one, per_leaf):
            s, d = hits(td)
            assert np.array_equal(d, ed) and np.array_equal(s, es.view(np.uint32)), (filtered, qi)


def test_exact_search_override_serves_cost_le_k_leaves_on_the_device(shard):
    leaves, rows, masks = shard
    q = O.synth(0, 1, DIM, 960, 3)[0]
    gq = LU.GpuKnnFloatVectorQuery("v", q, K, lambda lf: masks[lf.ord])
    for ordinal in (4, 7, 9):
        lf = leaves[ordinal]
        acc = gq._accept(lf)
        td = gq.exact_search(lf, acc)
        es, ed, _ = O.exact_search(rows[ordinal], q, K, int(COS), accept_bits=O.bits_from_bool(acc))
        s, d = hits(td)
        assert len(d) == int(acc.sum()) <= K
        assert np.array_equal(d, ed + lf.doc_base) and np.array_equal(s, es.view(np.uint32))


def test_view_cache_is_evicted_when_a_reader_closes_and_shared_under_concurrency():
    """The query's per-leaf-set view cache: concurrent rewrites of one leaf set share one view, and the
    reader-closed listener releases every view over a closed segment (no HBM pinned by stale views)."""
    import threading

    LU.GpuKnnFloatVectorQuery.release_views()
    rows = [O.synth(0, n, DIM, 950 + i, 3) for i, n in enumerate([700, 900])]
    readers = [LU.GpuFlatVectorsReader("v", r, COS) for r in rows]
    leaves = [LU.LeafReaderContext(0, 0, readers[0]), LU.LeafReaderContext(1, 700, readers[1])]
    q = O.synth(0, 1, DIM, 960, 3)[0]
    outs, errs = [], []

    def run():
        try:
            outs.append(LU.GpuKnnFloatVectorQuery("v", q, K).rewrite(leaves))
        except Exception as e:   # pragma: no cover - reported below
            errs.append(e)
    try:
        ts = [threading.Thread(target=run) for _ in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
        assert LU.GpuKnnFloatVectorQuery.cached_views() == 1
        assert all([sd.doc for sd in o.score_docs] == [sd.doc for sd in outs[0].score_docs] for o in outs)
        readers[0].close()
        assert LU.GpuKnnFloatVectorQuery.cached_views() == 0
    finally:
        for r in readers:
            r.close()
        LU.GpuKnnFloatVectorQuery.release_views()


def test_evicted_view_stays_open_until_its_last_search_finishes():
    """A reader that closes while a rewrite holds its cached view evicts the entry at once, but the view
    itself closes only when that rewrite releases it (no view closed under a search)."""
    LU.GpuKnnFloatVectorQuery.release_views()
    rows = [O.synth(0, n, DIM, 970 + i, 3) for i, n in enumerate([600, 500])]
    readers = [LU.GpuFlatVectorsReader("v", r, COS) for r in rows]
    leaves = [LU.LeafReaderContext(0, 0, readers[0]), LU.LeafReaderContext(1, 600, readers[1])]
    q = O.synth(0, 1, DIM, 971, 3)[0]
    gq = LU.GpuKnnFloatVectorQuery("v", q, K)
    try:
        e = gq._acquire_view(leaves)   # a rewrite in flight
        readers[1].close()             # the reader-closed listener runs under it
        assert LU.GpuKnnFloatVectorQuery.cached_views() == 0 and e.evicted
        assert e.view._h.value         # still open: its user has not finished
        s, d, _, c, _, _ = e.view.search(q, K, 0, K)
        es, ed = oracle(leaves, rows, q, gq._accept)
        assert np.array_equal(d[0, :c[0]], ed) and np.array_equal(np.asarray(s[0, :c[0]], np.float32).view(np.uint32),
                                                                  es.view(np.uint32))
        gq._release_view(e)
        assert not e.view._h.value     # the last user closed it
    finally:
        for r in readers:
            r.close()
        LU.GpuKnnFloatVectorQuery.release_views()
