"""GPU parity of single-query filtered searches (the C5 configuration as benchmarked).

A float32 query with an accept bitset takes one of two scans (both run by every test here):
  * gather (default, tune filter_gather 1): the accepted ordinals of every segment are compacted first
    (osk_filter.hip: count per tile, prefix, write) and `sq8_scan<…, kScanGather>` runs over gather
    tiles of that list; an overflowed list is re-scanned exactly over the same compacted range;
  * window walk (filter_gather 0): `sq8_scan<…, kScanQueue>` queues the accepted rows of sparse
    64-row windows across windows (one `ds_permute` append each) and scans the queue 64 rows at a
    time, flushing when the next window would overflow it.
These tests drive exactly that call (`search_batch(q[i:i+1])`, `DeviceShardSet.search` with one query)
and compare docs and score bits against

  * the fp32 streaming scan of the same call (tune "sq8" 0), and
  * the oracle's [L] exactSearch restatement (`O.exact_search(..., accept_bits=...)`, ORDER_DEVICE),

over selectivities 0.1 % … 100 %, bitsets built to straddle every queue edge (windows of 1…64
accepted rows, queue fills of exactly 64, overflowing appends, dense windows with and without a
non-empty queue, runs crossing wave and tile boundaries) and multi-segment views where some leaves
have no bitset.  Reference semantics: [L] AbstractKnnVectorQuery.exactSearch over AcceptDocs, driven
from S/search/internal/ContextIndexSearcher.java:203-218.
"""
import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

COS = LU.VectorSimilarityFunction.COSINE
SIMS = [LU.VectorSimilarityFunction(s) for s in range(4)]


def corpus(n, dim, sim, seed):
    return O.synth(0, n, dim, seed, {0: 1, 1: 3, 2: 3, 3: 2}[int(sim)])


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def assert_same(a, b):
    for x, y in zip(a, b):
        x, y = np.asarray(x), np.asarray(y)
        if x.dtype == np.float32:
            assert np.array_equal(bits(x), bits(y)), (x, y)
        else:
            assert np.array_equal(x, y), (x, y)


def sq8_off(fn):
    _lib.tune("sq8", 0)
    try:
        return fn()
    finally:
        _lib.tune("sq8", 1)


def edge_mask(n, rng):
    """Accept mask whose 64-row windows hold 0…64 accepted rows in patterns that hit every edge of
    the FQ queue: runs of sparse windows that fill the 64-entry queue exactly, appends that
    overflow it (qn + n > 64 → flush first), dense windows (≥ 16 rows) arriving with an empty and
    with a non-empty queue, and single accepted rows on window boundaries."""
    counts = []
    pattern = [1, 3, 7, 15, 16, 17, 31, 33, 40, 63, 64, 0, 0, 2, 62, 1, 1, 48, 5, 59, 60, 4]
    while len(counts) * 64 < n:
        counts += list(rng.permutation(pattern))
    mask = np.zeros(len(counts) * 64, bool)
    for w, c in enumerate(counts):
        if c:
            mask[w * 64 + rng.choice(64, c, replace=False)] = True
    # boundary rows: first and last row of some windows
    mask[::640] = True
    mask[63::704] = True
    return mask[:n]


def check_single(reader, rows, queries, k, sim, mask, ord_to_doc=None):
    ab = O.bits_from_bool(mask)
    for i in range(len(queries)):
        q = queries[i:i + 1]
        on = reader.search_batch(q, k, ab)
        off = sq8_off(lambda: reader.search_batch(q, k, ab))
        assert_same(on, off)
        os_, od, ov = O.exact_search(rows, queries[i], k, int(sim), ord_to_doc=ord_to_doc, accept_bits=ab)
        s, d, c, v = on
        assert c[0] == len(od)
        assert np.array_equal(d[0, : c[0]], od), (i, d[0, : c[0]], od)
        assert np.array_equal(bits(s[0, : c[0]]), bits(os_))
        assert v[0] == ov


@pytest.fixture(autouse=True, params=[1, 0], ids=["gather", "window_walk"])
def filter_mode(request):
    """Filtered single-query scans compact the accepted ordinals and scan them (tune filter_gather 1,
    the default, osk_filter.hip), or walk the bitset's 64-row windows with the cross-window queue
    instance (filter_gather 0)."""
    _lib.tune("filter_gather", request.param)
    yield request.param
    _lib.tune("filter_gather", 1)


@pytest.fixture(params=[0, 8], ids=["tiles_default", "tiles_8"])
def tiles(request):
    """Default tiling (≈1k rows per tile) and 8 large tiles (≈1.9k rows per wave: long queues)."""
    _lib.tune("tiles_target", request.param)
    yield request.param
    _lib.tune("tiles_target", 0)


@pytest.mark.parametrize("selectivity", [0.001, 0.01, 0.1, 0.5, 1.0])
@pytest.mark.parametrize("dim", [128, 768])
def test_single_query_filtered_dense(selectivity, dim, tiles):
    n = 60000
    rows = corpus(n, dim, COS, 101)
    queries = corpus(4, dim, COS, 102)
    rng = np.random.default_rng(int(selectivity * 1e4) + dim)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    try:
        check_single(r, rows, queries, 10, COS, rng.random(n) < selectivity)
    finally:
        r.close()


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
@pytest.mark.parametrize("dim", [17, 96, 384])
def test_single_query_filtered_queue_edges(sim, dim, tiles):
    n = 50000 + dim
    rows = corpus(n, dim, sim, 103)
    queries = corpus(3, dim, sim, 104)
    rng = np.random.default_rng(dim + int(sim))
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        for k in (1, 10, 12):
            check_single(r, rows, queries, k, sim, edge_mask(n, rng))
    finally:
        r.close()


def test_single_query_filtered_fewer_accepted_than_k():
    """AcceptDocs with ≤ k accepted docs ([L] the filter-cost ≤ k branch: exactSearch)."""
    n = 70000
    rows = corpus(n, 256, COS, 105)
    queries = corpus(3, 256, COS, 106)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    try:
        for n_acc in (0, 1, 5, 10):
            mask = np.zeros(n, bool)
            mask[np.random.default_rng(n_acc).choice(n, n_acc, replace=False)] = True
            check_single(r, rows, queries, 10, COS, mask)
    finally:
        r.close()


def test_single_query_filtered_multi_segment_view(tiles):
    """One query over a 3-shard view; some leaves have a bitset, others none (no deletions)."""
    sim = COS
    sizes = [30000, 700, 45000, 20000]
    segs = [corpus(s, 768, sim, 110 + i) for i, s in enumerate(sizes)]
    shard_of = [0, 0, 1, 2]
    leaves = [[], [], []]
    readers = []
    bases = [0, 0, 0]
    for rows, s in zip(segs, shard_of):
        rd = LU.GpuFlatVectorsReader("v", rows, sim)
        readers.append(rd)
        leaves[s].append(LU.LeafReaderContext(len(leaves[s]), bases[s], rd))
        bases[s] += len(rows)
    ds = LU.DeviceShardSet(leaves, [2, 0, 1])
    rng = np.random.default_rng(7)
    queries = corpus(3, 768, sim, 120)
    try:
        for accept in ([rng.random(30000) < 0.01, None, rng.random(45000) < 0.1, None],
                       [None, None, None, None],
                       [edge_mask(30000, rng), rng.random(700) < 0.5, None, edge_mask(20000, rng)]):
            for i in range(len(queries)):
                q = queries[i:i + 1]
                on = ds.search(q, 10, 0, 10, accept=accept)
                off = sq8_off(lambda: ds.search(q, 10, 0, 10, accept=accept))
                assert_same(on, off)
                # oracle: per leaf exactSearch, per shard merge (docBase), coordinator merge
                per_shard = [[], [], []]
                for li, (rows, s) in enumerate(zip(segs, shard_of)):
                    ab = None if accept[li] is None else O.bits_from_bool(accept[li])
                    sc, dc, _ = O.exact_search(rows, queries[i], 10, int(sim), accept_bits=ab)
                    base = sum(len(segs[j]) for j in range(li) if shard_of[j] == s)
                    per_shard[s].append((sc, dc + base))
                shard_lists = [O.topdocs_merge(ps, 0, 10)[:2] for ps in per_shard]
                es, ed, esh, et, _ = O.topdocs_merge(shard_lists, 0, 10, [2, 0, 1])
                s_, d_, sh_, c_, t_, _ = on
                assert c_[0] == len(ed)
                assert np.array_equal(d_[0, : c_[0]], ed) and np.array_equal(sh_[0, : c_[0]], esh)
                assert np.array_equal(bits(s_[0, : c_[0]]), bits(es))
    finally:
        ds.close()
        for rd in readers:
            rd.close()


def test_single_query_filtered_sparse_field():
    """Sparse ord→doc with liveDocs: the FQ instance only serves dense fields; the sparse branch must
    agree with the oracle too (single query)."""
    n, max_doc = 40000, 90000
    rng = np.random.default_rng(9)
    rows = corpus(n, 768, COS, 130)
    docs = np.sort(rng.choice(max_doc, n, replace=False)).astype(np.int32)
    queries = corpus(3, 768, COS, 131)
    r = LU.GpuFlatVectorsReader("v", rows, COS, ord_to_doc=docs, max_doc=max_doc)
    try:
        check_single(r, rows, queries, 10, COS, rng.random(max_doc) < 0.05, ord_to_doc=docs)
    finally:
        r.close()


@pytest.mark.parametrize("nq", [1, 5])
def test_filtered_forced_exact_rescan_of_every_list(nq):
    """The settle's exact re-scan of an overflowed list, forced for every list (the testing build's
    sq8_force_fallback): in gather mode it walks the list's share of the compacted ordinals, in window
    mode its row range; both must equal the fp32 scan."""
    rows = corpus(40000, 128, COS, 140)
    queries = corpus(nq, 128, COS, 141)
    mask = np.random.default_rng(nq).random(40000) < 0.07
    ab = O.bits_from_bool(mask)
    with _lib.testing():
        _lib.tune("sq8_mfma_min", 0)   # batches on the VALU scan (the gather path's)
        r = LU.GpuFlatVectorsReader("v", rows, COS)
        try:
            off = sq8_off(lambda: r.search_batch(queries, 10, ab))
            _lib.tune("sq8_force_fallback", 1)
            forced = r.search_batch(queries, 10, ab)
            _lib.tune("sq8_force_fallback", 0)
            assert_same(forced, off)
            assert_same(r.search_batch(queries, 10, ab), off)
        finally:
            r.close()
            _lib.tune("sq8_mfma_min", 2)


def test_filtered_batches_on_the_valu_scan():
    """Filtered batches of 2…8 queries on the VALU scan (sq8_mfma_min 0) also take the gather path."""
    rows = corpus(50000, 384, COS, 150)
    queries = corpus(8, 384, COS, 151)
    mask = np.random.default_rng(4).random(50000) < 0.03
    ab = O.bits_from_bool(mask)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    _lib.tune("sq8_mfma_min", 0)
    try:
        for b in (2, 3, 8):
            on = r.search_batch(queries[:b], 10, ab)
            assert_same(on, sq8_off(lambda: r.search_batch(queries[:b], 10, ab)))
            for i in range(b):
                os_, od, _ = O.exact_search(rows, queries[i], 10, int(COS), accept_bits=ab)
                assert np.array_equal(on[1][i], od)
    finally:
        _lib.tune("sq8_mfma_min", 2)
        r.close()
