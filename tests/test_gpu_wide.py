"""GPU parity of the wide int8 MFMA prefilter (osk_sq8w.hip, 256 queries per launch).

Large unfiltered batches of float32 rows of ≤ 256 dims read the int8 corpus once per 256 queries.  Its
quick test is relaxed to per-step row maxima and its lists are per (quarter, query), so every result must
still equal the fp32 streaming scan (tune "sq8" 0), sq8_mfma (tune "sq8_wide_min" 0) and the oracle's
device-order exactSearch + TopDocs.merge bit for bit: docs, score bits, tie order, shard indices.
Covered: every similarity, dims 1…768 (KS = 2, 4, 8 and 12), batches that are not multiples of 16, 64 or 256
(partial query blocks, idle waves, several launches), k 1…12, ragged multi-segment multi-shard views with
partial 16-row groups and 1-row segments, heavy ties, zero and constant rows, a zero query, and the
pilot floor on data where most rows tie.
"""
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


def assert_same(a, b):
    for x, y in zip(a, b):
        x, y = np.asarray(x), np.asarray(y)
        if x.dtype == np.float32:
            assert np.array_equal(bits(x), bits(y)), (x, y)
        else:
            assert np.array_equal(x, y), (x, y)


def tuned(key, value, default, fn):
    _lib.tune(key, value)
    try:
        return fn()
    finally:
        _lib.tune(key, default)


def view_of(rows_list, sim, shard_of, shard_index=None):
    n_shards = max(shard_of) + 1
    leaves = [[] for _ in range(n_shards)]
    readers, bases = [], [0] * n_shards
    for rows, s in zip(rows_list, shard_of):
        r = LU.GpuFlatVectorsReader("v", rows, sim)
        readers.append(r)
        leaves[s].append(LU.LeafReaderContext(len(leaves[s]), bases[s], r))
        bases[s] += len(rows)
    return LU.DeviceShardSet(leaves, shard_index), readers


def close_all(ds, readers):
    ds.close()
    for r in readers:
        r.close()


def three_ways(ds, queries, k, from_=0, size=None):
    """wide vs sq8_mfma vs fp32 scan; returns the wide result and checks the wide kernel ran."""
    size = size or k
    w0 = ds.counter("sq8_wide_calls")
    wide = ds.search(queries, k, from_, size)
    assert ds.counter("sq8_wide_calls") == w0 + 1
    narrow = tuned("sq8_wide_min", 0, WIDE_MIN, lambda: ds.search(queries, k, from_, size))
    fp32 = tuned("sq8", 0, 1, lambda: ds.search(queries, k, from_, size))
    assert_same(wide, narrow)
    assert_same(wide, fp32)
    return wide


def oracle_merge(rows_list, shard_of, shard_index, q, k, sim):
    n_shards = max(shard_of) + 1
    lists = []
    for s in range(n_shards):
        segs = [i for i, t in enumerate(shard_of) if t == s]
        rows = np.concatenate([rows_list[i] for i in segs])
        lists.append(O.exact_search(rows, q, k, int(sim))[:2])
    return O.topdocs_merge(lists, 0, k, shard_index)


WIDE_MIN = 48   # the batches these tests send to the wide kernel


@pytest.fixture(autouse=True)
def defaults():
    _lib.tune("sq8_wide_min", WIDE_MIN)
    _lib.tune("sq8_wide_force", 1)   # (these views are small: the cost model alone would keep sq8_mfma)
    yield
    _lib.tune("sq8_wide_min", 64)
    _lib.tune("sq8_wide_force", 0)


@pytest.mark.parametrize("dim", [1, 17, 64, 96, 100, 128, 129, 200, 256, 257, 400, 512, 513, 700, 768])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_wide_equals_mfma_scan_and_oracle(dim, sim):
    sizes = [7001, 1, 2999, 16, 4100]
    rows_list = [corpus(n, dim, sim, 10 + i) for i, n in enumerate(sizes)]
    shard_of, shard_index = [0, 0, 1, 2, 2], [2, 0, 1]
    queries = corpus(77, dim, sim, 20)
    ds, readers = view_of(rows_list, sim, shard_of, shard_index)
    try:
        s, d, sh, c, _, _ = three_ways(ds, queries, 10)
        for i in range(0, 77, 19):
            es, ed, esh, _, _ = oracle_merge(rows_list, shard_of, shard_index, queries[i], 10, sim)
            assert np.array_equal(d[i, :c[i]], ed) and np.array_equal(sh[i, :c[i]], esh)
            assert np.array_equal(bits(s[i, :c[i]]), bits(es))
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("nq", [48, 63, 64, 65, 200, 256, 257, 520])
def test_wide_batch_shapes(nq):
    """Partial 16-query blocks, waves with no query, several launches of 256."""
    sim = LU.VectorSimilarityFunction.DOT_PRODUCT
    rows_list = [corpus(n, 96, sim, 30 + i) for i, n in enumerate([12000, 5003])]
    queries = corpus(nq, 96, sim, 40)
    ds, readers = view_of(rows_list, sim, [0, 1])
    try:
        three_ways(ds, queries, 10)
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("k", [1, 5, 12])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_wide_k_and_from_size(k, sim):
    rows_list = [corpus(n, 128, sim, 50 + i) for i, n in enumerate([9000, 3000, 6001])]
    queries = corpus(100, 128, sim, 60)
    ds, readers = view_of(rows_list, sim, [0, 1, 1], [1, 0])
    try:
        three_ways(ds, queries, k, 0, k)
        if k > 2:
            three_ways(ds, queries, k, 2, k - 2)
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_wide_ties_zero_rows_and_zero_query(sim):
    """Duplicated rows (exact ties broken by doc), zero and constant rows, and a zero query: the relaxed
    quick test passes every pair of a zero query or a zero row, the precise bound decides."""
    rng = np.random.default_rng(3)
    base = corpus(400, 64, sim, 70)
    rows = base[rng.integers(0, 400, 6000)].copy()
    rows[::97] = 0.0
    rows[5::101] = 0.25
    queries = corpus(80, 64, sim, 71)
    queries[3] = 0.0
    queries[40] = rows[10]
    ds, readers = view_of([rows[:3500], rows[3500:]], sim, [0, 1])
    try:
        three_ways(ds, queries, 10)
    finally:
        close_all(ds, readers)


def test_wide_many_tiles_at_size():
    """A device-generated 3.2M × 96 DOT view over 4 shards (thousands of quarters): the wide path (one
    launch of 256 after its pilot) equals sq8_mfma and the oracle on a sample of queries."""
    sim, rps, dim = LU.VectorSimilarityFunction.DOT_PRODUCT, 800_000, 96
    readers = [LU.GpuFlatVectorsReader.synthetic("v", rps, dim, sim, seed=91, dist=_lib.DIST_NORMALISH_UNIT,
                                                 row0=s * rps) for s in range(4)]
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], [3, 1, 0, 2])
    try:
        q = O.synth(0, 256, dim, 92, _lib.DIST_NORMALISH_UNIT)
        w0 = ds.counter("sq8_wide_calls")
        out = ds.search(q, 10, 0, 10)
        assert ds.counter("sq8_wide_calls") == w0 + 1
        assert ds.counter("sq8_fallback_queries") == 0
        assert_same(out, tuned("sq8_wide_min", 0, WIDE_MIN, lambda: ds.search(q, 10, 0, 10)))
        samp = [0, 77, 200, 255]
        lists = [[] for _ in samp]
        for s in range(4):
            rows = O.synth(s * rps, rps, dim, 91, _lib.DIST_NORMALISH_UNIT)
            sc, dc, cc = O.knn_batch(rows, q[samp], 10, int(sim), O.ORDER_DEVICE, 16)
            for j in range(len(samp)):
                lists[j].append((sc[j, :cc[j]], dc[j, :cc[j]]))
        for j, i in enumerate(samp):
            es, ed, esh, _, _ = O.topdocs_merge(lists[j], 0, 10, [3, 1, 0, 2])
            assert np.array_equal(out[1][i], ed) and np.array_equal(out[2][i], esh)
            assert np.array_equal(bits(out[0][i]), bits(es))
    finally:
        ds.close()
        for r in readers:
            r.close()


def _oracle_check(out, rows_list, shard_of, shard_index, queries, k, sim, every=1):
    s, d, sh, c, _, _ = out
    for i in range(0, len(queries), every):
        es, ed, esh, _, _ = oracle_merge(rows_list, shard_of, shard_index, queries[i], k, sim)
        assert c[i] == len(ed)
        assert np.array_equal(d[i, :c[i]], ed) and np.array_equal(sh[i, :c[i]], esh), i
        assert np.array_equal(bits(s[i, :c[i]]), bits(es)), i


def test_wide_with_few_scan_tiles():
    """tiles_target far below the wide kernel's quarter table (the scan tiles and the wide quarters are two
    tables): the pilot's key buffer is sized by the wide table, so results equal the oracle."""
    sim = LU.VectorSimilarityFunction.DOT_PRODUCT
    rows_list = [corpus(n, 96, sim, 80 + i) for i, n in enumerate([150_000, 90_001])]
    queries = corpus(256, 96, sim, 81)
    _lib.tune("tiles_target", 16)
    try:
        ds, readers = view_of(rows_list, sim, [0, 1], [1, 0])
    finally:
        _lib.tune("tiles_target", 0)
    try:
        out = three_ways(ds, queries, 10)
        _oracle_check(out, rows_list, [0, 1], [1, 0], queries, 10, sim, every=37)
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("sim", [LU.VectorSimilarityFunction.COSINE, LU.VectorSimilarityFunction.EUCLIDEAN],
                         ids=lambda s: s.name)
def test_wide_many_shards_global_floors_and_grid_doubling(sim):
    """20 shards (> kWideMaxFloorShards = 16: the per-(shard, query) floors live in global memory, not LDS),
    256-row quarters and a 1-workgroup grid, so one workgroup's quarter descriptors overflow the LDS cap and
    launch_sq8_wide doubles the grid until they fit; a second view keeps the default grid."""
    sizes = [9000 + 517 * i for i in range(20)]
    rows_list = [corpus(n, 128, sim, 200 + i) for i, n in enumerate(sizes)]
    shard_of = list(range(20))
    shard_index = list(np.random.default_rng(5).permutation(20))
    queries = corpus(130, 128, sim, 201)
    _lib.tune("sq8_wide_quarter_rows", 256)
    try:
        ds, readers = view_of(rows_list, sim, shard_of, shard_index)
        ds.search(queries[:64], 10, 0, 10)   # builds the wide table under the knob
    finally:
        _lib.tune("sq8_wide_quarter_rows", 0)
    try:
        default_grid = three_ways(ds, queries, 10)
        small = tuned("sq8_wide_grid", 1, 0, lambda: ds.search(queries, 10, 0, 10))
        assert_same(small, default_grid)
        _oracle_check(small, rows_list, shard_of, shard_index, queries, 10, sim, every=29)
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("defer", [0, 1])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_wide_immediate_and_deferred_insertions_agree(sim, defer):
    """The wide kernel defers its list insertions to each quarter's end when LDS allows (sq8_wide_defer 1, the
    default) or inserts at once (0); both equal sq8_mfma, the fp32 scan and the oracle.  Quarters of 256 rows
    and a 1-workgroup grid give each wave many quarters, drains and (few floors yet) full queues."""
    dim = {0: 128, 1: 96, 2: 768, 3: 200}[int(sim)]
    rows_list = [corpus(n, dim, sim, 300 + i) for i, n in enumerate([20000, 7777])]
    queries = corpus(140, dim, sim, 301)
    _lib.tune("sq8_wide_quarter_rows", 256)
    try:
        ds, readers = view_of(rows_list, sim, [0, 1], [1, 0])
        ds.search(queries[:64], 10, 0, 10)   # builds the wide table under the knob
    finally:
        _lib.tune("sq8_wide_quarter_rows", 0)
    _lib.tune("sq8_wide_defer", defer)
    try:
        out = three_ways(ds, queries, 10)
        small = tuned("sq8_wide_grid", 1, 0, lambda: ds.search(queries, 10, 0, 10))
        assert_same(small, out)
        _oracle_check(out, rows_list, [0, 1], [1, 0], queries, 10, sim, every=23)
    finally:
        _lib.tune("sq8_wide_defer", 1)
        close_all(ds, readers)


def test_glds16_run_destinations():
    """The one-statement LDS-DMA helper the wide kernel's ring runs on (glds16_run, osk_device.h): N = 1, 2, 4
    DMAs at the slab stride (1 KiB) and the bound-term stride (kAuxGroupF4 · 16 B) land exactly at their own
    out-of-order LDS destinations (M0 + immediate offset + lane·16 = the destination), nothing else written.
    Round 5's first one-statement build read the offset as global-only and faulted a box;
    a compiler or ISA change to that semantics fails here, not as a parity failure elsewhere."""
    import ctypes as C
    with _lib.testing() as T:
        bad = C.c_int64(-1)
        _lib.check(T.osk_testing_glds_probe(0, C.byref(bad)))
        assert bad.value == 0, f"{bad.value} LDS words differ from the expected DMA image"


def test_wide_copy_is_built_only_when_a_batch_takes_the_wide_kernel():
    """The group-scaled copy (codes + tiled bound terms, osk_sq8w.hip launch_sq8w_build) is the wide kernel's
    alone: warming the MFMA prefilter and running sq8_mfma batches leave it unbuilt; the first batch the cost
    model sends to the wide kernel builds it."""
    import ctypes as C
    n, dim = 5000, 96
    rows = corpus(n, dim, SIMS[1], 2601)
    q = corpus(64, dim, SIMS[1], 2602)
    ds, readers = view_of([rows], SIMS[1], [0])
    r = readers[0]

    def footprint():
        b = C.c_int64()
        _lib.check(_lib.lib().osk_seg_footprint(r.handle, C.byref(b)))
        return b.value

    try:
        _lib.check(_lib.lib().osk_view_warm(ds.handle, _lib.OSK_WARM_PREFILTER_MFMA))
        warmed = footprint()
        narrow = tuned("sq8_wide_min", 0, WIDE_MIN, lambda: ds.search(q, 10, 0, 10))
        assert footprint() == warmed and ds.counter("sq8_wide_calls") == 0
        wide = ds.search(q, 10, 0, 10)
        assert ds.counter("sq8_wide_calls") == 1
        groups = (n + 15) // 16
        assert footprint() == warmed + groups * 2 * 1024 + groups * 22 * 16   # KS = 2 slabs + kAuxGroupF4 terms
        assert_same(wide, narrow)
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("claim", [1, 0])
@pytest.mark.parametrize("qcap", [0, 1, 8, 64, 128])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_wide_rows_kernel_equals_the_ring_kernel(sim, qcap, claim):
    """≤ 128 dims run the pilot and the main passes on sq8_wide_rows (rows owned by waves, no step barrier,
    insertions queued to the query's owner wave).  Its results equal sq8_wide's (tune sq8_wide_rows 0), the fp32
    scan and sq8_mfma; with the queues shrunk (sq8_wide_rows_qcap: 1 or 8 entries — no sub-queues, a pool of
    1 / 8; 64 or 128 — sub-queues of 4 / 8 entries spilling into pools of 32 / 64) entries spill into the pool
    or are dropped and their (quarter, query) lists marked for the settle's exact re-scan — results still
    equal, bit for bit; with the groups dealt (claim 0) or claimed (claim 1)."""
    rows_list = [corpus(n, 96, sim, 80 + i) for i, n in enumerate([23001, 1, 7000, 16])]
    shard_of, shard_index = [0, 0, 1, 2], [1, 2, 0]
    queries = corpus(300, 96, sim, 90)
    queries[7] = 0.0
    ds, readers = view_of(rows_list, sim, shard_of, shard_index)
    try:
        _lib.tune("sq8_wide_rows_qcap", qcap)
        _lib.tune("sq8_wide_rows_claim", claim)
        try:
            rows = three_ways(ds, queries, 10)
        finally:
            _lib.tune("sq8_wide_rows_qcap", 0)
            _lib.tune("sq8_wide_rows_claim", 1)
        ring = tuned("sq8_wide_rows", 0, 1, lambda: ds.search(queries, 10, 0, 10))
        assert_same(rows, ring)
        for i in (0, 7, 299):
            es, ed, esh, _, _ = oracle_merge(rows_list, shard_of, shard_index, queries[i], 10, sim)
            s, d, sh, c, _, _ = rows
            assert np.array_equal(d[i, :c[i]], ed) and np.array_equal(sh[i, :c[i]], esh)
            assert np.array_equal(bits(s[i, :c[i]]), bits(es))
    finally:
        close_all(ds, readers)
