"""GPU parity of the 6-bit first tier of the certified prefilter (osk_sq6.hip).

Single unfiltered float32 queries over views of ≥ 512 dims scan 6-bit codes (576 + 16 B per 768-dim
row instead of 768 + 16 B) and settle exactly as the int8 tier does, so every result must equal the
int8 tier (tune "sq6" 0), the fp32 streaming scan (tune "sq8" 0) and the oracle's device-order
exactSearch bit for bit: docs, score bits, tie order, visited counts.  Covered: every similarity,
dims with and without a tier (padding to 256 dims per lane set), ragged multi-segment multi-shard
views (partial 8-row blocks, 1-row segments), sparse ord→doc maps, k 1…12, heavy ties, constant and
zero rows, adversarial dynamic range (a bound so wide the settle re-scans lists exactly), and a view
of many tiles where the tier must certify with a bounded number of re-scored rows.
"""
import ctypes as C

import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIMS = [LU.VectorSimilarityFunction(s) for s in range(4)]
COS = LU.VectorSimilarityFunction.COSINE


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


def tuned(key, value, fn):
    old = {"sq6": 1, "sq8": 1, "sq8_force_fallback": 0}[key]
    _lib.tune(key, value)
    try:
        return fn()
    finally:
        _lib.tune(key, old)


def one_by_one(search, queries):
    """Single-query calls (the tier serves batch 1), stacked like one batched result."""
    outs = [search(queries[i:i + 1]) for i in range(len(queries))]
    return tuple(np.concatenate([o[j] for o in outs]) for j in range(len(outs[0])))


def three_ways(search, queries):
    six = one_by_one(search, queries)
    eight = tuned("sq6", 0, lambda: one_by_one(search, queries))
    fp32 = tuned("sq8", 0, lambda: one_by_one(search, queries))
    assert_same(six, eight)
    assert_same(six, fp32)
    return six


def view_of(rows_list, sim, shard_of=None, shard_index=None, docs_list=None, max_docs=None):
    shard_of = shard_of or [0] * len(rows_list)
    n_shards = max(shard_of) + 1
    leaves = [[] for _ in range(n_shards)]
    readers, bases = [], [0] * n_shards
    for i, (rows, s) in enumerate(zip(rows_list, shard_of)):
        kw = {}
        if docs_list and docs_list[i] is not None:
            kw = dict(ord_to_doc=docs_list[i], max_doc=max_docs[i])
        r = LU.GpuFlatVectorsReader("v", rows, sim, **kw)
        readers.append(r)
        leaves[s].append(LU.LeafReaderContext(len(leaves[s]), bases[s], r))
        bases[s] += max_docs[i] if (docs_list and docs_list[i] is not None) else len(rows)
    return LU.DeviceShardSet(leaves, shard_index), readers


def close_all(ds, readers):
    ds.close()
    for r in readers:
        r.close()


@pytest.mark.parametrize("dim", [512, 520, 600, 768, 1000, 1024, 1536, 2048])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_single_queries_equal_int8_fp32_and_oracle(dim, sim):
    n = 2600 + dim % 13
    rows = corpus(n, dim, sim, 40 + dim)
    queries = corpus(4, dim, sim, 41 + dim)
    ds, readers = view_of([rows], sim)
    try:
        before = ds.counter("sq6_calls")
        s, d, sh, c, t, _ = three_ways(lambda q: ds.search(q, 10, 0, 10), queries)
        has_tier = dim in (512, 768, 1000, 1024, 1536)
        # the tier exists where 6-bit rows are ≤ 0.8 × the int8 rows (dims padded to 256 per lane set)
        assert (ds.counter("sq6_calls") - before == len(queries)) == has_tier
        for i in range(len(queries)):
            os_, od, _ = O.exact_search(rows, queries[i], 10, int(sim), O.ORDER_DEVICE)
            assert np.array_equal(d[i, :c[i]], od) and np.array_equal(bits(s[i, :c[i]]), bits(os_))
    finally:
        close_all(ds, readers)


@pytest.mark.parametrize("k", [1, 3, 10, 12])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_ragged_segments_shards_and_sparse_docs(k, sim):
    """Segments of 1, 3, 7 and 8·m + 5 rows (partial 8-row blocks and tiles ending inside a block),
    a sparse field, permuted shard indices, from/size cuts."""
    dim = 768
    sizes = [4005, 1, 3, 7, 1237, 2900]
    segs = [corpus(n, dim, sim, 60 + i) for i, n in enumerate(sizes)]
    rng = np.random.default_rng(k)
    docs = [None] * len(sizes)
    maxd = [None] * len(sizes)
    docs[4] = np.sort(rng.choice(5000, sizes[4], replace=False)).astype(np.int32)
    maxd[4] = 5000
    ds, readers = view_of(segs, sim, [0, 0, 1, 1, 2, 2], [2, 0, 1], docs, maxd)
    queries = corpus(3, dim, sim, 70)
    try:
        for f, sz in [(0, k), (min(2, k - 1), k - min(2, k - 1))]:
            three_ways(lambda q: ds.search(q, k, f, sz), queries)
        assert ds.counter("sq6_calls") >= 3
    finally:
        close_all(ds, readers)


def test_segment_reader_and_visited_counts():
    sim = COS
    rows = corpus(5003, 768, sim, 80)
    queries = corpus(3, 768, sim, 81)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        s, d, c, v = three_ways(lambda q: r.search_batch(q, 10), queries)
        for i in range(3):
            os_, od, ov = O.exact_search(rows, queries[i], 10, int(sim))
            assert np.array_equal(d[i], od) and np.array_equal(bits(s[i]), bits(os_)) and v[i] == ov == 5003
    finally:
        r.close()


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_heavy_ties(sim):
    base = corpus(600, 512, sim, 90)
    rows = np.concatenate([base, base[::-1], base])
    queries = np.concatenate([base[:2], corpus(2, 512, sim, 91)])
    ds, readers = view_of([rows], sim)
    try:
        _, d, _, c, _, _ = three_ways(lambda q: ds.search(q, 12, 0, 12), queries)
        for i in range(len(queries)):
            _, od, _ = O.exact_search(rows, queries[i], 12, int(sim))
            assert np.array_equal(d[i, :c[i]], od)
    finally:
        close_all(ds, readers)


def test_constant_zero_and_adversarial_rows():
    rng = np.random.default_rng(13)
    adv = rng.standard_normal((5000, 768)).astype(np.float32) * 1e-3
    adv[:, 0] = 1000.0   # one huge component: 6-bit codes of the rest are all 0, the bound is very wide
    const = np.ones((900, 768), np.float32)
    const[100:200] = 0.0
    for rows, sims in [(adv, SIMS), (const, [LU.VectorSimilarityFunction.EUCLIDEAN,
                                              LU.VectorSimilarityFunction.DOT_PRODUCT,
                                              LU.VectorSimilarityFunction.MAXIMUM_INNER_PRODUCT])]:
        queries = np.concatenate([rng.standard_normal((3, 768)).astype(np.float32),
                                  np.zeros((1, 768), np.float32), rows[5:6]])
        for sim in sims:
            ds, readers = view_of([rows], sim)
            try:
                three_ways(lambda q: ds.search(q, 10, 0, 10), queries)
            finally:
                close_all(ds, readers)


def test_forced_exact_lists_is_exact():
    sim = LU.VectorSimilarityFunction.EUCLIDEAN
    rows = corpus(12000, 768, sim, 95)
    queries = corpus(3, 768, sim, 96)
    with _lib.testing():
        ds, readers = view_of([rows[:5000], rows[5000:]], sim, [0, 1], [1, 0])
        try:
            off = tuned("sq8", 0, lambda: one_by_one(lambda q: ds.search(q, 10, 0, 10), queries))
            forced = tuned("sq8_force_fallback", 1, lambda: one_by_one(lambda q: ds.search(q, 10, 0, 10), queries))
            assert_same(forced, off)
            assert ds.counter("sq6_calls") == 3
        finally:
            close_all(ds, readers)


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_many_tiles_calibration_and_certificate(sim):
    """200k × 768 over 4 shards (hundreds of tiles).  The view's first 4 single queries calibrate the tier
    (rows re-bounded from the int8 copy per row scanned) and it stays on only where it pays: never for the
    uniform EUCLIDEAN corpus, whose 6-bit bounds do not separate.  Either way no list
    overflows its certificate, the exact re-score set is no larger than the int8 tier's (the wave lists
    carry int8 bounds; the floor only keeps rows out), and results equal the int8 tier and the oracle."""
    rows = corpus(200_000, 768, sim, 100)
    queries = corpus(7, 768, sim, 101)
    ds, readers = view_of([rows[i * 50_000:(i + 1) * 50_000] for i in range(4)], sim, [0, 1, 2, 3])
    try:
        def run(six, qs):
            r0, b0, c0 = ds.counter("sq8_rescored_rows"), ds.counter("sq6_rebound_rows"), ds.counter("sq6_calls")
            out = tuned("sq6", six, lambda: one_by_one(lambda q: ds.search(q, 10, 0, 10), qs))
            return (out, ds.counter("sq8_rescored_rows") - r0, ds.counter("sq6_rebound_rows") - b0,
                    ds.counter("sq6_calls") - c0)
        probe, _, rb_probe, c_probe = run(1, queries[:4])
        assert c_probe == 4
        keeps = rb_probe * 100 <= 4 * 200_000 * 10
        if sim == LU.VectorSimilarityFunction.EUCLIDEAN:
            assert not keeps, rb_probe   # uniform rows: the 6-bit bounds do not separate
        out6, rs6, rb6, c6 = run(1, queries[4:])
        out8, rs8, rb8, c8 = run(0, queries[4:])
        assert_same(out6, out8)
        assert_same(probe, tuned("sq6", 0, lambda: one_by_one(lambda q: ds.search(q, 10, 0, 10), queries[:4])))
        assert c6 == (3 if keeps else 0) and c8 == 0 and rb8 == 0
        assert ds.counter("sq8_fallback_queries") == 0
        assert 3 * 4 * 10 <= rs6 <= rs8 + 3 * 4 * 16, (rs6, rs8)
        want = [O.topdocs_merge([O.exact_search(rows[s * 50_000:(s + 1) * 50_000], queries[4 + i], 10, int(sim))[:2]
                                 for s in range(4)], 0, 10, [0, 1, 2, 3]) for i in range(3)]
        for i in range(3):
            assert np.array_equal(out6[1][i], want[i][1]) and np.array_equal(bits(out6[0][i]), bits(want[i][0]))
    finally:
        close_all(ds, readers)


def test_footprint_counts_the_tier():
    sim = COS
    r768 = LU.GpuFlatVectorsReader("v", corpus(1001, 768, sim, 110), sim)
    r128 = LU.GpuFlatVectorsReader("v", corpus(1001, 128, sim, 111), sim)
    try:
        def fp(r):
            b = C.c_int64()
            _lib.check(_lib.lib().osk_seg_footprint(r.handle, C.byref(b)))
            return b.value
        n = 1001
        rows_768 = n * 192 * 16 + n * 4 + n * 48 * 16 + n * 16   # fp32 rows, norms, int8 copy + terms
        assert fp(r768) == rows_768 + ((n + 7) // 8) * 3 * 1536 + n * 16
        assert fp(r128) == n * 32 * 16 + n * 4 + n * 8 * 16 + n * 16   # no 6-bit tier at 128 dims
    finally:
        r768.close()
        r128.close()


@pytest.mark.parametrize("sim", [COS, LU.VectorSimilarityFunction.MAXIMUM_INNER_PRODUCT], ids=lambda s: s.name)
def test_large_view_keeps_the_tier(sim):
    """2.4M × 768 in 2 shards, generated on the device, the tier kept whatever its calibration says
    (sq6_probe_pct 100): it certifies, and equals the int8 tier and the oracle's coordinator merge."""
    dist = {2: 3, 3: 2}[int(sim)]
    rps, dim = 1_200_000, 768
    readers = [LU.GpuFlatVectorsReader.synthetic("v", rps, dim, sim, seed=777, dist=dist, row0=s * rps)
               for s in range(2)]
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], [1, 0])
    queries = O.synth(0, 6, dim, 778, dist)
    _lib.tune("sq6_probe_pct", 100)
    try:
        b0 = ds.counter("sq6_rebound_rows")
        out = one_by_one(lambda q: ds.search(q, 10, 0, 10), queries)
        rb = ds.counter("sq6_rebound_rows") - b0
        print(f"int8 re-bounds per query: {rb / 6:.0f} of {2 * rps} rows")
        assert ds.counter("sq6_calls") == 6 and rb < 6 * 2 * rps // 2, rb
        assert ds.counter("sq8_fallback_queries") == 0
        assert_same(out, tuned("sq6", 0, lambda: one_by_one(lambda q: ds.search(q, 10, 0, 10), queries)))
        lists = [[] for _ in range(6)]
        for s in range(2):
            rows = O.synth(s * rps, rps, dim, 777, dist)
            sc, dc, cc = O.knn_batch(rows, queries, 10, int(sim), O.ORDER_DEVICE, 16)
            for i in range(6):
                lists[i].append((sc[i, :cc[i]], dc[i, :cc[i]]))
            del rows
        for i in range(6):
            es, ed, esh, _, _ = O.topdocs_merge(lists[i], 0, 10, [1, 0])
            assert np.array_equal(out[1][i], ed) and np.array_equal(out[2][i], esh)
            assert np.array_equal(bits(out[0][i]), bits(es))
    finally:
        _lib.tune("sq6_probe_pct", 10)
        ds.close()
        for r in readers:
            r.close()


def _footprint(reader):
    b = C.c_int64()
    _lib.check(_lib.lib().osk_seg_footprint(reader.handle, C.byref(b)))
    return b.value


@pytest.mark.parametrize("sim", [LU.VectorSimilarityFunction.EUCLIDEAN, COS], ids=lambda s: s.name)
def test_calibration_is_per_segment_and_shared_by_views(sim):
    """The tier's calibration lives on the segments, not on a view object: the first view's probes decide
    for every segment (read back asynchronously, folded by later calls), a second view over the same
    segments and the replicas that concurrent host calls lease follow that decision without probing again,
    and a segment whose tier turned off (uniform EUCLIDEAN rows) frees its 6-bit copy."""
    import threading

    rows = corpus(120_000, 768, sim, 120)
    queries = corpus(12, 768, sim, 121)
    ds, readers = view_of([rows[:60_000], rows[60_000:]], sim, [0, 1])
    ds2 = None
    try:
        fp0 = [_footprint(r) for r in readers]
        out = one_by_one(lambda q: ds.search(q, 10, 0, 10), queries[:5])   # 4 probes, the 5th call folds
        c1 = ds.counter("sq6_calls")
        keeps = sim == COS
        assert c1 == (5 if keeps else 4), c1
        fp1 = [_footprint(r) for r in readers]
        sq6 = [((60_000 + 7) // 8) * 3 * 1536 + 60_000 * 16] * 2
        assert fp1 == (fp0 if keeps else [a - b for a, b in zip(fp0, sq6)]), (fp0, fp1)
        # a second view over the same segments: no probes, the segments' decision
        ds2 = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, readers[0])], [LU.LeafReaderContext(0, 0, readers[1])]])
        out2 = one_by_one(lambda q: ds2.search(q, 10, 0, 10), queries[:5])
        assert ds2.counter("sq6_calls") == (5 if keeps else 0)
        assert_same(out, out2)
        # concurrent host calls lease replicas of the first view: every slot follows the segments' state.
        # Each call asks a distinct (from, size) page, so the host entry's opportunistic batching (which
        # merges concurrent calls of equal k, from, size into one launch chain) keeps them single queries.
        res, errs = {}, []
        page = [(i % 4, 1 + i // 4) for i in range(16)]

        def worker(i):
            try:
                res[i] = ds.search(queries[5 + i % 7:6 + i % 7], 10, page[i][0], page[i][1])
            except Exception as e:   # pragma: no cover - reported below
                errs.append(e)
        ts = [threading.Thread(target=worker, args=(i,)) for i in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
        assert ds.counter("sq6_calls") - c1 == (16 if keeps else 0)
        for i in range(16):
            want = tuned("sq6", 0, lambda: ds.search(queries[5 + i % 7:6 + i % 7], 10, page[i][0], page[i][1]))
            assert_same(res[i], want)
    finally:
        if ds2 is not None:
            ds2.close()
        close_all(ds, readers)


def test_first_device_call_returns_before_its_work_completes():
    """A calibration probe is asynchronous: the view's first osk_view_search_device call (after warm) returns
    while its launches are still running, and its counts are folded by a later call without a wait."""
    import torch
    rps, dim = 2_000_000, 768
    readers = [LU.GpuFlatVectorsReader.synthetic("v", rps, dim, COS, seed=31, dist=3, row0=s * rps) for s in range(2)]
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers])
    try:
        _lib.check(_lib.lib().osk_view_warm(ds.handle, _lib.OSK_WARM_PREFILTER))
        q = torch.from_numpy(O.synth(0, 1, dim, 32, 3)).cuda()
        keys = torch.zeros((1, 2, 10), dtype=torch.int64, device="cuda")
        counts = torch.zeros((1, 2), dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            _lib.check(_lib.lib().osk_view_search_device(ds.handle, q.data_ptr(), 1, 10, None, keys.data_ptr(),
                                                         counts.data_ptr(), None, st.cuda_stream))
            pending = not st.query()
        st.synchronize()
        assert pending, "the probe call waited for its own work"
        assert ds.counter("sq6_calls") == 1
        assert counts.cpu().numpy().tolist() == [[10, 10]]
        want = ds.search(q.cpu().numpy(), 10, 0, 10)   # (a later call: folds the probe)
        got = np.sort(keys.cpu().numpy().view(np.uint64).reshape(-1))[::-1][:10]
        sc, dc = LU.decode_keys(got)
        assert np.array_equal(bits(sc), bits(want[0][0]))
    finally:
        ds.close()
        for r in readers:
            r.close()


def test_tier_off_frees_its_copy_without_waiting_for_other_streams():
    """A segment whose calibration turns the tier off frees its 6-bit copy stream-ordered (hipFreeAsync behind
    the events of the launches that read it), not with a device-wide synchronisation: while a neighbouring
    view's searches are queued on another stream, the call that folds the last probe and frees the copy
    returns before that stream's work completes.  Results stay exact after the free (int8 tier)."""
    import torch
    sim = LU.VectorSimilarityFunction.EUCLIDEAN   # uniform rows: the probes turn the tier off
    rows = corpus(120_000, 768, sim, 130)
    queries = corpus(8, 768, sim, 131)
    ds, readers = view_of([rows[:60_000], rows[60_000:]], sim, [0, 1])
    rps = 2_000_000
    big = [LU.GpuFlatVectorsReader.synthetic("v", rps, 768, COS, seed=33, dist=3, row0=s * rps) for s in range(2)]
    dsb = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in big])
    try:
        fp0 = [_footprint(r) for r in readers]
        first = one_by_one(lambda q: ds.search(q, 10, 0, 10), queries[:4])   # the 4 probes (not yet folded)
        assert ds.counter("sq6_calls") == 4
        qb = torch.from_numpy(O.synth(0, 1, 768, 34, 3)).cuda()
        keys = torch.zeros((1, 2, 10), dtype=torch.int64, device="cuda")
        counts = torch.zeros((1, 2), dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()
        L = _lib.lib()
        for _ in range(6):   # the neighbour's own probes and builds, done before the timed part
            _lib.check(L.osk_view_search_device(dsb.handle, qb.data_ptr(), 1, 10, None, keys.data_ptr(),
                                                counts.data_ptr(), None, st.cuda_stream))
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            for _ in range(60):   # ≈ 60 × 0.1 ms of queued work on the neighbour's stream
                _lib.check(L.osk_view_search_device(dsb.handle, qb.data_ptr(), 1, 10, None, keys.data_ptr(),
                                                    counts.data_ptr(), None, st.cuda_stream))
        out5 = ds.search(queries[4:5], 10, 0, 10)   # folds the 4th probe: the tier turns off, the copy is freed
        neighbour_pending = not st.query()
        st.synchronize()
        assert neighbour_pending, "the call that freed the 6-bit copy waited for another stream's work"
        assert ds.counter("sq6_calls") == 4
        sq6 = [((60_000 + 7) // 8) * 3 * 1536 + 60_000 * 16] * 2
        assert [_footprint(r) for r in readers] == [a - b for a, b in zip(fp0, sq6)]
        assert counts.cpu().numpy().tolist() == [[10, 10]]
        rest = one_by_one(lambda q: ds.search(q, 10, 0, 10), queries[5:])
        assert ds.counter("sq6_calls") == 4
        want = tuned("sq6", 0, lambda: one_by_one(lambda q: ds.search(q, 10, 0, 10), queries))
        got = tuple(np.concatenate([a, b, c]) for a, b, c in zip(first, out5, rest))
        assert_same(got, want)
    finally:
        dsb.close()
        for r in big:
            r.close()
        close_all(ds, readers)


def _rebound_variants(ds, queries, k):
    """sq6_rebound's schedules (list assignment × workgroups per CU) and its final-floor re-test on and off,
    on single queries."""
    outs = {}
    try:
        for stride, wgs, retest in [(1, 0, 1), (0, 0, 1), (1, 1, 1), (0, 1, 1), (1, 0, 0)]:
            _lib.tune("sq6_rebound_stride", stride)
            _lib.tune("sq6_rebound_wgs", wgs)
            _lib.tune("sq6_rebound_retest", retest)
            outs[(stride, wgs, retest)] = one_by_one(lambda q: ds.search(q, k, 0, k), queries)
    finally:
        _lib.tune("sq6_rebound_stride", 1)
        _lib.tune("sq6_rebound_wgs", 0)
        _lib.tune("sq6_rebound_retest", 1)
    return outs


@pytest.mark.parametrize("layout", ["ragged", "70_shards", "70_segments"])
def test_rebound_schedules_agree_with_the_oracle(layout):
    """sq6_rebound's schedules — contiguous or strided lists, as many workgroups per CU as fit or one (every
    wave walks many lists), the final-floor re-test on or off — give identical results, equal to the oracle; with more than 64 shards the floors and with more than 64 segments the
    per-segment counts leave LDS for their global fallbacks."""
    sim, dim, k = COS, 768, 10
    if layout == "ragged":
        sizes = [9001, 5, 3333, 12000, 77]
        shard_of = [0, 1, 1, 2, 0]
    elif layout == "70_shards":
        sizes = [450 + 7 * i for i in range(70)]
        shard_of = list(range(70))
    else:
        sizes = [300 + 11 * i for i in range(70)]
        shard_of = [i % 3 for i in range(70)]
    segs = [corpus(n, dim, sim, 300 + i) for i, n in enumerate(sizes)]
    n_shards = max(shard_of) + 1
    ds, readers = view_of(segs, sim, shard_of, list(range(n_shards)))
    queries = corpus(3, dim, sim, 399)
    _lib.tune("sq6_probe_pct", 100)   # (the small segments keep the tier whatever their probes count)
    try:
        for i in range(4):   # the calibration probes
            ds.search(queries[:1], k, 0, k)
        c0 = ds.counter("sq6_calls")
        outs = _rebound_variants(ds, queries, k)
        assert ds.counter("sq6_calls") - c0 == 5 * len(queries)
        ref = outs[(1, 0, 1)]
        for o in outs.values():
            assert_same(o, ref)
        s, d, sh, c, t, _ = ref
        for i in range(len(queries)):
            lists = []
            for si in range(n_shards):
                rows = np.concatenate([segs[j] for j in range(len(segs)) if shard_of[j] == si])
                sc, dc, _ = O.exact_search(rows, queries[i], k, int(sim), O.ORDER_DEVICE)
                lists.append((sc, dc))
            es, ed, esh, et, _ = O.topdocs_merge(lists, 0, k, list(range(n_shards)))
            assert np.array_equal(d[i, :c[i]], ed) and np.array_equal(sh[i, :c[i]], esh)
            assert np.array_equal(bits(s[i, :c[i]]), bits(es)) and t[i] == et
    finally:
        _lib.tune("sq6_probe_pct", 10)
        close_all(ds, readers)


def test_scan_profile_samples_every_nth_call():
    """osk_view_profile(view, N) stamps the scan launches of every N-th device search (bench.py's
    --profile-every): N = 3 over 9 calls gives 3 sampled calls, N = 1 every call, N = 0 none; N < 0 is refused."""
    import torch
    sim = COS
    rows = corpus(6000, 768, sim, 510)
    queries = torch.from_numpy(corpus(9, 768, sim, 511)).cuda()
    ds, readers = view_of([rows], sim)
    L = _lib.lib()
    try:
        view = ds._h
        keys = torch.empty((1, 1, 10), dtype=torch.int64, device="cuda")
        counts = torch.empty((1, 1), dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()

        def run(n):
            _lib.check(L.osk_view_profile(view, n))
            for i in range(9):
                _lib.check(L.osk_view_search_device(view, queries[i].data_ptr(), 1, 10, None, keys.data_ptr(),
                                                    counts.data_ptr(), None, st.cuda_stream))
            st.synchronize()
            ms, calls = C.c_double(), C.c_int64()
            _lib.check(L.osk_view_scan_time(view, C.byref(ms), C.byref(calls)))
            return ms.value, calls.value

        ms3, c3 = run(3)
        assert c3 == 3 and ms3 > 0.0
        ms1, c1 = run(1)
        assert c1 == 9 and ms1 > 0.0
        assert run(0) == (0.0, 0)
        assert L.osk_view_profile(view, -1) != 0
    finally:
        _lib.check(L.osk_view_profile(ds._h, 0))
        close_all(ds, readers)
