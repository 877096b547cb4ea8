"""GPU parity: libosknn's HIP path against the CPU oracle (oracle/lucene_oracle.c).

Bars:
  * ORDER_DEVICE oracle (the documented lane summation order): hit docs AND score bits identical.
  * byte vectors: exact int32 sums, so scores/docs identical to Lucene's arithmetic in any order.
  * ORDER_PANAMA512 / ORDER_SCALAR oracle (Lucene's own summation orders): scores within
    REL_TOL = 1e-5 relative (north_star), docs identical except swaps between hits whose oracle
    scores differ by ≤ TIE_ULPS ulps (a near-tie can legitimately reorder under another order).
Scoring parity vs Lucene itself is unpinned (no Lucene jar in the reference) — see DESIGN.md.
"""
import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

REL_TOL = 1e-5
TIE_ULPS = 8

F32, I8 = LU.VectorEncoding.FLOAT32, LU.VectorEncoding.BYTE
SIMS = [LU.VectorSimilarityFunction(s) for s in range(4)]


def corpus(n, dim, sim, seed, enc=F32):
    if enc == I8:
        return O.synth(0, n, dim, seed, 4)
    dist = 1 if sim == LU.VectorSimilarityFunction.EUCLIDEAN else 3
    if sim == LU.VectorSimilarityFunction.MAXIMUM_INNER_PRODUCT:
        dist = 2
    return O.synth(0, n, dim, seed, dist)


def bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


def assert_exact(reader, rows, queries, k, sim, accept=None, ord_to_doc=None, order=O.ORDER_DEVICE):
    s, d, c, v = reader.search_batch(queries, k, None if accept is None else O.bits_from_bool(accept))
    ab = None if accept is None else O.bits_from_bool(accept)
    for i in range(len(queries)):
        os_, od, ov = O.exact_search(rows, queries[i], k, int(sim), order, ord_to_doc=ord_to_doc, accept_bits=ab)
        assert c[i] == len(od), (i, c[i], len(od))
        assert np.array_equal(d[i, : c[i]], od), (i, d[i, : c[i]], od)
        assert bits_equal(s[i, : c[i]], os_), (i, s[i, : c[i]], os_)
        assert v[i] == ov
        assert np.all(np.isneginf(s[i, c[i]:])) and np.all(d[i, c[i]:] == 2**31 - 1)


@pytest.mark.parametrize("dim", [1, 3, 17, 96, 100, 128, 256, 384, 768, 1024, 1536, 4096])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_f32_bit_exact_device_order(dim, sim):
    n = 1500 + dim % 7
    rows = corpus(n, dim, sim, 11)
    queries = corpus(5, dim, sim, 12)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        assert_exact(r, rows, queries, 10, sim)
    finally:
        r.close()


@pytest.mark.parametrize("dim", [16, 100, 768])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_i8_exact(dim, sim):
    rows = corpus(2000, dim, sim, 21, I8)
    queries = corpus(4, dim, sim, 22, I8)
    r = LU.GpuFlatVectorsReader("v", rows, sim, I8)
    try:
        assert_exact(r, rows, queries, 10, sim)
    finally:
        r.close()


@pytest.mark.parametrize("stream", [1, 0], ids=["i8_stream", "scan_i8"])
@pytest.mark.parametrize("dim", [1, 15, 64, 96, 100, 257, 512, 768, 1000, 2048, 4096])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_i8_single_query_stream(dim, sim, stream):
    """One byte query per search, no filter: scan_i8_stream (exact-width lanes, 4 row groups in flight)
    and scan_i8 both equal the oracle; ragged row counts leave partial row groups at wave ends."""
    rows = corpus(3000 + dim % 13, dim, sim, 23, I8)
    queries = corpus(3, dim, sim, 24, I8)
    r = LU.GpuFlatVectorsReader("v", rows, sim, I8)
    _lib.tune("i8_stream", stream)
    try:
        for i in range(len(queries)):
            assert_exact(r, rows, queries[i: i + 1], 10 if i else 64, sim)
        rd = np.sort(np.random.default_rng(dim).choice(9000, len(rows), replace=False)).astype(np.int32)
        sp = LU.GpuFlatVectorsReader("v", rows, sim, I8, ord_to_doc=rd, max_doc=9000)
        try:
            assert_exact(sp, rows, queries[:1], 10, sim, ord_to_doc=rd)
        finally:
            sp.close()
    finally:
        _lib.tune("i8_stream", 1)
        r.close()


@pytest.mark.parametrize("nq", [1, 2, 3, 4, 7, 8, 9, 13, 32])
@pytest.mark.parametrize("dim", [128, 768])
def test_batch_sizes_same_bits(nq, dim):
    """Scores do not depend on how queries are batched (lane layout depends on dim only)."""
    sim = LU.VectorSimilarityFunction.COSINE
    rows = corpus(4000, dim, sim, 31)
    queries = corpus(nq, dim, sim, 32)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        s_all, d_all, _, _ = r.search_batch(queries, 10)
        for i in range(nq):
            s1, d1, _, _ = r.search_batch(queries[i : i + 1], 10)
            assert np.array_equal(d1[0], d_all[i]) and bits_equal(s1[0], s_all[i])
        assert_exact(r, rows, queries, 10, sim)
    finally:
        r.close()


@pytest.mark.parametrize("k", [1, 2, 10, 33, 64])
def test_k_values(k):
    sim = LU.VectorSimilarityFunction.EUCLIDEAN
    rows = corpus(5000, 96, sim, 41)
    queries = corpus(3, 96, sim, 42)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        assert_exact(r, rows, queries, k, sim)
    finally:
        r.close()


def test_k_larger_than_segment_and_tiny_segments():
    sim = LU.VectorSimilarityFunction.DOT_PRODUCT
    for n in [1, 2, 5, 63, 64, 65]:
        rows = corpus(n, 32, sim, 50 + n)
        q = corpus(2, 32, sim, 99)
        r = LU.GpuFlatVectorsReader("v", rows, sim)
        try:
            assert_exact(r, rows, q, 10, sim)
        finally:
            r.close()


def test_empty_segment():
    r = LU.GpuFlatVectorsReader("v", np.zeros((0, 8), np.float32), LU.VectorSimilarityFunction.EUCLIDEAN, max_doc=0)
    try:
        s, d, c, v = r.search_batch(np.ones((2, 8), np.float32), 5)
        assert list(c) == [0, 0] and list(v) == [0, 0]
    finally:
        r.close()


@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_exact_ties_lower_doc_wins(sim):
    """Duplicated vectors score identically; Lucene keeps / orders the lower doc first."""
    dim = 64
    base = corpus(300, dim, sim, 61)
    rows = np.concatenate([base, base[::-1], base[:50]], axis=0)   # every vector 2-3 times
    queries = np.concatenate([base[:2], corpus(2, dim, sim, 62)])  # some queries equal a row
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        assert_exact(r, rows, queries, 10, sim)
        s, d, c, _ = r.search_batch(queries, 10)
        for i in range(len(queries)):
            for j in range(c[i] - 1):
                assert s[i, j] > s[i, j + 1] or (s[i, j] == s[i, j + 1] and d[i, j] < d[i, j + 1])
    finally:
        r.close()


def test_constant_vectors_all_ties():
    dim = 24
    rows = np.ones((777, dim), np.float32)
    q = np.ones((1, dim), np.float32)
    for sim in SIMS:
        r = LU.GpuFlatVectorsReader("v", rows, sim)
        try:
            s, d, c, _ = r.search_batch(q, 10)
            assert list(d[0]) == list(range(10))
            assert_exact(r, rows, q, 10, sim)
        finally:
            r.close()


@pytest.mark.parametrize("selectivity", [0.0, 0.01, 0.1, 0.5, 1.0])
def test_filter_accept_bits(selectivity):
    sim = LU.VectorSimilarityFunction.COSINE
    rows = corpus(6000, 128, sim, 71)
    queries = corpus(3, 128, sim, 72)
    rng = np.random.default_rng(44)
    accept = rng.random(6000) < selectivity
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        assert_exact(r, rows, queries, 10, sim, accept=accept)
    finally:
        r.close()


def test_sparse_ord_to_doc_and_deletes():
    sim = LU.VectorSimilarityFunction.EUCLIDEAN
    n = 3000
    rng = np.random.default_rng(5)
    docs = np.sort(rng.choice(10000, n, replace=False)).astype(np.int32)
    rows = corpus(n, 48, sim, 81)
    queries = corpus(4, 48, sim, 82)
    live = rng.random(10000) < 0.8
    r = LU.GpuFlatVectorsReader("v", rows, sim, ord_to_doc=docs, max_doc=10000)
    try:
        assert_exact(r, rows, queries, 10, sim, ord_to_doc=docs)
        assert_exact(r, rows, queries, 10, sim, accept=live, ord_to_doc=docs)
    finally:
        r.close()


@pytest.mark.parametrize("order", [O.ORDER_PANAMA512, O.ORDER_SCALAR, O.ORDER_PANAMA512_NOFMA, O.ORDER_SCALAR_NOFMA],
                         ids=["panama512", "scalar", "panama512_nofma", "scalar_nofma"])
@pytest.mark.parametrize("sim", SIMS, ids=lambda s: s.name)
def test_lucene_orders_within_tolerance(order, sim):
    dim = 768
    rows = corpus(3000, dim, sim, 91)
    queries = corpus(4, dim, sim, 92)
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    try:
        s, d, c, _ = r.search_batch(queries, 10)
        for i in range(len(queries)):
            os_, od, _ = O.exact_search(rows, queries[i], 10, int(sim), order)
            np.testing.assert_allclose(s[i, : c[i]], os_, rtol=REL_TOL, atol=0)
            if not np.array_equal(d[i, : c[i]], od):
                # only near-ties may swap: every mismatching position must sit on a near-tie
                for j in np.nonzero(d[i, : c[i]] != od)[0]:
                    gap = np.abs(os_[max(j - 1, 0): j + 2] - os_[j]).min(initial=np.inf) if len(os_) > 1 else 0
                    ulp = np.spacing(np.float32(os_[j]))
                    assert gap <= TIE_ULPS * ulp, (i, j, d[i], od)
    finally:
        r.close()


def test_device_synth_matches_host():
    for dist, enc in [(0, F32), (1, F32), (2, F32), (3, F32), (4, I8)]:
        r = LU.GpuFlatVectorsReader.synthetic("v", 1000, 100, LU.VectorSimilarityFunction.EUCLIDEAN, enc,
                                              seed=7, dist=dist, row0=123)
        rows = O.synth(123, 1000, 100, 7, dist)
        q = O.synth(5000, 3, 100, 8, dist)
        try:
            assert_exact(r, rows, q, 10, LU.VectorSimilarityFunction.EUCLIDEAN)
        finally:
            r.close()


def test_multi_segment_multi_shard_merge():
    """Several shards × segments in one device view == per-leaf oracle exact search, per-leaf
    TopDocs.merge into the shard top-k, and the coordinator's TopDocs.merge(from, size)."""
    sim = LU.VectorSimilarityFunction.DOT_PRODUCT
    dim = 128
    rng = np.random.default_rng(3)
    shard_specs = [[700, 1300], [2500], [64, 1, 900], [1000]]   # rows per segment
    shard_leaves, rows_of = [], {}
    seed = 100
    for segs in shard_specs:
        leaves, base = [], 0
        for i, n in enumerate(segs):
            rows = corpus(n, dim, sim, seed)
            seed += 1
            live = rng.random(n) < 0.9
            reader = LU.GpuFlatVectorsReader("v", rows, sim)
            leaves.append(LU.LeafReaderContext(i, base, reader, live))
            rows_of[id(leaves[-1])] = rows
            base += n
        shard_leaves.append(leaves)
    shard_index = [2, 0, 3, 1]
    ds = LU.DeviceShardSet(shard_leaves, shard_index)
    queries = corpus(6, dim, sim, 555)
    for k, from_, size in [(10, 0, 10), (10, 5, 5), (10, 0, 3), (5, 2, 10), (64, 10, 30)]:
        s, d, sh, cnt, tot, mx = ds.search(queries, k, from_, size, accept=[lf.live_docs for lf in ds.leaves])
        for qi in range(len(queries)):
            shard_hits = []
            for leaves in shard_leaves:
                per_leaf = []
                for lf in leaves:
                    os_, od, _ = O.exact_search(rows_of[id(lf)], queries[qi], k, int(sim),
                                                O.ORDER_DEVICE, accept_bits=O.bits_from_bool(lf.live_docs))
                    per_leaf.append((os_, od + lf.doc_base))
                ms, md, _, _, _ = O.topdocs_merge(per_leaf, 0, k, shard_index=[0] * len(per_leaf))
                shard_hits.append((ms, md))
            es, ed, esh, etot, emx = O.topdocs_merge(shard_hits, from_, size, shard_index=shard_index)
            n = len(ed)
            assert cnt[qi] == n
            assert np.array_equal(d[qi, :n], ed) and np.array_equal(sh[qi, :n], esh)
            assert bits_equal(s[qi, :n], es)
            assert tot[qi] == etot
            assert bits_equal([mx[qi]], [emx])
    ds.close()
    for leaves in shard_leaves:
        for lf in leaves:
            lf.reader.close()


def test_knn_query_rewrite_mirror():
    """KnnFloatVectorQuery.rewrite over leaves (per-leaf search + TopDocs.merge(k))."""
    sim = LU.VectorSimilarityFunction.EUCLIDEAN
    sizes = [500, 1200, 33]
    leaves, all_rows, base = [], [], 0
    for i, n in enumerate(sizes):
        rows = corpus(n, 40, sim, 300 + i)
        leaves.append(LU.LeafReaderContext(i, base, LU.GpuFlatVectorsReader("v", rows, sim)))
        all_rows.append(rows)
        base += n
    q = corpus(1, 40, sim, 400)[0]
    td = LU.KnnFloatVectorQuery("v", q, 10).rewrite(leaves)
    os_, od, _ = O.exact_search(np.concatenate(all_rows), q, 10, int(sim))
    assert [h.doc for h in td.score_docs] == list(od)
    assert bits_equal([h.score for h in td.score_docs], os_)
    for lf in leaves:
        lf.reader.close()


def test_errors_are_codes_not_crashes():
    r = LU.GpuFlatVectorsReader("v", np.ones((10, 8), np.float32), LU.VectorSimilarityFunction.EUCLIDEAN)
    try:
        with pytest.raises(_lib.OskError):
            r.search_batch(np.ones((1, 8), np.float32), 0)
        with pytest.raises(_lib.OskError):
            r.search_batch(np.ones((1, 8), np.float32), _lib.OSK_MAX_K + 1)
        with pytest.raises(ValueError):
            r.search_batch(np.ones((1, 9), np.float32), 5)
    finally:
        r.close()


def _rand_lists(rng, world, nq, sl, k, tie_every=0):
    """Rank-major gathered image [world·nq, sl, k] of random best-first, zero-padded key lists."""
    keys = np.zeros((world * nq, sl, k), np.uint64)
    for r in range(world):
        for q in range(nq):
            for j in range(sl):
                c = int(rng.integers(0, k + 1))
                sc = np.sort(rng.integers(0, 6, c) if tie_every else rng.random(c)).astype(np.float32)[::-1]
                docs = np.sort(rng.choice(1000, c, replace=False)).astype(np.int64)
                # same score → ascending doc inside one list (as a shard returns them)
                order = np.lexsort((docs, -sc.astype(np.float64)))
                sc, docs = sc[order], docs[order]
                u = sc.view(np.uint32).astype(np.uint64)
                sortable = np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
                keys[r * nq + q, j, :c] = (sortable << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - docs.astype(np.uint64))
    return keys


@pytest.mark.parametrize("world,sl,k,from_,size,ties", [(1, 8, 10, 0, 10, 0), (2, 4, 10, 5, 8, 0), (3, 3, 16, 0, 12, 1),
                                                         (8, 1, 10, 0, 10, 1), (4, 2, 64, 10, 30, 0)])
def test_merge_device_ranked_matches_host_reduce(world, sl, k, from_, size, ties):
    """osk_merge_device_ranked straight over an all-gather image == the host reduce of the same lists
    (counts = non-zero keys; shardIndex = the owner's global shard numbers, pads INT32_MAX)."""
    import torch
    from opensearch_amd import distributed as D
    rng = np.random.default_rng(world * 100 + sl)
    nq = 5
    keys = _rand_lists(rng, world, nq, sl, k, ties)
    si = torch.tensor(rng.permutation(world * sl).astype(np.int32))
    host = D.ShardExchange(world, sl, nq, k, from_, size, si)
    want = [t.clone() for t in host.reduce(torch.from_numpy(keys.view(np.int64)))]
    dev = D.ShardExchange(world, sl, nq, k, from_, size, si, device=0)
    got = dev.reduce(torch.from_numpy(keys.view(np.int64)).cuda())
    torch.cuda.synchronize()
    for w, g in zip(want, got):
        g = g.cpu()
        if w.dtype == torch.float32:
            assert torch.equal(w.view(torch.int32), g.view(torch.int32)), (w, g)
        else:
            assert torch.equal(w, g), (w, g)


def test_merge_device_reference_known_answers():
    """The reference's own merge known answers fed straight into the device coordinator reduce
    (osk_merge_device): SearchPhaseControllerTests.testReduceTopNWithFromOffset (:1347-1392),
    FetchSearchPhaseTests.testFetchTwoDocument (:124-218) and the constant-score shardIndex/doc
    tie order of testSortDocsIsIdempotent (:255-298); tests/golden/merge_known_answers.json."""
    import json
    from pathlib import Path
    import torch
    cases = json.loads((Path(__file__).parent / "golden" / "merge_known_answers.json").read_text())
    for case in cases:
        shards = case["shards"]
        S = len(shards)
        k = max([len(s["scores"]) for s in shards] + [1])
        keys = np.zeros((1, S, k), np.uint64)
        counts = np.zeros((1, S), np.int32)
        for j, s in enumerate(shards):
            c = len(s["scores"])
            counts[0, j] = c
            sc = np.asarray(s["scores"], np.float32).view(np.uint32).astype(np.uint64)
            sortable = np.where(sc & 0x80000000, (~sc) & 0xFFFFFFFF, sc | 0x80000000)
            keys[0, j, :c] = (sortable << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - np.asarray(s["docs"], np.uint64))
        si = np.asarray([s["shard_index"] for s in shards], np.int32)
        size = case["size"]
        d_keys = torch.from_numpy(keys.view(np.int64)).cuda()
        d_counts = torch.from_numpy(counts).cuda()
        d_si = torch.from_numpy(si).cuda()
        o_s = torch.empty((1, size), dtype=torch.float32, device="cuda")
        o_d = torch.empty((1, size), dtype=torch.int32, device="cuda")
        o_sh = torch.empty((1, size), dtype=torch.int32, device="cuda")
        o_c = torch.empty(1, dtype=torch.int32, device="cuda")
        o_t = torch.empty(1, dtype=torch.int64, device="cuda")
        o_m = torch.empty(1, dtype=torch.float32, device="cuda")
        _lib.check(_lib.lib().osk_merge_device(0, d_keys.data_ptr(), d_counts.data_ptr(), d_si.data_ptr(), 1, S, k,
                                               case["from"], size, o_s.data_ptr(), o_d.data_ptr(), o_sh.data_ptr(),
                                               o_c.data_ptr(), o_t.data_ptr(), o_m.data_ptr(), None))
        torch.cuda.synchronize()
        n = int(o_c.item())
        if "expected_scores" in case:
            assert o_s[0, :n].cpu().tolist() == case["expected_scores"], (case["name"], o_s)
        if "expected_docs" in case:
            assert o_d[0, :n].cpu().tolist() == case["expected_docs"], (case["name"], o_d)
            assert o_sh[0, :n].cpu().tolist() == case["expected_shards"], (case["name"], o_sh)
        assert int(o_t.item()) == case["expected_total_hits"]
        assert float(o_m.item()) == case["expected_max_score"]
