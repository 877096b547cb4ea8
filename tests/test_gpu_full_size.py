"""Oracle parity at the EXACT benchmarked sizes (BASELINE.json configs C3, C4, C5), not proxies.

`test_gpu_configs_at_size.py` covers every path at 6.5M rows; this file runs the configs at the sizes the
bench and `tools/bench_configs.py` time them, on the same corpora:

* C3: 10M × 768 COSINE, 8 shards × 1.25M (shard s = global rows [s·1.25M, (s+1)·1.25M)), the bench's own
  seeds (rows 42, queries 43, `bench.py`), shardIndex = shard number.  Batch 1 on the 6-bit tier (a
  calibration probe, then the steady state with `sq6_calls` asserted), batch 32 on the int8 MFMA
  prefilter, batch 256 on whichever path the library picks (sampled queries).
* C5: the C3 corpus under 1 % and 50 % Bernoulli filters (compacted gather scan), and the 10M × 768
  byte-vector corpus (EUCLIDEAN, `scan_i8_stream`), batch 1.
* C4: 100M × 96 DOT_PRODUCT, 8 shards × 12.5M: batch 1024 on the wide int8 prefilter (32 sampled
  queries), batch 1 and batch 32; the same size under MAXIMUM_INNER_PRODUCT (raw rows), b1024 and b1.
* C1: 100k × 128 EUCLIDEAN, one shard, all 1,000 queries through `GpuKnnFloatVectorQuery.rewrite`, Lucene's
  per-leaf `KnnFloatVectorQuery` route over the GPU reader, and one batched C-ABI call.
* C2: 1M × 128 EUCLIDEAN (SIFT-like), one shard, single queries on `sq8_scan`.

The sampled batches are then checked whole: every query of C3 b256 and C4 b1024 equals the fp32 streaming
scan (`sq8` off), itself bit-exact to the oracle at these sizes (b1 cases above).

Every check is docs, shard indices and score bits of the coordinator merge against the oracle's
per-shard [L] exactSearch (device summation order) + TopDocs.merge
(`server/src/main/java/org/opensearch/action/search/SearchPhaseController.java:224-246`).  The oracle
regenerates each shard on the host with the device generator's twin (`O.synth_par`), one shard at a time
(4.8 GB host peak at C4), and scores it on 16 threads.
"""
import os

import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N_SHARDS = 8
SHARD_INDEX = list(range(N_SHARDS))   # the bench's: shard s is the s-th ShardId
THREADS = max(1, min(16, os.cpu_count() or 1))
SIM = LU.VectorSimilarityFunction
K = 10


def _readers(rps, dim, sim, seed, dist, enc=LU.VectorEncoding.FLOAT32):
    return [LU.GpuFlatVectorsReader.synthetic("v", rps, dim, sim, enc, seed=seed, dist=dist, row0=s * rps)
            for s in range(N_SHARDS)]


def _oracle(rps, dim, sim, seed, dist, query_sets, accepts=None):
    """Per (query set, filter) the coordinator merge of every query, shard by shard on the host.
    accepts: None (unfiltered) or a list of per-shard bool masks; with several filters, one result per filter
    for each query set."""
    filt = [None] if accepts is None else accepts
    lists = [[[[] for _ in range(len(q))] for q in query_sets] for _ in filt]
    for s in range(N_SHARDS):
        rows = O.synth_par(s * rps, rps, dim, seed, dist, THREADS)
        print(f"oracle shard {s}/{N_SHARDS} ({rps}x{dim})", flush=True)   # progress for long runs
        for fi, acc in enumerate(filt):
            for qi, qs in enumerate(query_sets):
                if acc is not None or rows.dtype == np.int8:
                    ab = None if acc is None else O.bits_from_bool(acc[s])
                    for i in range(len(qs)):
                        sc, dc, _ = O.exact_search(rows, qs[i], K, int(sim), accept_bits=ab)
                        lists[fi][qi][i].append((sc, dc))
                else:
                    sc, dc, cc = O.knn_batch(rows, qs, K, int(sim), O.ORDER_DEVICE, THREADS)
                    for i in range(len(qs)):
                        lists[fi][qi][i].append((sc[i, :cc[i]], dc[i, :cc[i]]))
        del rows
    res = [[[O.topdocs_merge(ls, 0, K, SHARD_INDEX) for ls in per_q] for per_q in per_f] for per_f in lists]
    return res[0] if accepts is None else res


def _check(out, want, rows_idx):
    s, d, sh, c, t, _ = out
    for j, i in enumerate(rows_idx):
        es, ed, esh, et, _ = want[j]
        assert c[i] == len(ed) == K, (i, c[i], len(ed))
        assert np.array_equal(d[i], ed), (i, d[i], ed)
        assert np.array_equal(sh[i], esh), (i, sh[i], esh)
        assert np.array_equal(np.asarray(s[i], np.float32).view(np.uint32), es.view(np.uint32)), i
        assert t[i] == et, (i, t[i], et)


def _sample(n, m, seed):
    return np.sort(np.random.default_rng(seed).choice(n, size=m, replace=False))


def _counted(ds, queries, counters, accept=None):
    before = {c: ds.counter(c) for c in counters}
    out = ds.search(queries, K, 0, K, accept=accept)
    return out, {c: ds.counter(c) - before[c] for c in before}


# ---------------------------------------------------------------------------------------------------
# C3 (and C5's filters): 10M × 768 COSINE, the bench's corpus and queries
# ---------------------------------------------------------------------------------------------------
C3_RPS, C3_DIM = 1_250_000, 768
DIST_UNIT = _lib.DIST_NORMALISH_UNIT


@pytest.fixture(scope="module")
def c3():
    readers = _readers(C3_RPS, C3_DIM, SIM.COSINE, 42, DIST_UNIT)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], SHARD_INDEX)
    pool = O.synth(0, 256, C3_DIM, 43, DIST_UNIT)          # the bench's query pool (first 256 of seed 43)
    q = {"b1": pool[:6], "b32": pool[:32], "b256": pool}
    samp = {"b1": list(range(6)), "b32": list(range(32)), "b256": list(_sample(256, 16, 11))}
    rng = np.random.default_rng(17)
    accepts = [[rng.random(C3_RPS) < sel for _ in range(N_SHARDS)] for sel in (0.01, 0.10, 0.50)]
    fq = O.synth(0, 1, C3_DIM, 907, DIST_UNIT)
    names = list(q)
    res =_oracle(C3_RPS, C3_DIM, SIM.COSINE, 42, DIST_UNIT, [q[n][samp[n]] for n in names])
    want = dict(zip(names, res))
    filt = _oracle(C3_RPS, C3_DIM, SIM.COSINE, 42, DIST_UNIT, [fq], accepts=accepts)
    want["f1"], want["f10"], want["f50"] = filt[0][0], filt[1][0], filt[2][0]
    yield ds, q, samp, want, fq, accepts
    ds.close()
    for r in readers:
        r.close()


def test_c3_full_b1_6bit_tier_probe_then_steady_state(c3):
    """The headline path at the headline size: single queries on the 6-bit tier — the first ones are the
    segments' calibration probes, the later ones run after the calibration kept the tier."""
    ds, q, samp, want, _, _ = c3
    counters = ("sq8_calls", "mfma_calls", "sq6_calls", "sq8_fallback_queries")
    for i in range(6):   # queries 0..3 probe (4 probes per segment), 4..5 are the steady state
        out, d = _counted(ds, q["b1"][i:i + 1], counters)
        assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq6_calls": 1, "sq8_fallback_queries": 0}, (i, d)
        _check(out, [want["b1"][i]], [0])
    # the tier stayed on for every segment after the probes (state 1 = kept)
    out, d = _counted(ds, q["b1"][:1], counters)
    assert d["sq6_calls"] == 1
    _check(out, [want["b1"][0]], [0])


def test_c3_full_b32_int8_mfma(c3):
    ds, q, samp, want, _, _ = c3
    out, d = _counted(ds, q["b32"], ("sq8_calls", "mfma_calls"))
    assert d == {"sq8_calls": 1, "mfma_calls": 0}, d
    _check(out, want["b32"], samp["b32"])


def test_c3_full_b256_library_path(c3):
    ds, q, samp, want, _, _ = c3
    out, d = _counted(ds, q["b256"], ("sq8_calls", "mfma_calls", "sq8_wide_calls"))
    assert d["sq8_calls"] + d["mfma_calls"] == 1, d
    _check(out, want["b256"], samp["b256"])
    _equals_fp32_scan(ds, q["b256"], out)


_MFMA_MIN_BATCH = 96   # the library's default (osk_internal.h)


def _equals_fp32_scan(ds, queries, out):
    """Every query of the batch (not only the oracle's sample) against the fp32 streaming scan — the
    prefilter off, `scan_f32`'s exact device order — docs, shard indices and score bits."""
    _lib.tune("sq8", 0)
    _lib.tune("mfma_min_batch", 0)   # and not the bf16×3 blocks: scan_f32, ≤ 8 queries per launch
    try:
        ref = ds.search(queries, K, 0, K)
    finally:
        _lib.tune("sq8", 1)
        _lib.tune("mfma_min_batch", _MFMA_MIN_BATCH)
    for a, b in zip(out, ref):
        a, b = np.asarray(a), np.asarray(b)
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("which", ["f1", "f10", "f50"])
def test_c5_full_filtered_b1(c3, which):
    """C5: 1 %, 10 % and 50 % accept bitsets over the 10M corpus (compacted gather scan)."""
    ds, _, _, want, fq, accepts = c3
    acc = accepts[{"f1": 0, "f10": 1, "f50": 2}[which]]
    out, d = _counted(ds, fq, ("sq8_calls",), accept=acc)
    assert d == {"sq8_calls": 1}, d
    _check(out, want[which], [0])


def test_c5_full_int8_b1():
    """C5 byte vectors: 10M × 768 int8 EUCLIDEAN (exact int32 arithmetic: identical in every order)."""
    readers = _readers(C3_RPS, C3_DIM, SIM.EUCLIDEAN, 5150, _lib.DIST_INT8, LU.VectorEncoding.BYTE)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], SHARD_INDEX)
    try:
        q = O.synth(0, 2, C3_DIM, 801, _lib.DIST_INT8)
        want = _oracle(C3_RPS, C3_DIM, SIM.EUCLIDEAN, 5150, _lib.DIST_INT8, [q])[0]
        for i in range(2):
            _check(ds.search(q[i:i + 1], K, 0, K), [want[i]], [0])
    finally:
        ds.close()
        for r in readers:
            r.close()


# ---------------------------------------------------------------------------------------------------
# C4: 100M × 96 DOT_PRODUCT, 8 shards × 12.5M (tools/bench_configs.py's corpus: seed 42, unit rows)
# ---------------------------------------------------------------------------------------------------
def test_c4_full_b1024_wide_b32_b1():
    rps, dim = 12_500_000, 96
    readers = _readers(rps, dim, SIM.DOT_PRODUCT, 42, DIST_UNIT)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], SHARD_INDEX)
    counters = ("sq8_calls", "mfma_calls", "sq8_wide_calls", "sq8_fallback_queries")
    try:
        q1024 = O.synth(0, 1024, dim, 43, DIST_UNIT)
        s1024 = list(_sample(1024, 32, 12))
        q32 = O.synth(0, 32, dim, 44, DIST_UNIT)
        q1 = O.synth(0, 2, dim, 45, DIST_UNIT)
        w1024, w32, w1 = _oracle(rps, dim, SIM.DOT_PRODUCT, 42, DIST_UNIT, [q1024[s1024], q32, q1])
        out, d = _counted(ds, q1024, counters)
        assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq8_wide_calls": 1, "sq8_fallback_queries": 0}, d
        _check(out, w1024, s1024)
        _equals_fp32_scan(ds, q1024, out)
        out, d = _counted(ds, q32, counters)
        assert d["sq8_calls"] == 1 and d["sq8_wide_calls"] == 0, d
        _check(out, w32, range(32))
        for i in range(2):
            out, d = _counted(ds, q1[i:i + 1], counters)
            assert d["sq8_calls"] == 1, d
            _check(out, [w1[i]], [0])
    finally:
        ds.close()
        for r in readers:
            r.close()


def test_c4_full_mip_b1024_wide_b1():
    """C4 at its size under MAXIMUM_INNER_PRODUCT (raw, unnormalised rows: the score transform's two branches):
    b1024 on the wide kernel (32 sampled queries, then all 1,024 against the fp32 scan) and b1."""
    rps, dim, seed, dist = 12_500_000, 96, 4242, _lib.DIST_NORMALISH
    readers = _readers(rps, dim, SIM.MAXIMUM_INNER_PRODUCT, seed, dist)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], SHARD_INDEX)
    counters = ("sq8_calls", "mfma_calls", "sq8_wide_calls", "sq8_fallback_queries")
    try:
        q1024 = O.synth(0, 1024, dim, 46, dist)
        s1024 = list(_sample(1024, 32, 13))
        q1 = O.synth(0, 2, dim, 47, dist)
        w1024, w1 = _oracle(rps, dim, SIM.MAXIMUM_INNER_PRODUCT, seed, dist, [q1024[s1024], q1])
        out, d = _counted(ds, q1024, counters)
        assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq8_wide_calls": 1, "sq8_fallback_queries": 0}, d
        _check(out, w1024, s1024)
        _equals_fp32_scan(ds, q1024, out)
        for i in range(2):
            out, d = _counted(ds, q1[i:i + 1], counters)
            assert d["sq8_calls"] == 1 and d["sq8_wide_calls"] == 0, d
            _check(out, [w1[i]], [0])
    finally:
        ds.close()
        for r in readers:
            r.close()


# ---------------------------------------------------------------------------------------------------
# C1 (100k × 128 L2, one shard, 1k queries) and C2 batch 1 (1M × 128 L2): tools/bench_configs.py's corpora
# ---------------------------------------------------------------------------------------------------
def _one_shard_oracle(n, dim, seed, dist, queries):
    rows = O.synth_par(0, n, dim, seed, dist, THREADS)
    sc, dc, cc = O.knn_batch(rows, queries, K, int(SIM.EUCLIDEAN), O.ORDER_DEVICE, THREADS)
    return sc, dc, cc


def test_c1_full_1k_queries():
    """BASELINE configs[0] on the HIP path: all 1,000 queries (seeds 42 / 43) three ways —
    (1) the plugin's `GpuKnnFloatVectorQuery.rewrite` (one device call per shard, ContextIndexSearcher.rewrite,
        `server/src/main/java/org/opensearch/search/internal/ContextIndexSearcher.java:203-218`) over a shard
        of three segments, then the shard's query phase;
    (2) Lucene's per-leaf `KnnFloatVectorQuery.rewrite` over the same leaves (one `KnnVectorsReader.search`
        per leaf on the GPU reader, `TopDocs.merge(k, perLeaf)`);
    (3) one batched C-ABI call over the single-segment shard (`osk_view_search`, 1,000 queries).
    Each equals the oracle's exactSearch over the whole 100k rows: docs and score bits."""
    n, dim, nq = 100_000, 128, 1_000
    dist = _lib.DIST_UNIFORM01
    queries = O.synth(0, nq, dim, 43, dist)
    sc, dc, cc = _one_shard_oracle(n, dim, 42, dist, queries)
    assert np.all(cc == K)
    bounds = (0, 37_000, 71_500, n)
    segs = [LU.GpuFlatVectorsReader.synthetic("v", bounds[i + 1] - bounds[i], dim, SIM.EUCLIDEAN, seed=42,
                                              dist=dist, row0=bounds[i]) for i in range(3)]
    leaves = [LU.LeafReaderContext(i, bounds[i], segs[i]) for i in range(3)]
    whole = LU.GpuFlatVectorsReader.synthetic("v", n, dim, SIM.EUCLIDEAN, seed=42, dist=dist)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, whole)]], [0])
    try:
        def same(td, i):
            d = np.array([h.doc for h in td.score_docs], np.int32)
            s = np.array([h.score for h in td.score_docs], np.float32)
            assert np.array_equal(d, dc[i]), (i, d, dc[i])
            assert np.array_equal(s.view(np.uint32), sc[i].view(np.uint32)), i

        for i in range(nq):
            same(LU.shard_query_phase(LU.GpuKnnFloatVectorQuery("v", queries[i], K), leaves, 0, K), i)
        for i in range(0, nq, 7):          # the per-leaf route: 3 reader calls per query
            same(LU.KnnFloatVectorQuery("v", queries[i], K).rewrite(leaves), i)
        s, d, sh, c, t, _ = ds.search(queries, K, 0, K)
        assert np.all(c == K) and np.all(sh == 0)
        assert np.array_equal(d, dc) and np.array_equal(s.view(np.uint32), sc.view(np.uint32))
    finally:
        LU.GpuKnnFloatVectorQuery.release_views()
        ds.close()
        whole.close()
        for r in segs:
            r.close()


def test_c2_full_b1():
    """C2 batch 1: 1M × 128 SIFT-like EUCLIDEAN rows, single queries on `sq8_scan` (the bench's corpus and
    query pool)."""
    n, dim = 1_000_000, 128
    dist = _lib.DIST_UNIFORM01_X128
    q = O.synth(0, 8, dim, 43, dist)
    sc, dc, cc = _one_shard_oracle(n, dim, 42, dist, q)
    r = LU.GpuFlatVectorsReader.synthetic("v", n, dim, SIM.EUCLIDEAN, seed=42, dist=dist)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    try:
        for i in range(len(q)):
            out, d = _counted(ds, q[i:i + 1], ("sq8_calls", "mfma_calls", "sq8_wide_calls"))
            assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq8_wide_calls": 0}, d
            s, dd, sh, c, t, _ = out
            assert c[0] == K and np.array_equal(dd[0], dc[i]), (i, dd[0], dc[i])
            assert np.array_equal(s[0].view(np.uint32), sc[i].view(np.uint32)), i
    finally:
        ds.close()
        r.close()
