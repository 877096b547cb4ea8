"""Oracle parity at the benchmarked sizes, in the large-tile regime, for every BASELINE config.

Every view here is at least CUs × 24 × 1,024 rows (≈ 6.29M on an MI355X, the large-tile rule of
osk_view_create) or is the benchmarked config itself, and each path the bench takes at
that size is checked against the oracle — docs, shard indices and score bits of the coordinator merge:

* C3-shaped 6.5M × 768 COSINE, 8 shards: batch 1 on the 6-bit tier (sq6_pilot + sq6_scan + the int8
  re-bound, DESIGN.md §3f — the headline kernel), both on a calibration probe and in the steady state
  after the segments' calibration has kept the tier, batch 32 on
  the int8 MFMA prefilter (sq8_mfma, register path at 768 dims), batches 128 / 160 / 192 / 256 on
  whichever path the library's cost model picks (the wide int8 prefilter at KS = 12; the test restates
  the model and asserts the choice), b256 also forced onto the bf16×3 MFMA candidate path, and a
  10 %-filtered single query (compacted gather scan);
* C4-shaped 6.5M × 96, DOT_PRODUCT and MAXIMUM_INNER_PRODUCT: batches 32 and 1024 on the LDS-DMA
  ring instance of sq8_mfma;
* C2 1M × 128 EUCLIDEAN (SIFT-like), one shard, batch 256 on bf16×3;
* C5 int8 6.5M × 768 EUCLIDEAN byte vectors, batch 1 on scan_i8_stream.

Large batches check a sample of their queries (every query of the batch is computed in the same
launches).  The corpora are generated on the device by the counter generator and shard by shard on
the host by its twin (O.synth), so host memory stays at one shard.  The oracle is the per-shard
[L] exactSearch (O.knn_batch, device summation order, multi-threaded) and the coordinator
TopDocs.merge (SearchPhaseController.java:224-246).
"""
import os

import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N_SHARDS = 8
SHARD_INDEX = [3, 1, 4, 0, 6, 2, 7, 5]      # permuted sorted-ShardId ranks
THREADS = max(1, min(16, os.cpu_count() or 1))
SIM = LU.VectorSimilarityFunction


def _readers(rows_per_shard, dim, sim, seed, dist, enc=LU.VectorEncoding.FLOAT32):
    return [LU.GpuFlatVectorsReader.synthetic("v", rows_per_shard, dim, sim, enc, seed=seed, dist=dist,
                                              row0=s * rows_per_shard) for s in range(N_SHARDS)]


def _oracle(rows_per_shard, dim, sim, seed, dist, query_sets, k, n_shards=N_SHARDS, shard_index=SHARD_INDEX,
            accept=None):
    """Per query set: the coordinator merge of every query, shard by shard on the host."""
    lists = [[[] for _ in range(len(q))] for q in query_sets]
    for s in range(n_shards):
        rows = O.synth(s * rows_per_shard, rows_per_shard, dim, seed, dist)
        print(f"oracle shard {s}/{n_shards} ({rows_per_shard}x{dim})", flush=True)   # progress for long runs
        for qi, qs in enumerate(query_sets):
            if accept is not None or rows.dtype == np.int8:
                for i in range(len(qs)):
                    ab = None if accept is None else O.bits_from_bool(accept[s])
                    sc, dc, _ = O.exact_search(rows, qs[i], k, int(sim), accept_bits=ab)
                    lists[qi][i].append((sc, dc))
            else:
                sc, dc, cc = O.knn_batch(rows, qs, k, int(sim), O.ORDER_DEVICE, THREADS)
                for i in range(len(qs)):
                    lists[qi][i].append((sc[i, :cc[i]], dc[i, :cc[i]]))
        del rows
    return [[O.topdocs_merge(ls, 0, k, shard_index) for ls in per_q] for per_q in lists]


def _check(out, want, rows_idx, k):
    s, d, sh, c, t, _ = out
    for j, i in enumerate(rows_idx):
        es, ed, esh, et, _ = want[j]
        assert c[i] == len(ed) == k, (i, c[i], len(ed))
        assert np.array_equal(d[i], ed), (i, d[i], ed)
        assert np.array_equal(sh[i], esh), (i, sh[i], esh)
        assert np.array_equal(np.asarray(s[i], np.float32).view(np.uint32), es.view(np.uint32)), i
        assert t[i] == et


def _sample(n, m, seed):
    return np.sort(np.random.default_rng(seed).choice(n, size=m, replace=False))


# ---- the library's path cost model, restated (osk_api.hip view_search_device) -------
def _wide_ks(dim):
    u8 = (dim + 15) // 16
    return 2 if u8 <= 8 else 4 if u8 <= 16 else 8 if u8 <= 32 else 12


def _wide_us(rows, dim, nq):
    return ((nq + 255) // 256) * (rows * _wide_ks(dim) * 0.031e-3 + 300.0)


def _narrow_us(rows, dim, nq):
    return ((nq + 31) // 32) * (rows * (16.0 * ((dim + 15) // 16) + 16.0) / 4.3e6 + 165.0 + 0.28 * dim)


def _takes_wide(rows, dim, nq):
    """osk_api.hip sq8_wide_pick: unfiltered batches of >= 64 queries of <= 768 dims, when cheaper."""
    return dim <= 768 and nq >= 64 and _wide_us(rows, dim, nq) <= _narrow_us(rows, dim, nq)


def _takes_bf16x3(rows, dim, nq, k=10):
    if nq < 96 or k > 12:
        return False
    sq8_us = _wide_us(rows, dim, nq) if _takes_wide(rows, dim, nq) else _narrow_us(rows, dim, nq)
    bf_us = ((nq + 255) // 256) * (rows * (0.153 + 0.00119 * dim) * 1e-3 + 325.0)
    return bf_us <= sq8_us


# ---------------------------------------------------------------------------------------------------
# C3-shaped: 6.5M × 768 COSINE, 8 shards
# ---------------------------------------------------------------------------------------------------
C3_RPS, C3_DIM, C3_SEED = 812_500, 768, 4242


@pytest.fixture(scope="module")
def c3():
    readers = _readers(C3_RPS, C3_DIM, SIM.COSINE, C3_SEED, _lib.DIST_NORMALISH_UNIT)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], SHARD_INDEX)
    q = {"b1": O.synth(0, 1, C3_DIM, 501, 3), "b32": O.synth(0, 32, C3_DIM, 502, 3),
         "b256": O.synth(0, 256, C3_DIM, 503, 3), "b128": O.synth(0, 128, C3_DIM, 504, 3),
         "b160": O.synth(0, 160, C3_DIM, 505, 3), "b192": O.synth(0, 192, C3_DIM, 506, 3)}
    samp = {"b1": [0], "b32": list(range(32)), "b256": list(_sample(256, 16, 1)), "b128": list(_sample(128, 8, 2)),
            "b160": list(_sample(160, 8, 3)), "b192": list(_sample(192, 8, 4))}
    names = list(q)
    want = _oracle(C3_RPS, C3_DIM, SIM.COSINE, C3_SEED, 3, [q[n][samp[n]] for n in names], 10)
    yield ds, q, samp, dict(zip(names, want))
    ds.close()
    for r in readers:
        r.close()


def _search_counted(ds, queries, k=10, counters=("sq8_calls", "mfma_calls")):
    before = {c: ds.counter(c) for c in counters}
    out = ds.search(queries, k, 0, k)
    return out, {c: ds.counter(c) - before[c] for c in before}


def test_c3_b1_6bit_tier_probe_and_steady_state(c3):
    """The headline path at C3 shape: a single query on the 6-bit tier, first as one of the segments'
    calibration probes, then again once the calibration (4 probes, folded asynchronously by later calls)
    has kept the tier — both equal the oracle bit for bit."""
    ds, q, samp, want = c3
    counters = ("sq8_calls", "mfma_calls", "sq6_calls")
    out, d = _search_counted(ds, q["b1"], counters=counters)
    assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq6_calls": 1}, d
    _check(out, want["b1"], samp["b1"], 10)
    for i in range(5):   # more probes (the 5th call folds the 4th), other queries
        ds.search(q["b32"][i:i + 1], 10, 0, 10)
    out, d = _search_counted(ds, q["b1"], counters=counters)
    assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq6_calls": 1}, d   # the calibration kept the tier
    _check(out, want["b1"], samp["b1"], 10)


def test_c3_b32_sq8_mfma(c3):
    ds, q, samp, want = c3
    out, d = _search_counted(ds, q["b32"])
    assert d == {"sq8_calls": 1, "mfma_calls": 0}
    _check(out, want["b32"], samp["b32"], 10)


def test_c3_b256_wide_and_bf16x3(c3):
    """C3 b256: the cost model's pick is the wide int8 prefilter at 768 dims (KS = 12, one corpus pass per 256
    queries); bf16×3 forced (the prefilter priced out) equals the oracle too."""
    ds, q, samp, want = c3
    counters = ("sq8_calls", "mfma_calls", "sq8_wide_calls")
    assert _takes_wide(N_SHARDS * C3_RPS, C3_DIM, 256) and not _takes_bf16x3(N_SHARDS * C3_RPS, C3_DIM, 256)
    out, d = _search_counted(ds, q["b256"], counters=counters)
    assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq8_wide_calls": 1}, d
    _check(out, want["b256"], samp["b256"], 10)
    _lib.tune("sq8_cost_pct", 100000)
    try:
        out, d = _search_counted(ds, q["b256"], counters=counters)
    finally:
        _lib.tune("sq8_cost_pct", 100)
    assert d == {"sq8_calls": 0, "mfma_calls": 1, "sq8_wide_calls": 0}, d
    _check(out, want["b256"], samp["b256"], 10)


@pytest.mark.parametrize("b", [128, 160, 192])
def test_c3_path_choice_follows_the_cost_model(c3, b):
    ds, q, samp, want = c3
    rows = N_SHARDS * C3_RPS
    wide, bf = _takes_wide(rows, C3_DIM, b), _takes_bf16x3(rows, C3_DIM, b)
    assert wide and not bf   # 768-dim batches of ≥ 64 take the wide kernel
    out, d = _search_counted(ds, q[f"b{b}"], counters=("sq8_calls", "mfma_calls", "sq8_wide_calls"))
    assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq8_wide_calls": 1}, d
    _check(out, want[f"b{b}"], samp[f"b{b}"], 10)


def test_c3_filtered_10pct_single_query(c3):
    ds, _, _, _ = c3
    rng = np.random.default_rng(7)
    accept = [rng.random(C3_RPS) < 0.10 for _ in range(N_SHARDS)]
    qs = O.synth(0, 1, C3_DIM, 507, 3)
    want = _oracle(C3_RPS, C3_DIM, SIM.COSINE, C3_SEED, 3, [qs], 10, accept=accept)[0]
    out = ds.search(qs, 10, 0, 10, accept=accept)
    _check(out, want, [0], 10)


# ---------------------------------------------------------------------------------------------------
# C4-shaped: 6.5M × 96, DOT_PRODUCT (unit rows) and MAXIMUM_INNER_PRODUCT (raw rows); the ring sq8_mfma
# ---------------------------------------------------------------------------------------------------
C4_RPS, C4_DIM = 812_500, 96


@pytest.mark.parametrize("sim,dist", [(SIM.DOT_PRODUCT, _lib.DIST_NORMALISH_UNIT),
                                      (SIM.MAXIMUM_INNER_PRODUCT, _lib.DIST_NORMALISH)])
def test_c4_prefilter_b32_sq8_mfma_b1024_wide(sim, dist):
    """C4 shape: b32 on sq8_mfma (the LDS-DMA ring), b1024 on the wide kernel (four launches of 256, each one
    corpus pass) — the cost model's picks at this size and at C4's own 100M rows — and b1024 forced onto
    bf16×3; all equal the oracle bit for bit."""
    seed = 9600 + int(sim)
    readers = _readers(C4_RPS, C4_DIM, sim, seed, dist)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], SHARD_INDEX)
    counters = ("sq8_calls", "mfma_calls", "sq8_wide_calls")
    try:
        q32 = O.synth(0, 32, C4_DIM, 601, dist)
        q1024 = O.synth(0, 1024, C4_DIM, 602, dist)
        s1024 = list(_sample(1024, 32, 5))
        want32, want1024 = _oracle(C4_RPS, C4_DIM, sim, seed, dist, [q32, q1024[s1024]], 10)
        out, d = _search_counted(ds, q32, counters=counters)
        assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq8_wide_calls": 0}, d
        _check(out, want32, range(32), 10)
        for rows in (N_SHARDS * C4_RPS, 100_000_000):
            assert _takes_wide(rows, C4_DIM, 1024) and not _takes_bf16x3(rows, C4_DIM, 1024)
        assert not _takes_wide(100_000_000, C4_DIM, 32)
        out, d = _search_counted(ds, q1024, counters=counters)
        assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq8_wide_calls": 1}, d
        assert ds.counter("sq8_fallback_queries") == 0
        _check(out, want1024, s1024, 10)
        _lib.tune("sq8_cost_pct", 100000)   # the prefilter priced out: bf16×3 blocks
        try:
            out, d = _search_counted(ds, q1024, counters=counters)
        finally:
            _lib.tune("sq8_cost_pct", 100)
        assert d == {"sq8_calls": 0, "mfma_calls": 1, "sq8_wide_calls": 0}, d
        _check(out, want1024, s1024, 10)
    finally:
        ds.close()
        for r in readers:
            r.close()


# ---------------------------------------------------------------------------------------------------
# C2: SIFT-shaped 1M × 128 EUCLIDEAN, one shard, batch 256 on bf16×3
# ---------------------------------------------------------------------------------------------------
def test_c2_b256_wide_and_bf16x3():
    """C2 b256: the cost model's pick is the wide int8 prefilter (one corpus pass, 0.39 ms against bf16×3's
    0.46); bf16×3 forced (the prefilter priced out) equals the oracle too."""
    rows_n, dim, seed = 1_000_000, 128, 1280
    r = LU.GpuFlatVectorsReader.synthetic("v", rows_n, dim, SIM.EUCLIDEAN, seed=seed, dist=_lib.DIST_UNIFORM01_X128)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    counters = ("sq8_calls", "mfma_calls", "sq8_wide_calls")
    try:
        q = O.synth(0, 256, dim, 701, _lib.DIST_UNIFORM01_X128)
        samp = list(_sample(256, 16, 6))
        assert _takes_wide(rows_n, dim, 256) and not _takes_bf16x3(rows_n, dim, 256)
        want = _oracle(rows_n, dim, SIM.EUCLIDEAN, seed, _lib.DIST_UNIFORM01_X128, [q[samp]], 10, n_shards=1,
                       shard_index=[0])[0]
        out, d = _search_counted(ds, q, counters=counters)
        assert d == {"sq8_calls": 1, "mfma_calls": 0, "sq8_wide_calls": 1}, d
        _check(out, want, samp, 10)
        _lib.tune("sq8_cost_pct", 100000)
        try:
            out, d = _search_counted(ds, q, counters=counters)
        finally:
            _lib.tune("sq8_cost_pct", 100)
        assert d == {"sq8_calls": 0, "mfma_calls": 1, "sq8_wide_calls": 0}, d
        _check(out, want, samp, 10)
    finally:
        ds.close()
        r.close()


# ---------------------------------------------------------------------------------------------------
# C5 int8: 6.5M × 768 EUCLIDEAN byte vectors, batch 1 on scan_i8_stream
# ---------------------------------------------------------------------------------------------------
def test_c5_int8_stream_b1():
    rps, dim, seed = 812_500, 768, 5150
    readers = _readers(rps, dim, SIM.EUCLIDEAN, seed, _lib.DIST_INT8, LU.VectorEncoding.BYTE)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], SHARD_INDEX)
    try:
        q = O.synth(0, 2, dim, 801, _lib.DIST_INT8)
        want = _oracle(rps, dim, SIM.EUCLIDEAN, seed, _lib.DIST_INT8, [q], 10)[0]
        for i in range(2):
            out = ds.search(q[i:i + 1], 10, 0, 10)
            _check(out, [want[i]], [0], 10)
    finally:
        ds.close()
        for r in readers:
            r.close()
