"""GPU parity in the large-view tile regime (the C3/C4/C5 headline regime, as benchmarked).

Views of at least CUs × tile_large_slots × tile_min_rows rows (256 × 24 × 1024 ≈ 6.29M on an
MI355X) get CUs × 24 workgroup tiles instead of whole rounds of 4 slots per CU (osk_view_create,
DESIGN.md §3c).  Every other GPU test uses views far below that size, so here a 6.5M × 128 COSINE
corpus in 8 shards (one segment each, generated on the device by the counter generator; the host
twin feeds the oracle) is searched through every path the bench takes — the single-query int8
prefilter (sq8_scan), the batched int8 MFMA prefilter (sq8_mfma), the fp32 streaming scan, a 1 %
filtered single query (the FQ instance) — and each query is compared against the oracle's
per-shard [L] exactSearch + coordinator TopDocs.merge (SearchPhaseController.java:224-246),
docs, shard indices and score bits.
"""
import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

N_SHARDS = 8
ROWS_PER_SHARD = 812_500          # 6.5M rows in total
DIM = 128
COS = LU.VectorSimilarityFunction.COSINE


@pytest.fixture(scope="module")
def big():
    readers = [LU.GpuFlatVectorsReader.synthetic("v", ROWS_PER_SHARD, DIM, COS, seed=42,
                                                 dist=_lib.DIST_NORMALISH_UNIT, row0=s * ROWS_PER_SHARD)
               for s in range(N_SHARDS)]
    shard_index = [3, 1, 4, 0, 6, 2, 7, 5]   # permuted sorted-ShardId ranks
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], shard_index)
    rows = O.synth(0, N_SHARDS * ROWS_PER_SHARD, DIM, 42, 3)
    yield ds, rows, shard_index
    ds.close()
    for r in readers:
        r.close()


def oracle_merge(rows, q, k, shard_index, accept=None):
    lists = []
    for s in range(N_SHARDS):
        part = rows[s * ROWS_PER_SHARD:(s + 1) * ROWS_PER_SHARD]
        ab = None if accept is None else O.bits_from_bool(accept[s])
        sc, dc, _ = O.exact_search(part, q, k, int(COS), accept_bits=ab)
        lists.append((sc, dc))
    return O.topdocs_merge(lists, 0, k, shard_index)


def check(out, rows, queries, k, shard_index, accept=None):
    s, d, sh, c, t, _ = out
    for i in range(len(queries)):
        es, ed, esh, et, _ = oracle_merge(rows, queries[i], k, shard_index, accept)
        assert c[i] == len(ed) == k
        assert np.array_equal(d[i], ed), (i, d[i], ed)
        assert np.array_equal(sh[i], esh), (i, sh[i], esh)
        assert np.array_equal(np.asarray(s[i], np.float32).view(np.uint32), es.view(np.uint32))


def test_large_view_is_in_the_large_tile_regime(big):
    import torch
    ds, _, _ = big
    # CUs × 24 tiles (6,144 on 256 CUs; the small-view rule would give 4 rounds = CUs × 16), 4 wave
    # lists per tile, settle slices of 32 lists that never span shards (768 lists per shard here)
    ds.search(O.synth(0, 1, DIM, 43, 3), 10, 0, 10)
    assert ds.counter("sq8_calls") >= 1
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert ds.counter("sq8_slices") * 32 == 4 * 24 * cus, (ds.counter("sq8_slices"), cus)


@pytest.mark.parametrize("nq", [1, 3])
def test_large_view_prefilter_single_and_batched(big, nq):
    ds, rows, si = big
    queries = O.synth(0, nq, DIM, 43 + nq, 3)
    calls = ds.counter("sq8_calls")
    out = ds.search(queries, 10, 0, 10)
    assert ds.counter("sq8_calls") == calls + 1
    check(out, rows, queries, 10, si)


def test_large_view_fp32_stream(big):
    ds, rows, si = big
    queries = O.synth(0, 2, DIM, 50, 3)
    _lib.tune("sq8", 0)
    try:
        out = ds.search(queries, 10, 0, 10)
    finally:
        _lib.tune("sq8", 1)
    check(out, rows, queries, 10, si)


def test_large_view_filtered_single_query(big):
    ds, rows, si = big
    rng = np.random.default_rng(5)
    accept = [rng.random(ROWS_PER_SHARD) < 0.01 for _ in range(N_SHARDS)]
    queries = O.synth(0, 2, DIM, 51, 3)
    for i in range(len(queries)):
        out = ds.search(queries[i:i + 1], 10, 0, 10, accept=accept)
        check(out, rows, queries[i:i + 1], 10, si, accept)
