"""COSINE zero vectors score NaN, and a NaN is never a hit — on every device path.

[L] AbstractKnnVectorQuery.exactSearch collects a doc only when `score > topDoc.score` against a HitQueue prefilled
with −∞ sentinels, which is false for NaN, and drops the sentinels left over: a zero query under COSINE returns
no hit at all (every score is 0/0), and a zero row is visited but never collected.  The oracle restates exactly
that (`oracle/lucene_oracle.c` HitQueue); before round 6 the device paths kept NaN keys — the fp32 scan returned
one NaN hit for a zero query, the prefilter paths ten — found by tests/test_gpu_wide.py's zero-query case.

Every path is checked against the oracle's per-shard exactSearch + TopDocs.merge
(`server/src/main/java/org/opensearch/action/search/SearchPhaseController.java:224-246`): the fp32 scan (prefilter
off), sq8_scan (b1), the 6-bit tier (≥ 512 dims), sq8_mfma (b32), the wide kernels (b300, both), the select path
(k = 40) and byte COSINE vectors.
"""
import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu
COS = LU.VectorSimilarityFunction.COSINE


def _view(rows_list, shard_of, enc=LU.VectorEncoding.FLOAT32):
    n_shards = max(shard_of) + 1
    leaves = [[] for _ in range(n_shards)]
    readers, bases = [], [0] * n_shards
    for rows, s in zip(rows_list, shard_of):
        r = LU.GpuFlatVectorsReader("v", rows, COS, enc)
        readers.append(r)
        leaves[s].append(LU.LeafReaderContext(len(leaves[s]), bases[s], r))
        bases[s] += len(rows)
    return LU.DeviceShardSet(leaves, list(range(n_shards))), readers


def _oracle(rows_list, shard_of, q, k):
    lists = []
    for s in range(max(shard_of) + 1):
        rows = np.concatenate([rows_list[i] for i, t in enumerate(shard_of) if t == s])
        lists.append(O.exact_search(rows, q, k, int(COS))[:2])
    return O.topdocs_merge(lists, 0, k, list(range(len(lists))))


def _check(out, rows_list, shard_of, queries, k, idx):
    s, d, sh, c, t, _ = out
    for i in idx:
        es, ed, esh, et, _ = _oracle(rows_list, shard_of, queries[i], k)
        assert c[i] == len(ed), (i, c[i], len(ed))
        assert np.array_equal(d[i, :c[i]], ed) and np.array_equal(sh[i, :c[i]], esh), i
        assert np.array_equal(s[i, :c[i]].view(np.uint32), es.view(np.uint32)), i
        assert not np.isnan(s[i, :c[i]]).any()


def _data(dim, n_rows=(9000, 4001), seed=7, enc=LU.VectorEncoding.FLOAT32):
    dist = _lib.DIST_INT8 if enc == LU.VectorEncoding.BYTE else _lib.DIST_NORMALISH_UNIT
    rows_list = [O.synth(0, n, dim, seed + i, dist) for i, n in enumerate(n_rows)]
    for r in rows_list:
        r[::53] = 0          # zero rows: NaN under COSINE, never hits
    q = O.synth(0, 300, dim, seed + 9, dist)
    q[0] = 0                 # a zero query: no hit at all
    q[1] = rows_list[0][5]
    return rows_list, q


@pytest.mark.parametrize("dim", [96, 768])
def test_zero_vectors_every_float_path(dim):
    rows_list, q = _data(dim)
    shard_of = [0, 1]
    ds, readers = _view(rows_list, shard_of)
    try:
        # single queries: the fp32 scan (prefilter off), then the prefilter (sq8_scan; the 6-bit tier at 768 dims)
        for sq8 in (0, 1):
            _lib.tune("sq8", sq8)
            try:
                for i in (0, 1, 2):
                    _check(ds.search(q[i:i + 1], 10, 0, 10), rows_list, shard_of, q[i:i + 1], 10, [0])
            finally:
                _lib.tune("sq8", 1)
        _check(ds.search(q[:32], 10, 0, 10), rows_list, shard_of, q, 10, [0, 1, 2, 31])   # sq8_mfma
        for rows in (1, 0):   # the wide kernels (forced: the view is small)
            _lib.tune("sq8_wide_force", 1)
            _lib.tune("sq8_wide_rows", rows)
            try:
                _check(ds.search(q, 10, 0, 10), rows_list, shard_of, q, 10, [0, 1, 2, 299])
            finally:
                _lib.tune("sq8_wide_force", 0)
                _lib.tune("sq8_wide_rows", 1)
        _check(ds.search(q[:2], 40, 0, 40), rows_list, shard_of, q[:2], 40, [0, 1])   # the select path (k > 12)
    finally:
        ds.close()
        for r in readers:
            r.close()


def test_zero_vectors_byte_cosine():
    enc = LU.VectorEncoding.BYTE
    rows_list, q = _data(256, enc=enc)
    shard_of = [0, 1]
    ds, readers = _view(rows_list, shard_of, enc)
    try:
        for i in (0, 1, 2):
            _check(ds.search(q[i:i + 1], 10, 0, 10), rows_list, shard_of, q[i:i + 1], 10, [0])
        _check(ds.search(q[:8], 10, 0, 10), rows_list, shard_of, q[:8], 10, range(8))
    finally:
        ds.close()
        for r in readers:
            r.close()
