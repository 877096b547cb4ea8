"""BASELINE.json configs[0] on the CPU: 100k × 128 fp32 EUCLIDEAN, one shard, k = 10, 1,000 queries through
`KnnFloatVectorQuery` (plumbing, no GPU).

This is the reference's own CPU route, restated with the host pieces of this repo:

* [L] `AbstractKnnVectorQuery.rewrite` → one `KnnVectorsReader.search` per leaf, docBase added, then
  `TopDocs.merge(k, perLeaf)` (`opensearch_amd/lucene.py` `_KnnVectorQuery.rewrite`; the merge runs in
  libosknn's host reduce `osk_topdocs_merge`);
* the shard's query phase, `numDocs = min(from + size, …)`
  (`server/src/main/java/org/opensearch/search/query/TopDocsCollectorContext.java:866-891`), reached from
  `ContextIndexSearcher.rewrite` (`server/src/main/java/org/opensearch/search/internal/ContextIndexSearcher.java:203-218`);
* the coordinator's `SearchPhaseController.mergeTopDocs`
  (`server/src/main/java/org/opensearch/action/search/SearchPhaseController.java:224-246`) over the one shard.

The per-leaf scorer stands where Lucene's CPU `exactSearch` stands: the oracle's Panama-512 order (Lucene's
`PanamaVectorUtilSupport`, the order a CPU run of the reference uses).  It is a test stand-in only — the
product reader (`GpuFlatVectorsReader`) needs a gfx950 device, and `tests/test_gpu_full_size.py::
test_c1_full_1k_queries` runs the same corpus and queries through it.  The expected answer is one exact search
over the whole 100k rows: splitting the shard into leaves must not change a doc, a score bit or the tie order.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

N, DIM, K, NQ = 100_000, 128, 10, 1_000
SEED_ROWS, SEED_QUERIES = 42, 43          # tools/bench_configs.py's C1 corpus and query pool
LEAVES = (0, 37_000, 71_500, N)           # three segments of the shard (ragged, not 64-aligned)


class _CpuFlatVectorsReader:
    """Test stand-in for a Lucene flat-vector reader on the CPU ([L] exactSearch, Panama order)."""

    def __init__(self, field, rows):
        self.field, self.rows = field, rows
        self.max_doc = len(rows)

    def search(self, field, target, k, accept_docs=None):
        assert field == self.field
        ab = None if accept_docs is None else O.bits_from_bool(accept_docs)
        sc, dc, vis = O.exact_search(self.rows, target, k, int(LU.VectorSimilarityFunction.EUCLIDEAN),
                                     O.ORDER_PANAMA512, accept_bits=ab)
        return LU.TopDocs(LU.TotalHits(vis), [LU.ScoreDoc(int(d), float(s)) for s, d in zip(sc, dc)])


@pytest.fixture(scope="module")
def c1():
    rows = O.synth(0, N, DIM, SEED_ROWS, _lib.DIST_UNIFORM01)
    queries = O.synth(0, NQ, DIM, SEED_QUERIES, _lib.DIST_UNIFORM01)
    leaves = [LU.LeafReaderContext(i, LEAVES[i], _CpuFlatVectorsReader("v", rows[LEAVES[i]:LEAVES[i + 1]]))
              for i in range(len(LEAVES) - 1)]
    sc, dc, cc = O.knn_batch(rows, queries, K, int(LU.VectorSimilarityFunction.EUCLIDEAN), O.ORDER_PANAMA512, 8)
    return rows, queries, leaves, (sc, dc, cc)


def _shard_phase(leaves, q, accept=None):
    flt = None if accept is None else (lambda leaf: accept[leaf.doc_base:leaf.doc_base + leaf.max_doc])
    query = LU.KnnFloatVectorQuery("v", q, K, filter=flt)
    return LU.shard_query_phase(query, leaves, 0, K)


def test_c1_all_1k_queries_through_knn_float_vector_query(c1):
    rows, queries, leaves, (sc, dc, cc) = c1
    with ThreadPoolExecutor(8) as ex:    # the search pool: queries run concurrently, each rewrite is per leaf
        got = list(ex.map(lambda i: _shard_phase(leaves, queries[i]), range(NQ)))
    for i, td in enumerate(got):
        assert cc[i] == K
        assert td.total_hits.value == K               # the rewritten DocAndScoreQuery matches k docs
        d = np.array([h.doc for h in td.score_docs], np.int32)
        s = np.array([h.score for h in td.score_docs], np.float32)
        assert np.array_equal(d, dc[i]), (i, d, dc[i])
        assert np.array_equal(s.view(np.uint32), sc[i].view(np.uint32)), i
    # the coordinator's mergeTopDocs over the one shard (shardIndex 0) keeps the shard's order
    for i in (0, 1, NQ - 1):
        ms, md, msh, tot, mx = O.topdocs_merge([(sc[i], dc[i])], 0, K, [0])
        assert np.array_equal(md, dc[i]) and np.all(msh == 0) and tot == K and mx == sc[i][0]


def test_c1_leaves_split_never_changes_the_answer_with_a_filter(c1):
    """A filter pushed into every leaf's AcceptDocs ([L] liveDocs ∩ filter) — the per-leaf route still equals
    one filtered exact search over the whole shard."""
    rows, queries, leaves, _ = c1
    acc = np.random.default_rng(5).random(N) < 0.3
    ab = O.bits_from_bool(acc)
    for i in range(0, NQ, 97):
        td = _shard_phase(leaves, queries[i], accept=acc)
        es, ed, _ = O.exact_search(rows, queries[i], K, int(LU.VectorSimilarityFunction.EUCLIDEAN),
                                   O.ORDER_PANAMA512, accept_bits=ab)
        assert [h.doc for h in td.score_docs] == ed.tolist()
        assert np.array_equal(np.array([h.score for h in td.score_docs], np.float32).view(np.uint32),
                              es.view(np.uint32))
