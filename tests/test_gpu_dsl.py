"""End to end through the plugin DSL on the GPU: a `knn_vector` mapping, documents in two shards of two
segments each, a `knn` query body with a filter over doc values → KnnQueryBuilder.do_to_query → the
Lucene query's per-leaf rewrite on the GPU readers → the shard collector cut → the coordinator's
TopDocs.merge — compared with the oracle's exactSearch over the same accepted docs."""
import numpy as np
import pytest

from opensearch_amd import dsl as Q, lucene as LU, search as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_knn_query_body_end_to_end():
    rng = np.random.default_rng(11)
    mapping = {"emb": {"type": "knn_vector", "dimension": 96, "space_type": "cosinesimil"},
               "color": "keyword", "price": "long"}
    ctx_map = {"emb": Q.parse_knn_vector_mapping("emb", mapping["emb"]), "color": "keyword", "price": "long"}
    shards = []
    for s in range(2):
        leaves, base = [], 0
        for g in range(2):
            n = int(rng.integers(3000, 6000))
            rows = np.stack([Q.parse_document_vector(ctx_map["emb"], v) for v in O.synth(0, n, 96, 20 + 2 * s + g, 3)])
            leaf = LU.LeafReaderContext(g, base, LU.GpuFlatVectorsReader("emb", rows, LU.VectorSimilarityFunction.COSINE))
            leaf.rows = rows
            leaf.colors = rng.choice(np.array(["red", "blue", "green"]), n)
            leaf.prices = rng.integers(0, 100, n)
            leaves.append(leaf)
            base += n
        shards.append(leaves)

    def doc_values(leaf, f):
        return {"color": leaf.colors, "price": leaf.prices}[f]

    ctx = Q.QueryShardContext(ctx_map, doc_values)
    q = O.synth(0, 1, 96, 99, 3)[0]
    body = {"knn": {"emb": {"vector": q.tolist(), "k": 25,
                            "filter": {"bool": {"must": [{"range": {"price": {"gte": 10, "lt": 70}}}],
                                                "must_not": [{"term": {"color": "blue"}}]}}}}}
    builder = Q.parse_query(body)
    size, from_ = 20, 3
    try:
        shard_results = []
        for si, leaves in enumerate(shards):
            query = builder.do_to_query(ctx)
            td = LU.shard_query_phase(query, leaves, from_, size)
            S.set_shard_index(td, si)
            shard_results.append(td)
        hits = S.sort_docs(False, shard_results, from_, size)
        # oracle
        lists = []
        for leaves in shards:
            per = []
            for leaf in leaves:
                m = (leaf.prices >= 10) & (leaf.prices < 70) & (leaf.colors != "blue")
                sc, dc, _ = O.exact_search(leaf.rows, q, 25, int(LU.VectorSimilarityFunction.COSINE),
                                           accept_bits=O.bits_from_bool(m))
                per.append((sc, dc + leaf.doc_base))
            ms, md, _, _, _ = O.topdocs_merge(per, 0, 25)
            lists.append((ms[: from_ + size], md[: from_ + size]))
        es, ed, esh, _, _ = O.topdocs_merge(lists, from_, size, [0, 1])
        assert [h.doc for h in hits] == ed.tolist()
        assert [h.shard_index for h in hits] == esh.tolist()
        assert np.array_equal(np.array([h.score for h in hits], np.float32).view(np.uint32), es.view(np.uint32))
    finally:
        for leaves in shards:
            for leaf in leaves:
                leaf.reader.close()
