"""Contract tests of the `knn_vector` mapper and the `knn` query builder (opensearch_amd/dsl.py), in the
shape of the reference's plugin contract suites: AbstractQueryTestCase (testFromXContent :129,
testToQuery :440, testSerialization :597) and MapperTestCase (:176-399).  CPU only: toQuery returns
the Lucene query objects; executing them is tests/test_gpu_dsl.py."""
import json

import numpy as np
import pytest

from opensearch_amd import dsl as Q
from opensearch_amd.lucene import KnnByteVectorQuery, KnnFloatVectorQuery, VectorEncoding, VectorSimilarityFunction


def random_builder(rng):
    dim = int(rng.integers(1, 64))
    filt = rng.choice([None, {"term": {"color": "red"}}, {"range": {"price": {"gte": 1, "lt": 9}}},
                       {"bool": {"must": [{"terms": {"tag": [1, 2]}}], "must_not": [{"term": {"color": "blue"}}]}}])
    return Q.KnnQueryBuilder("emb", rng.standard_normal(dim).astype(np.float32).tolist(), int(rng.integers(1, 10001)),
                             filt, float(rng.choice([1.0, 2.5])), rng.choice([None, "q1"]))


@pytest.mark.parametrize("seed", range(20))
def test_from_xcontent_round_trip(seed):
    b = random_builder(np.random.default_rng(seed))
    parsed = Q.parse_query(json.dumps(b.to_xcontent()))
    assert parsed == b


@pytest.mark.parametrize("seed", range(20))
def test_serialization_round_trip(seed):
    b = random_builder(np.random.default_rng(100 + seed))
    assert Q.KnnQueryBuilder.read_from(b.write_to()) == b


def test_parse_errors():
    bad = [{"knn": {}}, {"knn": {"a": {"vector": [1.0]}}}, {"knn": {"a": {"k": 3}}}, {"knn": {"a": {"vector": [1], "k": 0}}},
           {"knn": {"a": {"vector": [1], "k": 10001}}}, {"knn": {"a": {"vector": [], "k": 1}}},
           {"knn": {"a": {"vector": [1], "k": 1, "bogus": 1}}}, {"knn": {"a": {"vector": [1], "k": 1},
                                                                         "b": {"vector": [1], "k": 1}}},
           {"knn": {"a": {"vector": [1], "k": 1, "filter": {"script": {}}}}}, {"match": {}}]
    for body in bad:
        with pytest.raises(Q.ParsingException):
            Q.parse_query(body)


def test_mapping_parse_and_round_trip():
    ft = Q.parse_knn_vector_mapping("emb", {"type": "knn_vector", "dimension": 768, "space_type": "cosinesimil",
                                           "method": {"name": "flat", "engine": "gpu"}})
    assert (ft.dimension, ft.encoding, ft.similarity) == (768, VectorEncoding.FLOAT32, VectorSimilarityFunction.COSINE)
    assert Q.parse_knn_vector_mapping("emb", ft.to_xcontent()) == ft
    fb = Q.parse_knn_vector_mapping("b", {"type": "knn_vector", "dimension": 8, "data_type": "byte",
                                         "space_type": "innerproduct"})
    assert (fb.encoding, fb.similarity) == (VectorEncoding.BYTE, VectorSimilarityFunction.MAXIMUM_INNER_PRODUCT)
    for bad in [{"type": "dense_vector", "dimension": 3}, {"type": "knn_vector"}, {"type": "knn_vector", "dimension": 0},
                {"type": "knn_vector", "dimension": 5000}, {"type": "knn_vector", "dimension": 3, "space_type": "l1"},
                {"type": "knn_vector", "dimension": 3, "data_type": "half"},
                {"type": "knn_vector", "dimension": 3, "method": {"name": "hnsw"}},
                {"type": "knn_vector", "dimension": 3, "m": 16}]:
        with pytest.raises(Q.MapperParsingException):
            Q.parse_knn_vector_mapping("x", bad)


def test_document_vectors():
    ft = Q.parse_knn_vector_mapping("f", {"type": "knn_vector", "dimension": 3})
    assert Q.parse_document_vector(ft, [1, 2, 3]).dtype == np.float32
    fb = Q.parse_knn_vector_mapping("b", {"type": "knn_vector", "dimension": 2, "data_type": "byte"})
    assert Q.parse_document_vector(fb, [-128, 127]).tolist() == [-128, 127]
    for ftx, v in [(ft, [1, 2]), (ft, [1, float("nan"), 2]), (fb, [1.5, 2]), (fb, [200, 0])]:
        with pytest.raises(Q.MapperParsingException):
            Q.parse_document_vector(ftx, v)


def test_to_query():
    ctx = Q.QueryShardContext({"emb": Q.parse_knn_vector_mapping("emb", {"type": "knn_vector", "dimension": 4}),
                               "bytes": Q.parse_knn_vector_mapping("bytes", {"type": "knn_vector", "dimension": 4,
                                                                             "data_type": "byte"}),
                               "color": "keyword"},
                              doc_values=lambda leaf, f: np.zeros(leaf.max_doc))
    q = Q.KnnQueryBuilder("emb", [1, 2, 3, 4], 5, {"term": {"color": "x"}}).do_to_query(ctx)
    assert isinstance(q, KnnFloatVectorQuery) and q.k == 5 and q.target.dtype == np.float32 and q.filter is not None
    qb = Q.KnnQueryBuilder("bytes", [1, 2, 3, 4], 3).do_to_query(ctx)
    assert isinstance(qb, KnnByteVectorQuery) and qb.target.dtype == np.int8 and qb.filter is None
    with pytest.raises(Q.QueryShardException, match="invalid dimension"):
        Q.KnnQueryBuilder("emb", [1, 2, 3], 5).do_to_query(ctx)
    with pytest.raises(Q.QueryShardException, match="not knn_vector"):
        Q.KnnQueryBuilder("color", [1, 2, 3, 4], 5).do_to_query(ctx)
    with pytest.raises(Q.QueryShardException, match="failed to find field"):
        Q.KnnQueryBuilder("nope", [1, 2, 3, 4], 5).do_to_query(ctx)
