"""The coordinator reduce mirror (opensearch_amd/search.py) against the reference's own tests:
SearchPhaseControllerTests (server/src/test/java/org/opensearch/action/search/
SearchPhaseControllerTests.java) and FetchSearchPhaseTests.java."""
import math

import numpy as np
import pytest

from opensearch_amd import lucene as LU
from opensearch_amd import search as SP
from oracle import oracle as O


def _result(shard, scores, docs=None, from_=0, size=10):
    docs = docs if docs is not None else [0] * len(scores)
    td = LU.TopDocs(LU.TotalHits(len(scores)), [LU.ScoreDoc(d, float(s)) for s, d in zip(scores, docs)])
    return SP.QuerySearchResult(shard, td, float(scores[0]) if len(scores) else math.nan, from_, size)


@pytest.mark.parametrize("batch", [2, 3, 4, 512])
def test_reduce_top_n_with_from_offset(batch):
    """testReduceTopNWithFromOffset (:1347-1392): 4 shards × 3 docs, scores 100…89, from 5, size 5."""
    c = SP.QueryPhaseResultConsumer(4, from_=5, size=5, batch_reduce_size=batch)
    score = 100
    for i in range(4):
        c.consume_result(_result(i, [score, score - 1, score - 2], from_=5, size=5))
        score -= 3
    r = c.reduce()
    assert [d.score for d in r.score_docs] == [95.0, 94.0, 93.0, 92.0, 91.0]
    assert r.max_score == 100.0 and r.total_hits.value == 12


@pytest.mark.parametrize("seed", range(5))
def test_consumer_only_hits(seed):
    """testConsumerOnlyHits (:1285-1333): one hit per shard, size 1 → the max score wins."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 100))
    c = SP.QueryPhaseResultConsumer(n, size=1, batch_reduce_size=int(rng.integers(2, 200)))
    mx = 0
    for i in range(n):
        num = int(rng.integers(1, 1001))
        mx = max(mx, num)
        c.consume_result(_result(i, [num], size=1))
    r = c.reduce()
    assert len(r.score_docs) == 1 and r.score_docs[0].score == mx
    assert r.max_score == mx and r.total_hits.value == n


def test_fetch_two_document_order():
    """FetchSearchPhaseTests.testFetchTwoDocument (:124-218): (42, 1.0) on shard 0, (84, 2.0) on 1."""
    c = SP.QueryPhaseResultConsumer(2)
    c.consume_result(_result(0, [1.0], [42]))
    c.consume_result(_result(1, [2.0], [84]))
    r = c.reduce()
    assert [d.doc for d in r.score_docs] == [84, 42] and r.total_hits.value == 2


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("constant", [False, True])
def test_sort_docs_idempotent_and_matches_oracle(seed, constant):
    """testSortDocsIsIdempotent (:255-298): same inputs → same docs/shards/scores; constant scores
    order by shardIndex then doc.  Also equals the oracle's TopDocs.merge."""
    rng = np.random.default_rng(seed)
    n_shards = int(rng.integers(1, 20))
    size = int(rng.integers(1, n_shards * 2 + 1))

    def gen():
        tds, raw = [], []
        r2 = np.random.default_rng(seed + 1000)
        for s in range(n_shards):
            n = int(r2.integers(0, size + 1))
            sc = np.ones(n, np.float32) if constant else np.abs(r2.random(n)).astype(np.float32)
            sc = np.sort(sc)[::-1]
            td = LU.TopDocs(LU.TotalHits(n), [LU.ScoreDoc(i, float(v)) for i, v in enumerate(sc)])
            SP.set_shard_index(td, s)
            tds.append(td)
            raw.append((sc, np.arange(n, dtype=np.int32)))
        return tds, raw

    a, raw = gen()
    b, _ = gen()
    da = SP.sort_docs(False, a, 0, size)
    db = SP.sort_docs(False, b, 0, size)
    assert [(d.doc, d.shard_index, d.score) for d in da] == [(d.doc, d.shard_index, d.score) for d in db]
    if n_shards > 1:
        es, ed, esh, _, _ = O.topdocs_merge(raw, 0, size, list(range(n_shards)))
        assert [d.doc for d in da] == list(ed) and [d.shard_index for d in da] == list(esh)
        if constant:
            pairs = [(d.shard_index, d.doc) for d in da]
            assert pairs == sorted(pairs)


def test_batched_partial_reduce_equals_single_reduce():
    rng = np.random.default_rng(7)
    results = []
    for s in range(37):
        n = int(rng.integers(0, 11))
        sc = np.sort(rng.random(n).astype(np.float32))[::-1]
        results.append((s, sc))
    outs = []
    for batch in [2, 5, 512]:
        c = SP.QueryPhaseResultConsumer(37, from_=3, size=7, batch_reduce_size=batch)
        for i in rng.permutation(len(results)):   # shards answer in any order
            s, sc = results[i]
            c.consume_result(_result(s, sc, list(range(len(sc))), 3, 7) if len(sc) else
                             SP.QuerySearchResult(s, LU.TopDocs(LU.TotalHits(0), []), math.nan, 3, 7))
        r = c.reduce()
        outs.append([(d.doc, d.shard_index, d.score) for d in r.score_docs])
        assert r.total_hits.value == sum(len(sc) for _, sc in results)
    assert outs[0] == outs[1] == outs[2]


def test_single_shard_no_pagination_returned_as_is():
    td = LU.TopDocs(LU.TotalHits(3), [LU.ScoreDoc(5, 3.0), LU.ScoreDoc(1, 2.0), LU.ScoreDoc(9, 1.0)])
    assert SP.merge_top_docs([td], 2, 0) is td
    assert SP.merge_top_docs([], 2, 0) is None


def test_total_hits_tracking_threshold():
    st = SP.TopDocsStats(track_total_hits_up_to=5)
    st.add(LU.TopDocs(LU.TotalHits(4), []), 1.0)
    st.add(LU.TopDocs(LU.TotalHits(4), []), 2.0)
    th = st.get_total_hits()
    assert th.value == 5 and th.relation == LU.Relation.GREATER_THAN_OR_EQUAL_TO
    assert st.max_score == 2.0
    assert math.isnan(SP.TopDocsStats().max_score)


def _two_shard_fetch(fail_shard=None):
    """FetchSearchPhaseTests.testFetchTwoDocument (:124-218) / testFailFetchOneDoc (:220-313): shard 0
    returns (42, 1.0), shard 1 (84, 2.0), each with maxScore 2.0."""
    c = SP.QueryPhaseResultConsumer(2)
    for shard, doc, score in [(0, 42, 1.0), (1, 84, 2.0)]:
        td = LU.TopDocs(LU.TotalHits(1), [LU.ScoreDoc(doc, score)])
        c.consume_result(SP.QuerySearchResult(shard, td, 2.0))
    r = c.reduce()
    to_load = SP.fill_doc_ids_to_load(2, r.score_docs)
    fetched = {s: [SP.SearchHit(d) for d in docs] for s, docs in enumerate(to_load)
               if docs is not None and s != fail_shard}
    return r, to_load, SP.get_hits(r, fetched)


def test_fetch_two_document():
    r, to_load, hits = _two_shard_fetch()
    assert to_load == [[42], [84]]
    assert hits.total_hits.value == 2 and hits.max_score == 2.0
    assert [h.doc_id for h in hits.hits] == [84, 42]
    assert [h.score for h in hits.hits] == [2.0, 1.0] and [h.shard for h in hits.hits] == [1, 0]


def test_fail_fetch_one_doc():
    _, _, hits = _two_shard_fetch(fail_shard=0)
    assert hits.total_hits.value == 2
    assert [h.doc_id for h in hits.hits] == [84]


def test_fetch_with_from_offset():
    """testReduceTopNWithFromOffset's shards (:1347-1392) through the fetch handoff: the 5 hits of
    ranks 5…9, each fetched from its own shard in merged order."""
    c = SP.QueryPhaseResultConsumer(4, from_=5, size=5)
    score = 100
    for i in range(4):
        c.consume_result(_result(i, [score, score - 1, score - 2], [10 * i, 10 * i + 1, 10 * i + 2], 5, 5))
        score -= 3
    r = c.reduce()
    to_load = SP.fill_doc_ids_to_load(4, r.score_docs)
    hits = SP.get_hits(r, {s: [SP.SearchHit(d) for d in docs] for s, docs in enumerate(to_load) if docs})
    assert [h.score for h in hits.hits] == [95.0, 94.0, 93.0, 92.0, 91.0]
    assert [(h.shard, h.doc_id) for h in hits.hits] == [(1, 12), (2, 20), (2, 21), (2, 22), (3, 30)]
