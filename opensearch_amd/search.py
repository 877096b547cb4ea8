"""Coordinator-side reduce: a mirror of OpenSearch's SearchPhaseController / QueryPhaseResultConsumer
for the k-NN path (server/src/main/java/org/opensearch/action/search/).

  * set_shard_index     SearchPhaseController.java:248-253
  * merge_top_docs      SearchPhaseController.java:224-246 (→ [L] TopDocs.merge(from, topN, …))
  * sort_docs           SearchPhaseController.java:177-222 (no suggestions / collapse / field sort)
  * TopDocsStats        SearchPhaseController.java:839-901
  * QueryPhaseResultConsumer  QueryPhaseResultConsumer.java:160-277 (batched partial reduce,
                        default batched_reduce_size 512, SearchRequest.java:88)
  * fill_doc_ids_to_load / get_hits  the fetch handoff: SearchPhaseController.java:274-284 and
                        :340-405 as driven by FetchSearchPhase.innerRun (FetchSearchPhase.java:132-165)

The merges run in libosknn's host reduce; the device reduce (`osk_merge_device`) implements the same
ordering on the GPU after the RCCL all-gather (see distributed.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Sequence

from .lucene import Relation, ScoreDoc, TopDocs, TotalHits

TRACK_TOTAL_HITS_ACCURATE = 2**31 - 1
TRACK_TOTAL_HITS_DISABLED = -1
DEFAULT_TRACK_TOTAL_HITS_UP_TO = 10000


def set_shard_index(top_docs: TopDocs, shard_index: int) -> None:
    for sd in top_docs.score_docs:
        assert sd.shard_index == -1, "shardIndex is already set"
        sd.shard_index = shard_index


def merge_top_docs(results: Sequence[TopDocs], top_n: int, from_: int) -> TopDocs | None:
    if not results:
        return None
    if len(results) == 1 and from_ == 0:   # only one shard and no pagination: returned as is
        return results[0]
    return TopDocs.merge(from_, top_n, list(results))


def sort_docs(ignore_from: bool, top_docs: Sequence[TopDocs], from_: int, size: int) -> list[ScoreDoc]:
    if not top_docs:
        return []
    merged = merge_top_docs(top_docs, size, 0 if ignore_from else from_)
    return [] if merged is None else list(merged.score_docs)


@dataclass
class TopDocsStats:
    track_total_hits_up_to: int = DEFAULT_TRACK_TOTAL_HITS_UP_TO
    total_hits: int = 0
    relation: Relation = Relation.EQUAL_TO
    fetch_hits: int = 0
    _max_score: float = -math.inf

    @property
    def max_score(self) -> float:
        return math.nan if math.isinf(self._max_score) else self._max_score

    def get_total_hits(self) -> TotalHits | None:
        if self.track_total_hits_up_to == TRACK_TOTAL_HITS_DISABLED:
            return None
        if self.track_total_hits_up_to == TRACK_TOTAL_HITS_ACCURATE:
            return TotalHits(self.total_hits, self.relation)
        if self.total_hits <= self.track_total_hits_up_to:
            return TotalHits(self.total_hits, self.relation)
        return TotalHits(self.track_total_hits_up_to, Relation.GREATER_THAN_OR_EQUAL_TO)

    def add(self, top_docs: TopDocs, max_score: float) -> None:
        if self.track_total_hits_up_to != TRACK_TOTAL_HITS_DISABLED:
            self.total_hits += top_docs.total_hits.value
            if top_docs.total_hits.relation == Relation.GREATER_THAN_OR_EQUAL_TO:
                self.relation = Relation.GREATER_THAN_OR_EQUAL_TO
        self.fetch_hits += len(top_docs.score_docs)
        if not math.isnan(max_score):
            self._max_score = max(self._max_score, max_score)


@dataclass
class QuerySearchResult:
    """The slice of QuerySearchResult (S/search/query/QuerySearchResult.java:65,177-200) the reduce
    reads: shard index, per-shard TopDocs, maxScore, from and size."""
    shard_index: int
    top_docs: TopDocs
    max_score: float
    from_: int = 0
    size: int = 10


@dataclass
class ReducedQueryPhase:
    total_hits: TotalHits | None
    max_score: float
    score_docs: list[ScoreDoc]
    num_reduce_phases: int
    from_: int
    size: int
    fetch_hits: int = 0      # Σ shard hit-list lengths (TopDocsStats.fetchHits, SearchPhaseController.java:874)


class QueryPhaseResultConsumer:
    """Batched incremental reduce (QueryPhaseResultConsumer.java:160-277): shard results are buffered;
    every `batch_reduce_size` of them are merged (sorted by shardIndex, setShardIndex, mergeTopDocs
    with topN = from+size, from 0) into one partial result; reduce() finishes with sortDocs."""

    def __init__(self, expected_results: int, from_: int = 0, size: int = 10,
                 batch_reduce_size: int = 512,
                 track_total_hits_up_to: int = DEFAULT_TRACK_TOTAL_HITS_UP_TO):
        self.expected = expected_results
        self.from_ = from_
        self.size = size
        self.top_n = from_ + size
        self.batch_reduce_size = max(2, batch_reduce_size)
        self.stats = TopDocsStats(track_total_hits_up_to)
        self.buffer: list[QuerySearchResult] = []
        self.merged: TopDocs | None = None
        self.num_reduce_phases = 0

    def consume_result(self, result: QuerySearchResult) -> None:
        # PendingMerges.consume (QueryPhaseResultConsumer.java:389-419): the buffer (plus one slot
        # for a previous partial result) is reduced BEFORE the new result is buffered.
        pending = len(self.buffer) + (1 if self.merged is not None else 0)
        if pending >= self.batch_reduce_size:
            self._partial_reduce()
        self.buffer.append(result)

    def _partial_reduce(self) -> None:
        batch = sorted(self.buffer, key=lambda r: r.shard_index)
        self.buffer = []
        for r in batch:
            self.stats.add(r.top_docs, r.max_score)
        lst = [] if self.merged is None else [self.merged]
        for r in batch:
            set_shard_index(r.top_docs, r.shard_index)
            lst.append(r.top_docs)
        self.merged = merge_top_docs(lst, self.top_n, 0)
        self.num_reduce_phases += 1

    def reduce(self) -> ReducedQueryPhase:
        batch = sorted(self.buffer, key=lambda r: r.shard_index)
        self.buffer = []
        for r in batch:
            self.stats.add(r.top_docs, r.max_score)
        lst = [] if self.merged is None else [self.merged]
        for r in batch:
            set_shard_index(r.top_docs, r.shard_index)
            lst.append(r.top_docs)
        docs = sort_docs(False, lst, self.from_, self.size)
        return ReducedQueryPhase(self.stats.get_total_hits(), self.stats.max_score, docs,
                                 self.num_reduce_phases + 1, self.from_, self.size, self.stats.fetch_hits)


# ---- fetch handoff (adjacent to the hot path: maps the merged hits back to their shards) ----

def fill_doc_ids_to_load(num_shards: int, shard_docs: Sequence[ScoreDoc]) -> list[list[int] | None]:
    """SearchPhaseController.fillDocIdsToLoad (:274-284): per shard, the docs to fetch in merged
    order (None for a shard with nothing to fetch)."""
    out: list[list[int] | None] = [None] * num_shards
    for sd in shard_docs:
        if out[sd.shard_index] is None:
            out[sd.shard_index] = []
        out[sd.shard_index].append(sd.doc)
    return out


@dataclass
class SearchHit:
    """The slice of SearchHit the merge sets: docId, score and the shard it came from."""
    doc_id: int
    score: float = math.nan
    shard: int | None = None


@dataclass
class SearchHits:
    hits: list[SearchHit]
    total_hits: TotalHits | None
    max_score: float


def get_hits(reduced: ReducedQueryPhase, fetch_results: dict[int, list[SearchHit]],
             ignore_from: bool = False) -> SearchHits:
    """SearchPhaseController.getHits (:340-405) for score-sorted (k-NN) results: walks the merged
    ScoreDocs in order, takes the next fetched hit of each one's shard (each shard answered its
    docIdsToLoad in that order), sets the hit's score from the ScoreDoc, and skips a hit whose shard
    failed during fetch (absent from `fetch_results`)."""
    counters = {s: 0 for s in fetch_results}
    from_ = 0 if ignore_from else reduced.from_
    n = min(reduced.fetch_hits - from_, reduced.size)
    n = min(len(reduced.score_docs), n)
    hits: list[SearchHit] = []
    if fetch_results:
        for sd in reduced.score_docs[: max(0, n)]:
            fetched = fetch_results.get(sd.shard_index)
            if fetched is None:   # shard failure during fetch: the hit is dropped
                continue
            i = counters[sd.shard_index]
            counters[sd.shard_index] = i + 1
            hit = fetched[i]
            hit.shard = sd.shard_index
            hit.score = sd.score
            hits.append(hit)
    return SearchHits(hits, reduced.total_hits, reduced.max_score)
