"""Shard-result wire format — a mirror of OpenSearch's `Lucene.writeTopDocs` / `Lucene.readTopDocs`
(server/src/main/java/org/opensearch/common/lucene/Lucene.java:407-447, :314-357) for the plain
TopDocs a k-NN shard returns (type byte 0).  The bytes are produced and parsed by libosknn
(`osk_topdocs_write` / `osk_topdocs_read`), so a Java plugin and this mirror share one encoder.

  byte 0 | vLong totalHits | vInt relation | int BE floatToIntBits(maxScore) | vInt n |
  n × (vInt doc, int BE floatToIntBits(score))

The encodings are StreamOutput's (libs/core/.../io/stream/StreamOutput.java:247-337, 480-482).
Errors raise `OskError` carrying StreamInput's / StreamOutput's message (an IOException /
IllegalStateException in the reference).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import check, lib, ptr
from .lucene import Relation, ScoreDoc, TopDocs, TotalHits


@dataclass
class TopDocsAndMaxScore:
    """S/common/lucene/search/TopDocsAndMaxScore.java: a shard's TopDocs plus its max score."""
    top_docs: TopDocs
    max_score: float


def write_top_docs(td: TopDocsAndMaxScore) -> bytes:
    """Lucene.writeTopDocs (:437-446) for a plain TopDocs."""
    sds = td.top_docs.score_docs
    n = len(sds)
    docs = np.asarray([sd.doc for sd in sds] or [0], np.int32)
    scores = np.asarray([sd.score for sd in sds] or [0.0], np.float32)
    th = td.top_docs.total_hits
    size = C.c_int64()
    check(lib().osk_topdocs_write(int(th.value), th.relation.value, float(td.max_score), n, ptr(docs),
                                  ptr(scores), None, 0, C.byref(size)))
    out = np.empty(max(1, size.value), np.uint8)
    check(lib().osk_topdocs_write(int(th.value), th.relation.value, float(td.max_score), n, ptr(docs),
                                  ptr(scores), ptr(out), size.value, C.byref(size)))
    return out[: size.value].tobytes()


def read_top_docs(buf: bytes, max_hits: int = 1 << 16) -> tuple[TopDocsAndMaxScore, int]:
    """Lucene.readTopDocs (:314-330) → (TopDocsAndMaxScore, bytes consumed)."""
    a = np.frombuffer(buf, np.uint8) if len(buf) else np.zeros(1, np.uint8)
    docs = np.empty(max(1, max_hits), np.int32)
    scores = np.empty(max(1, max_hits), np.float32)
    total, rel, mx, n, used = C.c_int64(), C.c_int32(), C.c_float(), C.c_int32(), C.c_int64()
    check(lib().osk_topdocs_read(ptr(a), len(buf), C.byref(total), C.byref(rel), C.byref(mx), max_hits,
                                 C.byref(n), ptr(docs), ptr(scores), C.byref(used)))
    sds = [ScoreDoc(int(docs[i]), float(scores[i])) for i in range(n.value)]
    td = TopDocs(TotalHits(total.value, Relation(rel.value)), sds)
    return TopDocsAndMaxScore(td, mx.value), used.value
