"""Pure-Python restatement of OpenSearch's shard-result wire format for a plain TopDocs.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of libosknn's osk_topdocs_write /
osk_topdocs_read — never by opensearch_amd/.  Follows, line by line in behaviour:
  * Lucene.writeTopDocs type 0       server/src/main/java/org/opensearch/common/lucene/Lucene.java:437-446
  * Lucene.writeTotalHits            Lucene.java:402-405 (vLong value, writeEnum(relation))
  * Lucene.writeScoreDoc             Lucene.java:525-531 (vInt doc, float score)
  * Lucene.readTopDocs type 0        Lucene.java:314-330; readTotalHits :308-312
  * StreamOutput.writeInt / writeVInt / writeVLong / writeFloat
        libs/core/src/main/java/org/opensearch/core/common/io/stream/StreamOutput.java:247-254,262-285,308-337,480-482
  * StreamInput.readVInt / readVLong / readEnum
        libs/core/src/main/java/org/opensearch/core/common/io/stream/StreamInput.java:218-244,267-319,1280-1290
Pinned by the reference's own encoding test (BytesStreamsTests.testVInt, server/src/test/java/org/
opensearch/common/io/stream/BytesStreamsTests.java:834-850: the "simple" 7-bit loop) and by the
hand-derived known answers in tests/golden/wire_known_answers.json.
"""
from __future__ import annotations

import math
import struct


def _vint(i: int) -> bytes:
    i &= 0xFFFFFFFF                    # Java int, >>> 7 on the unsigned bits
    out = bytearray()
    while i & ~0x7F:
        out.append((i & 0x7F) | 0x80)
        i >>= 7
    out.append(i)
    return bytes(out)


def _vlong(i: int) -> bytes:
    if i < 0:
        raise ValueError(f"Negative longs unsupported, use writeLong or writeZLong for negative numbers [{i}]")
    out = bytearray()
    while i & ~0x7F:
        out.append((i & 0x7F) | 0x80)
        i >>= 7
    out.append(i)
    return bytes(out)


def _float(f: float) -> bytes:
    bits = 0x7FC00000 if math.isnan(f) else struct.unpack(">I", struct.pack(">f", f))[0]
    return struct.pack(">I", bits)   # writeInt: big-endian


def write_top_docs(total_hits: int, relation: int, max_score: float, docs, scores) -> bytes:
    out = bytearray([0])
    out += _vlong(total_hits)
    out += _vint(relation)
    out += _float(max_score)
    out += _vint(len(docs))
    for d, s in zip(docs, scores):
        out += _vint(int(d))
        out += _float(float(s))
    return bytes(out)


def read_top_docs(buf: bytes):
    """→ (total_hits, relation, max_score, docs, scores, consumed); raises ValueError like StreamInput."""
    pos = 0

    def byte():
        nonlocal pos
        if pos >= len(buf):
            raise ValueError("EOF")
        b = buf[pos]
        pos += 1
        return b

    def vint():
        i = 0
        for sh in (0, 7, 14, 21):
            b = byte()
            i |= (b & 0x7F) << sh
            if not b & 0x80:
                return i - (1 << 32) if i & 0x80000000 else i
        b = byte()
        if b & 0x80:
            raise ValueError("Invalid vInt")
        i |= (b & 0x7F) << 28
        i &= 0xFFFFFFFF
        return i - (1 << 32) if i & 0x80000000 else i

    def vlong():
        i = 0
        for sh in range(0, 63, 7):
            b = byte()
            i |= (b & 0x7F) << sh
            if not b & 0x80:
                return i
        b = byte()
        if b not in (0, 1):
            raise ValueError("Invalid vlong")
        i |= b << 63
        return i - (1 << 64) if i & (1 << 63) else i

    def f32():
        return struct.unpack(">f", bytes(byte() for _ in range(4)))[0]

    t = byte()
    if t != 0:
        raise ValueError(f"Unknown type {t}")
    total = vlong()
    rel = vint()
    if rel < 0 or rel > 1:
        raise ValueError(f"Unknown Relation ordinal [{rel}]")
    mx = f32()
    n = vint()
    if n < 0:
        raise ValueError("negative count")
    docs, scores = [], []
    for _ in range(n):
        docs.append(vint())
        scores.append(f32())
    return total, rel, mx, docs, scores, pos
