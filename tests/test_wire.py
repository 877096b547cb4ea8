"""Shard-result wire format: libosknn's osk_topdocs_write / osk_topdocs_read vs
the pure-Python restatement (oracle/wire_oracle.py) and hand-derived known answers.  CPU only."""
import json
import math
import os
import struct

import numpy as np
import pytest

from opensearch_amd import wire
from opensearch_amd._lib import OskError
from opensearch_amd.lucene import Relation, ScoreDoc, TopDocs, TotalHits
from oracle import wire_oracle as WO

HERE = os.path.dirname(os.path.abspath(__file__))
KA = json.load(open(os.path.join(HERE, "golden", "wire_known_answers.json")))


def _td(total, rel, mx, docs, scores):
    sds = [ScoreDoc(int(d), float(s)) for d, s in zip(docs, scores)]
    return wire.TopDocsAndMaxScore(TopDocs(TotalHits(total, Relation(rel)), sds), mx)


@pytest.mark.parametrize("case", KA["encode"], ids=lambda c: c["name"])
def test_known_answers(case):
    mx = float("nan") if case["max_score"] == "NaN" else case["max_score"]
    args = (case["total_hits"], case["relation"], mx, case["docs"], case["scores"])
    want = bytes.fromhex(case["hex"])
    assert WO.write_top_docs(*args) == want          # the oracle is pinned by the known answer
    got = wire.write_top_docs(_td(*args))
    assert got == want
    td, used = wire.read_top_docs(got + b"\xde\xad")  # trailing bytes are left unread
    assert used == len(want)
    assert td.top_docs.total_hits == TotalHits(case["total_hits"], Relation(case["relation"]))
    assert [sd.doc for sd in td.top_docs.score_docs] == case["docs"]
    assert [sd.score for sd in td.top_docs.score_docs] == case["scores"]
    assert (math.isnan(td.max_score) and math.isnan(mx)) or td.max_score == mx


@pytest.mark.parametrize("case", KA["decode_errors"], ids=lambda c: c["name"])
def test_decode_errors(case):
    with pytest.raises(OskError) as e:
        wire.read_top_docs(bytes.fromhex(case["hex"]))
    assert e.value.code == case["code"]
    assert case["message"] in str(e.value)


def test_negative_total_hits_rejected_like_write_vlong():
    with pytest.raises(OskError, match=r"Negative longs unsupported.*\[-5\]"):
        wire.write_top_docs(_td(-5, 0, 1.0, [], []))


def test_vint_matches_reference_simple_loop():
    # BytesStreamsTests.testVInt (BytesStreamsTests.java:834-850): writeVInt ≡ the plain 7-bit loop,
    # for random ints incl. negatives; checked through the doc field of a one-hit TopDocs
    rng = np.random.default_rng(7)
    vals = [0, 1, 127, 128, 16383, 16384, 2**31 - 1, -1, -(2**31)] + rng.integers(-2**31, 2**31, 200).tolist()
    for v in vals:
        got = wire.write_top_docs(_td(1, 0, 1.0, [v], [1.0]))
        i, simple = v & 0xFFFFFFFF, bytearray()
        while i & ~0x7F:
            simple.append((i & 0x7F) | 0x80)
            i >>= 7
        simple.append(i)
        assert got[8:8 + len(simple)] == bytes(simple)
        td, _ = wire.read_top_docs(got)
        assert td.top_docs.score_docs[0].doc == v


def test_random_round_trips_against_oracle():
    rng = np.random.default_rng(3)
    for _ in range(300):
        n = int(rng.integers(0, 40))
        docs = rng.integers(-2**31, 2**31, n).tolist()
        scores = rng.standard_normal(n).astype(np.float32).tolist()
        if n and rng.random() < 0.2:
            scores[0] = float("nan")
        total = int(rng.integers(0, 2**62)) if rng.random() < 0.5 else int(rng.integers(0, 1000))
        rel = int(rng.integers(0, 2))
        mx = float(np.float32(rng.standard_normal()))
        want = WO.write_top_docs(total, rel, mx, docs, scores)
        got = wire.write_top_docs(_td(total, rel, mx, docs, scores))
        assert got == want
        t2, r2, m2, d2, s2, used = WO.read_top_docs(got)
        td, used2 = wire.read_top_docs(got)
        assert used == used2 == len(got)
        assert td.top_docs.total_hits.value == t2 == total
        assert [sd.doc for sd in td.top_docs.score_docs] == d2 == docs
        # NaN scores are canonicalised by floatToIntBits; everything else round-trips bit for bit
        for a, b in zip([sd.score for sd in td.top_docs.score_docs], scores):
            pa = struct.pack(">f", a)
            assert pa == (b"\x7f\xc0\x00\x00" if math.isnan(b) else struct.pack(">f", b))
