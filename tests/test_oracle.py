"""The CPU oracle, pinned: against the committed golden fixtures, against the reference's own merge
known-answer tests, and against an independent float64 numpy restatement of Lucene's formulas.
(Scoring parity with Lucene itself is unpinned — no Lucene jar or vector fixture in the reference.)
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN / "knn_golden.npz", allow_pickle=False)


def _f64_scores(rows, q, sim, enc):
    """Lucene's VectorSimilarityFunction formulas evaluated in float64 (independent of summation order)."""
    r = rows.astype(np.float64)
    q = q.astype(np.float64)
    dot = r @ q
    if sim == 0:
        d2 = ((r - q) ** 2).sum(1)
        return 1.0 / (1.0 + d2)
    if sim == 1:
        if enc == "i8":
            return 0.5 + dot / (len(q) * 2**15)
        return np.maximum((1 + dot) / 2, 0)
    if sim == 2:
        c = dot / np.sqrt((r * r).sum(1) * (q * q).sum())
        return (1 + c) / 2 if enc == "i8" else np.maximum((1 + c) / 2, 0)
    return np.where(dot < 0, 1 / (1 - dot), dot + 1)


def test_generator_pinned(golden):
    for dist in range(5):
        blk = O.synth(12345, 64, 96, 42, dist)
        assert np.array_equal(np.frombuffer(hashlib.sha256(blk.tobytes()).digest(), np.uint8),
                              golden[f"synth_sha_{dist}"])


def test_oracle_matches_golden(golden):
    keys = sorted({k.rsplit("_rows", 1)[0] for k in golden.files if k.endswith("_rows")})
    assert len(keys) == 20
    for key in keys:
        enc, sim, dim = key.split("_")
        sim = int(sim)
        rows, qs = golden[f"{key}_rows"], golden[f"{key}_queries"]
        o2d, acc = golden[f"{key}_ord_to_doc"], golden[f"{key}_accept"]
        orders = [O.ORDER_DEVICE, O.ORDER_SCALAR, O.ORDER_PANAMA512] if enc == "f32" else [O.ORDER_DEVICE]
        for order in orders:
            for variant in ["dense", "sparse_filtered"]:
                es = golden[f"{key}_o{order}_{variant}_scores"]
                ed = golden[f"{key}_o{order}_{variant}_docs"]
                ec = golden[f"{key}_o{order}_{variant}_count"]
                for i in range(len(qs)):
                    if variant == "dense":
                        s, d, _ = O.exact_search(rows, qs[i], 7, sim, order)
                    else:
                        s, d, _ = O.exact_search(rows, qs[i], 7, sim, order, ord_to_doc=o2d, accept_bits=acc)
                    assert len(d) == ec[i]
                    assert np.array_equal(d, ed[i, : ec[i]])
                    assert np.array_equal(s.view(np.uint32), es[i, : ec[i]].view(np.uint32))


@pytest.mark.parametrize("order", [O.ORDER_DEVICE, O.ORDER_SCALAR, O.ORDER_PANAMA512])
@pytest.mark.parametrize("sim", [0, 1, 2, 3])
def test_oracle_scores_vs_float64(order, sim):
    for dim in [3, 33, 128, 768]:
        dist = {0: 1, 1: 3, 2: 3, 3: 2}[sim]
        rows = O.synth(0, 50, dim, 7, dist)
        q = O.synth(0, 1, dim, 8, dist)[0]
        ref = _f64_scores(rows, q, sim, "f32")
        got = np.array([O.score(q, rows[i], sim, order) for i in range(len(rows))])
        # fp32 summation error is bounded relative to Σ|q·x| (cancellation in signed sums); every
        # score transform has |d score / d sum| ≤ 1
        mag = np.abs(rows.astype(np.float64) * q.astype(np.float64)).sum(1)
        assert np.all(np.abs(got - ref) <= 2e-6 * np.abs(ref) + 1e-6 * mag + 1e-7)


@pytest.mark.parametrize("sim", [0, 1, 2, 3])
def test_oracle_byte_scores_exact(sim):
    rows = O.synth(0, 60, 40, 9, 4)
    q = O.synth(0, 1, 40, 10, 4)[0]
    ref = _f64_scores(rows, q, sim, "i8").astype(np.float32)
    got = np.array([O.score(q, rows[i], sim) for i in range(len(rows))], np.float32)
    # integer sums are exact; only the final float transform rounds
    np.testing.assert_allclose(got, ref, rtol=1e-6)


def test_exact_search_tie_semantics():
    """[L] exactSearch: strict '>' replacement ⇒ among equal scores the lower doc wins, and the result
    is ordered score desc then doc asc."""
    rows = np.ones((20, 4), np.float32)
    rows[7] = 2.0
    q = np.ones(4, np.float32)
    s, d, v = O.exact_search(rows, q, 5, 1)            # DOT_PRODUCT
    assert list(d) == [7, 0, 1, 2, 3] and v == 20
    assert s[0] > s[1] and len(set(s[1:].tolist())) == 1


def test_exact_search_k_larger_than_segment_drops_sentinels():
    rows = O.synth(0, 3, 8, 1, 1)
    s, d, v = O.exact_search(rows, rows[0], 10, 0)
    assert len(d) == 3 and d[0] == 0 and s[0] == 1.0


def test_exact_search_filter_and_sparse_docs():
    rows = O.synth(0, 100, 16, 2, 1)
    o2d = np.arange(100, dtype=np.int32) * 3 + 1
    acc = np.zeros(400, bool)
    acc[o2d[::2]] = True
    s, d, v = O.exact_search(rows, rows[4], 10, 0, ord_to_doc=o2d, accept_bits=O.bits_from_bool(acc))
    assert v == 50 and d[0] == o2d[4] and all(x in set(o2d[::2]) for x in d)


def test_merge_known_answers_from_reference_tests():
    for case in json.loads((GOLDEN / "merge_known_answers.json").read_text()):
        shards = [(np.array(s["scores"], np.float32), np.array(s["docs"], np.int32)) for s in case["shards"]]
        sidx = [s["shard_index"] for s in case["shards"]]
        sc, dc, sh, tot, mx = O.topdocs_merge(shards, case["from"], case["size"], sidx)
        if "expected_scores" in case:
            assert list(sc) == case["expected_scores"]
        if "expected_docs" in case:
            assert list(dc) == case["expected_docs"] and list(sh) == case["expected_shards"]
        assert tot == case["expected_total_hits"] and mx == case["expected_max_score"]


def test_cpu_baseline_driver_matches_single_thread():
    rows = O.synth(0, 3000, 64, 3, 3)
    qs = O.synth(0, 4, 64, 4, 3)
    sc, dc, cc = O.knn_batch(rows, qs, 10, 2, O.ORDER_PANAMA512, 4)
    for i in range(4):
        s, d, _ = O.exact_search(rows, qs[i], 10, 2, O.ORDER_PANAMA512)
        assert np.array_equal(dc[i], d) and np.array_equal(sc[i], s)


@pytest.mark.parametrize("sim", range(4))
def test_nofma_orders_differ_only_by_rounding(sim):
    """Lucene fuses multiply-adds only where the CPU has fast FMA (Constants.HAS_FAST_*_FMA): the
    *_NOFMA orders (multiply, then add) must stay within the north star's 1e-5 of the fused ones, and
    must actually round differently somewhere (the flag is live)."""
    dist = {0: 1, 1: 3, 2: 3, 3: 2}[sim]
    rows = O.synth(0, 3000, 768, 31, dist)
    qs = O.synth(0, 4, 768, 32, dist)
    differ = False
    for fused, plain in ((O.ORDER_SCALAR, O.ORDER_SCALAR_NOFMA), (O.ORDER_PANAMA512, O.ORDER_PANAMA512_NOFMA)):
        for q in qs:
            a = np.array([O.score(q, x, sim, fused) for x in rows[:200]], np.float32)
            b = np.array([O.score(q, x, sim, plain) for x in rows[:200]], np.float32)
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=0)
            differ |= not np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert differ
