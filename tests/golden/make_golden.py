#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

  python tests/golden/make_golden.py

1. merge_known_answers.json — the reference's own known-answer tests for the coordinator merge,
   restated as data (inputs + expected outputs):
     * SearchPhaseControllerTests.testReduceTopNWithFromOffset
       (server/src/test/java/org/opensearch/action/search/SearchPhaseControllerTests.java:1347-1392)
     * FetchSearchPhaseTests.testFetchTwoDocument (FetchSearchPhaseTests.java:124-218, merged order)
     * constant-score tie breaking of testSortDocsIsIdempotent (:255-298): equal scores order by
       shardIndex then doc.
2. knn_golden.npz — exact k-NN results of the CPU oracle (oracle/lucene_oracle.c) on small corpora:
   every similarity × {float32, int8}, sparse ord→doc, deletes/filters, duplicates (exact ties).
   LABEL: restatement of Lucene 10.3.0 semantics — NOT produced by Lucene (no JDK / lucene-core jar
   exists in this image).  They pin the oracle against silent change and give the
   GPU path fixed vectors to match.
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402


def merge_known_answers():
    cases = []
    # testReduceTopNWithFromOffset: 4 shards × 3 docs (doc 0), scores 100..89, from 5, size 5
    shards, score = [], 100
    for i in range(4):
        shards.append({"shard_index": i, "scores": [float(score - j) for j in range(3)], "docs": [0, 0, 0],
                       "total_hits": 3})
        score -= 3
    cases.append({"name": "testReduceTopNWithFromOffset", "from": 5, "size": 5, "shards": shards,
                  "expected_scores": [95.0, 94.0, 93.0, 92.0, 91.0], "expected_total_hits": 12,
                  "expected_max_score": 100.0})
    # testFetchTwoDocument: shard0 (doc 42, 1.0), shard1 (doc 84, 2.0) → 84 then 42
    cases.append({"name": "testFetchTwoDocument", "from": 0, "size": 10,
                  "shards": [{"shard_index": 0, "scores": [1.0], "docs": [42], "total_hits": 1},
                             {"shard_index": 1, "scores": [2.0], "docs": [84], "total_hits": 1}],
                  "expected_docs": [84, 42], "expected_shards": [1, 0], "expected_total_hits": 2,
                  "expected_max_score": 2.0})
    # constant scores (generateQueryResults(useConstantScore=true): docs 0..n-1, score 1.0)
    cs = [{"shard_index": s, "scores": [1.0] * n, "docs": list(range(n)), "total_hits": n}
          for s, n in enumerate([3, 0, 2, 4])]
    exp = [(s, d) for s, n in enumerate([3, 0, 2, 4]) for d in range(n)]
    cases.append({"name": "constantScoreTieBreak", "from": 2, "size": 6, "shards": cs,
                  "expected_docs": [d for _, d in exp[2:8]], "expected_shards": [s for s, _ in exp[2:8]],
                  "expected_total_hits": 9, "expected_max_score": 1.0})
    return cases


def knn_cases():
    out = {}
    specs = []
    for enc in ["f32", "i8"]:
        for sim in range(4):
            for dim in ([5, 40, 100] if enc == "f32" else [16, 40]):
                specs.append((enc, sim, dim))
    idx = 0
    rng = np.random.default_rng(2024)
    for enc, sim, dim in specs:
        n, nq, k = 200, 3, 7
        if enc == "i8":
            rows = O.synth(0, n, dim, 1000 + idx, 4)
            qs = O.synth(0, nq, dim, 2000 + idx, 4)
        else:
            dist = {0: 1, 1: 3, 2: 3, 3: 2}[sim]
            rows = O.synth(0, n, dim, 1000 + idx, dist)
            qs = O.synth(0, nq, dim, 2000 + idx, dist)
        rows[150:170] = rows[10:30]          # exact duplicates → exact ties
        ord_to_doc = np.sort(rng.choice(400, n, replace=False)).astype(np.int32)
        accept = rng.random(400) < 0.7
        key = f"{enc}_{sim}_{dim}"
        out[f"{key}_rows"] = rows
        out[f"{key}_queries"] = qs
        out[f"{key}_ord_to_doc"] = ord_to_doc
        out[f"{key}_accept"] = O.bits_from_bool(accept)
        orders = [O.ORDER_DEVICE, O.ORDER_SCALAR, O.ORDER_PANAMA512] if enc == "f32" else [O.ORDER_DEVICE]
        for order in orders:
            for variant in ["dense", "sparse_filtered"]:
                sc = np.full((nq, k), -np.inf, np.float32)
                dc = np.full((nq, k), 2**31 - 1, np.int32)
                cnt = np.zeros(nq, np.int32)
                for i in range(nq):
                    if variant == "dense":
                        s, d, _ = O.exact_search(rows, qs[i], k, sim, order)
                    else:
                        s, d, _ = O.exact_search(rows, qs[i], k, sim, order, ord_to_doc=ord_to_doc,
                                                 accept_bits=out[f"{key}_accept"])
                    sc[i, : len(s)] = s
                    dc[i, : len(d)] = d
                    cnt[i] = len(d)
                out[f"{key}_o{order}_{variant}_scores"] = sc
                out[f"{key}_o{order}_{variant}_docs"] = dc
                out[f"{key}_o{order}_{variant}_count"] = cnt
        idx += 1
    # generator pin: sha256 of a block of every distribution
    for dist in range(5):
        blk = O.synth(12345, 64, 96, 42, dist)
        out[f"synth_sha_{dist}"] = np.frombuffer(hashlib.sha256(blk.tobytes()).digest(), np.uint8)
    return out


def main():
    (HERE / "merge_known_answers.json").write_text(json.dumps(merge_known_answers(), indent=1))
    np.savez_compressed(HERE / "knn_golden.npz", **knn_cases())
    print("wrote", HERE / "merge_known_answers.json", HERE / "knn_golden.npz")


if __name__ == "__main__":
    main()
