"""Per-leaf route vs one call per shard, on a many-segment shard.

Lucene's KnnFloatVectorQuery runs one KnnVectorsReader.search per leaf (osk_seg_search per segment, then
TopDocs.merge on the host); the plugin's GpuKnnFloatVectorQuery makes one osk_view_search over every
leaf of the shard.  Both return identical hits; this prints their per-query
latency (one search thread) and throughput (8 threads) as JSON lines.

    python tools/shard_calls.py [--segments 20] [--rows 1250000] [--dim 768] [--queries 200]
"""
import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from opensearch_amd import _lib, lucene as LU   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=20)
    ap.add_argument("--rows", type=int, default=1_250_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=200)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    # a log-normal spread of segment sizes, as tiered merging leaves them
    w = rng.lognormal(0.0, 1.0, a.segments)
    sizes = np.maximum(1000, (w / w.sum() * a.rows).astype(np.int64))
    readers, leaves, base, row0 = [], [], 0, 0
    for i, n in enumerate(sizes):
        r = LU.GpuFlatVectorsReader.synthetic("v", int(n), a.dim, LU.VectorSimilarityFunction.COSINE, seed=7,
                                              dist=_lib.DIST_NORMALISH_UNIT, row0=row0)
        readers.append(r)
        leaves.append(LU.LeafReaderContext(i, base, r))
        base += int(n)
        row0 += int(n)
    queries = LU.synth_host(10**9, a.queries, a.dim, 8, _lib.DIST_NORMALISH_UNIT)

    def per_leaf(q):
        return LU.KnnFloatVectorQuery("v", q, 10).rewrite(leaves)

    def one_call(q):
        return LU.GpuKnnFloatVectorQuery("v", q, 10).rewrite(leaves)

    # identical hits
    for i in range(5):
        x, y = per_leaf(queries[i]), one_call(queries[i])
        assert [(h.doc, np.float32(h.score)) for h in x.score_docs] == [(h.doc, np.float32(h.score)) for h in y.score_docs]
    for name, fn in (("per_leaf_osk_seg_search", per_leaf), ("one_osk_view_search", one_call)):
        for q in queries[:10]:
            fn(q)
        t0 = time.perf_counter()
        for q in queries:
            fn(q)
        lat = (time.perf_counter() - t0) / len(queries)
        done = [0]
        lock = threading.Lock()

        def worker(t):
            for j in range(t, len(queries), a.threads):
                fn(queries[j])
                with lock:
                    done[0] += 1

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        qps = done[0] / (time.perf_counter() - t0)
        print(json.dumps({"route": name, "segments": a.segments, "rows": int(sizes.sum()), "dim": a.dim,
                          "ms_per_query_1_thread": round(lat * 1e3, 3), f"qps_{a.threads}_threads": round(qps, 1),
                          "segment_rows_min_max": [int(sizes.min()), int(sizes.max())]}), flush=True)
    LU.GpuKnnFloatVectorQuery.release_views()
    for r in readers:
        r.close()


if __name__ == "__main__":
    main()
