#!/usr/bin/env python3
"""Throughput of the host entries under concurrent search threads — the way a Java KnnVectorsReader /
coordinator calls libosknn from the `search` pool (S/threadpool/ThreadPool.java:106): T threads each
issue single-query osk_view_search calls (host buffers, synchronous) on ONE shared view; the library
leases each concurrent call a workspace slot and stream (osk_objects.h ViewLease).

  python tools/host_threads.py [--rows-per-shard N] [--threads 1,2,4,8] [--calls 200]

Prints one JSON line per thread count: QPS, mean latency per call, workspace slots leased.
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib  # noqa: E402
from opensearch_amd._lib import check, lib, ptr  # noqa: E402
from opensearch_amd.lucene import synth_host  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-per-shard", type=int, default=1_250_000)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--threads", default="1,2,4,8")
    ap.add_argument("--calls", type=int, default=200, help="calls per thread")
    ap.add_argument("--batching", type=int, default=1, help="osk_tune host_batching (opportunistic batching of "
                    "concurrent calls; 0 = each call alone)")
    ap.add_argument("--leaders", type=int, default=0, help="osk_tune host_batch_leaders (0 = library default)")
    a = ap.parse_args()
    L = lib()
    _lib.tune("host_batching", a.batching)
    if a.leaders:
        _lib.tune("host_batch_leaders", a.leaders)
    segs = []
    for s in range(a.shards):
        h = C.c_void_p()
        check(L.osk_seg_synth(0, a.rows_per_shard, a.dim, _lib.FLOAT32, _lib.COSINE, 42, _lib.DIST_NORMALISH_UNIT,
                              s * a.rows_per_shard, C.byref(h)))
        segs.append(h.value)
    arr = (C.c_void_p * len(segs))(*segs)
    ss = np.arange(len(segs), dtype=np.int32)
    view = C.c_void_p()
    check(L.osk_view_create(arr, len(segs), ptr(ss), None, len(segs), None, C.byref(view)))
    pool = synth_host(0, 64, a.dim, 43, _lib.DIST_NORMALISH_UNIT)

    def one(i, out):
        q = np.ascontiguousarray(pool[i % 64:i % 64 + 1])
        sc, dc, sh = (np.empty((1, 10), np.float32), np.empty((1, 10), np.int32), np.empty((1, 10), np.int32))
        cnt, tot, mx = np.empty(1, np.int32), np.empty(1, np.int64), np.empty(1, np.float32)
        check(L.osk_view_search(view, ptr(q), 1, 10, 0, 10, None, ptr(sc), ptr(dc), ptr(sh), ptr(cnt), ptr(tot),
                                ptr(mx)))
        out.append(int(cnt[0]))

    for i in range(8):   # warm the first slot
        one(i, [])
    for T in [int(x) for x in a.threads.split(",")]:
        outs = [[] for _ in range(T)]
        barrier = threading.Barrier(T + 1)

        def worker(t):
            barrier.wait()
            for c in range(a.calls):
                one(t * 131 + c, outs[t])

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for th in ths:
            th.start()
        barrier.wait()
        t0 = time.perf_counter()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        assert all(c == 10 for o in outs for c in o)
        slots, nb, nr = C.c_int64(), C.c_int64(), C.c_int64()
        check(L.osk_view_counter(view, b"host_slots", C.byref(slots)))
        check(L.osk_view_counter(view, b"host_batches", C.byref(nb)))
        check(L.osk_view_counter(view, b"host_batched_requests", C.byref(nr)))
        n = T * a.calls
        print(json.dumps({"threads": T, "calls": n, "qps": n / dt, "latency_ms": dt / a.calls * 1e3,
                          "host_slots": slots.value, "batching": a.batching, "leaders": a.leaders,
                          "requests_per_batch_so_far": nr.value / max(1, nb.value),
                          "rows": a.rows_per_shard * a.shards, "dim": a.dim}), flush=True)
    L.osk_view_release(view)
    for h in segs:
        L.osk_seg_release(C.c_void_p(h))


if __name__ == "__main__":
    main()
