#!/usr/bin/env python3
"""A/B the streaming scan's variants in ONE process, interleaved (cdna_hip_programming.md §5.4 rule 24).

  python tools/scan_ab.py [--rows-per-shard N] [--rounds R] [--iters I]

Stages the C3 corpus once (8 shards × 1.25M × 768 fp32 COSINE on the device), builds one osk_view per
tile-count variant, and times scan launches (HIP events on the launch stream, osk_view_profile) for
every (nt, tiles, batch) variant, round-robin.  Prints median GB/s of algorithmic bytes per variant.
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib  # noqa: E402
from opensearch_amd.lucene import synth_host  # noqa: E402

L = _lib.lib()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-per-shard", type=int, default=1_250_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--sim", type=int, default=_lib.COSINE)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tiles", default="1024,2048,4096")
    ap.add_argument("--batches", default="1")
    ap.add_argument("--nt", default="0,1")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dim, nsh, n = a.dim, 8, a.rows_per_shard
    segs = []
    for s in range(nsh):
        h = C.c_void_p()
        _lib.check(L.osk_seg_synth(0, n, dim, _lib.FLOAT32, a.sim, 42, _lib.DIST_NORMALISH_UNIT, s * n, C.byref(h)))
        segs.append(h.value)
    arr = (C.c_void_p * nsh)(*segs)
    import numpy as np
    seg_shard = np.arange(nsh, dtype=np.int32)
    views = {}
    for t in [int(x) for x in a.tiles.split(",")]:
        _lib.check(L.osk_tune_set(b"tiles_target", t))
        v = C.c_void_p()
        _lib.check(L.osk_view_create(arr, nsh, seg_shard.ctypes.data, None, nsh, None, C.byref(v)))
        views[t] = v
    batches = [int(x) for x in a.batches.split(",")]
    qs = torch.from_numpy(synth_host(0, max(batches) * 4, dim, 43, _lib.DIST_NORMALISH_UNIT)).cuda()
    keys = torch.empty((max(batches), nsh, 10), dtype=torch.int64, device="cuda")
    cnt = torch.empty((max(batches), nsh), dtype=torch.int32, device="cuda")
    torch.cuda.set_stream(torch.cuda.Stream())   # non-null: 0 would mean the library's own stream
    stream = torch.cuda.current_stream().cuda_stream
    variants = [(nt, t, b) for nt in [int(x) for x in a.nt.split(",")] for t in views for b in batches]
    res = {v: [] for v in variants}
    for r in range(a.rounds):
        for (nt, t, b) in variants:
            _lib.check(L.osk_tune_set(b"scan_nt", nt))
            view = views[t]
            for _ in range(2):   # warm
                _lib.check(L.osk_view_search_device(view, qs.data_ptr(), b, 10, None, keys.data_ptr(), cnt.data_ptr(), None, stream))
            _lib.check(L.osk_view_profile(view, 1))
            for i in range(a.iters):
                _lib.check(L.osk_view_search_device(view, qs.data_ptr(), b, 10, None, keys.data_ptr(), cnt.data_ptr(), None, stream))
            ms, calls = C.c_double(), C.c_int64()
            _lib.check(L.osk_view_scan_time(view, C.byref(ms), C.byref(calls)))
            _lib.check(L.osk_view_profile(view, 0))
            avg = ms.value / calls.value
            gbs = nsh * n * dim * 4 * ((b + 7) // 8) / (avg * 1e-3) / 1e9
            res[(nt, t, b)].append(gbs)
        print(f"round {r} done", file=sys.stderr, flush=True)
    out = []
    for v, xs in res.items():
        out.append({"nt": v[0], "tiles": v[1], "batch": v[2], "gbs_median": statistics.median(xs),
                    "gbs_min": min(xs), "gbs_max": max(xs)})
        print(f"nt={v[0]} tiles={v[1]:5d} batch={v[2]:2d}  median {statistics.median(xs):7.1f} GB/s  "
              f"[{min(xs):.1f}, {max(xs):.1f}]")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
