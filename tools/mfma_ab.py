#!/usr/bin/env python3
"""A/B the batched MFMA candidate kernel in one process (interleaved rounds): ablations and unit counts.

  python tools/mfma_ab.py [--rows-per-shard N] [--batch 256] [--ablate 0,1,2,4,6] [--units 512]

ablate bits: 1 = skip the epilogue (scores + selection), 2 = skip query (B) staging, 4 = skip corpus (A) staging.
Ablated runs produce wrong candidates; only the kernel time (HIP events, osk_view_profile) matters.
"""
import os
os.environ.setdefault("OSK_TESTING_LIB", "1")   # A/B knobs live in libosknn_testing.so
import argparse
import ctypes as C
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib  # noqa: E402
from opensearch_amd.lucene import synth_host  # noqa: E402

L = _lib.lib()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-per-shard", type=int, default=1_250_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ablate", default="0,1,2,4,6,7")
    ap.add_argument("--units", default="512")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    nsh, n, dim = 8, a.rows_per_shard, a.dim
    segs = []
    for s in range(nsh):
        h = C.c_void_p()
        _lib.check(L.osk_seg_synth(0, n, dim, _lib.FLOAT32, _lib.COSINE, 42, _lib.DIST_NORMALISH_UNIT, s * n, C.byref(h)))
        segs.append(h.value)
    arr = (C.c_void_p * nsh)(*segs)
    ss = np.arange(nsh, dtype=np.int32)
    views = {}
    for u in [int(x) for x in a.units.split(",")]:
        _lib.tune("mfma_units", u)
        v = C.c_void_p()
        _lib.check(L.osk_view_create(arr, nsh, ss.ctypes.data, None, nsh, None, C.byref(v)))
        views[u] = v
    B = a.batch
    qs = torch.from_numpy(synth_host(0, B, dim, 43, _lib.DIST_NORMALISH_UNIT)).cuda()
    keys = torch.empty((B, nsh, 10), dtype=torch.int64, device="cuda")
    cnt = torch.empty((B, nsh), dtype=torch.int32, device="cuda")
    torch.cuda.set_stream(torch.cuda.Stream())   # non-null: 0 would mean the library's own stream
    stream = torch.cuda.current_stream().cuda_stream
    variants = [(ab, u) for ab in [int(x) for x in a.ablate.split(",")] for u in views]
    res = {v: [] for v in variants}
    for r in range(a.rounds):
        for ab, u in variants:
            _lib.tune("mfma_ablate", ab)
            view = views[u]
            _lib.check(L.osk_view_search_device(view, qs.data_ptr(), B, 10, None, keys.data_ptr(), cnt.data_ptr(), None, stream))
            _lib.check(L.osk_view_profile(view, 1))
            for _ in range(a.iters):
                _lib.check(L.osk_view_search_device(view, qs.data_ptr(), B, 10, None, keys.data_ptr(), cnt.data_ptr(), None, stream))
            ms, calls = C.c_double(), C.c_int64()
            _lib.check(L.osk_view_scan_time(view, C.byref(ms), C.byref(calls)))
            _lib.check(L.osk_view_profile(view, 0))
            res[(ab, u)].append(ms.value / calls.value)
        print(f"round {r} done", file=sys.stderr, flush=True)
    _lib.tune("mfma_ablate", 0)
    for (ab, u), xs in res.items():
        print(f"ablate={ab} units={u:5d} batch={B}: median {statistics.median(xs):8.3f} ms  [{min(xs):.3f}, {max(xs):.3f}]")


if __name__ == "__main__":
    main()
