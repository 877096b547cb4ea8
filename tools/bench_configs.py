#!/usr/bin/env python3
"""Measure every BASELINE.json config on one MI355X (bench.py measures the headline C3 only).

  python tools/bench_configs.py [--only C2,C3,...] [--steps N]

Prints one JSON line per (config, batch): QPS (with --inflight F batches in flight, each on its own
stream and view, as concurrent search threads issue them), ms per batch, the scan's mean duration per batch
(HIP events, osk_view_profile), the fp32-equivalent rate (rows × dim × 4 B per 256 queries ÷ that time:
what an fp32 scan would have to stream, so it exceeds HBM peak on the int8 prefilter path) and, on the
prefilter path, the rate of the bytes it actually reads (int8_prefilter_GBps).  Synthetic data from the device generator:
  C1  100k × 128 fp32 L2, 1 shard, k=10                      (the CPU plumbing config, run here on the GPU)
  C2  1M × 128 fp32 L2 (U[0,1)·128, SIFT-like), 1 shard       batch 1 and 256
  C3  10M × 768 fp32 COSINE, 8 shards                         batch 1 and 256
  C4  100M × 96 fp32 DOT_PRODUCT (unit rows), 8 shards        batch 1 and 1024 (one GPU holds all 100M)
  C5f 10M × 768 COSINE, Bernoulli(s) accept bitsets, s ∈ {1%, 10%, 50%}, batch 1
  C5i 10M × 768 int8 (U{−128..127}), EUCLIDEAN, batch 1
  C3o C3 with outlier dimensions (robustness of the int8 prefilter): N(0,1) rows whose `dims` evenly
      spaced dimensions are scaled ×`scale` before the rows are L2-normalised (--outlier dims:scale,...),
      batch 1, prefilter on and off (the fp32 scan), with rescored rows and exactly re-scanned lists
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib  # noqa: E402
from opensearch_amd.lucene import bits_from_bool, synth_host  # noqa: E402

L = _lib.lib()


class View:
    def __init__(self, n_shards, rows_per_shard, dim, sim, enc, dist, seed=42):
        self.segs = []
        for s in range(n_shards):
            h = C.c_void_p()
            _lib.check(L.osk_seg_synth(0, rows_per_shard, dim, enc, sim, seed, dist, s * rows_per_shard, C.byref(h)))
            self.segs.append(h.value)
        arr = (C.c_void_p * n_shards)(*self.segs)
        ss = np.arange(n_shards, dtype=np.int32)
        self.v = C.c_void_p()
        _lib.check(L.osk_view_create(arr, n_shards, ss.ctypes.data, None, n_shards, None, C.byref(self.v)))
        self.n_shards, self.rows, self.dim, self.enc = n_shards, rows_per_shard, dim, enc
        self.extra = []

    def views(self, n):
        """n views over the same segments (own workspaces): one per query in flight."""
        while len(self.extra) < n - 1:
            arr = (C.c_void_p * self.n_shards)(*self.segs)
            ss = np.arange(self.n_shards, dtype=np.int32)
            v = C.c_void_p()
            _lib.check(L.osk_view_create(arr, self.n_shards, ss.ctypes.data, None, self.n_shards, None, C.byref(v)))
            self.extra.append(v)
        return [self.v] + self.extra[:n - 1]

    def close(self):
        for v in self.extra:
            L.osk_view_release(v)
        L.osk_view_release(self.v)
        for h in self.segs:
            L.osk_seg_release(C.c_void_p(h))


class TorchView(View):
    """A view whose shards are staged from device tensors (make(s) -> [rows, dim] float32 on cuda)."""

    def __init__(self, n_shards, rows_per_shard, dim, sim, make):
        self.segs = []
        for s in range(n_shards):
            x = make(s).contiguous()
            torch.cuda.synchronize()   # the library's stream does not wait on torch's (osknn.h)
            h = C.c_void_p()
            _lib.check(L.osk_seg_stage_device(0, x.data_ptr(), dim * 4, rows_per_shard, dim, _lib.FLOAT32, sim, None,
                                              rows_per_shard, C.byref(h)))
            torch.cuda.synchronize()
            del x
            self.segs.append(h.value)
        arr = (C.c_void_p * n_shards)(*self.segs)
        ss = np.arange(n_shards, dtype=np.int32)
        self.v = C.c_void_p()
        _lib.check(L.osk_view_create(arr, n_shards, ss.ctypes.data, None, n_shards, None, C.byref(self.v)))
        self.n_shards, self.rows, self.dim, self.enc = n_shards, rows_per_shard, dim, _lib.FLOAT32
        self.extra = []


def outlier_rows(n, dim, n_out, scale, seed):
    """N(0,1) rows, n_out evenly spaced dimensions ×scale, then L2-normalised."""
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    x = torch.randn((n, dim), generator=g, device="cuda", dtype=torch.float32)
    if n_out:
        x[:, torch.arange(n_out, device="cuda") * (dim // n_out)] *= scale
    return x / x.norm(dim=1, keepdim=True)


def qpool_dev(n, dim, dist):
    return torch.from_numpy(synth_host(0, n, dim, 43, dist)).cuda()


INFLIGHT = 1
HOST_MS = 0.0
HOST_ISSUE = 0.0


def run_slots(view, queries, batch, steps, warmup, accept_ptrs, k, slots):
    """ms per batch with `slots` queries in flight (round-robin over views and streams) and the scan
    kernel's mean launch duration."""
    S = view.n_shards
    views = view.views(slots)
    keys = [torch.empty((batch, S, k), dtype=torch.int64, device="cuda") for _ in range(slots)]
    cnt = [torch.empty((batch, S), dtype=torch.int32, device="cuda") for _ in range(slots)]
    streams = [torch.cuda.Stream() for _ in range(slots)]   # non-null: 0 would mean the library's own stream
    nq_pool = queries.shape[0] // batch
    acc = None if accept_ptrs is None else accept_ptrs.data_ptr()

    def step(i):
        j = i % slots
        q = queries[(i % nq_pool) * batch:(i % nq_pool + 1) * batch]
        _lib.check(L.osk_view_search_device(views[j], q.data_ptr(), batch, k, acc, keys[j].data_ptr(),
                                            cnt[j].data_ptr(), None, streams[j].cuda_stream))

    for i in range(max(warmup, slots)):
        step(i)
    torch.cuda.synchronize()
    for v in views:
        _lib.check(L.osk_view_profile(v, 1))
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    global HOST_MS
    HOST_MS = (time.perf_counter() - t0) / steps * 1e3   # issue time per batch (host-bound if ≈ ms per batch)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tot, n = 0.0, 0
    for v in views:
        ms, calls = C.c_double(), C.c_int64()
        _lib.check(L.osk_view_scan_time(v, C.byref(ms), C.byref(calls)))
        _lib.check(L.osk_view_profile(v, 0))
        tot, n = tot + ms.value, n + calls.value
    assert all(int(c.min()) >= 0 for c in cnt)
    return dt / steps * 1e3, tot / max(1, n)


PATH_COUNTERS = ("sq8_calls", "sq8_wide_calls", "sq6_calls", "mfma_calls", "select_calls")
PATH = {}


def run(view, queries, batch, steps, warmup, accept_ptrs=None, k=10):
    """(ms per batch with INFLIGHT queries in flight, the scan's isolated mean launch duration)."""
    before = {c: counter(view, c) for c in PATH_COUNTERS}
    ms, km = run_slots(view, queries, batch, steps, warmup, accept_ptrs, k, INFLIGHT)
    global HOST_ISSUE
    HOST_ISSUE = HOST_MS
    PATH.clear()
    PATH.update({c: counter(view, c) - before[c] for c in PATH_COUNTERS if counter(view, c) != before[c]})
    if INFLIGHT > 1:   # overlapped launches share HBM: the kernel's own duration from a one-in-flight pass
        _, km = run_slots(view, queries, batch, max(3, steps // 2), 2, accept_ptrs, k, 1)
    return ms, km


def counter(view, name):
    tot = 0
    for h in [view.v] + view.extra:
        v = C.c_int64()
        _lib.check(L.osk_view_counter(h, name.encode(), C.byref(v)))
        tot += v.value
    return tot


def emit(name, view, batch, ms_step, kernel_ms, bytes_per_launch, extra=None):
    rec = {"config": name, "batch": batch, "inflight": INFLIGHT, "qps": batch / (ms_step * 1e-3),
           "ms_per_batch": ms_step, "host_issue_ms_per_batch": HOST_ISSUE,
           "kernel_ms": kernel_ms, "fp32_equiv_GBps": bytes_per_launch / (kernel_ms * 1e-3) / 1e9,
           "rows": view.n_shards * view.rows, "dim": view.dim, "shards": view.n_shards,
           "path_calls": dict(PATH)}
    rows = view.n_shards * view.rows
    if view.enc == _lib.FLOAT32 and batch < 96 and not (extra or {}).get("selectivity"):
        # the certified int8 prefilter's own bytes: int8 rows (16-B units) + 16-B bound terms, read
        # once per launch of ≤ 8 (sq8_scan, batch 1) or ≤ 32 (sq8_mfma) queries
        per = 8 if batch < 2 else 32
        b8 = rows * (-(-view.dim // 16) * 16 + 16) * -(-batch // per)
        rec["int8_prefilter_GBps"] = b8 / (kernel_ms * 1e-3) / 1e9
    if batch >= 96:   # the bf16×3 candidate pass: tiles whose epilogue took the staging path, all calls so far
        rec["mfma_full_tiles"] = counter(view, "mfma_full_tiles")
    if extra:
        rec.update(extra)
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C1,C2,C3,C4,C5f,C5i")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--c4-batches", default="1,1024")
    ap.add_argument("--c2-batches", default="1,256")
    ap.add_argument("--c3-batches", default="1,256")
    ap.add_argument("--c5i-k", default="10", help="C5i k values (k > 12: the select path's exact mode)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--c5f-sel", default="0.01,0.1,0.5", help="C5f selectivities")
    ap.add_argument("--outlier", default="0:1,8:10,8:30,32:10", help="C3o corpora dims:scale, comma-separated")
    ap.add_argument("--c5f-modes", default="1:0,0:0",
                    help="C5f filter modes filter_gather:gather_min, comma-separated (1:0 = compacted gather, 0:0 = "
                         "bitset window walk)")
    ap.add_argument("--inflight", type=int, default=1, help="queries (batches) in flight: one view + stream each")
    a = ap.parse_args()
    global INFLIGHT
    INFLIGHT = a.inflight
    a.c5f_modes = [tuple(int(x) for x in m.split(":")) for m in a.c5f_modes.split(",")]
    for kv in a.tune:
        key, val = kv.split("=")
        _lib.tune(key, int(val))
    only = set(a.only.split(","))
    torch.cuda.set_device(0)
    st, wu = a.steps, 6   # ≥ kSq6Probes + 1: the 6-bit tier's calibration calls (synchronous) stay out of the timing

    def qpool(n, dim, dist, enc=_lib.FLOAT32):
        return torch.from_numpy(synth_host(0, n, dim, 43, dist)).cuda()

    if "C1" in only:
        v = View(1, 100_000, 128, _lib.EUCLIDEAN, _lib.FLOAT32, _lib.DIST_UNIFORM01)
        q = qpool(64, 128, _lib.DIST_UNIFORM01)
        ms, km = run(v, q, 1, st * 5, wu)
        emit("C1", v, 1, ms, km, 100_000 * 128 * 4)
        v.close()
    if "C2" in only:
        v = View(1, 1_000_000, 128, _lib.EUCLIDEAN, _lib.FLOAT32, _lib.DIST_UNIFORM01_X128)
        q = qpool(1024, 128, _lib.DIST_UNIFORM01_X128)
        for b in [int(x) for x in a.c2_batches.split(",")]:
            ms, km = run(v, q, b, st * 5 if b == 1 else st, wu)
            emit("C2", v, b, ms, km, 1_000_000 * 128 * 4 * ((b + 255) // 256))
        v.close()
    if "C3" in only or "C5f" in only:
        v = View(8, 1_250_000, 768, _lib.COSINE, _lib.FLOAT32, _lib.DIST_NORMALISH_UNIT)
        q = qpool(512, 768, _lib.DIST_NORMALISH_UNIT)
        if "C3" in only:
            for b in [int(x) for x in a.c3_batches.split(",")]:
                c0, s0, b0 = counter(v, "sq8_calls"), counter(v, "sq6_calls"), counter(v, "sq6_rebound_rows")
                ms, km = run(v, q, b, st, wu)
                n6 = counter(v, "sq6_calls") - s0
                emit("C3", v, b, ms, km, 10_000_000 * 768 * 4,
                     {"sq6_share_of_calls": n6 / max(1, counter(v, "sq8_calls") - c0),
                      "rebound_rows_per_query": (counter(v, "sq6_rebound_rows") - b0) / n6 if n6 else None})
        if "C5f" in only:
            rng = np.random.default_rng(44)
            for sel in [float(x) for x in a.c5f_sel.split(",")]:
                bits = [torch.from_numpy(bits_from_bool(rng.random(1_250_000) < sel).view(np.int64)).cuda()
                        for _ in range(8)]
                ptrs = torch.tensor([b.data_ptr() for b in bits], dtype=torch.int64, device="cuda")
                for gmode, gmin in a.c5f_modes:   # compacted gather scan vs the bitset window walk
                    _lib.tune("filter_gather", gmode)
                    _lib.tune("gather_min", gmin)
                    r0, x0 = counter(v, "sq8_rescored_rows"), counter(v, "sq8_exact_tiles")
                    c0 = counter(v, "sq8_calls")
                    ms, km = run(v, q, 1, st, wu, accept_ptrs=ptrs)
                    nc = max(1, counter(v, "sq8_calls") - c0)
                    # the prefilter's own bytes: accepted int8 rows + 16-B bound terms + the bitset
                    b8 = int(10_000_000 * sel) * (768 + 16) + 10_000_000 // 8
                    emit(f"C5f-{int(sel * 100)}%", v, 1, ms, km, int(10_000_000 * sel) * 768 * 4 + 10_000_000 // 8,
                         {"selectivity": sel, "filter_gather": gmode, "gather_min": gmin,
                          "rescored_rows_per_query": (counter(v, "sq8_rescored_rows") - r0) / nc,
                          "exact_lists_per_query": (counter(v, "sq8_exact_tiles") - x0) / nc,
                          "int8_prefilter_GBps": b8 / (km * 1e-3) / 1e9})
                _lib.tune("filter_gather", 1)
                _lib.tune("gather_min", 0)
        v.close()
    if "C3o" in only:
        for spec in a.outlier.split(","):
            n_out, scale = (float(x) for x in spec.split(":"))
            n_out = int(n_out)
            v = TorchView(8, 1_250_000, 768, _lib.COSINE, lambda s: outlier_rows(1_250_000, 768, n_out, scale, 100 + s))
            q = outlier_rows(512, 768, n_out, scale, 99)
            for sq8, sq6 in ((1, 1), (1, 0), (0, 0)):   # 6-bit tier (if the view keeps it), int8 tier, fp32
                _lib.tune("sq8", sq8)
                _lib.tune("sq6", sq6)
                r0, x0 = counter(v, "sq8_rescored_rows"), counter(v, "sq8_exact_tiles")
                f0 = counter(v, "sq8_fallback_queries")
                c0, s0, b0 = counter(v, "sq8_calls"), counter(v, "sq6_calls"), counter(v, "sq6_rebound_rows")
                ms, km = run(v, q, 1, st, wu)
                nc = max(1, counter(v, "sq8_calls") - c0)
                n6 = counter(v, "sq6_calls") - s0
                emit(f"C3o-{n_out}x{scale:g}", v, 1, ms, km, 10_000_000 * 768 * 4,
                     {"outlier_dims": n_out, "outlier_scale": scale, "prefilter": sq8,
                      "tier": "6-bit" if n6 else "int8" if sq8 else "fp32",
                      "sq6_share_of_calls": n6 / nc if sq8 else None,
                      "rebound_rows_per_query": (counter(v, "sq6_rebound_rows") - b0) / max(1, n6) if n6 else None,
                      "rescored_rows_per_query": (counter(v, "sq8_rescored_rows") - r0) / nc,
                      "exact_lists_per_query": (counter(v, "sq8_exact_tiles") - x0) / nc,
                      "fallback_queries": counter(v, "sq8_fallback_queries") - f0})
            _lib.tune("sq8", 1)
            _lib.tune("sq6", 1)
            v.close()
    if "C4" in only:
        v = View(8, 12_500_000, 96, _lib.DOT_PRODUCT, _lib.FLOAT32, _lib.DIST_NORMALISH_UNIT)
        q = qpool(2048, 96, _lib.DIST_NORMALISH_UNIT)
        for b in [int(x) for x in a.c4_batches.split(",")]:
            ms, km = run(v, q, b, st if b < 64 else max(3, st // 4), wu if b < 64 else 2)
            emit("C4", v, b, ms, km, 100_000_000 * 96 * 4 * ((b + 255) // 256))
        v.close()
    if "C5i" in only:
        v = View(8, 1_250_000, 768, _lib.EUCLIDEAN, _lib.BYTE, _lib.DIST_INT8)
        q = torch.from_numpy(synth_host(0, 64, 768, 43, _lib.DIST_INT8)).cuda()
        for kk in [int(x) for x in a.c5i_k.split(",")]:
            ms, km = run(v, q, 1, st, wu, k=kk)
            emit("C5i", v, 1, ms, km, 10_000_000 * 768, {"k": kk})
        v.close()


if __name__ == "__main__":
    main()
