"""The C-ABI's threading, stream and lifetime contract (include/osknn.h).

OpenSearch calls the reader from the `search` and `index_searcher` thread pools
(S/threadpool/ThreadPool.java:106,126) many at a time, and refreshes open and drop segments under
live searches (S/index/engine/InternalEngine.java:584-589).  Here:
  * 8 threads × 100 searches on shared segments and views (ctypes releases the GIL, so the calls
    really overlap) return exactly the serial results;
  * searches on one view alternating between two caller streams return exactly the serial results
    (the view reuses its workspace; the library orders a call after the previous call's stream);
  * a segment released by its reader while a view still groups it stays valid until the view goes;
  * warming builds the derived copies ahead of the first search (footprint grows, results unchanged).
"""
import threading

import numpy as np
import pytest
import torch

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

COS = LU.VectorSimilarityFunction.COSINE
L2 = LU.VectorSimilarityFunction.EUCLIDEAN


def same(a, b):
    for x, y in zip(a, b):
        x, y = np.asarray(x), np.asarray(y)
        if x.dtype == np.float32:
            x, y = x.view(np.uint32), y.view(np.uint32)
        if not np.array_equal(x, y):
            return False
    return True


def test_eight_threads_hundred_searches_each():
    rows_a = O.synth(0, 20000, 256, 200, 3)
    rows_b = O.synth(0, 15000, 256, 201, 3)
    rows_c = O.synth(0, 8000, 96, 202, 1)
    ra, rb = LU.GpuFlatVectorsReader("v", rows_a, COS), LU.GpuFlatVectorsReader("v", rows_b, COS)
    rc = LU.GpuFlatVectorsReader("v", rows_c, L2)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, ra)], [LU.LeafReaderContext(0, 0, rb)]], [1, 0])
    pool = O.synth(0, 64, 256, 203, 3)
    pool_c = O.synth(0, 64, 96, 204, 1)
    rng = np.random.default_rng(0)
    filt = rng.random(20000) < 0.05

    # the calls each thread makes: (kind, query index, batch)
    def call(kind, i, b):
        if kind == 0:
            return ds.search(pool[i:i + b], 10, 0, 10)
        if kind == 1:
            return ra.search_batch(pool[i:i + b], 10)
        if kind == 2:
            return ds.search(pool[i:i + b], 10, 0, 10, accept=[filt, None])
        return rc.search_batch(pool_c[i:i + b], 7)

    plans = [[(int(rng.integers(4)), int(rng.integers(48)), int(rng.choice([1, 1, 2, 5, 16]))) for _ in range(100)]
             for _ in range(8)]
    try:
        serial = {p: call(*p) for plan in plans for p in plan}
        errors = []

        def worker(plan):
            try:
                for p in plan:
                    if not same(call(*p), serial[p]):
                        errors.append(("mismatch", p))
            except Exception as e:   # noqa: BLE001 - reported below
                errors.append(("error", repr(e)))

        threads = [threading.Thread(target=worker, args=(pl,)) for pl in plans]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        assert not errors, errors[:5]
    finally:
        ds.close()
        for r in (ra, rb, rc):
            r.close()


def test_searches_alternating_between_two_streams():
    rows = O.synth(0, 30000, 768, 210, 3)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    queries = torch.from_numpy(O.synth(0, 40, 768, 211, 3)).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    k = 10
    try:
        def run(i, st):
            keys = torch.empty((1, 1, k), dtype=torch.int64, device="cuda")
            cnt = torch.empty((1, 1), dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            _lib.check(_lib.lib().osk_view_search_device(ds.handle, queries[i].data_ptr(), 1, k, None, keys.data_ptr(),
                                                         cnt.data_ptr(), None, st.cuda_stream))
            return keys, cnt

        serial = []
        for i in range(40):
            keys, cnt = run(i, streams[0])
            streams[0].synchronize()
            serial.append(keys.cpu().clone())
        outs = [run(i, streams[i % 2]) for i in range(40)]
        torch.cuda.synchronize()
        for i, (keys, _) in enumerate(outs):
            assert torch.equal(keys.cpu(), serial[i]), i
    finally:
        ds.close()
        r.close()


def test_segment_released_under_a_live_view_stays_valid():
    rows = O.synth(0, 5000, 128, 220, 3)
    q = O.synth(0, 3, 128, 221, 3)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    want = ds.search(q, 10, 0, 10)
    r.close()                              # the reader goes (segment merged away); the view keeps it
    got = ds.search(q, 10, 0, 10)
    assert same(want, got)
    ds.close()                             # last reference: freed now


def test_warm_builds_copies_ahead_and_results_do_not_change():
    import ctypes as C
    rows = O.synth(0, 20000, 768, 230, 3)
    queries = O.synth(0, 40, 768, 231, 3)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])

    def footprint():
        b = C.c_int64()
        _lib.check(_lib.lib().osk_seg_footprint(r.handle, C.byref(b)))
        return b.value

    try:
        staged = footprint()
        # rows (768·4 B) + norms (4 B) + the int8 prefilter copy built at staging (768 + 16 B)
        assert staged >= 20000 * (768 * 4 + 4 + 768 + 16)
        before = [ds.search(queries[:b], 10, 0, 10) for b in (1, 8, 40)]
        _lib.check(_lib.lib().osk_view_warm(ds.handle, _lib.OSK_WARM_ALL))
        warmed = footprint()
        assert warmed >= staged + 20000 * 768 * 2   # + tiled int8 twin and bf16 hi/lo split
        after = [ds.search(queries[:b], 10, 0, 10) for b in (1, 8, 40)]
        assert all(same(a, b) for a, b in zip(before, after))
        assert footprint() == warmed
    finally:
        ds.close()
        r.close()


def test_host_entries_lease_concurrent_workspaces():
    """Concurrent synchronous host calls on ONE view / ONE segment each lease a workspace slot (the
    view or a replica over the same segments) with its own stream (osk_objects.h ViewLease): they run
    concurrently on the device, more slots appear under load (≤ 8), and every result equals the
    serial one."""
    rows = O.synth(0, 60000, 384, 210, 3)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    pool = O.synth(0, 32, 384, 211, 3)
    want_v = [ds.search(pool[i:i + 1], 10, 0, 10) for i in range(32)]
    want_s = [r.search_batch(pool[i:i + 1], 10) for i in range(32)]
    errors, barrier = [], threading.Barrier(8)

    def worker(t):
        try:
            barrier.wait()
            for rep in range(40):
                i = (t * 7 + rep) % 32
                if (t + rep) % 2:
                    got = ds.search(pool[i:i + 1], 10, 0, 10)
                    if not same(got, want_v[i]):
                        errors.append(("view", t, rep))
                else:
                    got = r.search_batch(pool[i:i + 1], 10)
                    if not same(got, want_s[i]):
                        errors.append(("seg", t, rep))
        except Exception as e:   # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    try:
        assert not errors, errors[:5]
        slots = ds.counter("host_slots")
        assert 1 <= slots <= 8
    finally:
        ds.close()
        r.close()


def test_host_calls_batch_opportunistically():
    """Concurrent unfiltered host calls on one view are batched while the device is busy (same k /
    from / size only): some batches carry several requests, and every caller gets
    exactly its serial result, whatever it was batched with."""
    rows = O.synth(0, 200000, 256, 220, 3)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    pool = O.synth(0, 48, 256, 221, 3)
    shapes = [(10, 0, 10), (5, 0, 5), (10, 2, 8)]
    want = {(i, sh): ds.search(pool[i:i + 1], sh[0], sh[1], sh[2]) for i in range(48) for sh in shapes}
    want_seg = {i: r.search_batch(pool[i:i + 2], 7) for i in range(0, 46, 2)}
    b0, q0 = ds.counter("host_batches"), ds.counter("host_batched_requests")
    errors, barrier = [], threading.Barrier(8)

    def worker(t):
        try:
            barrier.wait()
            for rep in range(60):
                i = (t * 5 + rep * 3) % 48
                if t == 7:   # a segment-level caller with 2 queries per call
                    j = (i // 2) * 2
                    if j > 44:
                        j = 44
                    if not same(r.search_batch(pool[j:j + 2], 7), want_seg[j]):
                        errors.append(("seg", t, rep))
                    continue
                sh = shapes[(t + rep) % 3]
                if not same(ds.search(pool[i:i + 1], sh[0], sh[1], sh[2]), want[(i, sh)]):
                    errors.append(("view", t, rep, sh))
        except Exception as e:   # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    try:
        assert not errors, errors[:5]
        nb, nq = ds.counter("host_batches") - b0, ds.counter("host_batched_requests") - q0
        assert nq == 7 * 60 and nb < nq   # every view call went through the batcher; some were merged
    finally:
        ds.close()
        r.close()


def test_batched_host_call_errors_stay_with_their_caller():
    """A request that fails (here k = 0) fails alone: the batcher groups by (k, from, size), so the
    valid concurrent calls still get their exact results, and the failing caller gets the error code
    and its own message."""
    rows = O.synth(0, 50000, 128, 230, 3)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    pool = O.synth(0, 16, 128, 231, 3)
    want = [ds.search(pool[i:i + 1], 10, 0, 10) for i in range(16)]
    results, barrier = {}, threading.Barrier(6)

    def worker(t):
        barrier.wait()
        for rep in range(20):
            i = (t + rep) % 16
            try:
                if t == 0:
                    ds.search(pool[i:i + 1], 0, 0, 10)
                    results[(t, rep)] = "no error"
                else:
                    results[(t, rep)] = same(ds.search(pool[i:i + 1], 10, 0, 10), want[i])
            except _lib.OskError as e:
                results[(t, rep)] = ("error", str(e))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    try:
        for (t, rep), v in results.items():
            if t == 0:
                assert isinstance(v, tuple) and v[0] == "error" and "k must be" in v[1], v
            else:
                assert v is True, (t, rep, v)
    finally:
        ds.close()
        r.close()


def test_counters_sum_over_leased_replicas_and_call_timing():
    """Counters of a view sum over the replica slots its host entries leased (osk_view_counter), and the
    per-call device time of a host search is exported for the query profiler (osk_last_call_device_ns;
    SearchPlugin.getQueryProfileMetricsProvider, S/plugins/SearchPlugin.java:108)."""
    import time
    rows = O.synth(0, 60000, 256, 240, 3)
    r = LU.GpuFlatVectorsReader("v", rows, COS)
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]], [0])
    pool = O.synth(0, 16, 256, 241, 3)
    _lib.tune("host_batching", 0)
    try:
        c0 = ds.counter("sq8_calls")
        barrier = threading.Barrier(8)

        def worker(t):
            barrier.wait()
            for rep in range(10):
                ds.search(pool[(t + rep) % 16:(t + rep) % 16 + 1], 10, 0, 10)

        threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        assert ds.counter("sq8_calls") - c0 == 80   # every call, whichever slot served it
        assert ds.counter("host_slots") >= 1
        _lib.tune("call_timing", 0)
        ds.search(pool[:1], 10, 0, 10)
        assert _lib.last_call_device_ns() == (-1, 0)
        _lib.tune("call_timing", 1)
        t0 = time.perf_counter_ns()
        want = ds.search(pool[:1], 10, 0, 10)
        wall = time.perf_counter_ns() - t0
        ns, shared = _lib.last_call_device_ns()
        assert shared == 1 and 0 < ns <= wall
        # the timing knob changes nothing but the timing
        assert same(ds.search(pool[:1], 10, 0, 10), want)
        # batched host calls report the shared launch chain's time and how many requests it served
        _lib.tune("host_batching", 1)
        got = {}

        def timed(t):
            barrier.wait()
            ds.search(pool[t:t + 1], 10, 0, 10)
            got[t] = _lib.last_call_device_ns()

        threads = [threading.Thread(target=timed, args=(t,)) for t in range(8)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        assert all(ns > 0 and 1 <= sh <= 8 for ns, sh in got.values()), got
    finally:
        _lib.tune("call_timing", 0)
        _lib.tune("host_batching", 1)
        ds.close()
        r.close()
