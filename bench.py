#!/usr/bin/env python3
"""Headline benchmark: exact k-NN QPS@k=10 on the Cohere-shaped corpus (BASELINE.json config C3).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
  (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N)

Workload (config C3): 10,000,000 × 768 fp32 vectors, COSINE, 8 index shards of
1,250,000 docs (shard s = global rows [s·1.25M, (s+1)·1.25M) as local docs 0…1.25M−1, one segment
each), k = 10, from = 0, size = 10.  Synthetic data generated on the device by libosknn's counter
generator (Irwin–Hall(4) ≈ N(0,1), rows L2-normalised; queries from seed 43).  Shard s lives on
rank s·N/8, so the total corpus is fixed and each GPU scans 10M/N rows ("strong" scaling).

One step = one batch of B queries (default 1: the single-query path the north star targets) through
the whole hot path with inputs resident in HBM: per-shard exact scan + top-k on every GPU, per-shard
merge, RCCL all-gather of the per-shard top-k lists, device coordinator merge (TopDocs.merge) — one
C-ABI call per rank (osk_shards_search_merge_device; libosknn owns the RCCL communicator).
value = queries answered by the whole job per second.  Queries are issued as a serving node's search
threads issue them: F = 4 in flight (--inflight), each a separate single-query C-ABI call on its own
stream with its own view (workspace) over the shared segments, round-robin — one query's settle, merge
and exchange run under the next one's scan instead of idling the chip.  The same run also times the
steps strictly one after another ("one_in_flight": per-query latency).

Path (the library's own choice): a single unfiltered query — the headline —
takes the certified prefilter's 6-bit tier (sq6_pilot seeds per-shard floors from 1 % of the rows on the int8
copy, sq6_scan streams 6-bit codes + 16-B bound terms and keeps the rows whose upper bound reaches the floor,
sq6_rebound re-bounds them on the int8 copy, the settle re-scores the surviving candidates exactly in fp32);
results are bit-identical to the fp32 streaming scan, which the bench re-runs on the same queries and
compares.  Batches of 2…~160 take the int8 MFMA prefilter (sq8_mfma, 32 queries per corpus pass), larger ones
the wide int8 prefilter (≤ 768 dims, 256 queries per pass) or the bf16×3 MFMA path, by the library's cost model.
roofline: the dominant kernel is HBM-bound; algorithmic bytes per launch = rows scanned × (576 + 16) B for
sq6_scan (6-bit codes + 16-B bound terms, one query per launch; rows × (768 + 16) B for sq8_scan's int8 tier;
rows × 768 × 4 B for the fp32 scan).  Its average duration is measured live from the kernel's own
dispatch-packet timestamps (hipExtLaunchKernelGGL events, osk_view_profile) of every 8th search
(`--profile-every`: a stamped launch costs a few µs of stream time, so the timed loop samples) in the
one-in-flight timed pass (overlapped launches share HBM with their neighbours, so their individual durations
overstate the kernel's time); the whole step's sustained rate (bytes per step ÷ ms per step of the headline pass) is reported
beside it.  `--rank-share R/W` stages only the shards rank R of a W-GPU run owns (one shard of 1.25M rows
at W = 8) on this one GPU: the per-GPU share of that run, without its all-gather.
cpu_baseline: rank 0 at N = 1 only — the oracle's Lucene-equivalent restatement (Panama-512 order,
not Lucene: no JDK/jar on the box) on a bounded sample, scaled to the full corpus by rows.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from opensearch_amd import _lib  # noqa: E402
from opensearch_amd import distributed as D  # noqa: E402
from opensearch_amd.lucene import synth_host  # noqa: E402

N_SHARDS = 8
ROWS_PER_SHARD = 1_250_000
DIM = 768
K = 10
FROM, SIZE = 0, 10
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md; 6.29 TB/s measured float4 copy)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_traffic_c3_b1.json")


def pmc_traffic(rows_local: int, batch: int, prefilter: bool, six: bool = False):
    """HBM bytes per scan launch from the committed rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes of this
    same command (tools/pmc_traffic.py; gfx950 ×2 FETCH correction applied), scaled to this rank's rows.
    The passes were taken at N=1 (10M rows, batch 1).  None when absent or for another batch size."""
    path = PMC_SUMMARY_SQ6 if six else PMC_SUMMARY
    if batch != 1 or not os.path.exists(path):
        return None, None
    data = json.load(open(path))
    # (a prefix: the headline instance is sq8_scan<16, 3, 1, 4, MODE>)
    want = "sq6_scan<3, 3>" if six else "sq8_scan<16, 3, 1, 4" if prefilter else "scan_f32<16, 12, 1, false"
    for name, v in data.items():
        if want in name:
            return v["hbm_bytes"] * rows_local / (N_SHARDS * ROWS_PER_SHARD), os.path.relpath(path, ROOT)
    return None, None


READ_CEILING = os.path.join(ROOT, "profiles", "r02j", "hbm_read_ceiling.json")
# the 6-bit tier's pass (tools/gpu_run.sh pmc: FETCH_SIZE / WRITE_SIZE of this bench at N = 1, round 6)
PMC_SUMMARY_SQ6 = os.path.join(ROOT, "profiles", "r06", "pmc", "pmc_traffic.json")


def read_ceiling():
    """The best pure HBM read stream measured on this MI355X (tools/hbm_read.hip: 16-B non-temporal loads,
    8 GB buffer), GB/s — the practical ceiling a streaming scan can reach, beside the 8 TB/s spec."""
    if not os.path.exists(READ_CEILING):
        return None
    return max(r["TBps"] for r in json.load(open(READ_CEILING))["results"]) * 1000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_info() -> tuple[str, str]:
    """(CPU model, vector ISA that sets Lucene's Panama species width) of this host."""
    model, flags = "unknown", set()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and model == "unknown":
                model = line.split(":", 1)[1].strip()
            elif line.startswith("flags") and not flags:
                flags = set(line.split(":", 1)[1].split())
    except OSError:
        pass
    isa = ("AVX-512 (16 fp32 lanes)" if "avx512f" in flags else "AVX2 (8 fp32 lanes)" if "avx2" in flags
           else "SSE/other")
    return model, isa


def _cpulist(text: str) -> list[int]:
    out = []
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out += list(range(int(a), int(b or a) + 1))
    return out


def numa_cores(threads: int) -> tuple[int, list[int]]:
    """One NUMA node's CPUs for the baseline's threads: the node with the most CPUs this process may use,
    one hardware thread per physical core first (SMT siblings only if the node has too few cores)."""
    allowed = os.sched_getaffinity(0)
    best = (-1, [])
    for d in sorted(Path("/sys/devices/system/node").glob("node[0-9]*")):
        try:
            cpus = [c for c in _cpulist((d / "cpulist").read_text()) if c in allowed]
        except OSError:
            continue
        if len(cpus) > len(best[1]):
            best = (int(d.name[4:]), cpus)
    node, cpus = best
    if not cpus:
        return -1, sorted(allowed)[:threads]
    first, rest = [], []
    for c in cpus:
        try:
            sib = _cpulist(Path(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read_text())
        except OSError:
            sib = [c]
        (first if c == min(s for s in sib if s in allowed or s == c) else rest).append(c)
    return node, (first + rest)[:threads]


def cpu_baseline(sample_rows: int, n_queries: int, threads: int, passes: int = 15) -> dict:
    """The oracle's Lucene-equivalent exact search (Panama-512 summation order, one thread per row slice
    like the index_searcher pool's slices) over a bounded C3 sample that is far larger than the host's
    caches.  The AVX-512 build of the restatement runs where the host has AVX-512 (Lucene's 16-lane
    FLOAT_SPECIES there); the threads are pinned to one NUMA node (the sample is first-touched there), and
    `passes` passes are timed on `threads` threads (median reported; min/max beside it: the box's host is
    shared), then 3 on 1 thread."""
    from oracle import oracle as O
    isa = O.use_build("v4")
    node, cores = numa_cores(threads)
    prev_aff = os.sched_getaffinity(0)
    threads = len(cores)
    os.sched_setaffinity(0, cores)   # this thread, and the threads it creates, on the node's cores
    try:
        return _cpu_baseline_pinned(O, sample_rows, n_queries, threads, passes, isa, node, cores)
    finally:
        os.sched_setaffinity(0, prev_aff)


def _cpu_baseline_pinned(O, sample_rows, n_queries, threads, passes, isa, node, cores) -> dict:
    t0 = time.perf_counter()
    rows = O.synth(0, sample_rows, DIM, 42, 3)
    qs = O.synth(0, n_queries, DIM, 43, 3)
    log(f"cpu_baseline: generated {sample_rows}x{DIM} in {time.perf_counter() - t0:.1f}s")
    O.knn_batch(rows, qs, K, 2, O.ORDER_PANAMA512, threads)   # warm-up pass (pages, threads, clocks)

    def median_qps(nq, nthreads, n_passes):
        rates = []
        for _ in range(n_passes):
            t0 = time.perf_counter()
            O.knn_batch(rows, qs[:nq], K, 2, O.ORDER_PANAMA512, nthreads)
            rates.append(nq / (time.perf_counter() - t0))
        return float(np.median(rates)), rates

    qps_n, rates_n = median_qps(n_queries, threads, passes)
    nq1 = max(4, n_queries // threads)
    qps_1, rates_1 = median_qps(nq1, 1, 3)
    total_rows = N_SHARDS * ROWS_PER_SHARD
    scale = sample_rows / total_rows
    model, _ = cpu_info()
    return {
        "value": qps_n * scale,
        "unit": "queries/s",
        "cores": threads,
        "kind": "port",
        "value_1thread": qps_1 * scale,
        "min_max_of_passes": [min(rates_n) * scale, max(rates_n) * scale],
        "host_cpus": os.cpu_count(),
        "numa_node": node,
        "pinned_cpus": cores,
        "cpu_model": model,
        "isa": isa,
        "passes_qps_on_sample": [round(r, 2) for r in rates_n],
        "best_of_passes": max(rates_n) * scale,   # least disturbed by other tenants of the shared host
        "passes_1thread_qps_on_sample": [round(r, 2) for r in rates_1],
        "sample": (f"median of {passes} passes of {n_queries} queries × {sample_rows} rows × {DIM} fp32 COSINE k={K} "
                   f"({sample_rows * DIM * 4 / 1e9:.2f} GB, far beyond the LLC) on {threads} threads "
                   f"({qps_n:.1f} QPS on the sample; 1 thread: median of 3 passes of {nq1} queries, "
                   f"{qps_1:.2f} QPS), scaled ×{sample_rows}/{total_rows} to the 10M corpus (exact search is "
                   f"linear in rows); Lucene-equivalent restatement (Panama-512 order), not Lucene: no JDK/jar "
                   f"on the box"),
    }


def main():
    global K, SIZE
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--k", type=int, default=K, help="k (and size); the headline is k = 10. k > 12 takes the "
                    "select path (osk_select.hip), k ≤ 12 the prefilter's wave lists")
    ap.add_argument("--rows-per-shard", type=int, default=ROWS_PER_SHARD)
    ap.add_argument("--rank-share", default="", metavar="R/W",
                    help="stage only the shards rank R of a W-GPU run owns (shard s on rank s·W/8), on this one GPU: "
                         "the per-GPU share of an N = W run measured without its collective (e.g. 0/8: one shard "
                         "of 1.25M rows)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="queries in flight: search threads issuing round-robin, each on its own stream with its "
                         "own view (workspace) over the shared segments; 1 = strictly one query after another")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-every", type=int, default=8,
                    help="stamp the scan launches of every N-th search with HIP events (osk_view_profile N); the "
                         "stamps cost a few µs of stream time around the stamped launch, so the timed loop samples")
    ap.add_argument("--no-sq8", action="store_true", help="measure the fp32 streaming scan as the main path")
    ap.add_argument("--exchange", choices=["osk", "torch"], default="osk",
                    help="osk: the C-ABI step osk_shards_search_merge_device (RCCL all-gather inside libosknn; "
                         "torch.distributed/gloo only carries the communicator id and the timing barriers); "
                         "torch: torch.distributed.all_gather_into_tensor + osk_merge_device_ranked")
    ap.add_argument("--dist-backend", default="nccl",
                    help="--exchange torch only: nccl (= RCCL over xGMI, one GPU per rank); gloo to rehearse "
                         "N > 1 ranks on one GPU")
    ap.add_argument("--dump", default="", help="rank 0 writes the merged results of batches 0..7 to this .npz "
                    "(cross-N parity: the N-rank result must equal the 1-GPU result)")
    ap.add_argument("--mfma-min-batch", type=int, default=0,
                    help="A/B: batches ≥ this take the bf16×3 MFMA path (osk_tune mfma_min_batch; 0 = library default)")
    ap.add_argument("--sq8-mfma-min", type=int, default=-1,
                    help="A/B: prefilter batches ≥ this scan on int8 MFMA (osk_tune sq8_mfma_min; -1 = library default)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="A/B: extra osk_tune knobs (e.g. sq8_mfma_nt=0)")
    ap.add_argument("--tiles", type=int, default=0, help="A/B: workgroup tiles per view (osk_tune tiles_target)")
    # ≈15 s of CPU work (5 passes on the box's 16-thread share + 3 single-thread passes): a bounded C3 sample
    ap.add_argument("--cpu-sample-rows", type=int, default=524_288)
    ap.add_argument("--cpu-queries", type=int, default=256)
    a = ap.parse_args()

    K = SIZE = a.k
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.dist_backend == "gloo" and a.exchange == "torch":   # rehearsal: several ranks may share one GPU
        local_rank %= torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    if world > 1:
        if a.exchange == "osk" or a.dist_backend == "gloo":
            dist.init_process_group("gloo")   # host-side coordination only (id broadcast, barriers, max)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    if a.tiles:
        _lib.tune("tiles_target", a.tiles)
    for kv in a.tune:
        key, val = kv.split("=")
        _lib.tune(key, int(val))
    mfma_min_batch = a.mfma_min_batch or 96   # the library default (osk_internal.h)
    _lib.tune("mfma_min_batch", mfma_min_batch)
    sq8_mfma_min = 2 if a.sq8_mfma_min < 0 else a.sq8_mfma_min
    _lib.tune("sq8_mfma_min", sq8_mfma_min)
    t0 = time.perf_counter()
    s_rank, s_world = rank, world
    if a.rank_share:
        if world != 1:
            raise SystemExit("--rank-share emulates one rank's share on one GPU: run it with --gpus 1")
        s_rank, s_world = (int(x) for x in a.rank_share.split("/"))
    shards = D.LocalShards(s_rank, s_world, N_SHARDS, a.rows_per_shard, DIM, _lib.COSINE, _lib.FLOAT32, 42,
                           _lib.DIST_NORMALISH_UNIT, local_rank)
    torch.cuda.synchronize()
    rows_local = len(shards.shards) * a.rows_per_shard
    log(f"rank {rank}: staged shards {shards.shards} ({rows_local} rows) in {time.perf_counter() - t0:.1f}s")

    n_pool = 64
    qpool = torch.from_numpy(synth_host(0, n_pool * a.batch, DIM, 43, _lib.DIST_NORMALISH_UNIT)).cuda()
    B = a.batch
    keys = torch.empty((B, shards.s_pad, K), dtype=torch.int64, device="cuda")
    counts = torch.empty((B, shards.s_pad), dtype=torch.int32, device="cuda")
    # Queries in flight: F search "threads", each with its own stream and its own view over the same
    # staged segments (own workspace), issued round-robin — consecutive queries overlap on the device
    # (one query's settle / merge / exchange under the next one's scan), as concurrent requests from the
    # search pool do.  Explicit streams throughout: the null stream's handle is 0, which the C-ABI reads
    # as "the library's own (non-blocking) stream".
    F = 1 if a.exchange == "torch" else max(1, a.inflight)
    streams = [torch.cuda.Stream() for _ in range(F)]
    torch.cuda.set_stream(streams[0])
    views = [shards.view] + [shards.add_view() for _ in range(F - 1)]
    comm = None
    if a.exchange == "osk":
        # libosknn's own RCCL communicator (world 1: no collective runs, the local lists are the image)
        comm = (D.DeviceComm.from_process_group(local_rank) if world > 1
                else D.DeviceComm.init_rank(local_rank, 0, 1, D.DeviceComm.unique_id()))
        comm.set_device_limits(B, K, shards.s_pad)   # (every rank: the exchange block's fixed size)
        xsteps = [D.ShardSearchMerge(comm, v, shards.s_pad, B, K, FROM, SIZE, device=local_rank) for v in views]
    else:
        xchg = D.ShardExchange(world, shards.s_pad, B, K, FROM, SIZE, shards.global_shard_index, device=local_rank)

    def step(i, slots=F):
        q = qpool[(i % n_pool) * B:(i % n_pool + 1) * B]
        j = i % slots
        if comm is not None:   # scan + ONE RCCL all-gather of the per-shard top-k + device TopDocs.merge
            return xsteps[j](q.data_ptr(), streams[j].cuda_stream)
        shards.search(q.data_ptr(), B, K, keys, counts, streams[0].cuda_stream)
        return xchg(keys, streams[0].cuda_stream)   # torch all-gather of the per-shard top-k + device TopDocs.merge

    def profile(enable):
        for v in views:
            _lib.check(_lib.lib().osk_view_profile(v, enable))

    # setup: the first single queries calibrate the 6-bit tier per segment (asynchronous probes, folded by
    # later calls; osk_seg::sq6_state); issue them here, with the other one-time builds, not inside the warmup
    for i in range(4 * F):
        step(n_pool - 1 - (i % n_pool), F)
    torch.cuda.synchronize()

    def timed(steps, warmup, offset=0, slots=F):
        """W untimed steps, then K steps between barrier + synchronize; returns the max-over-ranks wall
        time, the mean scan-launch duration (HIP events on the launch streams), the GPU event time and
        the last step's output."""
        out = None
        for i in range(max(warmup, slots)):
            out = step(offset + i, slots)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        profile(max(1, a.profile_every))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t_start = time.perf_counter()
        ev0.record(streams[0])
        for s in streams[1:slots]:
            s.wait_stream(streams[0])
        for i in range(steps):
            out = step(offset + warmup + i, slots)
            if (i + 1) % 200 == 0:
                log(f"rank {rank}: step {i + 1}/{steps}")
        for s in streams[1:slots]:
            streams[0].wait_stream(s)
        ev1.record(streams[0])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        tot_ms, tot_calls = 0.0, 0
        for v in views:
            scan_ms, calls = C.c_double(), C.c_int64()
            _lib.check(_lib.lib().osk_view_scan_time(v, C.byref(scan_ms), C.byref(calls)))
            tot_ms, tot_calls = tot_ms + scan_ms.value, tot_calls + calls.value
        profile(0)
        t = torch.tensor([elapsed], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)   # max over ranks (host tensor: gloo or nccl)
        return float(t.item()), tot_ms / max(1, tot_calls), ev0.elapsed_time(ev1), out

    def counter(name):
        tot = 0
        for view in views:
            v = C.c_int64()
            _lib.check(_lib.lib().osk_view_counter(view, name.encode(), C.byref(v)))
            tot += v.value
        return tot

    _lib.tune("sq8", 0 if a.no_sq8 else 1)
    fb0, rs0, calls0 = counter("sq8_fallback_queries"), counter("sq8_rescored_rows"), counter("sq8_calls")
    sel0, six0, rb0 = counter("select_calls"), counter("sq6_calls"), counter("sq6_rebound_rows")
    elapsed_max, ovl_scan_ms, ev_ms, out = timed(a.steps, a.warmup)
    # The same steps one at a time (one query in flight): the per-query latency, and the scan kernel's
    # isolated launch duration — the roofline's denominator.  With F > 1 the launches of neighbouring
    # queries overlap on the device and share HBM, so their individual durations overstate the kernel's
    # time; the whole step's sustained rate is reported beside it.
    n_lat = min(a.steps, 50)
    if F > 1:
        lat_el, scan_avg_ms, _, _ = timed(n_lat, 2, slots=1)
    else:
        lat_el, scan_avg_ms, n_lat = elapsed_max, ovl_scan_ms, a.steps
    # the path the library chose (prefilter searches count sq8_calls, select-path searches select_calls;
    # else bf16×3 from batch 96, else fp32)
    prefilter = counter("sq8_calls") > calls0
    select = counter("select_calls") > sel0
    six = prefilter and counter("sq6_calls") > six0   # single queries on the 6-bit tier
    batched = not prefilter and not select and B >= 96 and K <= 12
    sq8_mfma = prefilter and sq8_mfma_min > 0 and B >= sq8_mfma_min
    # sanity on the last step: every query got `SIZE` hits from the 10M corpus
    cnt = out[3].cpu().numpy()
    assert np.all(cnt == SIZE), cnt

    u8 = (DIM + 15) // 16
    if select:
        passes = B
        bytes_per_launch = rows_local * (u8 * 16 + 16 + 8) * passes
        kernel_name = ("sel_bounds<16,3> select path writer (k > 12): int8 rows + 16-B bound terms read, 8-B LB/UB "
                       "written per row, one query per launch; then radix select, collect, exact re-score, sort")
    elif sq8_mfma:
        passes = (B + 31) // 32
        bytes_per_launch = rows_local * (u8 * 16 + 16) * passes
        kernel_name = ("sq8_mfma<KS=12,QB=2> certified int8 prefilter on v_mfma_i32_16x16x64_i8 (bytes = int8 rows "
                       "(tiled copy) + 16-B bound terms per row, once per launch of ≤ 32 queries; time = pilot + "
                       "pilot merge + main pass)")
    elif six:
        # the 6-bit codes (3/4 of the int8 row, dims padded to 256 per lane set) + 16-B bound terms of every
        # row, plus the int8 rows + bound terms the scan re-bounded (counted on the device, per launch)
        passes = B
        bytes_per_launch = rows_local * (((DIM + 255) // 256) * 192 + 16)
        kernel_name = ("sq6_scan<C=3,U=3> the 6-bit pass of the certified prefilter (bytes = 6-bit codes + 16-B "
                       "bound terms per row, one query per launch; its pilot and int8 re-bound kernels read "
                       "≈ 1 % more: sq6_pilot 0.021 GB, sq6_rebound 0.047 GB after its final-floor re-test, profiles/r06/pmc/)")
    elif prefilter:
        passes = (B + 7) // 8
        bytes_per_launch = rows_local * (u8 * 16 + 16) * passes
        kernel_name = (f"sq8_scan<L=16,V=3,NQ={min(8, 1 << max(0, (B - 1).bit_length()))}> certified int8 prefilter "
                       "(bytes = int8 rows + 16-B bound terms per row, once per launch of ≤ 8 queries)")
    elif batched:
        passes = (B + 255) // 256
        bytes_per_launch = rows_local * DIM * 4 * passes
        kernel_name = "mfma_cand (bf16x3 split MFMA candidates; bytes = the hi/lo copy read once per 256 queries)"
    else:
        passes = (B + 7) // 8
        bytes_per_launch = rows_local * DIM * 4 * passes
        kernel_name = "scan_f32<L=16,V=12,NQ=min(B,8),dot,nt>"
    achieved = bytes_per_launch / (scan_avg_ms * 1e-3) / 1e9
    mfma_tflops = (3 * 2 * B * rows_local * DIM) / (scan_avg_ms * 1e-3) / 1e12 if batched else None

    extra = {}
    if prefilter:
        n_calls = counter("sq8_calls") - calls0
        extra["prefilter"] = {
            "tier": "6-bit + int8 re-bound" if six else "int8",
            "int8_rebound_rows_per_query": ((counter("sq6_rebound_rows") - rb0) /
                                            max(1, counter("sq6_calls") - six0)) if six else None,
            "fallback_queries": counter("sq8_fallback_queries") - fb0,
            "rescored_rows_per_query": (counter("sq8_rescored_rows") - rs0) / max(1, n_calls * B),
            "searches": n_calls,
        }
        # the fp32 streaming scan on the same queries, same run: its own roofline, and the results
        # of both paths compared bit for bit (docs, scores, shard indices) on a sample of batches
        _lib.tune("sq8", 0)
        s_el, s_scan, _, _ = timed(min(a.steps, 50), 2, slots=1)
        mism = 0
        for i in range(min(8, n_pool)):
            ref = [t.clone() for t in step(i, 1)]
            _lib.tune("sq8", 1)
            got = step(i, 1)
            _lib.tune("sq8", 0)
            for j, (x, y) in enumerate(zip(got, ref)):
                same = torch.equal(x.view(torch.int32) if x.dtype == torch.float32 else x,
                                   y.view(torch.int32) if y.dtype == torch.float32 else y)
                if not same:
                    mism += 1
                    if mism <= 4:
                        log(f"mismatch batch {i} output {j}: prefilter {x.flatten()[:10].tolist()} "
                            f"fp32 {y.flatten()[:10].tolist()}")
        _lib.tune("sq8", 1)
        s_bytes = rows_local * DIM * 4 * ((B + 7) // 8)
        extra["fp32_stream"] = {
            "value": min(a.steps, 50) * B / s_el, "scan_ms_avg": s_scan,
            "roofline_achieved_GBps": s_bytes / (s_scan * 1e-3) / 1e9,
            "roofline_frac": s_bytes / (s_scan * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "kernel": "scan_f32<L=16,V=12,NQ=min(B,8),dot,nt>",
            "identical_to_prefilter_on_8_batches": mism == 0,
        }
        assert mism == 0, f"prefilter and fp32 scan results differ in {mism} tensors"

    if a.dump:
        outs = [[t.cpu().numpy().copy() for t in step(i, 1)] for i in range(min(8, n_pool))]
        if rank == 0:
            np.savez(a.dump, scores=np.stack([o[0] for o in outs]), docs=np.stack([o[1] for o in outs]),
                     shard=np.stack([o[2] for o in outs]), count=np.stack([o[3] for o in outs]),
                     total=np.stack([o[4] for o in outs]), max_score=np.stack([o[5] for o in outs]))

    traffic, traffic_src = pmc_traffic(rows_local, B, prefilter, six)
    ceiling = read_ceiling()
    if rank == 0:
        res = {
            "metric": "exact k-NN QPS@k=10 (recall=1.0), 10M×768 fp32, 1/2/4/8 GPUs; % HBM roofline",
            "value": a.steps * B / elapsed_max,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed_max / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device counter generator: Irwin-Hall(4)≈N(0,1), rows L2-normalised; seed 42/43)",
            "config": {"workload": f"C3 Cohere-shaped exact k-NN: 10M×768 fp32 COSINE, 8 shards, k={K}, from=0, size={SIZE}",
                       "batch": B, "rows": N_SHARDS * a.rows_per_shard, "dim": DIM, "shards": N_SHARDS,
                       "k": K,
                       "rank_share": (f"rank {s_rank} of {s_world}: shards {shards.shards} only, no collective "
                                      f"(the per-GPU share of an N = {s_world} run)") if a.rank_share else None,
                       "path": ("prefilter" if prefilter else "select" if select else "mfma" if batched
                                else "fp32_stream"),
                       "parallelism": (f"8 shards over {world} GPU(s); " + (
                           ("one C-ABI step per rank: scan + libosknn RCCL all-gather + device merge" if world > 1
                            else "one GPU: scan + device merge, no collective")
                           if a.exchange == "osk" else f"torch.distributed {a.dist_backend} all-gather + device merge"))},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "measured_read_ceiling_GBps": ceiling,
                         "frac_of_measured_read_ceiling": achieved / ceiling if ceiling else None,
                         "read_ceiling_source": os.path.relpath(READ_CEILING, ROOT) if ceiling else None,
                         "kernel": kernel_name, "scan_ms_avg": scan_avg_ms,
                         "scan_ms_measured_in": ("the one-in-flight pass of this run (isolated launches)" if F > 1
                                                 else "the timed region")
                         + f", every {max(1, a.profile_every)}th search's launch sampled",
                         "sustained_GBps": bytes_per_launch / (elapsed_max / a.steps) / 1e9,
                         "sustained_frac": bytes_per_launch / (elapsed_max / a.steps) / 1e9 / HBM_PEAK_GBS,
                         "overlapped_scan_ms_avg": ovl_scan_ms if F > 1 else None,
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "bf16_mfma_tflops": mfma_tflops},
            "gpu_event_ms_per_step": ev_ms / a.steps,
            "inflight": F,
        }
        res["one_in_flight"] = {"value": n_lat * B / lat_el, "latency_ms_per_step": lat_el / n_lat * 1e3}
        res.update(extra)
        if world == 1 and not a.no_cpu_baseline:
            # the GPU box grants 16 host threads per GPU (OMP_NUM_THREADS there); nproc shows the whole host
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
            res["cpu_baseline"] = cpu_baseline(a.cpu_sample_rows, a.cpu_queries, threads)
        print(json.dumps(res), flush=True)
    shards.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
