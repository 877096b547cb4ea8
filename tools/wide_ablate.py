"""A/B timing of the wide int8 MFMA prefilter (osk_sq8w.hip) and its insertion-event counts.

    python tools/wide_ablate.py [C4|C2|C3] [batch]      (ABLATE="0,1,2,3" sq8_mfma_ablate values)

C4: 8 × 12.5M × 96 DOT_PRODUCT unit rows; C2: 1 × 1M × 128 EUCLIDEAN U[0,1)·128.  Runs on the testing build
(ablations; the kernel's event counters).  Reports per search: pilot + merge + main pass time
(osk_view_scan_time), insertion events (queries with a passing pair per 16-row group and wave) and
quick-test passes (pairs), each also per (query, quarter).  OSK_TESTING_LIB=0: the shipped library (ABLATE=0
only; its counters read 0) — the SQ counter passes of the shipped kernels (tools/pmc_wide_sq.sh)."""
import os
os.environ.setdefault("OSK_TESTING_LIB", "1")
import ctypes as C
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib, distributed as D  # noqa: E402
from opensearch_amd._lib import check, lib  # noqa: E402
from opensearch_amd.lucene import synth_host  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
K = 10
NS, RPS, DIM, SIM, DIST = {"C4": (8, 12_500_000, 96, _lib.DOT_PRODUCT, _lib.DIST_NORMALISH_UNIT),
                           "C2": (1, 1_000_000, 128, _lib.EUCLIDEAN, _lib.DIST_UNIFORM01_X128),
                           "C3": (8, 1_250_000, 768, _lib.COSINE, _lib.DIST_NORMALISH_UNIT)}[cfg]
_lib.tune("sq8_wide_min", 2)
_lib.tune("sq8_wide_force", 1)
for kv in filter(None, os.environ.get("TUNE", "").split(",")):
    _lib.tune(kv.split("=")[0], int(kv.split("=")[1]))
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
st = s.cuda_stream
shards = D.LocalShards(0, 1, NS, RPS, DIM, SIM, _lib.FLOAT32, 42, DIST, 0)
q = torch.from_numpy(synth_host(0, B, DIM, 43, DIST)).cuda()
kk = torch.empty((B, NS, K), dtype=torch.int64, device="cuda")
cc = torch.empty((B, NS), dtype=torch.int32, device="cuda")


SHIPPED = os.environ.get("OSK_TESTING_LIB") == "0"


def counter(name):
    v = C.c_int64()
    rc = lib().osk_view_counter(shards.view, name.encode(), C.byref(v))
    if SHIPPED and rc:   # (the shipped library has no testing counters)
        return 0
    check(rc)
    return v.value


tiles = C.c_int64()
for ab in [int(x) for x in os.environ.get("ABLATE", "0,1,2,3").split(",")]:
    if not SHIPPED:
        _lib.tune("sq8_mfma_ablate", ab)
    elif ab:
        raise SystemExit("the shipped library takes no ablation")
    for _ in range(2):
        shards.search(q.data_ptr(), B, K, kk, cc, st)
    torch.cuda.synchronize()
    e0, p0, w0 = counter("sq8_wide_events"), counter("sq8_wide_pairs"), counter("sq8_wide_calls")
    x0 = [counter(c) for c in ("sq8_fallback_queries", "sq8_exact_tiles", "sq8_rescored_rows")]
    cyc0 = [counter("sq8_wide_" + c + "_cycles") for c in ("wait", "loop", "slow", "drain")]
    slow0 = counter("sq8_wide_slow_steps")
    RC = ("total", "setup", "quarter_end", "first_wait", "setup_barrier", "setup_fragment")
    rows0 = [counter("sq8_rows_" + c + "_cycles") for c in RC]
    check(lib().osk_view_profile(shards.view, 1))
    n = 5
    for _ in range(n):
        shards.search(q.data_ptr(), B, K, kk, cc, st)
    torch.cuda.synchronize()
    ms, calls = C.c_double(), C.c_int64()
    check(lib().osk_view_scan_time(shards.view, C.byref(ms), C.byref(calls)))
    check(lib().osk_view_profile(shards.view, 0))
    ev, pr, wc = counter("sq8_wide_events") - e0, counter("sq8_wide_pairs") - p0, counter("sq8_wide_calls") - w0
    launches = max(1, wc) * ((B + 255) // 256)
    print(f"{cfg} b{B} ablate={ab}: {ms.value / max(1, calls.value):.3f} ms per search (pilot+merge+main), "
          f"wide calls {wc}/{n}, events/search {ev / n:.0f}, pairs/search {pr / n:.0f}", flush=True)
    x1 = [counter(c) - c0 for c0, c in zip(x0, ("sq8_fallback_queries", "sq8_exact_tiles", "sq8_rescored_rows"))]
    print(f"   settle per search: fallback queries {x1[0] / n:.1f}, exactly re-scanned lists {x1[1] / n:.1f}, "
          f"re-scored rows {x1[2] / n:.0f}", flush=True)
    cyc = [counter("sq8_wide_" + c + "_cycles") - c0 for c0, c in zip(cyc0, ("wait", "loop", "slow", "drain"))]
    slow = counter("sq8_wide_slow_steps") - slow0
    rows = NS * RPS
    wave_steps = launches * (rows / 16.0) * 8 / ({96: 8, 128: 8, 768: 2}.get(DIM, 4))
    print(f"   wave-steps on the slow path per search: {slow / n:.0f} ({slow / max(1.0, wave_steps):.3f} of "
          f"≈{wave_steps / n:.0f})", flush=True)
    # wave 0's shader clocks summed over workgroups (pilot + main): per workgroup per search, and the split
    wgs = 256 * 2 * n
    print(f"   clocks per wg-launch (wave 0): loop {cyc[1] / wgs:.0f}, wait+barrier {cyc[0] / wgs:.0f} "
          f"({cyc[0] / max(1, cyc[1]):.2f}), slow-path enqueues {cyc[2] / wgs:.0f} ({cyc[2] / max(1, cyc[1]):.2f}), "
          f"quarter-end drains + flushes {cyc[3] / wgs:.0f} ({cyc[3] / max(1, cyc[1]):.2f})", flush=True)
    rows = [counter("sq8_rows_" + c + "_cycles") - c0 for c0, c in zip(rows0, RC)]
    if rows[0]:   # sq8_wide_rows (main passes): wave 0 per workgroup-launch, 2 launches per search
        rw = 256 * 2 * n
        print(f"   sq8_wide_rows clocks per wg-launch (wave 0): total {rows[0] / rw:.0f}, setup {rows[1] / rw:.0f}, "
              f"quarter ends {rows[2] / rw:.0f}, first-group waits {rows[3] / rw:.0f} (setup: to the barrier "
              f"{rows[4] / rw:.0f}, then the fragments {rows[5] / rw:.0f})", flush=True)
if not SHIPPED:
    _lib.tune("sq8_mfma_ablate", 0)
shards.close()
