"""A/B timing of the 6-bit prefilter tier at C3 (8 × 1.25M × 768 COSINE, single queries): the int8 scan
(sq8_scan) against the 6-bit scan (sq6_scan) and its ablations (tune sq8_mfma_ablate in the testing
build: 1 drop the int8 re-bound queue, 2 no floor, 3 both — results wrong, kernel time only).
Prints one JSON line per variant: mean scan launch (HIP events, osk_view_scan_time), int8 re-bounds
and exactly re-scored rows per query."""
import os
os.environ.setdefault("OSK_TESTING_LIB", "1")   # A/B knobs live in libosknn_testing.so
import ctypes as C
import json
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib, distributed as D  # noqa: E402
from opensearch_amd._lib import check, lib  # noqa: E402

RPS = int(os.environ.get("RPS", "1250000"))
DIM, K, N = 768, 10, int(os.environ.get("N", "40"))
for kv in filter(None, os.environ.get("TUNE", "").split(",")):
    _lib.tune(kv.split("=")[0], int(kv.split("=")[1]))
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
st = s.cuda_stream
shards = D.LocalShards(0, 1, 8, RPS, DIM, _lib.COSINE, _lib.FLOAT32, 42, _lib.DIST_NORMALISH_UNIT, 0)
g = torch.Generator(device="cuda").manual_seed(43)
q = torch.randn(N, DIM, device="cuda", generator=g)
q = q / q.norm(dim=1, keepdim=True)
kk = torch.empty((1, 8, K), dtype=torch.int64, device="cuda")
cc = torch.empty((1, 8), dtype=torch.int32, device="cuda")


def counter(name):
    v = C.c_int64()
    check(lib().osk_view_counter(shards.view, name.encode(), C.byref(v)))
    return v.value


_lib.tune("sq6_probe_pct", 100)   # keep the tier whatever the calibration says (A/B)
VARIANTS = [("int8", 0, 0), ("sq6", 1, 0), ("sq6_no_rebound", 1, 1), ("sq6_no_floor", 1, 2),
            ("sq6_no_store", 1, 4), ("sq6_no_lb", 1, 8), ("sq6_no_store_no_lb", 1, 12), ("sq6_loads_only", 1, 1 | 2 | 16), ("sq6_no_cand", 1, 1 | 2), ("sq6", 1, 0), ("int8", 0, 0)]
only = os.environ.get("ONLY")   # e.g. ONLY=sq6 (rocprof runs)
for name, six, ab in VARIANTS:
    if only and name not in only.split(","):
        continue
    _lib.tune("sq6", six)
    _lib.tune("sq8_mfma_ablate", ab)
    for i in range(6):
        shards.search(q[i % N].data_ptr(), 1, K, kk, cc, st)
    torch.cuda.synchronize()
    rb0, rs0 = counter("sq6_rebound_rows"), counter("sq8_rescored_rows")
    check(lib().osk_view_profile(shards.view, 1))
    for i in range(N):
        shards.search(q[i].data_ptr(), 1, K, kk, cc, st)
    torch.cuda.synchronize()
    ms, calls = C.c_double(), C.c_int64()
    check(lib().osk_view_scan_time(shards.view, C.byref(ms), C.byref(calls)))
    check(lib().osk_view_profile(shards.view, 0))
    print(json.dumps({"variant": name, "scan_ms": ms.value / max(1, calls.value), "calls": calls.value,
                      "rebound_per_query": (counter("sq6_rebound_rows") - rb0) / N,
                      "rescored_per_query": (counter("sq8_rescored_rows") - rs0) / N}), flush=True)
_lib.tune("sq8_mfma_ablate", 0)
shards.close()
