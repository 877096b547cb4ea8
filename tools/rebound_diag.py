"""Single-query chain time on the 6-bit tier (C3 10M × 768 COSINE) and sq6_rebound's counters.

    TUNE=sq6_rebound_stride=0 python tools/rebound_diag.py [n_queries]

Reports the GPU time of one search (HIP events around the whole chain, one in flight), the 6-bit candidates
per search, how many of them survive the re-test against the final floor (the rows gathered from the int8
copy), and on the testing build (OSK_TESTING_LIB=1, the default) the 8-row passes and the slowest
workgroup's shader clocks."""
import os
os.environ.setdefault("OSK_TESTING_LIB", "1")
import ctypes as C
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib, distributed as D  # noqa: E402
from opensearch_amd._lib import check, lib  # noqa: E402
from opensearch_amd.lucene import synth_host  # noqa: E402

NQ = int(sys.argv[1]) if len(sys.argv) > 1 else 64
NS, RPS, DIM, K = 8, 1_250_000, 768, 10
for kv in filter(None, os.environ.get("TUNE", "").split(",")):
    _lib.tune(kv.split("=")[0], int(kv.split("=")[1]))
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
st = s.cuda_stream
shards = D.LocalShards(0, 1, NS, RPS, DIM, _lib.COSINE, _lib.FLOAT32, 42, _lib.DIST_NORMALISH_UNIT, 0)
q = torch.from_numpy(synth_host(0, NQ + 8, DIM, 43, _lib.DIST_NORMALISH_UNIT)).cuda()
kk = torch.empty((1, NS, K), dtype=torch.int64, device="cuda")
cc = torch.empty((1, NS), dtype=torch.int32, device="cuda")


def counter(name):
    v = C.c_int64()
    check(lib().osk_view_counter(shards.view, name.encode(), C.byref(v)))
    return v.value


for i in range(8):   # the calibration probes and warm-up
    shards.search(q[i].data_ptr(), 1, K, kk, cc, st)
torch.cuda.synchronize()
r0, g0, p0 = counter("sq6_rebound_rows"), counter("sq6_rebound_gathered_rows"), counter("sq6_rebound_passes")
ms = []
for i in range(NQ):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    shards.search(q[8 + i].data_ptr(), 1, K, kk, cc, st)
    e1.record(s)
    e1.synchronize()
    ms.append(e0.elapsed_time(e1))
ms.sort()
reb, gat = counter("sq6_rebound_rows") - r0, counter("sq6_rebound_gathered_rows") - g0
passes = counter("sq6_rebound_passes") - p0
waves = 4 * 4 * 256
print(f"{os.environ.get('TUNE', '')}: chain median {ms[len(ms) // 2] * 1e3:.1f} us, min {ms[0] * 1e3:.1f} us over "
      f"{NQ} queries; sq6 calls {counter('sq6_calls')}", flush=True)
print(f"   6-bit candidates/search {reb / NQ:.0f}, gathered after the final-floor re-test {gat / NQ:.0f}; "
      f"passes/search {passes / NQ:.0f} (mean per wave {passes / NQ / waves:.2f}); slowest workgroup ever: "
      f"{counter('sq6_rebound_max_wg_cycles')} clocks", flush=True)
