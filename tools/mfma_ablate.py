"""A/B timing of the int8 MFMA prefilter's main pass (C3, 16 queries per search): full kernel vs
ablations (tune sq8_mfma_ablate: 1 no epilogue, 2 no MFMA, 3 loads only).  Results of ablated runs
are wrong; only the kernel time (osk_view_scan_time: pilot + merge + main) is reported."""
import os
os.environ.setdefault("OSK_TESTING_LIB", "1")   # A/B knobs live in libosknn_testing.so
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib, distributed as D  # noqa: E402
from opensearch_amd._lib import check, lib  # noqa: E402

# argv: [C3|C4|C2] [batch]  (C3: 8 × 1.25M × 768 COSINE; C4: 8 × 12.5M × 96 DOT_PRODUCT; C2: 8 × 125k × 128 L2)
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
K = 10
RPS, DIM, SIM = {"C3": (1_250_000, 768, _lib.COSINE), "C4": (12_500_000, 96, _lib.DOT_PRODUCT),
                 "C2": (125_000, 128, _lib.EUCLIDEAN)}[cfg]
# TUNE="key=value,..." sets library knobs (osk_tune_set) before staging
for kv in filter(None, os.environ.get("TUNE", "").split(",")):
    _lib.tune(kv.split("=")[0], int(kv.split("=")[1]))
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
st = s.cuda_stream
shards = D.LocalShards(0, 1, 8, RPS, DIM, SIM, _lib.FLOAT32, 42, _lib.DIST_NORMALISH_UNIT, 0)
q = torch.randn(B, DIM, device="cuda")
q = q / q.norm(dim=1, keepdim=True)
kk = torch.empty((B, 8, K), dtype=torch.int64, device="cuda")
cc = torch.empty((B, 8), dtype=torch.int32, device="cuda")
for ab in [int(x) for x in os.environ.get("ABLATE", "0,1,2,3,0").split(",")]:
    _lib.tune("sq8_mfma_ablate", ab)
    for _ in range(3):
        shards.search(q.data_ptr(), B, K, kk, cc, st)
    torch.cuda.synchronize()
    check(lib().osk_view_profile(shards.view, 1))
    for _ in range(10):
        shards.search(q.data_ptr(), B, K, kk, cc, st)
    torch.cuda.synchronize()
    ms, n = C.c_double(), C.c_int64()
    check(lib().osk_view_scan_time(shards.view, C.byref(ms), C.byref(n)))
    check(lib().osk_view_profile(shards.view, 0))
    print(f"{cfg} b{B} {os.environ.get('TUNE', '')} ablate={ab}: {ms.value / max(1, n.value):.3f} ms per scan (pilot+merge+main)", flush=True)
_lib.tune("sq8_mfma_ablate", 0)
shards.close()
