"""A/B timing of the int8 MFMA prefilter's main pass (C3, 16 queries per search): full kernel vs
ablations (tune sq8_mfma_ablate: 1 no epilogue, 2 no MFMA, 3 loads only).  Results of ablated runs
are wrong; only the kernel time (osk_view_scan_time: pilot + merge + main) is reported."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib, distributed as D  # noqa: E402
from opensearch_amd._lib import check, lib  # noqa: E402

torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
st = s.cuda_stream
B, K = 16, 10
shards = D.LocalShards(0, 1, 8, 1_250_000, 768, _lib.COSINE, _lib.FLOAT32, 42, _lib.DIST_NORMALISH_UNIT, 0)
q = torch.randn(B, 768, device="cuda")
q = q / q.norm(dim=1, keepdim=True)
kk = torch.empty((B, 8, K), dtype=torch.int64, device="cuda")
cc = torch.empty((B, 8), dtype=torch.int32, device="cuda")
for ab in (0, 1, 2, 3, 0):
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
    print(f"ablate={ab}: {ms.value / max(1, n.value):.3f} ms per 16-query scan (pilot+merge+main)", flush=True)
_lib.tune("sq8_mfma_ablate", 0)
shards.close()
