#!/usr/bin/env python3
"""Debug the batched MFMA path on a small case: compare the approx candidates it kept with numpy."""
import os
os.environ.setdefault("OSK_TESTING_LIB", "1")   # A/B knobs live in libosknn_testing.so
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib, lucene as LU  # noqa: E402
from oracle import oracle as O  # noqa: E402

n, dim, nq, sim = int(os.environ.get("N", 4096)), int(os.environ.get("DIM", 128)), 16, int(os.environ.get("SIM", 2))
rows = O.synth(0, n, dim, 7, 3)
qs = O.synth(0, nq, dim, 8, 3)
r = LU.GpuFlatVectorsReader("v", rows, sim)
ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)]])
out = ds.search(qs, 10, 0, 10)
print("stats", ds.stats())
KC = 16
ak = np.zeros(nq * KC, np.uint64)
_lib.check(_lib.lib().osk_view_debug_copy(ds.handle, b"akeys", ak.ctypes.data, ak.nbytes))
fl = np.zeros(nq, np.int32)
_lib.check(_lib.lib().osk_view_debug_copy(ds.handle, b"flags", fl.ctypes.data, fl.nbytes))
print("flags", fl)
ak = ak.reshape(nq, KC)
hi = (ak >> np.uint64(32)).astype(np.uint32)
lo = (ak & np.uint64(0xFFFFFFFF)).astype(np.uint32)
vrow = (0xFFFFFFFF - lo).astype(np.int64)
sa = np.where(hi & 0x80000000, hi & 0x7FFFFFFF, ~hi).astype(np.uint32).view(np.float32)
x = rows.astype(np.float64)
for q in range(3):
    qq = qs[q].astype(np.float64)
    cos = (x @ qq) / np.linalg.norm(x, axis=1) / np.linalg.norm(qq)
    score = (1 + cos) / 2
    top = np.argsort(-score)[:KC]
    print(f"q{q} approx rows {vrow[q][:8]} approx s {sa[q][:4]} (16th {sa[q][-1]:.6f})")
    print(f"    true rows  {top[:8]} true s {score[top[:4]]} (16th {score[top[-1]]:.6f})")
    print(f"    true score of approx rows {score[vrow[q][:4].clip(0, n - 1)]}")
    print("    result docs", out[1][q][:5], "scores", out[0][q][:3])
