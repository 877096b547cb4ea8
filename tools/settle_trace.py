"""Phase timestamps of the prefilter settle (tune "settle_trace"): where a (slice, query) block spends
its time.  python tools/settle_trace.py [rows_per_shard] [batch]"""
import os
os.environ.setdefault("OSK_TESTING_LIB", "1")   # A/B knobs live in libosknn_testing.so
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from opensearch_amd import _lib, distributed as D  # noqa: E402
from opensearch_amd.lucene import synth_host  # noqa: E402

rps = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 1
torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
STREAM = torch.cuda.current_stream().cuda_stream
sh = D.LocalShards(0, 1, 8, rps, 768, _lib.COSINE, _lib.FLOAT32, 42, _lib.DIST_NORMALISH_UNIT, 0)
q = torch.from_numpy(synth_host(0, 16 * nq, 768, 43, _lib.DIST_NORMALISH_UNIT)).cuda()
keys = torch.zeros((nq, 8, 10), dtype=torch.int64, device="cuda")
counts = torch.zeros((nq, 8), dtype=torch.int32, device="cuda")
for i in range(8):   # warm-up (builds the int8 copy)
    sh.search(q[i * nq:(i + 1) * nq].data_ptr(), nq, 10, keys, counts, STREAM)
_lib.tune("settle_trace", 1)
for i in range(8, 16):
    sh.search(q[i * nq:(i + 1) * nq].data_ptr(), nq, 10, keys, counts, STREAM)
    torch.cuda.synchronize()
_lib.tune("settle_trace", 0)
v = C.c_int64()
_lib.check(_lib.lib().osk_view_counter(sh.view, b"sq8_slices", C.byref(v)))
ns = v.value
tr = np.zeros(nq * ns * 8, np.uint64)
_lib.check(_lib.lib().osk_view_debug_copy(sh.view, b"settle_trace", tr.ctypes.data, tr.nbytes))
tr = tr.reshape(nq * ns, 8).astype(np.int64)
t0 = tr[:, 0].min()
ns_ = lambda x: x * 10   # wall clock: 100 MHz
start = ns_(tr[:, 0] - t0)
end = ns_(tr[:, 4] - t0)
ph = [ns_(tr[:, i + 1] - tr[:, i]) for i in range(4)]
names = ["loads+max(a)", "rank+(b)", "(c) rescore", "(c')+(d)"]
print(f"slices={ns} batch={nq} blocks={nq * ns}  kernel span ≈ {end.max() / 1e3:.1f} us")
print(f"block start: p50 {np.percentile(start, 50) / 1e3:.1f} p90 {np.percentile(start, 90) / 1e3:.1f} "
      f"max {start.max() / 1e3:.1f} us")
for n, p in zip(names, ph):
    print(f"  {n:14s} p50 {np.percentile(p, 50) / 1e3:6.2f}  p90 {np.percentile(p, 90) / 1e3:6.2f}  "
          f"max {p.max() / 1e3:6.2f} us")
print(f"  block total    p50 {np.percentile(end - start, 50) / 1e3:6.2f}  max {(end - start).max() / 1e3:6.2f} us")
print(f"  candidates/block: mean {tr[:, 5].mean():.2f} max {tr[:, 5].max()}")
