"""Micro-benchmark of the per-step latency kernels at batch 1 (run under rocprofv3 --kernel-trace --stats):
the coordinator merge alone (osk_merge_device_ranked, 8 shards × k=10, one query), and a 1.25M-row
8-shard prefilter search step (prep, scan, settle, settle_merge) followed by the merge."""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opensearch_amd import _lib, distributed as D  # noqa: E402
from opensearch_amd._lib import check, lib  # noqa: E402

torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
st = s.cuda_stream
S, K = 8, 10
keys = torch.randint(1, 2**62, (1, S, K), dtype=torch.int64, device="cuda")
keys = keys.sort(dim=2, descending=True).values
si = torch.arange(S, dtype=torch.int32, device="cuda")
out = [torch.empty(10, dtype=torch.float32, device="cuda"), torch.empty(10, dtype=torch.int32, device="cuda"),
       torch.empty(10, dtype=torch.int32, device="cuda"), torch.empty(1, dtype=torch.int32, device="cuda"),
       torch.empty(1, dtype=torch.int64, device="cuda"), torch.empty(1, dtype=torch.float32, device="cuda")]
for n in (20, 500):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        check(lib().osk_merge_device_ranked(0, keys.data_ptr(), 1, S, si.data_ptr(), 1, K, 0, 10,
                                            *[o.data_ptr() for o in out], st))
    torch.cuda.synchronize()
print(f"merge_coord back-to-back: {(time.perf_counter() - t) / 500 * 1e6:.2f} us/launch")

shards = D.LocalShards(0, 1, 8, 156250, 768, _lib.COSINE, _lib.FLOAT32, 42, _lib.DIST_NORMALISH_UNIT, 0)
q = torch.randn(1, 768, device="cuda")
kk = torch.empty((1, 8, K), dtype=torch.int64, device="cuda")
cc = torch.empty((1, 8), dtype=torch.int32, device="cuda")
x = D.ShardExchange(1, 8, 1, K, 0, 10, shards.global_shard_index, device=0)
for n in (20, 300):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        shards.search(q.data_ptr(), 1, K, kk, cc, st)
        x(kk, st)
    torch.cuda.synchronize()
print(f"1.25M-row step: {(time.perf_counter() - t) / 300 * 1e6:.1f} us/step")
shards.close()
