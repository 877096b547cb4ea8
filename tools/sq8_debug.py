"""Diagnose prefilter vs fp32-scan differences on the bench corpus (per-shard keys)."""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from opensearch_amd import _lib, distributed as D  # noqa: E402
from opensearch_amd.lucene import synth_host  # noqa: E402

rps = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 4
torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
STREAM = torch.cuda.current_stream().cuda_stream
sh = D.LocalShards(0, 1, 8, rps, 768, _lib.COSINE, _lib.FLOAT32, 42, _lib.DIST_NORMALISH_UNIT, 0)
q = torch.from_numpy(synth_host(0, nq, 768, 43, _lib.DIST_NORMALISH_UNIT)).cuda()
K = 10


def run(sq8):
    _lib.tune("sq8", sq8)
    keys = torch.zeros((nq, 8, K), dtype=torch.int64, device="cuda")
    counts = torch.zeros((nq, 8), dtype=torch.int32, device="cuda")
    for b in range(nq):
        sh.search(q[b:b + 1].data_ptr(), 1, K, keys[b:b + 1], counts[b:b + 1], STREAM)
    torch.cuda.synchronize()
    return keys.cpu().numpy().view(np.uint64), counts.cpu().numpy()


def counter(name):
    v = C.c_int64()
    _lib.check(_lib.lib().osk_view_counter(sh.view, name.encode(), C.byref(v)))
    return v.value


k1, c1 = run(1)
print("counters", {n: counter(n) for n in ["sq8_calls", "sq8_fallback_queries", "sq8_rescored_rows"]})
k0, c0 = run(0)
bad = 0
for b in range(nq):
    for s in range(8):
        if not np.array_equal(k1[b, s], k0[b, s]) or c1[b, s] != c0[b, s]:
            bad += 1
            if bad <= 6:
                def dec(k):
                    return [(float(np.uint32(x >> 32).view(np.float32)) if False else hex(int(x >> 32)), 0xFFFFFFFF - int(x & 0xFFFFFFFF)) for x in k]
                print(f"q{b} shard{s} counts {c1[b, s]} vs {c0[b, s]}")
                print("  sq8 :", dec(k1[b, s]))
                print("  fp32:", dec(k0[b, s]))
print("mismatching (query, shard) pairs:", bad, "of", nq * 8)
