"""Diagnostics for sq8_wide_rows: which queries differ from the fp32 scan, per similarity / queue cap / zero query."""
import sys

import numpy as np

sys.path.insert(0, ".")
from opensearch_amd import _lib, lucene as LU  # noqa: E402
from oracle import oracle as O  # noqa: E402

SIM = LU.VectorSimilarityFunction


def corpus(n, dim, sim, seed):
    dist = {0: 1, 1: 3, 2: 3, 3: 2}[int(sim)]
    return O.synth(0, n, dim, seed, dist)


def run(sim, zero_query, nq, sizes):
    rows_list = [corpus(n, 96, sim, 80 + i) for i, n in enumerate(sizes)]
    n_shards = 3 if len(sizes) == 4 else 1
    shard_of = [0, 0, 1, 2][:len(sizes)] if n_shards == 3 else [0] * len(sizes)
    leaves = [[] for _ in range(n_shards)]
    readers, bases = [], [0] * n_shards
    for rows, s in zip(rows_list, shard_of):
        r = LU.GpuFlatVectorsReader("v", rows, sim)
        readers.append(r)
        leaves[s].append(LU.LeafReaderContext(len(leaves[s]), bases[s], r))
        bases[s] += len(rows)
    ds = LU.DeviceShardSet(leaves, None)
    q = corpus(nq, 96, sim, 90)
    if zero_query:
        q[7] = 0.0
    _lib.tune("sq8", 0)
    ref = ds.search(q, 10, 0, 10)
    _lib.tune("sq8", 1)
    for rows_on in (1, 0):
        _lib.tune("sq8_wide_rows", rows_on)
        out = ds.search(q, 10, 0, 10)
        bad = [i for i in range(nq) if not (np.array_equal(out[1][i], ref[1][i]) and
                                           np.array_equal(out[0][i].view(np.uint32), ref[0][i].view(np.uint32)))]
        print(f"sim={sim.name} zero={zero_query} nq={nq} sizes={sizes} rows={rows_on}: {len(bad)} differ {bad[:12]}",
              flush=True)
        for i in bad[:2]:
            print("   got ", out[1][i].tolist(), out[0][i].tolist())
            print("   want", ref[1][i].tolist(), ref[0][i].tolist())
    _lib.tune("sq8_wide_rows", 1)
    ds.close()
    for r in readers:
        r.close()


_lib.tune("sq8_wide_min", 48)
_lib.tune("sq8_wide_force", 1)
for sim in (SIM.COSINE, SIM.DOT_PRODUCT):
    for zero in (True, False):
        for nq in (300, 256):
            run(sim, zero, nq, [23001, 1, 7000, 16])
run(SIM.COSINE, False, 256, [23001])
