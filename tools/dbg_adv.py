import numpy as np, sys
sys.path.insert(0, "/root/repo")
from opensearch_amd import _lib, lucene as LU
rng = np.random.default_rng(13)
rows = rng.standard_normal((5000, 64)).astype(np.float32) * 1e-3
rows[:, 0] = 1000.0
queries = rng.standard_normal((4, 64)).astype(np.float32)
for sim in [LU.VectorSimilarityFunction(s) for s in range(4)]:
    r = LU.GpuFlatVectorsReader("v", rows, sim)
    a = r.search_batch(queries, 10)
    _lib.tune("sq8", 0); b = r.search_batch(queries, 10); _lib.tune("sq8", 1)
    for q in range(4):
        if not np.array_equal(a[0][q].view(np.uint32), b[0][q].view(np.uint32)) or not np.array_equal(a[1][q], b[1][q]):
            print(sim.name, "q", q, "\n pre", a[1][q], a[0][q], "\n ref", b[1][q], b[0][q])
    r.close()
