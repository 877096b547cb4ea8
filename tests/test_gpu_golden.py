"""The HIP path against the committed golden fixtures (tests/golden/knn_golden.npz, made by
tests/golden/make_golden.py from the CPU oracle; label: restatement of Lucene 10.3.0 semantics — not
produced by Lucene, parity unpinned for scoring).

Every similarity × {float32 at dims 5/40/100, int8 at dims 16/40}, 200 rows with 20 exact duplicates
(exact ties), dense and sparse (ord→doc over 400 docs) with an accept bitset, k = 7, 3 queries:
  * the device summation order (o0): docs AND score bits identical;
  * Lucene's Panama-512 (o2) and scalar (o1) orders (float32): scores within the north star's 1e-5
    relative tolerance, position by position.
The fixtures are frozen, so a change in either the oracle or the library shows up here.
"""
from pathlib import Path

import numpy as np
import pytest

from opensearch_amd import lucene as LU

pytestmark = pytest.mark.gpu

GOLDEN = np.load(Path(__file__).resolve().parent / "golden" / "knn_golden.npz")
KEYS = sorted({k.rsplit("_", 1)[0] for k in GOLDEN.files if k.endswith("_rows")})
K = 7
REL_TOL = 1e-5


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("key", KEYS)
@pytest.mark.parametrize("variant", ["dense", "sparse_filtered"])
def test_golden_vectors(key, variant):
    enc, sim, _dim = key.split("_")
    rows, queries = GOLDEN[f"{key}_rows"], GOLDEN[f"{key}_queries"]
    encoding = LU.VectorEncoding.FLOAT32 if enc == "f32" else LU.VectorEncoding.BYTE
    similarity = LU.VectorSimilarityFunction(int(sim))
    if variant == "dense":
        reader = LU.GpuFlatVectorsReader("v", rows, similarity, encoding)
        accept = None
    else:
        reader = LU.GpuFlatVectorsReader("v", rows, similarity, encoding, ord_to_doc=GOLDEN[f"{key}_ord_to_doc"],
                                         max_doc=400)
        accept = GOLDEN[f"{key}_accept"]
    try:
        s, d, c, _ = reader.search_batch(queries, K, accept)
    finally:
        reader.close()
    want_c = GOLDEN[f"{key}_o0_{variant}_count"]
    want_d = GOLDEN[f"{key}_o0_{variant}_docs"]
    want_s = GOLDEN[f"{key}_o0_{variant}_scores"]
    assert np.array_equal(c, want_c)
    for i in range(len(queries)):
        n = c[i]
        assert np.array_equal(d[i, :n], want_d[i, :n]), (i, d[i, :n], want_d[i, :n])
        assert np.array_equal(bits(s[i, :n]), bits(want_s[i, :n])), (i, s[i, :n], want_s[i, :n])
        if enc == "f32":
            for order in (1, 2):   # Lucene's scalar and Panama-512 summation orders
                ls = GOLDEN[f"{key}_o{order}_{variant}_scores"][i, :n]
                np.testing.assert_allclose(s[i, :n], ls, rtol=REL_TOL, atol=1e-30)
