"""The C-ABI library on a machine without a GPU: it loads, exports every symbol include/osknn.h
declares, its host-only entry points (reduce, key decode, generator) are right, and every device
entry point fails loudly with OSK_ERR_NO_DEVICE instead of falling back to the CPU."""
import ctypes as C
import json
import re
from pathlib import Path

import numpy as np
import pytest
import torch

from opensearch_amd import _lib, lucene as LU
from oracle import oracle as O

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "osknn.h"
GOLDEN = ROOT / "tests" / "golden"

no_gpu = pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device error path")


def header_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(osk_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    syms = header_symbols()
    assert len(syms) >= 20
    L = C.CDLL(str(_lib.LIB_PATH))
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_lib.SIGNATURES) == syms, "ctypes table out of sync with include/osknn.h"


def test_abi_version_and_constants():
    assert _lib.lib().osk_abi_version() == _lib.OSK_ABI_VERSION == 2
    text = HEADER.read_text()
    for name in ["OSK_ABI_VERSION", "OSK_COMM_ID_BYTES", "OSK_WARM_PREFILTER", "OSK_WARM_PREFILTER_MFMA", "OSK_WARM_BATCHED",
                 "OSK_WARM_ALL", "OSK_MAX_K", "OSK_EUCLIDEAN", "OSK_DOT_PRODUCT", "OSK_COSINE", "OSK_MAXIMUM_INNER_PRODUCT",
                 "OSK_FLOAT32", "OSK_BYTE", "OSK_ERR_NO_DEVICE"]:
        val = int(re.search(rf"#define {name}\s+(-?\d+)", text).group(1))
        py = name if name.startswith(("OSK_ERR", "OSK_MAX_", "OSK_COMM", "OSK_WARM", "OSK_ABI")) else name[4:]
        assert getattr(_lib, py) == val


@no_gpu
def test_device_entry_points_fail_loudly_without_gpu():
    with pytest.raises(_lib.OskError) as e:
        LU.GpuFlatVectorsReader("v", np.ones((4, 8), np.float32), LU.VectorSimilarityFunction.COSINE)
    assert e.value.code == _lib.OSK_ERR_NO_DEVICE
    h = C.c_void_p()
    rc = _lib.lib().osk_seg_synth(0, 10, 8, 0, 0, 1, 0, 0, C.byref(h))
    assert rc == _lib.OSK_ERR_NO_DEVICE and "no HIP device" in _lib.lib().osk_last_error().decode()
    assert _lib.lib().osk_merge_device(0, None, None, None, 1, 1, 10, 0, 10, *([None] * 7)) != 0
    uid = (C.c_uint8 * _lib.OSK_COMM_ID_BYTES)()
    assert _lib.lib().osk_comm_unique_id(uid) == _lib.OSK_ERR_NO_DEVICE
    comm = C.c_void_p()
    assert _lib.lib().osk_comm_init_rank(0, 0, 1, uid, C.byref(comm)) == _lib.OSK_ERR_NO_DEVICE


def test_testing_knobs_only_in_the_testing_build():
    """The shipped library refuses the result-corrupting A/B and test knobs; the testing build takes them."""
    for key in ["sq8_force_fallback", "sq8_mfma_ablate", "mfma_ablate", "settle_trace"]:
        assert _lib.lib().osk_tune_set(key.encode(), 1) == _lib.OSK_ERR_UNSUPPORTED
        with _lib.testing() as T:
            assert T.osk_tune_set(key.encode(), 1) == 0 and T.osk_tune_set(key.encode(), 0) == 0
    assert _lib.lib().osk_view_debug_copy(None, b"qc", None, 0) == _lib.OSK_ERR_UNSUPPORTED
    for key, bad in [("sq8", 2), ("sq8_mfma_queries", 24), ("tiles_target", -1), ("nope", 0)]:
        assert _lib.lib().osk_tune_set(key.encode(), bad) == _lib.OSK_ERR_INVALID


def test_host_generator_matches_oracle_generator():
    for dist in range(5):
        assert np.array_equal(LU.synth_host(11, 33, 70, 9, dist), O.synth(11, 33, 70, 9, dist))


def _key(score, doc):
    u = np.float32(score).view(np.uint32).item()
    s = (~u & 0xFFFFFFFF) if u & 0x80000000 else (u | 0x80000000)
    return (s << 32) | (0xFFFFFFFF - doc)


def test_key_order_is_lucene_order_and_decodes():
    hits = [(0.5, 7), (0.5, 3), (1.0, 100), (0.25, 0), (0.0, 1), (3.5, 2**31 - 2)]
    keys = np.array([_key(s, d) for s, d in hits], np.uint64)
    order = sorted(range(len(hits)), key=lambda i: -int(keys[i]))   # larger key = better hit
    assert [hits[i] for i in order] == sorted(hits, key=lambda h: (-h[0], h[1]))
    s, d = LU.decode_keys(np.append(keys, np.uint64(0)))
    assert list(d[:-1]) == [h[1] for h in hits] and np.allclose(s[:-1], [h[0] for h in hits])
    assert np.isneginf(s[-1]) and d[-1] == 2**31 - 1


def test_host_reduce_reference_known_answers():
    for case in json.loads((GOLDEN / "merge_known_answers.json").read_text()):
        tds = [LU.TopDocs(LU.TotalHits(s["total_hits"]),
                          [LU.ScoreDoc(d, sc, s["shard_index"]) for sc, d in zip(s["scores"], s["docs"])])
               for s in case["shards"]]
        m = LU.TopDocs.merge(case["from"], case["size"], tds)
        if "expected_scores" in case:
            assert [h.score for h in m.score_docs] == case["expected_scores"]
        if "expected_docs" in case:
            assert [h.doc for h in m.score_docs] == case["expected_docs"]
            assert [h.shard_index for h in m.score_docs] == case["expected_shards"]
        assert m.total_hits.value == case["expected_total_hits"]


@pytest.mark.parametrize("seed", range(20))
def test_host_reduce_matches_oracle_randomized(seed):
    """SearchPhaseControllerTests.testSortDocs-style randomized merges (ties included) vs the oracle."""
    rng = np.random.default_rng(seed)
    n_shards = int(rng.integers(1, 20))
    shards = []
    for s in range(n_shards):
        n = int(rng.integers(0, 12))
        sc = np.sort(rng.choice([0.25, 0.5, 1.0, 2.0], n) if seed % 2 else rng.random(n).astype(np.float32))[::-1]
        shards.append((np.asarray(sc, np.float32), np.arange(n, dtype=np.int32) * 3))
    sidx = rng.permutation(n_shards).astype(np.int32)
    from_, size = int(rng.integers(0, 8)), int(rng.integers(1, 15))
    es, ed, esh, etot, emx = O.topdocs_merge(shards, from_, size, sidx)
    counts = np.array([len(s[0]) for s in shards], np.int32)
    stride = max(1, counts.max())
    sc = np.zeros((n_shards, stride), np.float32)
    dc = np.zeros((n_shards, stride), np.int32)
    for i, (s, d) in enumerate(shards):
        sc[i, : len(s)], dc[i, : len(d)] = s, d
    os_, od, osh = np.empty(size, np.float32), np.empty(size, np.int32), np.empty(size, np.int32)
    cnt, tot, mx = C.c_int32(), C.c_int64(), C.c_float()
    _lib.check(_lib.lib().osk_topdocs_merge(n_shards, counts.ctypes.data, sc.ctypes.data, dc.ctypes.data, stride,
                                            sidx.ctypes.data, None, from_, size, os_.ctypes.data, od.ctypes.data,
                                            osh.ctypes.data, C.byref(cnt), C.byref(tot), C.byref(mx)))
    n = cnt.value
    assert n == len(ed) and np.array_equal(od[:n], ed) and np.array_equal(osh[:n], esh)
    assert np.array_equal(os_[:n], es) and tot.value == etot
    assert (np.isnan(mx.value) and np.isnan(emx)) or mx.value == emx
    assert np.all(osh[n:] == -1) and np.all(np.isneginf(os_[n:]))


def test_host_reduce_rejects_bad_arguments():
    cnt, tot, mx = C.c_int32(), C.c_int64(), C.c_float()
    rc = _lib.lib().osk_topdocs_merge(-1, None, None, None, 1, None, None, 0, 0, None, None, None,
                                      C.byref(cnt), C.byref(tot), C.byref(mx))
    assert rc == _lib.OSK_ERR_INVALID and "bad argument" in _lib.lib().osk_last_error().decode()
