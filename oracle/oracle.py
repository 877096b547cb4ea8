"""ctypes wrapper of liboracle.so — the CPU restatement of Lucene's exact k-NN semantics.

TEST INFRASTRUCTURE ONLY (see lucene_oracle.c's header): imported by tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg — never by opensearch_amd/.
Scoring parity is UNPINNED (no Lucene jar / JDK / vector fixture exists in the reference);
the merge is pinned by the reference's SearchPhaseController / FetchSearchPhase known-answer tests.
"""
from __future__ import annotations

import ctypes as C
import subprocess
import threading
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"

ORDER_DEVICE = 0
ORDER_SCALAR = 1
ORDER_PANAMA512 = 2
ORDER_SCALAR_NOFMA = 3      # Lucene's orders where Constants.HAS_FAST_*_FMA is false: multiply, then add
ORDER_PANAMA512_NOFMA = 4

LIB_V4_PATH = HERE / "liboracle_v4.so"   # same source, x86-64-v4 (AVX-512) build: the CPU baseline's
_lock = threading.Lock()
_lib = None
_variant = "v3"


def build(force: bool = False) -> Path:
    src = HERE / "lucene_oracle.c"
    stale = any(not p.exists() or p.stat().st_mtime < src.stat().st_mtime for p in (LIB_PATH, LIB_V4_PATH))
    if force or stale:
        subprocess.run(["make", "-s", "-B" if force else "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def host_has_avx512() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    return " avx512f " in line + " "
    except OSError:
        pass
    return False


def use_build(variant: str) -> str:
    """Select the build before the first call: "v4" (AVX-512, only where the host has avx512f) or "v3"
    (AVX2, the default).  Returns the ISA label of the build that will be loaded."""
    global _variant
    with _lock:
        if _lib is not None:
            raise RuntimeError("the oracle library is already loaded")
        _variant = "v4" if variant == "v4" and host_has_avx512() else "v3"
    return isa()


def isa() -> str:
    return ("AVX-512, x86-64-v4 build (16 fp32 lanes)" if _variant == "v4"
            else "AVX2, x86-64-v3 build (8 fp32 lanes)")


def lib() -> C.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            build()
            L = C.CDLL(str(LIB_V4_PATH if _variant == "v4" else LIB_PATH))
            P, I32, I64, U64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
            L.orc_synth.argtypes = [P, I64, I64, I32, U64, I32]
            L.orc_score_f32.argtypes = [P, P, I32, I32, I32]
            L.orc_score_f32.restype = C.c_float
            L.orc_score_i8.argtypes = [P, P, I32, I32]
            L.orc_score_i8.restype = C.c_float
            L.orc_exact_search_f32.argtypes = [P, I64, I32, P, P, P, I32, I32, I32, P, P, P]
            L.orc_exact_search_i8.argtypes = [P, I64, I32, P, P, P, I32, I32, P, P, P]
            L.orc_topdocs_merge.argtypes = [I32, P, P, P, I32, P, I32, I32, P, P, P, P, P]
            L.orc_knn_batch_f32.argtypes = [P, I64, I32, P, I32, I32, I32, I32, I32, P, P, P]
            _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def synth(row0: int, n: int, dim: int, seed: int, dist: int) -> np.ndarray:
    out = np.empty((n, dim), np.int8 if dist == 4 else np.float32)
    lib().orc_synth(_p(out), row0, n, dim, seed, dist)
    return out


def synth_par(row0: int, n: int, dim: int, seed: int, dist: int, nthreads: int = 8) -> np.ndarray:
    """synth() in row chunks on `nthreads` threads (the generator is a counter hash of the global row
    index, so chunking does not change a byte; ctypes drops the GIL for each call)."""
    from concurrent.futures import ThreadPoolExecutor
    out = np.empty((n, dim), np.int8 if dist == 4 else np.float32)
    step = max(1, -(-n // max(1, nthreads)))
    L = lib()

    def run(i0):
        L.orc_synth(out.ctypes.data + i0 * out.strides[0], row0 + i0, min(step, n - i0), dim, seed, dist)

    with ThreadPoolExecutor(max(1, nthreads)) as ex:
        list(ex.map(run, range(0, n, step)))
    return out


def score(q: np.ndarray, x: np.ndarray, sim: int, order: int = ORDER_DEVICE) -> float:
    if q.dtype == np.int8:
        return float(lib().orc_score_i8(_p(np.ascontiguousarray(q)), _p(np.ascontiguousarray(x)), len(q), sim))
    q = np.ascontiguousarray(q, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    return float(lib().orc_score_f32(_p(q), _p(x), len(q), sim, order))


def exact_search(rows: np.ndarray, query: np.ndarray, k: int, sim: int, order: int = ORDER_DEVICE,
                 ord_to_doc: np.ndarray | None = None, accept_bits: np.ndarray | None = None):
    """[L] AbstractKnnVectorQuery.exactSearch on one leaf → (scores, docs, visited)."""
    rows = np.ascontiguousarray(rows)
    n, dim = rows.shape
    sc = np.empty(k, np.float32)
    dc = np.empty(k, np.int32)
    vis = C.c_int64()
    o2d = None if ord_to_doc is None else np.ascontiguousarray(ord_to_doc, np.int32)
    ab = None if accept_bits is None else np.ascontiguousarray(accept_bits, np.uint64)
    if rows.dtype == np.int8:
        q = np.ascontiguousarray(query, np.int8)
        c = lib().orc_exact_search_i8(_p(rows), n, dim, _p(o2d), _p(ab), _p(q), k, sim, _p(sc), _p(dc),
                                      C.byref(vis))
    else:
        q = np.ascontiguousarray(query, np.float32)
        c = lib().orc_exact_search_f32(_p(rows), n, dim, _p(o2d), _p(ab), _p(q), k, sim, order, _p(sc),
                                       _p(dc), C.byref(vis))
    return sc[:c].copy(), dc[:c].copy(), vis.value


def topdocs_merge(shards, from_: int, size: int, shard_index=None):
    """shards: list of (scores, docs) → (scores, docs, shard_idx, total_hits, max_score)."""
    n = len(shards)
    stride = max([len(s[0]) for s in shards] + [1])
    counts = np.array([len(s[0]) for s in shards] or [0], np.int32)
    sc = np.zeros((max(n, 1), stride), np.float32)
    dc = np.zeros((max(n, 1), stride), np.int32)
    for i, (s, d) in enumerate(shards):
        sc[i, : len(s)] = s
        dc[i, : len(d)] = d
    si = None if shard_index is None else np.ascontiguousarray(shard_index, np.int32)
    os_ = np.empty(max(size, 1), np.float32)
    od = np.empty(max(size, 1), np.int32)
    osh = np.empty(max(size, 1), np.int32)
    tot = C.c_int64()
    mx = C.c_float()
    c = lib().orc_topdocs_merge(n, _p(counts), _p(sc), _p(dc), stride, _p(si), from_, size, _p(os_), _p(od),
                                _p(osh), C.byref(tot), C.byref(mx))
    return os_[:c].copy(), od[:c].copy(), osh[:c].copy(), tot.value, mx.value


def knn_batch(rows: np.ndarray, queries: np.ndarray, k: int, sim: int, order: int, nthreads: int):
    """Multi-threaded exact search (CPU baseline) → (scores[nq,k], docs[nq,k], counts[nq])."""
    rows = np.ascontiguousarray(rows, np.float32)
    queries = np.ascontiguousarray(queries, np.float32)
    nq = queries.shape[0]
    sc = np.empty((nq, k), np.float32)
    dc = np.empty((nq, k), np.int32)
    cc = np.empty(nq, np.int32)
    lib().orc_knn_batch_f32(_p(rows), rows.shape[0], rows.shape[1], _p(queries), nq, k, sim, order, nthreads,
                            _p(sc), _p(dc), _p(cc))
    return sc, dc, cc


def bits_from_bool(mask: np.ndarray) -> np.ndarray:
    mask = np.asarray(mask, dtype=bool)
    nwords = max(1, (len(mask) + 63) // 64)
    packed = np.packbits(mask, bitorder="little")
    buf = np.zeros(nwords * 8, np.uint8)
    buf[: len(packed)] = packed
    return buf.view(np.uint64).copy()
