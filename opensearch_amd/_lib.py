"""ctypes binding of libosknn.so (the C-ABI in include/osknn.h).

This is the Python twin of the Panama FFM binding a Java plugin would use.
The library is built in-tree (`python -m opensearch_amd.build`); if it is missing we fail loudly —
there is no CPU fallback for the search path.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading
from pathlib import Path

# OSKNN_LIB: another build of the same ABI (A/B timing of two builds in one GPU call; tools only)
LIB_PATH = Path(os.environ.get("OSKNN_LIB") or Path(__file__).resolve().with_name("libosknn.so")).resolve()
# same ABI plus the test/A-B-only knobs (osknn.h): loaded only inside `with testing():`
TESTING_LIB_PATH = Path(__file__).resolve().with_name("libosknn_testing.so")

OSK_OK = 0
OSK_ERR_INVALID = -1
OSK_ERR_DEVICE = -2
OSK_ERR_OOM = -3
OSK_ERR_UNSUPPORTED = -4
OSK_ERR_NO_DEVICE = -5
OSK_MAX_K = 10000
OSK_ABI_VERSION = 2        # include/osknn.h OSK_ABI_VERSION
OSK_MAX_DIM = 4096
OSK_COMM_ID_BYTES = 128

OSK_WARM_PREFILTER = 1
OSK_WARM_PREFILTER_MFMA = 2
OSK_WARM_BATCHED = 4
OSK_WARM_ALL = 7

FLOAT32 = 0
BYTE = 1

EUCLIDEAN = 0
DOT_PRODUCT = 1
COSINE = 2
MAXIMUM_INNER_PRODUCT = 3

DIST_UNIFORM01 = 0
DIST_UNIFORM01_X128 = 1
DIST_NORMALISH = 2
DIST_NORMALISH_UNIT = 3
DIST_INT8 = 4

_P = C.c_void_p
_I32 = C.c_int32
_I64 = C.c_int64
_U64 = C.c_uint64
_PI32 = C.POINTER(C.c_int32)
_PI64 = C.POINTER(C.c_int64)
_PF = C.POINTER(C.c_float)

# name → (restype, argtypes); every symbol include/osknn.h declares
SIGNATURES = {
    "osk_abi_version": (_I32, []),
    "osk_last_error": (C.c_char_p, []),
    "osk_device_count": (_I32, [_PI32]),
    "osk_seg_stage": (_I32, [_I32, _P, _I64, _I32, _I32, _I32, _P, _I32, C.POINTER(_P)]),
    "osk_seg_stage_file": (_I32, [_I32, C.c_char_p, _I64, _I64, _I32, _I32, _I32, _P, _I32, C.POINTER(_P)]),
    "osk_seg_stage_device": (_I32, [_I32, _P, _I64, _I64, _I32, _I32, _I32, _P, _I32, C.POINTER(_P)]),
    "osk_seg_synth": (_I32, [_I32, _I64, _I32, _I32, _I32, _U64, _I32, _I64, C.POINTER(_P)]),
    "osk_seg_release": (_I32, [_P]),
    "osk_seg_retain": (_I32, [_P]),
    "osk_seg_footprint": (_I32, [_P, _PI64]),
    "osk_seg_warm": (_I32, [_P, _I32]),
    "osk_view_warm": (_I32, [_P, _I32]),
    "osk_comm_unique_id": (_I32, [_P]),
    "osk_comm_init_rank": (_I32, [_I32, _I32, _I32, _P, C.POINTER(_P)]),
    "osk_comm_init_all": (_I32, [_P, _I32, C.POINTER(_P)]),
    "osk_comm_release": (_I32, [_P]),
    "osk_comm_info": (_I32, [_P, _PI32, _PI32, _PI32]),
    "osk_comm_all_gather": (_I32, [_P, _P, _P, _I64, _P]),
    "osk_comm_status": (_I32, [_P, _PI64]),
    "osk_comm_set_device_limits": (_I32, [_P, _I32, _I32, _I32]),
    "osk_comm_init_loopback": (_I32, [_I32, _I32, _I32, _P, _I64, C.POINTER(_P)]),
    "osk_comm_init_all_loopback": (_I32, [_P, _I32, C.POINTER(_P)]),
    "osk_testing_glds_probe": (_I32, [_I32, _PI64]),
    "osk_shards_search_merge": (_I32, [_P, _P, _I32, _P, _I32, _I32, _P, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "osk_shards_search_merge_device": (_I32, [_P, _P, _P, _I32, _I32, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P,
                                              _P]),
    "osk_seg_info": (_I32, [_P, _PI64, _PI32, _PI32, _PI32, _PI32, _PI32]),
    "osk_synth_host": (_I32, [_P, _I64, _I64, _I32, _U64, _I32]),
    "osk_seg_search": (_I32, [_P, _P, _I32, _I32, _P, _P, _P, _P, _P]),
    "osk_view_create": (_I32, [_P, _I32, _P, _P, _I32, _P, C.POINTER(_P)]),
    "osk_view_release": (_I32, [_P]),
    "osk_view_search_device": (_I32, [_P, _P, _I32, _I32, _P, _P, _P, _P, _P]),
    "osk_merge_device": (_I32, [_I32, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "osk_merge_device_ranked": (_I32, [_I32, _P, _I32, _I32, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "osk_view_search": (_I32, [_P, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "osk_topdocs_merge": (_I32, [_I32, _P, _P, _P, _I32, _P, _P, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "osk_decode_keys": (_I32, [_P, _I64, _P, _P]),
    "osk_topdocs_write": (_I32, [_I64, _I32, C.c_float, _I32, _P, _P, _P, _I64, _PI64]),
    "osk_topdocs_read": (_I32, [_P, _I64, _PI64, _PI32, _PF, _I32, _PI32, _P, _P, _PI64]),
    "osk_view_profile": (_I32, [_P, _I32]),
    "osk_tune_set": (_I32, [C.c_char_p, _I64]),
    "osk_view_stats": (_I32, [_P, _PI64, _PI64]),
    "osk_view_counter": (_I32, [_P, C.c_char_p, _PI64]),
    "osk_view_debug_copy": (_I32, [_P, C.c_char_p, _P, _I64]),
    "osk_view_scan_time": (_I32, [_P, C.POINTER(C.c_double), _PI64]),
    "osk_last_call_device_ns": (_I32, [_PI64, _PI32]),
}


class OskError(RuntimeError):
    """A negative return code from libosknn (maps to an IOException / shard failure in Java)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libosknn error {code}: {msg}")
        self.code = code


_lock = threading.Lock()
_lib = None
_product = None
_testing = None


def _load(path: Path) -> C.CDLL:
    if not path.exists():
        raise RuntimeError(
            f"{path} is missing: build it with `python -m opensearch_amd.build` "
            "(libosknn has no CPU fallback)")
    L = C.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib() -> C.CDLL:
    """The library every call goes through: libosknn.so, or libosknn_testing.so inside `testing()`."""
    global _lib, _product
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            # tools that drive the A/B knobs (tools/mfma_ablate.py, settle_trace.py) set OSK_TESTING_LIB=1
            path = TESTING_LIB_PATH if os.environ.get("OSK_TESTING_LIB") == "1" else LIB_PATH
            _product = _product or _load(path)
            _lib = _product
    return _lib


@contextlib.contextmanager
def testing():
    """Route every call to libosknn_testing.so (same ABI plus the test-only knobs: sq8_force_fallback,
    the A/B ablations, settle traces, workspace debug copies).  Objects made inside must be used and
    released inside: the two libraries share no state."""
    global _lib, _testing
    lib()
    with _lock:
        _testing = _testing or _load(TESTING_LIB_PATH)
        prev, _lib = _lib, _testing
    try:
        yield _testing
    finally:
        with _lock:
            _lib = prev


def check(rc: int) -> None:
    if rc != OSK_OK:
        msg = lib().osk_last_error()
        raise OskError(rc, msg.decode() if msg else "")


def ptr(a) -> int | None:
    """Address of a numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data


def tune(key: str, value: int) -> None:
    """Process-wide tuning knob (osk_tune_set): scan_nt, tiles_target, mfma_min_batch, mfma_units."""
    check(lib().osk_tune_set(key.encode(), int(value)))


def last_call_device_ns() -> tuple[int, int]:
    """(device ns, requests sharing it) of this thread's last host search (tune("call_timing", 1))."""
    ns, shared = C.c_int64(), C.c_int32()
    check(lib().osk_last_call_device_ns(C.byref(ns), C.byref(shared)))
    return ns.value, shared.value


def device_count() -> int:
    n = C.c_int32(0)
    check(lib().osk_device_count(C.byref(n)))
    return n.value
