"""Build libosknn.so in-tree with hipcc for gfx950.

    python -m opensearch_amd.build          # build if sources are newer than the .so
    python -m opensearch_amd.build --force  # always rebuild

The product library lands at opensearch_amd/libosknn.so (git-ignored, shipped to the GPU box by
gpurun).  A second library, opensearch_amd/libosknn_testing.so, links the same objects except the C-ABI
and prefilter translation units, which are compiled with -DOSK_TESTING: it adds the result-corrupting
A/B and test knobs (ablations, forced exact fallback, settle traces, workspace debug copies) that the shipped
library refuses.  Objects are compiled in parallel into build/osknn/.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
LIB = PKG / "libosknn.so"
LIB_TESTING = PKG / "libosknn_testing.so"
# the sources whose objects differ in the testing build (the C-ABI's test knobs; sq8_mfma's A/B ablations;
# the loopback transport of the multi-rank exchange)
TESTING_VARIANTS = ("osk_api.hip", "osk_sq8.hip", "osk_sq8w.hip", "osk_sq6.hip", "osk_comm.hip")
OBJDIR = ROOT / "build" / "osknn"

SOURCES = ["osk_kernels.hip", "osk_mfma.hip", "osk_sq8.hip", "osk_sq8w.hip", "osk_sq6.hip", "osk_filter.hip", "osk_select.hip", "osk_api.hip", "osk_comm.hip", "osk_host.cpp"]
HEADERS = ["osk_common.h", "osk_internal.h", "osk_wave.h", "osk_objects.h", "osk_device.h"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -ffp-contract=off: every fused multiply-add in the scoring path is an explicit fmaf, so the
# summation order (and the bits of every score) is exactly the one DESIGN.md documents.
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-result",
          f"-I{INCLUDE}", f"-I{CSRC}"]


def _stale() -> bool:
    if not LIB.exists() or not LIB_TESTING.exists():
        return True
    t = min(LIB.stat().st_mtime, LIB_TESTING.stat().st_mtime)
    deps = [CSRC / s for s in SOURCES + HEADERS] + [INCLUDE / "osknn.h", Path(__file__)]
    return any(d.stat().st_mtime > t for d in deps)


def _compile(job) -> Path:
    src, testing = job
    OBJDIR.mkdir(parents=True, exist_ok=True)
    obj = OBJDIR / (src + (".testing" if testing else "") + ".o")
    cmd = [HIPCC] + COMMON + (["-DOSK_TESTING"] if testing else [])
    if src.endswith(".hip"):
        cmd += [f"--offload-arch={ARCH}", "-x", "hip"]
    cmd += ["-c", str(CSRC / src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> Path:
    if not force and not _stale():
        return LIB
    jobs = [(s, False) for s in SOURCES] + [(s, True) for s in TESTING_VARIANTS]
    with cf.ThreadPoolExecutor(max_workers=len(jobs)) as ex:
        objs = dict(zip(jobs, ex.map(_compile, jobs)))
    for lib, testing in ((LIB, False), (LIB_TESTING, True)):
        parts = [objs[(s, testing and s in TESTING_VARIANTS)] for s in SOURCES]
        tmp = lib.with_suffix(".so.tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in parts]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, lib)
        if verbose:
            print(f"built {lib}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(force=a.force)
