"""Build libosknn.so in-tree with hipcc for gfx950.

    python -m opensearch_amd.build          # build if sources are newer than the .so
    python -m opensearch_amd.build --force  # always rebuild

The library lands at opensearch_amd/libosknn.so (git-ignored, shipped to the GPU box by gpurun).
Objects are compiled in parallel into build/osknn/ and linked once.
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
OBJDIR = ROOT / "build" / "osknn"

SOURCES = ["osk_kernels.hip", "osk_mfma.hip", "osk_sq8.hip", "osk_api.hip", "osk_host.cpp"]
HEADERS = ["osk_common.h", "osk_internal.h", "osk_wave.h"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -ffp-contract=off: every fused multiply-add in the scoring path is an explicit fmaf, so the
# summation order (and the bits of every score) is exactly the one DESIGN.md documents.
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-result",
          f"-I{INCLUDE}", f"-I{CSRC}"]


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = [CSRC / s for s in SOURCES + HEADERS] + [INCLUDE / "osknn.h", Path(__file__)]
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: str) -> Path:
    OBJDIR.mkdir(parents=True, exist_ok=True)
    obj = OBJDIR / (src + ".o")
    cmd = [HIPCC] + COMMON
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
    with cf.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(_compile, SOURCES))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(force=a.force)
