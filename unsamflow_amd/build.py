"""Build libunsamflow_hip.so in-tree with hipcc for gfx950.

The library is a plain C-ABI shared object (include/unsamflow_hip.h); it is
loaded with ctypes by :mod:`unsamflow_amd._lib`. No torch headers are used, so
the build needs only hipcc (cross-compiles without a GPU).

Usage: ``python -m unsamflow_amd.build [--force] [--verbose]``
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
LIB_DIR = PKG_DIR / "lib"
LIB_PATH = LIB_DIR / "libunsamflow_hip.so"
INCLUDE_DIR = PKG_DIR.parent / "include"

ARCH = os.environ.get("USF_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["corr.hip", "warp.hip", "photo.hip", "upsample.hip", "convex.hip", "stream.hip", "capi.cpp"]
HEADERS = ["usf_common.h", "warp_tap.h", "interp_tap.h"]

# -fno-slp-vectorize: the SLP vectorizer packs the kernels' independent FMAs into
# v_pk_fma_f32 / v_pk_add_f32, whose operands must sit in aligned register pairs:
# it then re-reads the correlation windows at odd LDS offsets (ds_read2_b32) and
# adds v_mov shuffles, and serialises each window's reads with its FMAs. The
# packing gains little FLOP rate on gfx950: plain v_fmac_f32 measured 102-107 TF,
# v_pk_fma_f32 106-122 TF (4-13 % more; profiles/r02_fma_rate.json), far less than
# those costs. Measured on the box (profiles/ab_r01/slp_*.json):
# corr bwd L4 54.8 -> 41.1 us, L3 40.3 -> 30.5 us; corr fwd L3 17.6 -> 15.7 us;
# photometric pair 91.5 -> 84.9 us; warp unchanged.
COMMON_FLAGS = [
    "-O3",
    "-std=c++17",
    "-fno-slp-vectorize",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-Wall",
    "-Wno-unused-function",
    f"-I{INCLUDE_DIR}",
]


def build_id() -> str:
    """Identity of the library this tree builds: sha256 (16 hex digits) over
    every source and header text, the compiler flags and the target. It is
    compiled into the library (usf_build_id) and stamped into the PMC
    summaries (tools/pmc_traffic.py), so bench.py never reports a traffic
    figure measured on another build."""
    h = hashlib.sha256()
    for f in [CSRC / s for s in SOURCES] + [CSRC / s for s in HEADERS] + [INCLUDE_DIR / "unsamflow_hip.h"]:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    h.update(" ".join(COMMON_FLAGS).encode())
    return h.hexdigest()[:16]


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_library(force: bool = False, verbose: bool = False) -> Path:
    """Compile every HIP source to an object file and link the shared library.

    Returns the path of the built library. Raises ``RuntimeError`` with the
    compiler output on failure.
    """
    LIB_DIR.mkdir(exist_ok=True)
    obj_dir = LIB_DIR / "obj"
    obj_dir.mkdir(exist_ok=True)
    headers = [CSRC / h for h in HEADERS] + [INCLUDE_DIR / "unsamflow_hip.h"]
    bid = build_id()
    stamp = obj_dir / "build_id.txt"
    id_changed = not stamp.exists() or stamp.read_text().strip() != bid
    objs = []
    for src in SOURCES:
        s = CSRC / src
        o = obj_dir / (s.stem + ".o")
        objs.append(o)
        # capi.cpp carries the build id: rebuilt whenever any source changed
        if force or _stale(o, [s] + headers) or (src == "capi.cpp" and id_changed):
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            extra = [f'-DUSF_BUILD_ID="{bid}"'] if src == "capi.cpp" else []
            cmd = [HIPCC, *COMMON_FLAGS, *extra, *lang, "-c", str(s), "-o", str(o)]
            _run(cmd, verbose)
    stamp.write_text(bid + "\n")
    if force or _stale(LIB_PATH, objs):
        tmp = LIB_PATH.with_suffix(".so.tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
        _run(cmd, verbose)
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"hipcc failed ({p.returncode}):\n{' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
    if verbose and (p.stdout or p.stderr):
        print(p.stdout + p.stderr, flush=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", "-v", action="store_true")
    a = ap.parse_args(argv)
    path = build_library(force=a.force, verbose=a.verbose)
    print(path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
