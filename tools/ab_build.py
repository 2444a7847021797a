"""Build A/B variants of libunsamflow_hip.so with compile-time knobs, for
side-by-side timing on the GPU box (load one with USF_LIB=<path>).

Usage: python tools/ab_build.py [--only=corr,warp] name:-DFLAG=V,-DFLAG2=V ...  -> unsamflow_amd/lib/ab/lib_<name>.so
"""
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
CSRC = REPO / "unsamflow_amd" / "csrc"
OUT = REPO / "unsamflow_amd" / "lib" / "ab"
sys.path.insert(0, str(REPO))
from unsamflow_amd.build import COMMON_FLAGS as FLAGS  # noqa: E402  (the library's flags; A/B defines on top)


def build(name, defines, only=None):
    """Sources in `only` (default: all) are compiled with the defines; the others
    link the library's own objects (unsamflow_amd/lib/obj, python -m unsamflow_amd.build)."""
    OUT.mkdir(parents=True, exist_ok=True)
    objs = []
    sys.path.insert(0, str(REPO))
    from unsamflow_amd.build import SOURCES

    for src in SOURCES:
        if only and Path(src).stem not in only:
            objs.append(str(REPO / "unsamflow_amd" / "lib" / "obj" / (Path(src).stem + ".o")))
            continue
        obj = OUT / f"{name}_{Path(src).stem}.o"
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *defines, *lang, "-c", str(CSRC / src), "-o", str(obj)],
                       check=True)
        objs.append(str(obj))
    so = OUT / f"lib_{name}.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o", str(so), *objs], check=True)
    print(so)


if __name__ == "__main__":
    args = sys.argv[1:]
    only = None
    if args and args[0].startswith("--only="):  # e.g. --only=corr: recompile corr.hip only
        only = args.pop(0).split("=", 1)[1].split(",")
    for arg in args:
        name, _, defs = arg.partition(":")
        build(name, [d for d in defs.split(",") if d], only)
