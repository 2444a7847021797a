"""VGPR / LDS budget and the occupancy it allows, per kernel instantiation.

Compiles a HIP source to gfx950 assembly and reads the .amdhsa_* directives:
waves/SIMD = min(8, 512 // vgpr_alloc) (unified 512-entry register file,
granule 8), workgroups/CU by LDS = 160 KiB // group segment size.

Usage: python tools/kernel_resources.py [unsamflow_amd/csrc/corr.hip ...]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def resources(src):
    with tempfile.TemporaryDirectory() as d:
        asm = Path(d) / "k.s"
        sys.path.insert(0, str(REPO))
        from unsamflow_amd.build import COMMON_FLAGS  # the library's own flags

        flags = [f for f in COMMON_FLAGS if f != "-fPIC"]
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-S", "-o", str(asm), str(src)],
                       check=True, capture_output=True)
        text = asm.read_text()
    out = []
    for name, body in re.findall(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", text, re.S):
        def g(k):
            return int(re.search(re.escape(k) + r"\s+(\d+)", body).group(1))
        v, lds = g(".amdhsa_next_free_vgpr"), g(".amdhsa_group_segment_fixed_size")
        scratch = g(".amdhsa_private_segment_fixed_size")
        out.append((re.sub(r"_ZN3usf12_GLOBAL__N_1\d+", "", name), v, lds, scratch))
    return out


if __name__ == "__main__":
    srcs = sys.argv[1:] or [REPO / "unsamflow_amd/csrc/corr.hip", REPO / "unsamflow_amd/csrc/warp.hip"]
    for src in srcs:
        for name, v, lds, scratch in resources(src):
            wps = min(8, 512 // (((v + 7) // 8) * 8))
            wg_lds = (160 * 1024) // lds if lds else 99
            print(f"{name[:64]:64s} vgpr={v:3d} waves/SIMD={wps} lds={lds:6d} wg/CU(lds)={wg_lds:2d} scratch={scratch}")
