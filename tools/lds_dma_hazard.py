"""LDS-DMA hazard check on the BUILT library's device code (no GPU).

Every ``buffer_load_dword{,x4} ... lds`` reads its buffer descriptor (and its
soffset) from SGPRs. A VMEM read needs 5 wait states behind a VALU write of an
SGPR it reads (``v_readfirstlane`` / ``v_readlane`` / ``v_cmp*`` with an SGPR
destination; cdna_hip_programming.md 5.7 item 2), and hipcc pads nothing in
front of inline asm. Round 4 faulted a box with a build whose register
allocation put a ``v_readlane`` spill reload right before a DMA (DESIGN.md
round-4 changes). corr.hip's DMA asm therefore opens with ``s_nop 4``; this
check proves, from the disassembly of the code objects inside
``libunsamflow_hip.so``, that every LDS-DMA is either directly preceded by
``s_nop N`` (N >= 4) or has 5 wait states of straight-line code (no branch
target in between) since the last VALU write of an SGPR it reads.

Usage: python tools/lds_dma_hazard.py [path/to/libunsamflow_hip.so]
"""
from __future__ import annotations

import re
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
LINE = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
DMA = re.compile(r"^buffer_load_dword\w*$")


def device_images(lib: Path, tmp: Path) -> list[Path]:
    """Extract the gfx950 code objects of a HIP fat binary (llvm-objdump --offloading
    writes them next to its input, so the input is copied into `tmp` first)."""
    src = tmp / lib.name
    shutil.copy(lib, src)
    subprocess.run([OBJDUMP, "--offloading", str(src)], check=True, capture_output=True, cwd=tmp)
    return sorted(p for p in tmp.iterdir() if "amdgcn" in p.name and "gfx950" in p.name)


def _sgprs(operands: str) -> set[str]:
    """SGPR names an operand string reads or writes: s5, s[16:19], m0, vcc."""
    out = set()
    for a, b in re.findall(r"\bs\[(\d+):(\d+)\]", operands):
        out.update(f"s{i}" for i in range(int(a), int(b) + 1))
    out.update(re.findall(r"\bs\d+\b", re.sub(r"\bs\[\d+:\d+\]", "", operands)))
    out.update(x for x in ("m0", "vcc") if re.search(rf"\b{x}\b", operands))
    return out


def _valu_sgpr_dst(mn: str, ops: str) -> set[str]:
    """SGPRs a VALU instruction writes (its first operand when that is an SGPR)."""
    if not mn.startswith("v_"):
        return set()
    first = ops.split(",")[0].strip() if ops else ""
    return _sgprs(first) if re.match(r"^(s\d|s\[|vcc|m0)", first) else set()


def check_image(path: Path) -> tuple[int, list[str]]:
    """(number of LDS-DMA instructions, list of violations) for one code object."""
    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(path)], check=True, capture_output=True,
                         text=True).stdout
    ins = []  # (addr, mnemonic, operands)
    for ln in dis.splitlines():
        m = LINE.match(ln)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return analyze(ins, path.name)


def analyze(ins: list[tuple[int, str, str]], name: str = "") -> tuple[int, list[str]]:
    """The check over one disassembled instruction stream [(address, mnemonic, operands)]."""
    targets = set()
    for addr, mn, ops in ins:
        if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
            imm = re.match(r"^(-?\d+)", ops)
            if imm:
                targets.add(addr + 4 + 4 * int(imm.group(1)))
    n, bad = 0, []
    for i, (addr, mn, ops) in enumerate(ins):
        if not (DMA.match(mn) and re.search(r"\blds\b", ops)):
            continue
        n += 1
        prev = ins[i - 1] if i else None
        if prev and prev[1] == "s_nop" and int(prev[2].split()[0], 0) >= 4:
            continue
        # straight-line distance from the last VALU write of an SGPR this DMA reads
        reads = _sgprs(ops) | {"m0"}
        ws, j, ok = 0, i - 1, True
        while j >= 0 and ws < 5:
            _, pmn, pops = ins[j]
            if ins[j + 1][0] in targets:
                ok = False  # a branch lands inside the window: the path in is not this one
                break
            if _valu_sgpr_dst(pmn, pops) & reads:
                ok = False
                break
            ws += int(pops.split()[0], 0) + 1 if pmn == "s_nop" else 1
            j -= 1
        if not ok:
            ctx = "; ".join(f"{x[1]} {x[2]}" for x in ins[max(0, i - 4):i + 1])
            bad.append(f"{name} @0x{addr:x}: {ctx}")
    return n, bad


def check_library(lib: Path) -> tuple[int, list[str]]:
    with tempfile.TemporaryDirectory() as d:
        total, bad = 0, []
        for img in device_images(lib, Path(d)):
            n, b = check_image(img)
            total += n
            bad += b
        return total, bad


if __name__ == "__main__":
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 else REPO / "unsamflow_amd" / "lib" / "libunsamflow_hip.so"
    n, bad = check_library(lib)
    print(f"{n} LDS-DMA instructions, {len(bad)} unguarded")
    for b in bad:
        print("  " + b)
    sys.exit(1 if bad else 0)
