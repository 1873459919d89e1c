"""gfx950 ISA audit of the built library (DESIGN.md §4 "64-bit shifts and the last VGPR").

A 64-bit shift (v_lshlrev_b64 / v_lshrrev_b64 / v_ashrrev_i64) reads its 32-bit shift amount as a
register pair; with the amount in the LAST VGPR of the wave's allocation the pair's second register lies
outside the allocation, and with other waves resident on the SIMD the shift then uses a wrong amount
(tools/last_vgpr_probe.hip, tools/shl64_hazard.hip; profiles/r06_shl64_hazard.jsonl).  The compiler
(ROCm 7.2 LLVM) does not avoid that register for gfx950.  This audit extracts every gfx950 code object
from the library, computes each kernel's VGPR allocation from its metadata, and lists the 64-bit shifts
whose amount operand is the allocation's last register.

    python tools/isa_audit.py [library.so]     (exit status 1 when a kernel has such a shift)
"""
from __future__ import annotations

import re
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
SHIFTS64 = ("v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64")


def _kernel_vgprs(code_object: Path) -> dict:
    """kernel symbol -> (vgpr_count, agpr_count) from the code object's AMDGPU metadata note."""
    notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(code_object)], capture_output=True, text=True,
                           check=True).stdout
    out, cur = {}, {}
    for line in notes.splitlines():
        s = line.strip().lstrip("- ").strip()
        m = re.match(r"\.(agpr_count|vgpr_count|symbol|name):\s*(\S+)", s)
        if not m:
            continue
        key, val = m.groups()
        if key == "agpr_count" and cur.get("symbol"):
            cur = {}  # (a kernel map starts with .agpr_count in sorted-key order)
        cur[key] = val
        if "symbol" in cur and "vgpr_count" in cur:
            out[cur["symbol"].removesuffix(".kd")] = (int(cur["vgpr_count"]), int(cur.get("agpr_count", 0)))
    return out


def allocation(vgprs: int, agprs: int) -> int:
    """Registers the hardware allocates per lane on gfx950: ArchVGPRs rounded to 4 (accum_offset) plus AGPRs,
    in granules of 8."""
    total = (vgprs + 3) // 4 * 4 + agprs if agprs else vgprs
    return (total + 7) // 8 * 8


def audit_code_object(co: Path) -> tuple:
    """(kernels read, [(kernel, allocation, instruction)]) for one gfx950 code object."""
    vg = _kernel_vgprs(co)
    dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)], capture_output=True, text=True,
                         check=True).stdout
    findings, kernel = [], None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            kernel = m.group(1)
            continue
        s = line.strip()
        if not kernel or kernel not in vg or not s.startswith(SHIFTS64):
            continue
        amount = s.split(None, 1)[1].split("//")[0].split(",")[1].strip()
        last = allocation(*vg[kernel]) - 1
        if amount == f"v{last}":
            findings.append((kernel, last + 1, s.split("//")[0].strip()))
    return len(vg), findings


def audit(lib: Path) -> list:
    """[(kernel, allocation, instruction)] for every 64-bit shift with its amount in the last allocated VGPR, over
    every gfx950 code object bundled in the library."""
    findings, kernels = [], 0
    with tempfile.TemporaryDirectory() as td:
        copy = Path(td) / lib.name
        shutil.copyfile(lib, copy)
        subprocess.run([str(LLVM / "llvm-objdump"), "--offloading", str(copy)], capture_output=True, check=True,
                       cwd=td)
        objs = sorted(Path(td).glob(lib.name + ".*gfx950*"))
        if not objs:
            raise RuntimeError(f"no gfx950 code object in {lib}")
        for co in objs:
            n, f = audit_code_object(co)
            kernels += n
            findings += f
    if kernels == 0:
        raise RuntimeError("no kernel metadata read")
    return findings


def main() -> int:
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 else Path(__file__).resolve().parent.parent / "dwarfs_amd/lib/libricepp_amd.so"
    found = audit(lib)
    for k, alloc, ins in found:
        print(f"{k} (allocation {alloc}): {ins}")
    print(f"{len(found)} 64-bit shift(s) with the amount in the last allocated VGPR")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main())
