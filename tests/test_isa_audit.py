"""The built library against the gfx950 64-bit-shift hazard (DESIGN.md §4 "64-bit shifts and the last VGPR";
tools/isa_audit.py): no v_lshlrev_b64 / v_lshrrev_b64 / v_ashrrev_i64 may take its shift amount from the last
VGPR of its kernel's allocation -- the round-5 bs 128 cs 2 encode fault.  CPU only (disassembly of the .so)."""

import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import isa_audit  # noqa: E402

LIB = ROOT / "dwarfs_amd" / "lib" / "libricepp_amd.so"


def test_no_64bit_shift_amount_in_the_last_allocated_vgpr():
    assert LIB.exists(), "build the library first (__graft_entry__.build())"
    found = isa_audit.audit(LIB)
    assert found == [], "\n".join(f"{k} (allocation {a}): {i}" for k, a, i in found)


@pytest.mark.parametrize("vgprs,amount,bad", [(136, "v135", True), (136, "v131", False), (137, "v135", False),
                                              (144, "v143", True), (120, "v119", True)])
def test_audit_detects_the_pattern(tmp_path, vgprs, amount, bad):
    """The detector itself, on a minimal kernel: the amount register is flagged exactly when it is the last of the
    allocation (136 -> v135; 137 VGPRs allocate 144, so v135 is not the last)."""
    top = vgprs - 1
    src = f"""
    .amdgcn_target "amdgcn-amd-amdhsa--gfx950"
    .text
    .globl k
    .p2align 8
    .type k,@function
k:
    v_mov_b32 v{top}, 0
    v_lshlrev_b64 v[2:3], {amount}, v[4:5]
    s_endpgm
    .rodata
    .p2align 6
    .amdhsa_kernel k
      .amdhsa_next_free_vgpr {vgprs}
      .amdhsa_next_free_sgpr 8
      .amdhsa_accum_offset {(vgprs + 3) // 4 * 4}
    .end_amdhsa_kernel
    .amdgpu_metadata
---
amdhsa.kernels:
  - .agpr_count:     0
    .name:           k
    .symbol:         k.kd
    .vgpr_count:     {vgprs}
    .sgpr_count:     8
    .kernarg_segment_size: 0
    .group_segment_fixed_size: 0
    .private_segment_fixed_size: 0
    .kernarg_segment_align: 8
    .wavefront_size: 64
    .max_flat_workgroup_size: 64
amdhsa.target:   amdgcn-amd-amdhsa--gfx950
amdhsa.version:
  - 1
  - 2
...
    .end_amdgpu_metadata
"""
    s = tmp_path / "k.s"
    s.write_text(src)
    o = tmp_path / "k.o"
    co = tmp_path / "k.co"
    subprocess.run([str(isa_audit.LLVM / "clang"), "--target=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", str(s), "-o",
                    str(o)], check=True)
    subprocess.run([str(isa_audit.LLVM / "ld.lld"), "-shared", str(o), "-o", str(co)], check=True)
    n, found = isa_audit.audit_code_object(co)
    assert n == 1
    assert bool(found) == bad, found
