"""Diagnostic (DESIGN.md §4 "64-bit shifts and the last VGPR"): builds libricepp_amd_<name>.so
from the RPP_DIAG_VALU_ANY build of ricepp_kernels.hip with its bs 128 cs 2
encode kernel's emission branches edited in the gfx950 assembly, to test
what the fault depends on.  Edits (before each `s_cbranch_vccz` that follows
the emission's `v_cmp_lt_u32 vcc, 32, vN`):
  none  reassembled unchanged (the pipeline itself reproduces the fault)
  vccw  `s_mov_b64 vcc, vcc`: VCC rewritten by the scalar unit (VCCZ recomputed)
  nop   `s_nop 7` x 4: only time between the compare and the branch
  drop  the branch removed: the slow (one code per shift) path always runs
  ldw   `s_waitcnt vmcnt(0)` after every global load of the kernel
  stw   `s_waitcnt vmcnt(0)` after every global store
  dsw   `s_waitcnt lgkmcnt(0)` after every LDS instruction
  dsn   `s_nop 4` after every LDS instruction
  vz    every VGPR but v0 (the work-item id) zeroed at kernel entry
  vf    every VGPR but v0 set to 0xffffffff at kernel entry
  valun `s_nop 1` after every vector ALU instruction
  ndpp / ndot / npk / nrl   `s_nop 4` after every DPP / v_dot2 / v_pk_* / v_readlane-v_readfirstlane
  lds8k / lds40k  the kernel's LDS allocation raised from 4 KiB to 8 KiB (same occupancy) / 40 KiB (4 per CU)
  sh64  every in-place 64-bit shift `v_lshlrev_b64 v[a:a+1], s, v[a:a+1]` shifts a copy in v[136:137] instead
  sh64s the same for `v_lshlrev_b64 v[a:a+1], va|va+1, v[x:y]` (shift amount in the destination)
  sh64d / sh64sd  controls: the same copies made, but the shift still reads its original registers
  vg144 / vg137 / acc140  no code change; the kernel's VGPR count in its descriptor and metadata set to 144 / 137
        (accum_offset 144 / 140), or only accum_offset raised to 140
Usage: python tools/asm_variant.py <edit>  (writes dwarfs_amd/lib/libricepp_amd_asm_<edit>.so)
Run on the round-6 investigation's source (git show bfbb877 -- the round-5 kernels with the RPP_DIAG_VALU_ANY
switch; today's source has neither the switch nor the 64-bit emission shift)."""
import re
import shlex
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL = "_ZN12_GLOBAL__N_117rpp_encode_kernelILj16ELj8ELj2ELb0EEEvNS_9EncParamsE"
edit = sys.argv[1]
tmp = Path(tempfile.mkdtemp(prefix="asmvar-"))
src = ROOT / "dwarfs_amd/csrc/ricepp_kernels.hip"
base = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++20", "--offload-arch=gfx950", "-fPIC", "-I", str(ROOT / "include"),
        "-DRPP_DIAG_VALU_ANY", "-c", str(src), "-o", str(tmp / "rk.o")]
out = subprocess.run(base + ["-###"], capture_output=True, text=True).stderr
cmds = [shlex.split(l) for l in out.splitlines() if l.startswith(' "')]
assert len(cmds) == 4, out
dev, lnk, bnd, host = cmds
# 1. device assembly
devs = [a if a != "-emit-obj" else "-S" for a in dev]
devs[devs.index("-o") + 1] = str(tmp / "dev.s")
subprocess.run(devs, check=True)
asm = (tmp / "dev.s").read_text().split("\n")
# 2. edit the kernel's emission branches
inside, sites, pending = False, 0, None
res = []
for i, line in enumerate(asm):
    if line.startswith(KERNEL + ":"):
        inside = True
    elif inside and line.startswith(".Lfunc_end"):
        inside = False
    if inside and re.match(r"\s*v_cmp_lt_u32_e32 vcc, 32, v\d+$", line):
        pending = i
    elif inside and pending is not None and re.search(r"\bvcc\b", line) and not line.strip().startswith("s_cbranch_vcc"):
        if not re.match(r"\s*v_cndmask", line):
            pending = None  # another vcc writer / reader in between: not this pattern
    if inside and pending is not None and line.strip().startswith("s_cbranch_vccz") and i - pending < 80:
        sites += 1
        if edit == "vccw":
            res.append("\ts_mov_b64 vcc, vcc")
        elif edit == "nop":
            res += ["\ts_nop 7"] * 4
        pending = None
        if edit == "drop":
            continue
    res.append(line)
    st = line.strip()
    m64 = re.match(r"v_lshlrev_b64 v\[(\d+):(\d+)\], (v\d+|s\d+|\d+), v\[(\d+):(\d+)\]$", st) if inside else None
    if m64 and edit in ("sh64", "sh64s", "sh64d", "sh64sd"):
        d0, d1, sh, s0, s1 = m64.groups()
        hit = (s0, s1) == (d0, d1) if edit in ("sh64", "sh64d") else sh in (f"v{d0}", f"v{d1}")
        if hit and edit in ("sh64d", "sh64sd"):
            res.pop()
            res += [f"\tv_mov_b32 v136, v{s0}", f"\tv_mov_b32 v137, v{s1}", "\t" + st]
            sites += 1
        elif hit:
            res.pop()
            if edit == "sh64":
                res += [f"\tv_mov_b32 v136, v{s0}", f"\tv_mov_b32 v137, v{s1}", f"\tv_lshlrev_b64 v[{d0}:{d1}], {sh}, v[136:137]"]
            else:
                res += [f"\tv_mov_b32 v136, {sh}", f"\tv_lshlrev_b64 v[{d0}:{d1}], v136, v[{s0}:{s1}]"]
            sites += 1
    if line.startswith(KERNEL + ":") and edit in ("vz", "vf"):
        res.append("; %bb.x:")
        res += [f"\tv_mov_b32 v{r}, {0 if edit == 'vz' else -1}" for r in range(1, 137)]
        sites += 1
    if inside and edit == "ldw" and st.startswith("global_load"):
        res.append("\ts_waitcnt vmcnt(0)"); sites += 1
    if inside and edit == "stw" and st.startswith("global_store"):
        res.append("\ts_waitcnt vmcnt(0)"); sites += 1
    if inside and edit == "dsw" and st.startswith("ds_"):
        res.append("\ts_waitcnt lgkmcnt(0)"); sites += 1
    if inside and st.startswith("v_") and (
            edit == "valun" or (edit == "ndpp" and "_dpp" in st) or (edit == "ndot" and st.startswith("v_dot"))
            or (edit == "npk" and st.startswith("v_pk_")) or (edit == "nrl" and st.startswith("v_read"))):
        res.append("\ts_nop 1" if edit == "valun" else "\ts_nop 4"); sites += 1
    if inside and edit == "dsn" and st.startswith("ds_"):
        res.append("\ts_nop 4"); sites += 1
if edit in ("lds8k", "lds40k"):
    kd = res.index(f"\t.amdhsa_kernel {KERNEL}") if f"\t.amdhsa_kernel {KERNEL}" in res else \
        next(i for i, l in enumerate(res) if l.strip() == f".amdhsa_kernel {KERNEL}")
    for i in range(kd, kd + 80):
        if "amdhsa_group_segment_fixed_size" in res[i]:
            res[i] = res[i].replace("4096", "8192" if edit == "lds8k" else "40960")
            sites += 1
            break
VG = {"sh64": (138, 140), "sh64s": (138, 140), "sh64d": (138, 140), "sh64sd": (138, 140),
      "vg144": (144, 144), "vg137": (137, 140), "acc140": (136, 140)}
if edit in VG:  # VGPR count / accum_offset: descriptor, symbol and metadata
    nv, acc = VG[edit]
    for i, l in enumerate(res):
        if l.strip() == f".amdhsa_kernel {KERNEL}":
            for j in range(i, i + 80):
                res[j] = re.sub(r"(amdhsa_next_free_vgpr) 136$", rf"\g<1> {nv}", res[j])
                res[j] = re.sub(r"(amdhsa_accum_offset) 136$", rf"\g<1> {acc}", res[j])
        if l.strip() == f".set {KERNEL}.num_vgpr, 136":
            res[i] = l.replace("136", str(nv))
        if l.strip() == f".name:           {KERNEL}":
            for j in range(i, i + 12):
                if ".vgpr_count:" in res[j]:
                    res[j] = res[j].replace("136", str(nv))
                    break
    sites += 1
print(f"{edit}: {sites} branch sites edited", flush=True)
assert sites > 0
(tmp / "dev_e.s").write_text("\n".join(res))
# 3. assemble, link, bundle, host
dobj = tmp / "dev_e.o"
subprocess.run(["/opt/rocm/lib/llvm/bin/clang", "--target=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", str(tmp / "dev_e.s"),
                "-o", str(dobj)], check=True)
li = [a for a in lnk]
li[-2] = str(dobj)  # the device object (before --no-whole-archive)
co = Path(li[li.index("-o") + 1])
subprocess.run(li, check=True)
subprocess.run(bnd, check=True)
subprocess.run(host, check=True)
# 4. the library: this object + the others as build_native compiles them
objs = [str(tmp / "rk.o")]
flags = ["-O3", "-std=c++20", "--offload-arch=gfx950", "-fPIC", "-I", str(ROOT / "include")]
for s in ["ricepp_decode2.hip", "fits_lsb.hip", "batch_image.hip", "pcm_transform.hip", "flac_kernels.hip",
          "ricepp_frame.cpp", "ricepp_facade.cpp"]:
    o = tmp / (s + ".o")
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-c", str(ROOT / "dwarfs_amd/csrc" / s), "-o", str(o)], check=True)
    objs.append(str(o))
lib = ROOT / f"dwarfs_amd/lib/libricepp_amd_asm_{edit}.so"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", str(lib), *objs], check=True)
print("wrote", lib)
