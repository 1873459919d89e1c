"""Diagnostic: instruction census of the decode fast loops in a gfx950 .s file.

Finds, inside one kernel's assembly, the innermost loops whose header block
holds every given marker (default: the bs-128 fs 5-7 loop: a dword buffer
store and a row_bcast DPP) and counts the instructions of the blocks from
the header to the first branch back to it, by class.
Usage: python tools/loop_census.py file.s [kernel-substring] [marker ...]"""
import re
import sys
from collections import Counter

path = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "rpp_decode_kernelILj1ELb0"
markers = sys.argv[3:] or ["buffer_store_dword v", "row_bcast:15"]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kname in l.split()[0] and l.split()[0].endswith(":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
lbl_re = re.compile(r"^(\.LBB\d+_\d+):")


def is_header(i: int) -> bool:
    if not lbl_re.match(body[i]):
        return False
    for j in range(i, min(i + 4, len(body))):
        if j > i and not body[j].strip().startswith(";"):
            break
        if "Loop Header" in body[j]:
            return True
    return False


headers = [(i, lbl_re.match(body[i]).group(1)) for i in range(len(body)) if is_header(i)]


def classify(ins: str) -> str:
    op = ins.split()[0]
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_setprio"):
        return "s_setprio"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if "_dpp" in op or " row_" in ins or "wave_shr" in ins:
        return "valu_dpp"
    if op.startswith("v_perm"):
        return "valu_perm"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "valu_lane"
    if op.startswith("v_") and (op.endswith("_e32") or op.endswith("_sdwa")):
        return "valu_vop2"
    if op.startswith("v_"):
        return "valu"
    return "other"


for hi, name in headers:
    # the loop: from the header to the last branch back to it
    back = max((j for j in range(hi, len(body)) if re.search(rf"{re.escape(name)}(?!\d)", body[j]) and
                body[j].strip().startswith(("s_cbranch", "s_branch"))), default=None)
    if back is None:
        continue
    seg = body[hi:back + 1]
    text = "\n".join(seg)
    if not all(m in text for m in markers):
        continue
    inner = [k for k in range(hi + 1, back + 1) if is_header(k)]
    if inner:
        continue
    c = Counter()
    for l in seg:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        c[classify(t)] += 1
    nops = sum(int(m.group(1)) + 1 for l in seg for m in [re.match(r"\s*s_nop (\d+)", l)] if m)
    print(f"{name}: {len(seg)} lines; " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())) + f"; nop wait states {nops}")
    # the hot path: the header block up to its first conditional branch, then
    # the fall-through blocks until the first branch back to the header or a
    # block that only the rare paths reach (heuristic: stop at the 3rd branch)
    h = Counter()
    nb = 0
    for l in seg:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        h[classify(t)] += 1
        if t.startswith("s_cbranch") or t.startswith("s_branch"):
            nb += 1
            if nb >= 3:
                break
    # SIMD cycles at 4 waves per SIMD, from tools/isa_rate (profiles/r04_isa_rate.txt):
    # VOP2 1.57, other VALU (VOP3, DPP, v_perm, lane reads) 2.66, SALU 2.57
    cyc = 1.57 * h["valu_vop2"] + 2.66 * (h["valu"] + h["valu_dpp"] + h["valu_perm"] + h["valu_lane"]) + 2.57 * h["salu"]
    print("   hot path (to the 3rd branch): " + ", ".join(f"{k} {v}" for k, v in sorted(h.items())) +
          f"; total {sum(h.values())}; est. SIMD cycles {cyc:.0f}")
