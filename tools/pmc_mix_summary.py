"""HBM bytes per call of the configs[3] mix's segmented encode and decode
from rocprofv3 --pmc runs of tools/prof_mix.py (one counter per run dir
gpurun_out/prof/mix_<COUNTER>/).  A decode call starts at its
rpp_seg_plan_kernel dispatch, an encode call at rpp_enc_units_kernel; every
rpp_ dispatch up to the next call's start belongs to the call.  The first
call of each kind (the checked round trip) is skipped.  Writes
profiles/pmc_mix.json (with the HIP sources' hash, as pmc_latest.json).
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md, HBM)."""
import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from bench import kernel_source_sha256  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
res = {}
per_kernel = {}
for counter in ("FETCH_SIZE", "WRITE_SIZE", "GRBM_GUI_ACTIVE"):
    f = ROOT / "gpurun_out" / "prof" / f"mix_{counter}" / "run_counter_collection.csv"
    if not f.exists():
        continue
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    # the marker-delimited segments after the checked round trip
    segs, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "rpp_" not in name:
            continue
        if "rpp_pcm_unpack_kernel" in name:
            cur = collections.Counter()
            segs.append(cur)
            continue
        if cur is not None:
            short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
            cur[short] += float(r["Counter_Value"])
    segs = [c for c in segs if c]  # (the last marker closes the last call)
    n_enc = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    calls = [("encode", c) for c in segs[:n_enc]] + [("decode", c) for c in segs[n_enc:]]
    for kind in ("encode", "decode"):
        cs = [c for k, c in calls if k == kind]
        if not cs:
            continue
        tot = sum(sum(c.values()) for c in cs) / len(cs)
        res.setdefault(kind, {})[counter] = tot
        keys = set().union(*cs)
        per_kernel.setdefault(kind, {})[counter] = {k: sum(c[k] for c in cs) / len(cs) for k in sorted(keys)}
        res[kind]["calls"] = len(cs)
out = {"source": f"profiles/{tag}_pmc_mix.txt", "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per call",
       "kernel_source_sha256": kernel_source_sha256()}
lines = []
for kind, v in res.items():
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        v["hbm_bytes_per_call"] = int((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024)
    out[kind] = v
    lines.append(f"{kind}: " + json.dumps(v))
    for counter, pk in per_kernel.get(kind, {}).items():
        lines.append(f"  {counter}:")
        for k, val in sorted(pk.items(), key=lambda kv: -kv[1]):
            lines.append(f"    {k:40s} {val:16.6g}")
(ROOT / "profiles" / f"{tag}_pmc_mix.txt").write_text("\n".join(lines) + "\n")
(ROOT / "profiles" / "pmc_mix.json").write_text(json.dumps(out, indent=1) + "\n")
print("\n".join(lines))
