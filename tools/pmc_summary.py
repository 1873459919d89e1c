"""Summarises rocprofv3 --pmc CSVs for the rpp_* kernels (mean per dispatch)."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/pmc_*/run_counter_collection.csv") + glob.glob(f"{root}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "rpp_" not in name:
            continue
        k = next((kk for kk in ("rpp_encode_kernel", "rpp_decode_kernel", "rpp_parse_kernel", "rpp_extract_kernel",
                                "rpp_lsb_or_kernel", "rpp_pcm") if kk in name), name.split("(")[0])
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in sorted(agg.items()):
    out[k] = {c: sum(v) / len(v) for c, v in sorted(d.items())}
    print(k)
    for c, v in out[k].items():
        print(f"   {c:28s} {v:14.6g}")
json.dump(out, open(f"{root}/pmc_summary.json", "w"), indent=1)
