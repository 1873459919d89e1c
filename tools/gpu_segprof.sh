# Kernel trace of the single-long-stream layouts of seg_bench (where the time of a segmented decode goes)
mkdir -p gpurun_out/segprof
export TMPDIR=/tmp
rm -rf gpurun_out/segprof/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segprof -o run -- python3 tools/seg_bench.py "one 16 MiB" > gpurun_out/segprof/log.txt 2>&1; rc=$?; echo "trace=$rc"
cat gpurun_out/segprof/log.txt | grep layout | cut -c1-200
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/segprof/run_kernel_trace.csv")))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"].split("(")[0][-60:]
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"{t:10.1f} us {c:5d}  {n}")
PY
