# Round-6 GPU session: the facade's 64 KiB reader pattern (16 threads x 64 KiB blocks) by pipeline depth
# (batches in flight per queue).  Output: gpurun_out/r06/facade64k_depth.jsonl
set -e
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/facade64k_depth.jsonl
for d in 2 4 8 16; do
  timeout -k 10 300 ./tests/cpp/build/facade_test --bench 4096 16 --trace --repeat=3 --depth=$d >> gpurun_out/r06/facade64k_depth.jsonl
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06/facade64k_depth.jsonl"):
    d = json.loads(l)
    t = d["decode_trace"]
    print(d["depth"], round(d["encode_GiBps"], 2), round(d["decode_GiBps"], 2), t["batches"], t["us_per_batch"], t["two_in_flight_frac"])
PY
