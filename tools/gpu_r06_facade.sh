# Round-6 GPU session: the facade's 16 MiB slow mode (16 threads x 16 MiB blocks, two processes of five runs,
# batch trace) and the 64 KiB reader pattern.  Output: gpurun_out/r06/facade_*.jsonl
set -e
mkdir -p gpurun_out/r06
for s in a b; do
  timeout -k 10 300 ./tests/cpp/build/facade_test --bench 64 --kib=16384 16 --trace --repeat=5 > gpurun_out/r06/facade_16m_$s.jsonl
done
timeout -k 10 300 ./tests/cpp/build/facade_test --bench 4096 16 --trace --repeat=3 > gpurun_out/r06/facade_64k.jsonl
python3 - <<'PY'
import json
for f in ["a", "b"]:
    for l in open(f"gpurun_out/r06/facade_16m_{f}.jsonl"):
        d = json.loads(l)
        print(f, round(d["encode_GiBps"], 1), round(d["decode_GiBps"], 1), d["encode_launches"], d["decode_launches"],
              d["decode_trace"]["requests"], d["decode_trace"]["two_in_flight_frac"], d["decode_trace"]["us_per_batch"])
for l in open("gpurun_out/r06/facade_64k.jsonl"):
    d = json.loads(l)
    print("64k", round(d["encode_GiBps"], 2), round(d["decode_GiBps"], 2), d["decode_trace"]["us_per_batch"], d["decode_trace"]["two_in_flight_frac"])
PY
