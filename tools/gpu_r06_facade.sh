# Round-6 GPU session: the facade's 16 MiB slow mode (16 threads x 16 MiB blocks, batch trace, buffer growth),
# two separate processes of five runs, after buffers sized by batch capacity; the facade test.
# Output: gpurun_out/r06/facade6_*.jsonl
set -e
mkdir -p gpurun_out/r06
for set in a b; do
  timeout -k 10 300 ./tests/cpp/build/facade_test --bench 64 --kib=16384 16 --trace --repeat=5 > gpurun_out/r06/facade6_16m_$set.jsonl
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06/facade6_16m_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        print(f.split("facade6_16m_")[-1][:-6], round(d["encode_GiBps"], 1), round(d["decode_GiBps"], 1),
              d["contexts_created"], d["buffer_grows"], d["buffer_grow_ms"], d["decode_trace"]["device_idle_frac"])
PY
timeout -k 10 300 ./tests/cpp/build/facade_test > gpurun_out/r06/facade_test_all3.txt 2>&1
tail -2 gpurun_out/r06/facade_test_all3.txt
