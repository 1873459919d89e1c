# Round-6 GPU session: the facade's 64 KiB reader pattern (16 threads x 64 KiB) by pipeline depth and the
# process's hardware queue count (GPU_MAX_HW_QUEUES, HIP's default 4): host-observed device time per
# batch vs the batch's device events.  Output: gpurun_out/r06/hwq.jsonl
set -e
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/hwq.jsonl
for q in 4 8 16; do
  for d in 2 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 ./tests/cpp/build/facade_test --bench 4096 16 --trace --repeat=2 --depth=$d | sed "s/^{/{\"hw_queues\": $q, /" >> gpurun_out/r06/hwq.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06/hwq.jsonl"):
    d = json.loads(l)
    print(d["hw_queues"], d["depth"], round(d["encode_GiBps"], 2), round(d["decode_GiBps"], 2), d["decode_us_per_batch"])
PY
