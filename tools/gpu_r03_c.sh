# Long-stream and mix workloads: seg_bench (bs 128 and 512), configs[3] mix bench (8 GiB, then 32 GiB)
mkdir -p gpurun_out
timeout -k 10 400 python tools/seg_bench.py > gpurun_out/seg_bench.jsonl 2> gpurun_out/seg_bench.err; echo "seg_bench=$?"; cat gpurun_out/seg_bench.jsonl
timeout -k 10 200 python tools/seg_bench.py --bs=512 "16 MiB Poisson" "generator stream" > gpurun_out/seg_bench512.jsonl 2>> gpurun_out/seg_bench.err; echo "seg_bench512=$?"; cat gpurun_out/seg_bench512.jsonl
timeout -k 10 300 python bench.py --workload mix --mix-gib 8 --steps 5 --warmup 1 > gpurun_out/bench_mix8.log 2>&1; echo "mix8=$?"; tail -1 gpurun_out/bench_mix8.log
timeout -k 10 500 python bench.py --workload mix --steps 3 --warmup 1 > gpurun_out/bench_mix32.log 2>&1; echo "mix32=$?"; tail -1 gpurun_out/bench_mix32.log
