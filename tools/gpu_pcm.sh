# PCM transformer GPU session: parity tests, throughput, rocprofv3 kernel stats.
set -u
mkdir -p gpurun_out/pcm
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pcm.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pcm/pytest.log 2>&1; rc=$?; echo "pytest=$rc"; tail -3 gpurun_out/pcm/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/pcm_bench.py > gpurun_out/pcm/bench.jsonl 2>&1; rc=$?; echo "bench=$rc"; cat gpurun_out/pcm/bench.jsonl
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/pcm/trace
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pcm/trace -o run -- python3 tools/pcm_bench.py 268435456 10 > gpurun_out/pcm/trace.log 2>&1; rc=$?; echo "trace=$rc"
exit $rc
