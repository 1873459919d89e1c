# host pipeline tests + PCIe-inclusive bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipeline.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_hp.log 2>&1; rc=$?; echo "pytest=$rc"; tail -8 gpurun_out/pytest_hp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/host_pipeline_bench.py 2>&1 | tee gpurun_out/host_pipeline.jsonl
