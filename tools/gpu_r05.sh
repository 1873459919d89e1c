# Round-5 GPU session steps (run through gpurun; outputs under gpurun_out/r05/).
# usage: bash tools/gpu_r05.sh step [step ...]
#   isa      instruction-rate microbenchmark (tools/isa_rate)
#   occ      fused-decode time vs waves per SIMD (tools/occupancy_sweep.py)
#   bench    bench line, the driver's short command and the default one (no CPU baseline)
#   variants bench line per library variant dwarfs_amd/lib/libricepp_amd_<v>.so (VARIANTS="a b")
#   facade   C++ facade test, then its throughput bench (64 KiB, 1 / 16 MiB blocks)
#   tests    the GPU test suite
#   trace    rocprofv3 kernel trace of the bench workload
#   pmc      PMC passes of the bench workload (tools/gpu_pmc.sh)
#   benchcpu the default bench line with its CPU baseline
#   sweep    configs[4] bs 16 / 32 / 128 x 10-16 bits (tools/workloads.py sweep)
#   f16      facade 16 MiB blocks at 8 / 16 / 32 threads: packed / slot-copy encode, 2 / 1 batches in flight
#   mix      bench.py --workload mix at 32 GiB, 10 steps
#   mixpmc   PMC passes of the 32 GiB mix (tools/gpu_pmc_mix.sh)
#   sbl      small-batch decode latency per path (tools/small_batch_latency.py)
#   paths    bs 16 / 32 decode per path (tools/workloads.py paths)
#   flac     the FLAC GPU tests, then tools/flac_bench.py
#   ftests   the facade GPU tests (C++ facade_test incl. exit with batches in flight) and the FLAC GPU tests
#   f16x5    facade 16 MiB blocks, 16 threads, five consecutive runs (bimodality check)
#   pmcq     one PMC pass of the bench workload per library (default + VARIANTS): cycles, LDS, VALU, SALU
#   dtests   the decode parity tests only (tests/test_gpu_parity.py, test_gpu_abi.py)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  tail -c 1500 "$O/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$O/$name.err"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    isa) run isa 60 ./tools/isa_rate ;;
    occ) run occ 240 python tools/occupancy_sweep.py ;;
    bench)
      run bench_short 240 python bench.py --no-cpu --steps 20 --warmup 5
      run bench_def 240 python bench.py --no-cpu ;;
    benchcpu) run bench_cpu 300 python bench.py ;;
    sweep) run sweep 600 python tools/workloads.py sweep ;;
    variants)
      for v in ${VARIANTS:-}; do
        RICEPP_AMD_LIB=$PWD/dwarfs_amd/lib/libricepp_amd_$v.so run "bench_$v" 240 python bench.py --no-cpu
      done ;;
    facade)
      run facade_test 300 ./tests/cpp/build/facade_test
      run facade_64k 300 ./tests/cpp/build/facade_test --bench 4096 16 64
      run facade_1m 300 ./tests/cpp/build/facade_test --bench 256 --kib=1024 16 64
      run facade_16m 300 ./tests/cpp/build/facade_test --bench 64 --kib=16384 4 16 ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    trace)
      rm -rf gpurun_out/prof/trace
      run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --no-cpu ;;
    pmc) run pmc 900 bash tools/gpu_pmc.sh ;;
    f16)
      run f16_main 300 ./tests/cpp/build/facade_test --bench 64 --kib=16384 8 16 32
      run f16_nopack 300 ./tests/cpp/build/facade_test --bench 64 --kib=16384 --pack-max-mib=16 8 16 32
      run f16_d1 300 ./tests/cpp/build/facade_test --bench 64 --kib=16384 --depth=1 8 16 32
      run f16_nopack_d1 300 ./tests/cpp/build/facade_test --bench 64 --kib=16384 --pack-max-mib=16 --depth=1 8 16 32 ;;
    mix) run bench_mix 600 python bench.py --workload mix --mix-gib 32 --steps 10 --warmup 2 ;;
    mixpmc) run mixpmc 1300 bash tools/gpu_pmc_mix.sh ;;
    sbl) run sbl 200 python tools/small_batch_latency.py ;;
    paths) run paths 400 python tools/workloads.py paths ;;
    flac)
      run flac_tests 600 python -u -m pytest tests/test_gpu_flac.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
      run flac_bench 300 python tools/flac_bench.py ;;
    pmcq)
      for v in base ${VARIANTS:-}; do
        if [ "$v" = base ]; then lib=$PWD/dwarfs_amd/lib/libricepp_amd.so; else lib=$PWD/dwarfs_amd/lib/libricepp_amd_$v.so; fi
        rm -rf gpurun_out/pmcq/$v
        RICEPP_AMD_LIB=$lib run "pmcq_$v" 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
          --output-format csv -d gpurun_out/pmcq/$v/p1 -o run -- python3 tools/prof_kernels.py 2
        python3 tools/pmc_summary.py gpurun_out/pmcq/$v > $O/pmcq_$v.txt; echo "== $v"; cat $O/pmcq_$v.txt
      done ;;
    ftests) run ftests 600 python -u -m pytest tests/test_gpu_block_codec.py tests/test_gpu_flac.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    f16x5)
      for i in 1 2 3 4 5; do run f16x5_$i 300 ./tests/cpp/build/facade_test --bench 64 --kib=16384 16; done ;;
    f64k) run f64k 300 ./tests/cpp/build/facade_test --bench 4096 16 64 ;;
    dtests) run dtests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abi.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
