# instruction counts of the bench kernels (one rocprofv3 pass)
mkdir -p gpurun_out/diag3
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/diag3/pmc_1 -o run -- python3 tools/prof_kernels.py 2 > gpurun_out/diag3/pmc_1.log 2>&1 || { tail -5 gpurun_out/diag3/pmc_1.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/diag3
