mkdir -p gpurun_out
timeout -k 10 180 python3 -u tools/seg_parse_diag.py > gpurun_out/diag.log 2>&1; echo "diag=$?"
grep -v amdgpu.ids gpurun_out/diag.log
