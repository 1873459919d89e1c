# Round-6 GPU session: where the time of one 7.5 Gbit stream's segmented decode goes (kernel trace), and
# the unit size.  Output: gpurun_out/r06/giant_*.
set -e
mkdir -p gpurun_out/r06
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/giant_prof -o giant -- python3 tools/giant_prof.py 0 3 > gpurun_out/r06/giant_prof.jsonl
cat gpurun_out/r06/giant_prof.jsonl


