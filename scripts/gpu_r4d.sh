# Round-4 GPU pass d: smoke(), then a rocprofv3 kernel trace of the headline bench (the agent's
# in-process probe with the 2048^3 overlap GEMM), kernel trace + stats only.
set -o pipefail
mkdir -p gpurun_out/r4d
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4d/smoke.txt 2>&1 && \
bash scripts/gpu_bench_prof.sh r4d/prof
