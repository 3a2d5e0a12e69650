# Round-4 GPU pass s: a 100-step headline soak on the final tree (tail latency), then a rocprofv3
# kernel trace + stats of a 10-step bench (kernel trace only, no PMC).
set -o pipefail
mkdir -p gpurun_out/r4s
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py --steps 100 --warmup 3 > gpurun_out/r4s/bench_soak100.json 2> gpurun_out/r4s/bench_soak100.err && \
bash scripts/gpu_bench_prof.sh r4s/prof
