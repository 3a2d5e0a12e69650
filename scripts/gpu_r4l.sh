# Round-4 GPU pass l: headline bench on the tree with the in-kernel counter reset (40 steps), then a
# rocprofv3 kernel trace + stats of it (kernel trace only, no PMC).
set -o pipefail
mkdir -p gpurun_out/r4l
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 > gpurun_out/r4l/bench.json 2> gpurun_out/r4l/bench.err && \
bash scripts/gpu_bench_prof.sh r4l/prof
