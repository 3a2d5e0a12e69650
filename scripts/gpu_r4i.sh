# Round-4 GPU pass i: probe idle-gap A/B, a 100-step headline bench soak, then the GPU tier
# and smoke on the current tree.
set -o pipefail
mkdir -p gpurun_out/r4i
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 180 python -u scripts/probe_idle_gap_ab.py 15 1.2 > gpurun_out/r4i/probe_idle_gap_ab.json 2> gpurun_out/r4i/idle.err && \
timeout -k 10 600 python -u bench.py --steps 100 --warmup 3 > gpurun_out/r4i/bench_soak.json 2> gpurun_out/r4i/bench_soak.err && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r4i/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4i/smoke.txt 2>&1
