# Round-4 GPU pass r: claim probes beside sweep-buffer (un)mapping with 1 GiB chunks (chunk timings
# traced), the whole GPU tier with the grouped GEMM tile order as default, smoke, and a 40-step
# bench that reports its slowest cycle's breakdown.
set -o pipefail
mkdir -p gpurun_out/r4r
export PYTHONPATH=$GRAFT_REPO_ROOT
GPUPOOL_SWEEP_TRACE=1 timeout -k 10 300 python -u scripts/probe_during_sweep_free.py > gpurun_out/r4r/sweep_1g.json 2> gpurun_out/r4r/sweep_1g_chunks.txt && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r4r/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4r/smoke.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 > gpurun_out/r4r/bench.json 2> gpurun_out/r4r/bench.err
