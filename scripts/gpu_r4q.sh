# Round-4 GPU pass q: sweep-buffer (un)mapping beside claim probes, with and without the chunk
# loop yielding to running probes (in-process A/B by environment), then the probe GPU tests.
set -o pipefail
mkdir -p gpurun_out/r4q
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/probe_during_sweep_free.py > gpurun_out/r4q/sweep_yield.json 2> gpurun_out/r4q/sweep_yield.err && \
GPUPOOL_SWEEP_NO_YIELD=1 timeout -k 10 300 python -u scripts/probe_during_sweep_free.py > gpurun_out/r4q/sweep_noyield.json 2> gpurun_out/r4q/sweep_noyield.err && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_probe_gpu.py > gpurun_out/r4q/pytest_probe_gpu.txt 2>&1 && \
timeout -k 10 300 python -u scripts/probe_gemm_group_ab.py 9 > gpurun_out/r4q/probe_gemm_group_ab.json 2> gpurun_out/r4q/gemm_group.err && \
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 > gpurun_out/r4q/bench.json 2> gpurun_out/r4q/bench.err
