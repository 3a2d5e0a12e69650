# Round-4 GPU pass m: ABFT accumulators zeroed by the operand kernel too — probe GPU tests, then the
# idle-gap A/B of the in-kernel reset vs memsets.
set -o pipefail
mkdir -p gpurun_out/r4m
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/gpu/test_probe_gpu.py > gpurun_out/r4m/pytest_probe_gpu.txt 2>&1 && \
timeout -k 10 240 python -u scripts/probe_idle_gap_ab.py --rounds 24 --gap 1.2 --variant zeroInKernel=1 --variant zeroInKernel=0 > gpurun_out/r4m/probe_idle_reset_ab.json 2> gpurun_out/r4m/idle.err
