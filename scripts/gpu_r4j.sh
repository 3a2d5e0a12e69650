# Round-4 GPU pass j: probe counter-reset path — the probe GPU tests (incl. reset-after-fault on
# both paths), then the idle-gap A/B of the two paths.
set -o pipefail
mkdir -p gpurun_out/r4j
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/gpu/test_probe_gpu.py > gpurun_out/r4j/pytest_probe_gpu.txt 2>&1 && \
timeout -k 10 240 python -u scripts/probe_idle_gap_ab.py 24 1.2 > gpurun_out/r4j/probe_idle_gap_ab.json 2> gpurun_out/r4j/idle.err
