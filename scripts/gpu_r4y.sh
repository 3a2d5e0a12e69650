# Round-4 GPU pass y: the final tree as the driver runs it — the whole GPU tier, smoke, and
# bench.py with no flags (the driver's N=1 defaults).
set -o pipefail
mkdir -p gpurun_out/r4y
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r4y/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4y/smoke.txt 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r4y/bench.json 2> gpurun_out/r4y/bench.err
