# Round-4 GPU pass o: the whole GPU tier, smoke and a 40-step headline bench on the tree with the
# in-kernel counter reset, the restart re-probe, fresh gRPC subchannels and the capped feed backoff.
set -o pipefail
mkdir -p gpurun_out/r4o
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r4o/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4o/smoke.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 > gpurun_out/r4o/bench.json 2> gpurun_out/r4o/bench.err
