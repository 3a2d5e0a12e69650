# Round-4 GPU pass w: the whole GPU tier, smoke and a 40-step bench on the tree with leader fencing,
# the any-GPU chunk yield and the VRAM-drop grace.
set -o pipefail
mkdir -p gpurun_out/r4w
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r4w/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4w/smoke.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 > gpurun_out/r4w/bench.json 2> gpurun_out/r4w/bench.err
