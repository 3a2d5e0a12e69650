# Round-4 GPU pass g: advertise A/B, then the whole GPU tier and smoke on the current tree.
set -o pipefail
mkdir -p gpurun_out/r4g
bash scripts/advertise_ab.sh r4g/advab && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r4g/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4g/smoke.txt 2>&1
