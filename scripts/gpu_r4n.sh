# Round-4 GPU pass n: where the claim span's probe time beyond the library's own clock goes — the
# binding's wall time (ctypes + JSON) after an idle gap vs back to back.
set -o pipefail
mkdir -p gpurun_out/r4n
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/probe_idle_gap_ab.py --rounds 16 --gap 1.2 --variant zeroInKernel=1 > gpurun_out/r4n/probe_idle_binding3.json 2> gpurun_out/r4n/idle.err && \
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_probe_gpu.py > gpurun_out/r4n/pytest_probe_gpu.txt 2>&1
