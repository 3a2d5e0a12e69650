# Round-4 GPU pass k: claim-probe launch order after an idle gap — MFMA phase enqueued after the
# whole HBM test (hbmFirst=1) vs after the first fill (2), both with in-kernel counter reset.
set -o pipefail
mkdir -p gpurun_out/r4k
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/probe_idle_gap_ab.py --rounds 32 --gap 1.2 --variant hbmFirst=1 --variant hbmFirst=2 \
  --variant hbmFirst=0 > gpurun_out/r4k/probe_idle_order_ab.json 2> gpurun_out/r4k/idle.err && \
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_probe_gpu.py > gpurun_out/r4k/pytest_probe_gpu.txt 2>&1
