set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probe_hbm_layout_ab.py 9 > gpurun_out/r4h_probe_hbm_layout_ab.json 2> gpurun_out/r4h_probe_hbm_layout_ab.err && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/gpu/test_probe_gpu.py > gpurun_out/r4h_pytest_probe.txt 2>&1
