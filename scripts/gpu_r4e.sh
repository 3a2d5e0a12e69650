# Round-4 GPU pass e: probe launch-order A/B + the probe GPU tests with the new default.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/probe_launch_order_ab.py 25 > gpurun_out/r4e_probe_launch_order_ab.json 2> gpurun_out/r4e_probe_launch_order_ab.err && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/gpu/test_probe_gpu.py > gpurun_out/r4e_pytest_probe.txt 2>&1
