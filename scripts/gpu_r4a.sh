set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/gpu/test_sharing_gpu.py > gpurun_out/r4a_sharing.txt 2>&1 && \
timeout -k 10 600 python -u scripts/xcd_interference_ab.py --rounds 3 --out gpurun_out/r4a_xcd_ab.json > gpurun_out/r4a_xcd_ab.log 2>&1
