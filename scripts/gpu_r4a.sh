# Round-4 GPU pass: isolated-sharing tests (XCD layout census, UUID-keyed account), the
# striped-vs-XCD interference A/B, then the whole GPU tier and a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/gpu/test_sharing_gpu.py > gpurun_out/r4a_sharing.txt 2>&1 && \
timeout -k 10 600 python -u scripts/xcd_interference_ab.py --rounds 3 --out gpurun_out/r4a_xcd_ab.json > gpurun_out/r4a_xcd_ab.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r4a_pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err
