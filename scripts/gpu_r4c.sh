# Round-4 GPU pass c: isolated-sharing tier, the masked-vs-time-sliced interference A/B, the
# claim-time probe GEMM A/B, the whole GPU tier and a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/gpu/test_sharing_gpu.py > gpurun_out/r4c_sharing.txt 2>&1 && \
timeout -k 10 240 python -u scripts/probe_gemm_overlap_ab.py 25 > gpurun_out/r4c_probe_gemm_overlap_ab.json 2> gpurun_out/r4c_probe_gemm_overlap_ab.err && \
timeout -k 10 600 python -u scripts/slot_interference_ab.py --rounds 3 --out gpurun_out/r4c_slot_ab.json > gpurun_out/r4c_slot_ab.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r4c_pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err
