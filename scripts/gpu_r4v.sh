# Round-4 GPU pass v: the probe GEMM with the transposed MFMA and 16-byte C stores vs the current
# epilogue (grouped order both), then the probe GPU tests (incl. the variant's exactness).
set -o pipefail
mkdir -p gpurun_out/r4v
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_probe_gpu.py > gpurun_out/r4v/pytest_probe_gpu.txt 2>&1 && \
GROUP_AB_VARIANTS=g4,v4 GROUP_AB_SIZES=2048,4096,8192 timeout -k 10 300 python -u scripts/probe_gemm_group_ab.py 11 > gpurun_out/r4v/gemm_vecc_ab.json 2> gpurun_out/r4v/v.err
