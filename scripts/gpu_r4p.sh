# Round-4 GPU pass p: the probe's MFMA GEMM against hipBLASLt (torch.matmul) on the same box.
set -o pipefail
mkdir -p gpurun_out/r4p
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u scripts/gemm_vs_hipblaslt.py 7 > gpurun_out/r4p/gemm_vs_hipblaslt.json 2> gpurun_out/r4p/gemm.err && \
timeout -k 10 300 python -u scripts/probe_during_sweep_free.py > gpurun_out/r4p/probe_during_sweep_free.json 2> gpurun_out/r4p/sweep.err
