# Round-4 GPU pass t: the grouped GEMM tile order at the claim-time size — standalone 2048^3 and
# the whole overlapped claim-time probe (HBM test beside it), grouped vs row-major.
set -o pipefail
mkdir -p gpurun_out/r4t
export PYTHONPATH=$GRAFT_REPO_ROOT
GROUP_AB_SIZES=2048 timeout -k 10 200 python -u scripts/probe_gemm_group_ab.py 9 > gpurun_out/r4t/gemm_group_2048.json 2> gpurun_out/r4t/g.err && \
timeout -k 10 300 python -u scripts/probe_idle_gap_ab.py --rounds 40 --gap 0.3 --variant gemmGroupM=0 --variant gemmGroupM=4 > gpurun_out/r4t/claim_probe_group_ab.json 2> gpurun_out/r4t/c.err
