# Round-4 GPU pass u: s_setprio around the probe GEMM's MFMA block (T5), in-process A/B at 4096^3
# and 8192^3 with the grouped tile order, plus the probe GPU tests.
set -o pipefail
mkdir -p gpurun_out/r4u
export PYTHONPATH=$GRAFT_REPO_ROOT
GROUP_AB_VARIANTS=g4,p4 timeout -k 10 300 python -u scripts/probe_gemm_group_ab.py 11 > gpurun_out/r4u/gemm_prio_ab.json 2> gpurun_out/r4u/p.err && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_probe_gpu.py > gpurun_out/r4u/pytest_probe_gpu.txt 2>&1
