# Round-4 GPU pass za: a 300-cycle headline soak on the final tree (tail latency after the RPC
# deadline fix).
set -o pipefail
mkdir -p gpurun_out/r4za
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench.py --steps 300 --warmup 3 > gpurun_out/r4za/bench_soak300.json 2> gpurun_out/r4za/bench_soak300.err
