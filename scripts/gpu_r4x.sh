# Round-4 GPU pass x: L2 hit/miss counters (rocprofv3 --pmc, one pass per variant, kernel trace
# only beside it) of the probe GEMM at 8192^3, row-major vs grouped tile order; then a 200-step
# headline soak on the final tree.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r4x
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/g0 -o g0 -- python3 $GRAFT_REPO_ROOT/scripts/gemm_l2_pmc.py 8192 0 > $O/g0.out 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/g4 -o g4 -- python3 $GRAFT_REPO_ROOT/scripts/gemm_l2_pmc.py 8192 4 > $O/g4.out 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u bench.py --steps 200 --warmup 3 > $O/bench_soak200.json 2> $O/bench_soak200.err
