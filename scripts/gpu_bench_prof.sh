#!/bin/bash
# rocprofv3 kernel trace + stats over the headline bench (real config 2 path: the agent's in-process
# probe kernels run in a child process, which the profiler follows). Kernel trace only, no PMC.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-benchprof}
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o bench -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 10 --warmup 2 --health-steps 0 > $O/bench.json 2> $O/bench.err
rc=$?; echo "rocprof rc=$rc" >> $O/bench.err; exit $rc
