#!/bin/bash
# rocprofv3 kernel stats for the probe (A/B script as the workload). Kernel trace only (no PMC here).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-probeprof}
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o probe -- \
  python3 $GRAFT_REPO_ROOT/scripts/probe_ab.py --rounds 3 --sizes 4096 > $O/probe_ab.json 2> $O/probe_ab.err
rc=$?; echo "rocprof rc=$rc" >> $O/probe_ab.err; exit $rc
