#!/bin/bash
# PMC counters for the HBM pattern kernels alone (1 GiB, HBM test only): bytes fetched and written
# per kernel vs the 1 GiB each moves (over-fetch / write amplification). One counter per pass
# (FETCH_SIZE takes 3 TCC counters, WRITE_SIZE 2; at most 4 per pass), kernel-trace only.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-hbmpmc}
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/g$i -o pmc -- \
    python3 $GRAFT_REPO_ROOT/scripts/probe_hbm_sweep.py 1:3 2 > $O/g$i.log 2>&1
  rc=$?; echo "group $i rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
done
