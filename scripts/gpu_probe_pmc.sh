#!/bin/bash
# PMC counters for the probe kernels (separate runs per counter group; kernel-trace/stats only).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc}
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/g$i -o pmc -- \
    python3 $GRAFT_REPO_ROOT/scripts/probe_ab.py --rounds 1 --sizes 4096 > $O/g$i.log 2>&1
  rc=$?; echo "group $i rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
done
