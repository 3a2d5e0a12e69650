#!/bin/bash
# GPU box: HBM pattern A/B (in one process), then the GPU tier / smoke / bench round.
set -u
O=gpurun_out/${1:-patab}
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 180 python -u scripts/probe_pattern_ab.py 9 > $O/pattern_ab.json 2> $O/pattern_ab.err
rc=$?; echo "ab rc=$rc" >> $O/pattern_ab.err; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_round.sh ${1:-patab}
