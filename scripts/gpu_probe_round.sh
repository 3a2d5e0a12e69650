#!/bin/bash
# Probe kernel A/B + GPU tier + bench, each GPU step time-limited, stop at the first failure.
set -u
O=gpurun_out/${1:-probe}
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 60 build/native/probe_selftest > $O/selftest.json 2>&1
rc=$?; echo "selftest rc=$rc" >> $O/selftest.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_ab.py --rounds 5 > $O/probe_ab.json 2> $O/probe_ab.err
rc=$?; echo "probe_ab rc=$rc" >> $O/probe_ab.err; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_round.sh ${1:-probe}
