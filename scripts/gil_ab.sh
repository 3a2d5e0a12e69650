#!/bin/bash
# A/B of the GIL switch interval in the agent + fake kubelet (real MI355X bench, config 2 only).
set -u
O=gpurun_out/${1:-gilab}
mkdir -p $O
export PYTHONPATH=$PWD
for sw in 0.005 0.0005 0.005 0.0005; do
  GPUPOOL_GIL_SWITCH_INTERVAL=$sw timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 3 \
    --scale-down-steps 0 --pool-steps 0 --health-steps 0 >> $O/bench_sw$sw.json 2>> $O/bench.err
  rc=$?; echo "sw=$sw rc=$rc" >> $O/bench.err; [ $rc -eq 0 ] || exit $rc
done
