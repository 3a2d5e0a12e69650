#!/bin/bash
# Real-MI355X bench (sweep + scale-down + health) plus the amd-smi RAS/bad-page shapes.
set -u
O=gpurun_out/${1:-bench2}
mkdir -p $O
export PYTHONPATH=$PWD
(amd-smi bad-pages --json > $O/amdsmi_bad_pages.json 2>&1; amd-smi metric --ecc --json > $O/amdsmi_metric_ecc.json 2>&1; amd-smi static --ras --json > $O/amdsmi_static_ras.json 2>&1; true)
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 3 --workdir $PWD/$O/bench > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/bench.err; cat $O/bench.json; exit $rc
