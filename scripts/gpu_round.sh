#!/bin/bash
# One GPU-box pass: pytest -m gpu, smoke(), real bench (config 2) with traces kept. Each GPU step is
# time-limited and the script stops at the first failure.
set -u
O=gpurun_out/${1:-round}
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v ${PYTEST_ARGS:-} --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 3 --workdir $PWD/$O/bench > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/bench.err; cat $O/bench.json; exit $rc
