#!/bin/bash
# GPU tier: pytest -m gpu, then the driver's smoke(), each step time-limited.
set -u
O=gpurun_out/gputests
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo "smoke rc=$?" >> $O/smoke.txt
