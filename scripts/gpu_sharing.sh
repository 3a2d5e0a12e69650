#!/bin/bash
# GPU box: isolated-sharing tests (libgpupool_share.so via HSA_TOOLS_LIB), time-limited.
set -u
O=gpurun_out/${1:-sharing}
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/gpu/test_sharing_gpu.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_sharing.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_sharing.txt; exit $rc
