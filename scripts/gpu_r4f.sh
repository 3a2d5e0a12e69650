# Round-4 GPU pass f: the libc-only share library on hardware (isolated-sharing tests incl. the
# operator's end-to-end isolated-slot test).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/gpu/test_sharing_gpu.py tests/gpu/test_operator_gpu.py -k "sharing or isolated or slot or time_sliced" > gpurun_out/r4f_sharing.txt 2>&1
