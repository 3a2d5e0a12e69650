# Round-4 GPU pass b: which CU masks an SPX MI355X applies (XCD-aligned vs striped), then the GPU
# tier (minus the XCD-layout census under investigation) and a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/cu_mask_layouts.py --out gpurun_out/r4b_cu_mask_layouts.json > gpurun_out/r4b_cu_mask_layouts.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests -k "not xcd_aligned" > gpurun_out/r4b_pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err
