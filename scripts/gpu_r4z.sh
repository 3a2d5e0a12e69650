# Round-4 GPU pass z: the GPU tier once more on the final tree (flake check after the RPC deadline
# fix); on a failure the test clusters' logs come back as a tarball.
set -o pipefail
mkdir -p gpurun_out/r4z
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
    --basetemp /tmp/r4z_pt -p no:cacheprovider tests > gpurun_out/r4z/pytest_gpu.txt 2>&1 || {
  rc=$?
  tar czf gpurun_out/r4z/pt_logs.tgz -C /tmp --exclude='*.sock' --exclude='*.so' r4z_pt 2>/dev/null
  exit $rc
}
