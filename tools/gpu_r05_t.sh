# round 5: the owner-computes exchange with rows over 2048 floats (kge_wide.inc)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05t"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_dp_owner_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$O/gpu_tests.log" 2>&1
