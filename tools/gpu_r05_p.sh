# round 5: rows over 2048 floats per (half-)row (kge_wide.inc) — the new wide
# tests, then the parity / rank / edge suites the shared code touches
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05p"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=10 > "$O/gpu_tests_wide.log" 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_edge_gpu.py tests/test_rank_parity_gpu.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider --durations=10 > "$O/gpu_tests.log" 2>&1 || exit $?
