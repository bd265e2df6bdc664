# round 5: the config-5 world-8 owner-computes test once more, with the failure
# report naming the owners / columns of any differing rows (r05r failed it once)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05s"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest "tests/test_partition_gpu.py::test_row_partition_yago3_10_shape[8-factors]" \
  "tests/test_partition_gpu.py::test_row_partition_yago3_10_shape[4-factors]" -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1
