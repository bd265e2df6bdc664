# round 6: does gloo order its async CUDA all-gathers on the caller's stream? (one run)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06a"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_collective_order_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/order.log" 2>&1
