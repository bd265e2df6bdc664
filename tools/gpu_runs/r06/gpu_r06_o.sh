# round 6: the filter index built on the GPU for test_step (torch unique / sort of the packed keys);
# ranking, edge and run.py GPU suites; the bench line without the CPU baseline (test_step block)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06o"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 800 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py tests/test_run_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || exit $?
