# round 5 final validation (after the tile staging change): the whole GPU suite, smoke, bench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05ai"
mkdir -p "$O"
cd "$ROOT"
( while true; do date >> "$O/heartbeat.txt"; sleep 30; done ) &
HB=$!
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --durations=15 > "$O/gpu_tests.log" 2>&1
rc=$?
kill $HB
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit $?
