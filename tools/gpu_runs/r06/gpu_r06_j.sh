# round 6 validation: the whole GPU suite, smoke(), the default bench line and the driver's window
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06j"
mkdir -p "$O"
cd "$ROOT"
( while true; do date >> "$O/heartbeat.txt"; sleep 30; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --durations=15 > "$O/gpu_tests.log" 2>&1
rc=$?
kill $HB
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > "$O/smoke.log" 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$O/bench_driver_window.json" 2> "$O/bench_driver_window.err" || exit $?
