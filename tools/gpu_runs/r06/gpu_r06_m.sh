# round 6 validation after the tile padding choice: the whole GPU suite, smoke(), RotatE / pRotatE
# ranking against the previous library (ab_prev/), the default bench line, the driver's window,
# and the bench's rocprofv3 kernel trace
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06m"
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
PREV="$ROOT/ab_prev/knowledgegraphembedding_amd/libkge_hip.so"
timeout -k 10 200 python3 tools/bench_rank.py --models RotatE --shape fb15k -d 1000 --gamma 24 --reps 3 >> "$O/fb_new.jsonl" 2>> "$O/err_fb.txt" || exit $?
KGE_HIP_LIB="$PREV" timeout -k 10 200 python3 tools/bench_rank.py --models RotatE --shape fb15k -d 1000 --gamma 24 --reps 3 >> "$O/fb_prev.jsonl" 2>> "$O/err_fb.txt" || exit $?
timeout -k 10 600 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$O/bench_driver_window.json" 2> "$O/bench_driver_window.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_default" -o run -- \
  python3 "$ROOT/bench.py" > "$O/bench_under_rocprof.json" 2> "$O/bench_under_rocprof.err" || exit $?
