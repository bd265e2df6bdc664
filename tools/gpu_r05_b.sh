# round 5: after removing the rejected kernel variants and correcting the split
# tile's lo·lo bound — the GPU parity / rank parity / run.py suites, then the
# bench line and the ranking kernels' trace
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05b"
mkdir -p "$O"
cd "$ROOT"
( while true; do date >> "$O/heartbeat.txt"; sleep 30; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  --durations=15 > "$O/gpu_tests.log" 2>&1
rc=$?
kill $HB
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_rank" -o run -- \
  python3 "$ROOT/tools/bench_rank.py" --models DistMult ComplEx --reps 5 > "$O/bench_rank.jsonl" 2> "$O/prof_rank.err" || exit $?
