# round 5: the register tile's counting pass stages its 64+64 rows through one buffer descriptor per operand (range check
# instead of zero-fill selects) — rank suites, then the FB15k and wn18rr ranking benches
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05ah"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py tests/test_wide_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_fb15k" -o run -- \
  python3 "$ROOT/tools/bench_rank.py" --models RotatE TransE --shape fb15k -d 1000 --gamma 24 --reps 3 > "$O/bench_rank_fb15k.jsonl" 2> "$O/bench_rank.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_protate" -o run -- \
  python3 "$ROOT/tools/bench_rank.py" --models pRotatE --shape wn18rr -d 500 --gamma 6 --reps 3 > "$O/bench_rank_protate.jsonl" 2>> "$O/bench_rank.err" || exit $?
timeout -k 10 300 python3 "$ROOT/tools/bench_rank.py" --models pRotatE --shape wn18rr -d 500 --gamma 6 --reps 3 --rank-trig device \
  >> "$O/bench_rank_protate.jsonl" 2>> "$O/bench_rank.err" || exit $?
cd "$ROOT"
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || exit $?
