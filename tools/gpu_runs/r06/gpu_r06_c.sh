# round 6: (1) rank parity / edge suites after the side-stream table work and the late copy;
# (2) ranking wall times A/B on one box: per direction / both / both without the side stream;
# (3) entity-pass drift: the round-4 tree (abr04/, temporary) against this tree, alternated, rocprofv3
#     kernel stats over 200 steps each; then k_row with the CSR serialised (KGE_CSR_SERIAL=1)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06c"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests.log" 2>&1 || exit $?
for rep in 1 2; do
  for m in DistMult ComplEx; do
    KGE_RANK_BOTH=0 timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 10 >> "$O/times_perdir.jsonl" 2>> "$O/err_t.txt" || exit $?
    timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 10 >> "$O/times_both.jsonl" 2>> "$O/err_t.txt" || exit $?
    KGE_RANK_SIDE=0 timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 10 >> "$O/times_both_noside.jsonl" 2>> "$O/err_t.txt" || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for m in DistMult ComplEx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/rprof_$m" -o run -- \
    python3 "$ROOT/tools/rank_timeline.py" --model $m --reps 5 > "$O/ptimes_$m.json" 2> "$O/err_$m.txt" || exit $?
done
run() {  # tag dir [env...]
  local tag=$1 dir=$2; shift 2
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$tag" -o run -- \
    python3 "$dir/bench.py" --no-rank --no-cpu-baseline --steps 200 --warmup 20 > "$O/bench_$tag.json" 2> "$O/err_$tag.txt"
}
run now1 "$ROOT" && run r04a "$ROOT/abr04" && run now2 "$ROOT" && run r04b "$ROOT/abr04" && \
run serial1 "$ROOT" KGE_CSR_SERIAL=1 && run now3 "$ROOT" && run serial2 "$ROOT" KGE_CSR_SERIAL=1 || exit $?
