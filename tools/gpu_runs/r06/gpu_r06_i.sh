# round 6: the split tile's error from the pieces' actual norms (narrower windows); rank parity,
# edge and wide-row suites; listed counts and whole-pass times against the previous commit's
# library (ab_prev/, KGE_HIP_LIB), alternated; rocprofv3 kernel stats of the both-direction pass
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06i"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py tests/test_wide_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests.log" 2>&1 || exit $?
PREV="$ROOT/ab_prev/knowledgegraphembedding_amd/libkge_hip.so"
timeout -k 10 200 python3 tools/bench_rank.py --models DistMult ComplEx --reps 3 > "$O/bench_rank_new.jsonl" 2>> "$O/err_b.txt" || exit $?
KGE_HIP_LIB="$PREV" timeout -k 10 200 python3 tools/bench_rank.py --models DistMult ComplEx --reps 3 > "$O/bench_rank_prev.jsonl" 2>> "$O/err_b.txt" || exit $?
for rep in 1 2 3; do
  for m in DistMult ComplEx; do
    timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 10 >> "$O/times_new.jsonl" 2>> "$O/err_t.txt" || exit $?
    KGE_HIP_LIB="$PREV" timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 10 >> "$O/times_prev.jsonl" 2>> "$O/err_t.txt" || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for m in DistMult ComplEx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/rprof_$m" -o run -- \
    python3 "$ROOT/tools/rank_timeline.py" --model $m --reps 5 > "$O/ptimes_$m.json" 2> "$O/err_$m.txt" || exit $?
done
