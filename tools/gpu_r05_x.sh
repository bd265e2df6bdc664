# round 5: the refinement with the next item's row prefetched into registers —
# rank parity / edge / wide tests, then the ranking pass traced as in r05w
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05x"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py tests/test_wide_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for m in DistMult ComplEx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof_$m" -o run -- \
    python3 "$ROOT/tools/rank_timeline.py" --model $m --reps 5 > "$O/times_$m.json" 2> "$O/err_$m.txt" || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_fb15k" -o run -- \
  python3 "$ROOT/tools/bench_rank.py" --models RotatE TransE --shape fb15k -d 1000 --gamma 24 --reps 3 > "$O/bench_rank_fb15k.jsonl" 2> "$O/bench_rank.err" || exit $?
