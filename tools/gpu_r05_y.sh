# round 5: refinement row prefetch (PQ per row length) against the plain
# (KGE_REF_PQ0 was read only by a temporary A/B build; the prefetch is the product form)
# staging (KGE_REF_PQ0=1, temporary A/B switch), alternated on one box
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05y"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py tests/test_wide_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for run in 1 2; do
  for v in 0 1; do
    KGE_REF_PQ0=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_pq0$v.$run" -o run -- \
      python3 "$ROOT/tools/bench_rank.py" --models DistMult ComplEx --reps 3 > "$O/bench_wn_pq0$v.$run.jsonl" 2>> "$O/err.txt" || exit $?
    KGE_REF_PQ0=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_fb_pq0$v.$run" -o run -- \
      python3 "$ROOT/tools/bench_rank.py" --models RotatE TransE --shape fb15k -d 1000 --gamma 24 --reps 2 > "$O/bench_fb_pq0$v.$run.jsonl" 2>> "$O/err.txt" || exit $?
  done
done
