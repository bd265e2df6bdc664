# round 6: pRotatE register tile with its LDS operands read one k ahead, against the unroll-4 loop
# (KGE_TILE_SPL=0, same library), alternated; rank parity suite
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06v"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests.log" 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_pipe.jsonl" 2>> "$O/err.txt" || exit $?
  KGE_TILE_SPL=0 timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_nopipe.jsonl" 2>> "$O/err.txt" || exit $?
done
