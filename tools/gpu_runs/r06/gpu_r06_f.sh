# round 6: sin_rn2 (near-midpoint candidates) in the screen and the selftest; the tile staging switch;
# rank parity + edge suites; pRotatE ranking A/B (fixed diagnostic path); CSR look-ahead A/B at the
# YAGO3-10 shape (config 5's single-GPU step)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06f"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests.log" 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_spl.jsonl" 2>> "$O/err_prot.txt" || exit $?
  KGE_TILE_SPL=0 timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_old.jsonl" 2>> "$O/err_prot.txt" || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload yago3-10-rowpart --no-rank --no-cpu-baseline --steps 100 --warmup 20 > "$O/yago_ahead_$i.json" 2> "$O/err_yago_ahead_$i.txt" || exit $?
  KGE_CSR_AHEAD=0 timeout -k 10 300 python3 bench.py --workload yago3-10-rowpart --no-rank --no-cpu-baseline --steps 100 --warmup 20 > "$O/yago_noahead_$i.json" 2> "$O/err_yago_noahead_$i.txt" || exit $?
done
