# round 6: pRotatE / TransE register tiles with pre-splatted staging — parity suites, then the bench's
# ranking sections A/B against round 5's staging (KGE_TILE_SPL=0), alternated, plus test_step
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06d"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py tests/test_wide_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_spl_$i.json" 2> "$O/err_spl_$i.txt" || exit $?
  KGE_TILE_SPL=0 timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_old_$i.json" 2> "$O/err_old_$i.txt" || exit $?
done
