# round 5: the entity table's Adam split from the gradient pass — the training
# parity suites, then the bench alternated with the fused form (KGE_ENT_FUSED_ADAM=1, diagnostic)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05f"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dp_factors_gpu.py tests/test_dp_owner_gpu.py \
  tests/test_dp_config4_gpu.py tests/test_edge_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$O/gpu_tests.log" 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-rank --steps 200 --warmup 100 > "$O/bench_split_$k.json" 2>> "$O/bench.err" || exit $?
  KGE_ENT_FUSED_ADAM=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-rank --steps 200 --warmup 100 > "$O/bench_fused_$k.json" 2>> "$O/bench.err" || exit $?
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-rank --steps 20 --warmup 5 > "$O/bench_split_20.json" 2>> "$O/bench.err" || exit $?
