# round 6: the occurrence CSR's kernels with capped grids beside k_row (KGE_CSR_BLOCKS), 200-step
# windows alternated on one box; training parity suite with a capped grid
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06p"
mkdir -p "$O"
cd "$ROOT"
KGE_CSR_BLOCKS=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/parity_cap32.log" 2>&1 || exit $?
for i in 1 2; do
  for c in 0 32 128 512; do
    KGE_CSR_BLOCKS=$c timeout -k 10 200 python3 bench.py --no-rank --no-cpu-baseline --steps 200 --warmup 20 > "$O/bench_cap${c}_$i.json" 2> "$O/err_cap${c}_$i.txt" || exit $?
  done
done
