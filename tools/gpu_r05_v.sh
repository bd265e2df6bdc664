# round 5: rehearsal of the driver's multi-GPU bench command on the one GPU
# (KGE_DIST_BACKEND=gloo: the ranks share the card, so the numbers are not a
# scaling measurement — the run checks that the N-rank path of bench.py runs
# the factor (N = 2) and owner (N = 4) exchanges and prints its line)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05v"
mkdir -p "$O"
cd "$ROOT"
export KGE_DIST_BACKEND=gloo GPU_MAX_HW_QUEUES=1
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 --no-cpu-baseline --no-rank \
    > "$O/bench_gloo_n$n.json" 2> "$O/bench_gloo_n$n.err" || exit $?
done
