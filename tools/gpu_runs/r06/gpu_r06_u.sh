# round 6: bench.py's multi-rank path rehearsed on one GPU with gloo (the driver's torchrun launch
# shape): N = 2 (factor exchange), N = 4 (owner exchange), config 5 row partition at N = 2; each line
# carries the replica check
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06u"
mkdir -p "$O"
cd "$ROOT"
export KGE_DIST_BACKEND=gloo
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 10 --warmup 3 --no-rank --no-cpu-baseline > "$O/bench_n2.json" 2> "$O/err_n2.txt" || exit $?
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 4 --steps 10 --warmup 3 --no-rank --no-cpu-baseline > "$O/bench_n4.json" 2> "$O/err_n4.txt" || exit $?
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 2 --steps 10 --warmup 3 --no-rank --no-cpu-baseline --workload yago3-10-rowpart > "$O/bench_yago_n2.json" 2> "$O/err_yago_n2.txt" || exit $?
