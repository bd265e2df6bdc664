# round 5: kernel trace of the training step with the entity Adam fused
# (KGE_ENT_FUSED_ADAM was read only by a temporary diagnostic build; the product
# entity pass always fuses the Adam step)
# (product) and split behind the gradient pass (diagnostic), to see where the
# split's extra 0.06 ms goes
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05g"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  KGE_ENT_FUSED_ADAM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_fused$v" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 30 --warmup 10 > "$O/bench_fused$v.json" 2> "$O/bench_fused$v.err" || exit $?
done
