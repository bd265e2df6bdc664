# round 4: k_row time per row against the batch (1024 rows = every block resident at once; 2048 / 4096 = two / four waves of blocks)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for BB in 1024 2048 4096 1024; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/rowb_$BB" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 40 --no-cpu-baseline --no-rank --batch $BB > "$GRAFT_REPO_ROOT/gpurun_out/rowb_$BB.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/rowb_$BB.err" || exit $?
done
