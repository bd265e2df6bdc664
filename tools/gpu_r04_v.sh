# round 4 final tree: the ranking kernels under rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04v_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_rank.py" --models DistMult ComplEx --reps 5 > "$GRAFT_REPO_ROOT/gpurun_out/r04v_rank.jsonl" 2>/dev/null || exit $?
