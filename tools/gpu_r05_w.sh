# round 5: kernel trace of bench.py's config-3 ranking pass (rank_queries_both)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05w"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for m in DistMult ComplEx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof_$m" -o run -- \
    python3 "$ROOT/tools/rank_timeline.py" --model $m --reps 5 > "$O/times_$m.json" 2> "$O/err_$m.txt" || exit $?
done
