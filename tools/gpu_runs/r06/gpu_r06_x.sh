# round 6: k_split_stats with four chunks' loads in flight (unrolled guard) and the pieces formed once;
# rank parity / edge suites; kernel stats of the both-direction DistMult / ComplEx pass
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06x"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for m in DistMult ComplEx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/rprof_$m" -o run -- \
    python3 "$ROOT/tools/rank_timeline.py" --model $m --reps 10 > "$O/ptimes_$m.json" 2> "$O/err_$m.txt" || exit $?
done
