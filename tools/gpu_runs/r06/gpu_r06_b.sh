# round 6: the two-direction ranking pass — rank parity / edge suites, then wall times and a kernel trace
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06b"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests.log" 2>&1 || exit $?
for m in DistMult ComplEx; do
  timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 8 > "$O/times_$m.json" 2> "$O/err_t_$m.txt" || exit $?
  KGE_RANK_BOTH=0 timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 8 > "$O/times_${m}_perdir.json" 2>> "$O/err_t_$m.txt" || exit $?
done
cd /tmp && export TMPDIR=/tmp
for m in DistMult ComplEx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof_$m" -o run -- \
    python3 "$ROOT/tools/rank_timeline.py" --model $m --reps 5 > "$O/ptimes_$m.json" 2> "$O/err_$m.txt" || exit $?
done
