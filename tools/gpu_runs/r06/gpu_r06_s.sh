# round 6: the split-bf16 tile with a 2-stage ring (KGE_XTILE_NST=2: one slab in flight, four
# workgroups per CU) against the 3-stage default (three per CU): rank parity with it, whole-pass
# times alternated, kernel stats
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06t"
mkdir -p "$O"
cd "$ROOT"
KGE_XTILE_NST=2 timeout -k 10 600 python -u -m pytest tests/test_rank_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests_nst2.log" 2>&1 || exit $?
for rep in 1 2 3; do
  for m in DistMult ComplEx; do
    timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 10 >> "$O/times_nst3.jsonl" 2>> "$O/err_t.txt" || exit $?
    KGE_XTILE_NST=2 timeout -k 10 120 python3 tools/rank_timeline.py --model $m --reps 10 >> "$O/times_nst2.jsonl" 2>> "$O/err_t.txt" || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for sps in 3 2; do
  KGE_XTILE_NST=$sps timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_sps$sps" -o run -- \
    python3 "$ROOT/tools/rank_timeline.py" --model DistMult --reps 5 > "$O/ptimes_sps$sps.json" 2> "$O/err_p$sps.txt" || exit $?
done
