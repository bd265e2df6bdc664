# round 4: the single-score window with the reference-order s_true: ranks, listed counts, whole-pass time
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r04o_rank.log 2>&1 || exit $?
for k in 1 2; do
  for v in 1 0; do
    KGE_RANK_TRUE_REF=$v timeout -k 10 200 python -u tools/bench_rank.py --models DistMult ComplEx --reps 5 > gpurun_out/r04o_tr_${v}_$k.jsonl 2>/dev/null || exit $?
    echo "TRUE_REF=$v run $k"; grep -o '"model": "[A-Za-z]*"\|"seconds": [0-9.e-]*\|"listed_per_query": [0-9.e-]*' gpurun_out/r04o_tr_${v}_$k.jsonl | paste - - -
  done
done > gpurun_out/r04o_ab.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04o_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_rank.py" --models DistMult ComplEx --reps 3 > /dev/null 2>&1 || exit $?
