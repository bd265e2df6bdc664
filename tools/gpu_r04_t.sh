# round 4: the merged-correction split tile (3 workgroups per CU): ranks, timing, listed counts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r04t_rank.log 2>&1 || exit $?
MODELS="DistMult ComplEx" bash tools/ab_rank.sh "KGE_XTILE_MERGE=0" "KGE_XTILE_MERGE=1" "KGE_XTILE_MERGE=0" "KGE_XTILE_MERGE=1" > gpurun_out/r04t_ab.txt 2>&1 || exit $?
for v in 0 1; do
  KGE_XTILE_MERGE=$v timeout -k 10 200 python -u tools/bench_rank.py --models DistMult ComplEx --reps 5 > gpurun_out/r04t_br_$v.jsonl 2>/dev/null || exit $?
done
