# round 4: s_true in reference order (k_rank_true_ref) against the gather-mode tile: ranks and whole-pass time
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04n_rank.log 2>&1 || exit $?
for k in 1 2; do
  for v in 1 0; do
    KGE_RANK_TRUE_REF=$v timeout -k 10 200 python -u tools/bench_rank.py --models DistMult ComplEx --reps 5 > gpurun_out/r04n_truref_$v_$k.jsonl 2>/dev/null || exit $?
    echo "TRUE_REF=$v run $k"; grep -o '"model": "[A-Za-z]*"\|"seconds": [0-9.e-]*' gpurun_out/r04n_truref_$v_$k.jsonl | paste - - 
  done
done > gpurun_out/r04n_ab.txt
