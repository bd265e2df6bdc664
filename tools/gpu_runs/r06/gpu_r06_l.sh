# round 6: register-tile k-rows padded for every model (pRotatE / RotatE staging-store bank
# conflicts); rank parity + edge suites; A/B against the library of commit dc94963 (ab_prev/),
# alternated; pRotatE / RotatE tile wave states
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06l"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py tests/test_wide_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests.log" 2>&1 || exit $?
PREV="$ROOT/ab_prev/knowledgegraphembedding_amd/libkge_hip.so"
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_new.jsonl" 2>> "$O/err_prot.txt" || exit $?
  KGE_HIP_LIB="$PREV" timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_prev.jsonl" 2>> "$O/err_prot.txt" || exit $?
  for m in RotatE TransE; do
    timeout -k 10 200 python3 tools/bench_rank.py --models $m --shape fb15k -d 1000 --gamma 24 --reps 3 >> "$O/fb_new.jsonl" 2>> "$O/err_fb.txt" || exit $?
    KGE_HIP_LIB="$PREV" timeout -k 10 200 python3 tools/bench_rank.py --models $m --shape fb15k -d 1000 --gamma 24 --reps 3 >> "$O/fb_prev.jsonl" 2>> "$O/err_fb.txt" || exit $?
  done
done
TAG=protate_pad COUNTERS="GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
  MODELS=pRotatE EXTRA="--gamma 6" bash tools/pmc_rank.sh > "$O/pmc_protate_pad.txt" 2>&1 || exit $?
TAG=rotate_pad COUNTERS="GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
  MODELS=RotatE EXTRA="--shape fb15k -d 1000 --gamma 24" bash tools/pmc_rank.sh > "$O/pmc_rotate_pad.txt" 2>&1 || exit $?
