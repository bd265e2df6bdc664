# round 6: pRotatE tile with the splats from the packed ops' operand selects (rank parity / edge
# suites, A/B against the previous commit's library, alternated); device sampler in the training
# loop against pre-staged batches (200-step windows, alternated); the bench's rocprofv3 trace + PMC
# traffic passes; the TransE tile's wave states with the pre-splatted staging
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06k"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/rank_tests.log" 2>&1 || exit $?
PREV="$ROOT/ab_prev/knowledgegraphembedding_amd/libkge_hip.so"
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_new.jsonl" 2>> "$O/err_prot.txt" || exit $?
  KGE_HIP_LIB="$PREV" timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_prev.jsonl" 2>> "$O/err_prot.txt" || exit $?
done
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-rank --no-cpu-baseline --steps 200 --warmup 20 > "$O/bench_staged_$i.json" 2> "$O/err_staged_$i.txt" || exit $?
  KGE_BENCH_SAMPLER=device timeout -k 10 200 python3 bench.py --no-rank --no-cpu-baseline --steps 200 --warmup 20 > "$O/bench_device_$i.json" 2> "$O/err_device_$i.txt" || exit $?
done
bash tools/profile.sh > "$O/profile.log" 2>&1 || exit $?
TAG=transe_spl COUNTERS="GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
  MODELS=TransE EXTRA="--shape fb15k -d 1000 --gamma 24" bash tools/pmc_rank.sh > "$O/pmc_transe_spl.txt" 2>&1 || exit $?
TAG=protate_sel COUNTERS="GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
  MODELS=pRotatE EXTRA="--gamma 6" bash tools/pmc_rank.sh > "$O/pmc_protate_sel.txt" 2>&1 || exit $?
