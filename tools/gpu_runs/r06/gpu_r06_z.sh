# round 6: KGEModel.test_step end to end at the FB15k evaluation shape for every model
# (tools/bench_test_step.py: 59,071 test triples, both directions, the GPU-built filter index)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06z"
mkdir -p "$O"
cd "$ROOT"
for m in RotatE TransE DistMult ComplEx; do
  timeout -k 10 240 python3 tools/bench_test_step.py --model $m >> "$O/test_step_models.jsonl" 2>> "$O/err.txt" || exit $?
done
timeout -k 10 240 python3 tools/bench_test_step.py --model pRotatE -d 500 --gamma 6 >> "$O/test_step_models.jsonl" 2>> "$O/err.txt" || exit $?
