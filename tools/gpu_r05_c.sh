# round 5: pRotatE's interval screen (three-call form), the tightened
# RotatE / TransE window, the 16x16x32 split-tile experiment — the ranking,
# edge and torch-op suites; then the ranking benches under rocprofv3 (split
# tile 32x32x16 vs 16x16x32, alternated) and pRotatE with library / device sin
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05c"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_edge_gpu.py tests/test_rank_parity_gpu.py tests/test_torch_ops_gpu.py \
  -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider --durations=10 > "$O/gpu_tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_rank.py --models pRotatE -d 500 --gamma 6 --reps 3 > "$O/bench_rank_protate.jsonl" 2> "$O/bench_rank.err" || exit $?
timeout -k 10 300 python -u tools/bench_rank.py --models pRotatE -d 500 --gamma 6 --reps 3 --rank-trig device > "$O/bench_rank_protate_device.jsonl" 2>> "$O/bench_rank.err" || exit $?
timeout -k 10 300 python -u tools/bench_rank.py --shape fb15k --models RotatE TransE -d 1000 --gamma 24 --reps 3 > "$O/bench_rank_fb15k.jsonl" 2>> "$O/bench_rank.err" || exit $?
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for p in auto mfma16; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_${p}_$k" -o run -- \
      python3 "$ROOT/tools/bench_rank.py" --models DistMult ComplEx --reps 5 --path $p > "$O/bench_rank_${p}_$k.jsonl" 2> "$O/prof_${p}_$k.err" || exit $?
  done
done
