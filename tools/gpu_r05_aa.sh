# round 5: pRotatE's interval screen bounded around the device sinf (no fp64
# sin): the sinf self-test, the rank parity / edge suites, and the pRotatE
# evaluation (library sin) under rocprofv3
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05aa"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_edge_gpu.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider --durations=5 > "$O/gpu_tests.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_prot" -o run -- \
  python3 "$ROOT/tools/bench_rank.py" --models pRotatE -d 500 --gamma 6 --reps 3 > "$O/bench_rank_protate.jsonl" 2> "$O/bench_rank.err" || exit $?
