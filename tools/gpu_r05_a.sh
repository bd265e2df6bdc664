# round 5: first box — the bench line with the distance-model ranking section,
# and kernel-trace summaries of the register-tile ranking (RotatE / TransE at the
# FB15k shape, pRotatE at the wn18rr shape with the library sin)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out/r05a"
O="$ROOT/gpurun_out/r05a"
cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$O/bench_default.json" 2> "$O/bench.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_fb15k" -o run -- \
  python3 "$ROOT/tools/bench_rank.py" --shape fb15k --models RotatE TransE -d 1000 --gamma 24 --reps 3 \
  > "$O/bench_rank_fb15k.jsonl" 2> "$O/prof_fb15k.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_wn18rr" -o run -- \
  python3 "$ROOT/tools/bench_rank.py" --models pRotatE -d 500 --gamma 6 --reps 3 \
  > "$O/bench_rank_protate.jsonl" 2> "$O/prof_wn18rr.err" || exit $?
