# round 5: split-bf16 tile with s_setprio(1) around each slab's MFMA block
# (KGE_XTILE_PRIO, temporary diagnostic build) against the plain tile,
# alternated on one box under rocprofv3
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05i"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for run in 1 2; do
  for v in 0 1; do
    KGE_XTILE_PRIO=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_prio${v}_$run" -o run -- \
      python3 "$ROOT/tools/bench_rank.py" --models DistMult ComplEx --reps 5 > "$O/bench_prio${v}_$run.jsonl" 2> "$O/err_prio${v}_$run.txt" || exit $?
  done
done
