#!/bin/bash
# A/B of the ranking tile under rocprofv3 kernel stats: one bench_rank run per
# env-variant string, e.g.  tools/ab_rank.sh "KGE_XTILE_TQ=2" "KGE_XTILE_TQ=1"
# Prints each variant's counting-tile min / max / mean launch time (µs).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i + 1))
  OUT="$ROOT/gpurun_out/abr_$i"
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/tools/bench_rank.py" --models ${MODELS:-DistMult} --reps 3 > "$OUT.jsonl" 2> "$OUT.err" || { tail -5 "$OUT.err"; exit 1; }
  python3 - "$OUT" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")):
    if "k_rank_mfma_x<false" in r["Name"] or "k_rank_mfma_xp" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], "min", round(float(r["MinNs"]) / 1e3, 1), "max", round(float(r["MaxNs"]) / 1e3, 1),
              "mean", round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
