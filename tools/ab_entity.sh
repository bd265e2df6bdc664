#!/bin/bash
# A/B of the entity pass under rocprofv3 kernel stats: one bench.py run (the
# training step only) per env-variant string, e.g.
#   tools/ab_entity.sh "KGE_ENT_VARIANT=0" "KGE_ENT_VARIANT=1"
# Prints each variant's k_entity_sl and k_row mean / min launch time (µs) and
# the bench line's scored-triples rate.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i + 1))
  OUT="$ROOT/gpurun_out/abe_$i"
  env $v timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/bench.py" --steps ${STEPS:-100} --warmup ${WARMUP:-60} --no-cpu-baseline --no-rank \
    > "$OUT.json" 2> "$OUT.err" || { tail -5 "$OUT.err"; exit 1; }
  python3 - "$OUT" "$v" <<'PY'
import csv, json, sys
line = [l for l in open(sys.argv[1] + ".json") if l.startswith("{")][-1]
rate = json.loads(line)["value"] / 1e6
for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")):
    if "k_entity_sl" in r["Name"] or "k_row<" in r["Name"]:
        print(sys.argv[2], r["Name"][:32], "calls", r["Calls"], "mean", round(float(r["AverageNs"]) / 1e3, 1),
              "min", round(float(r["MinNs"]) / 1e3, 1), "us", "rate_M", round(rate, 1))
PY
done
