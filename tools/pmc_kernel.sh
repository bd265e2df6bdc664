#!/bin/bash
# One rocprofv3 PMC pass per counter group over a short bench run, for A/B of a
# kernel's stall profile.  Usage: TAG=name COUNTERS="A B C" [ENVS="K=V ..."] tools/pmc_kernel.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for kv in ${ENVS:-}; do export "$kv"; done
timeout -k 10 300 rocprofv3 --pmc $COUNTERS --kernel-trace --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --steps 12 --warmup 2 --no-cpu-baseline --no-rank --no-stage-timer > "$OUT/bench.json" 2> "$OUT/err.log"
rc=$?; [ $rc -ne 0 ] && { tail -20 "$OUT/err.log"; exit $rc; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "k_entity" in k or "k_row<" in k:
        print(k[:50], {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
