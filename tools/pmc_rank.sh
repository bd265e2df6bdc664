#!/bin/bash
# PMC pass over tools/bench_rank.py (one counter group), for the ranking kernels.
# Usage: TAG=name COUNTERS="A B C" [MODELS="DistMult"] [EXTRA="--shape fb15k -d 1000 --gamma 24"] tools/pmc_rank.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmcr_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $COUNTERS --kernel-trace --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/tools/bench_rank.py" --models ${MODELS:-DistMult} --reps 1 ${EXTRA:-} > "$OUT/out.jsonl" 2> "$OUT/err.log"
rc=$?; [ $rc -ne 0 ] && { tail -20 "$OUT/err.log"; exit $rc; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "k_rank" in k:
        print(k[:60], {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
