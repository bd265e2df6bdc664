#!/bin/bash
# rocprofv3 passes over bench.py: kernel trace + stats, then one PMC pass per
# counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
STEPS=${STEPS:-20}
BARGS="$ROOT/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-rank"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/trace.err"; exit $rc; }
if [ "${PMC:-1}" = "1" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/pmc_$C" -o run -- python3 $BARGS > "$OUT/bench_$C.json" 2> "$OUT/pmc_$C.err"
    rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/pmc_$C.err"; exit $rc; }
  done
fi
if [ "${PMC:-1}" = "1" ]; then
  python3 "$ROOT/tools/pmc_traffic.py" "$OUT" --kernel k_row -o "$OUT/pmc_traffic.json" > /dev/null &&
  python3 "$ROOT/tools/pmc_traffic.py" "$OUT" --kernel k_entity_sl -o "$OUT/pmc_traffic_entity.json" > /dev/null
fi
find "$OUT" -name "*.csv" | head -20
