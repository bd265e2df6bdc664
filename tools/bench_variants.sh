#!/bin/bash
# A/B step variants in one GPU session (same device, back to back).
# VARIANTS: space-separated list of "ENV=VAL,ENV=VAL" items.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
k=0
for V in ${VARIANTS}; do
  k=$((k+1))
  env $(echo "$V" | tr ',' ' ') timeout -k 10 300 python bench.py --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --no-rank ${BENCH_ARGS:-} > gpurun_out/bv_$k.json 2>gpurun_out/bv_$k.err || { tail -5 gpurun_out/bv_$k.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bv_$k.json'));print('$V', round(d['value']/1e6,1), 'M/s', {k: round(v,4) for k,v in d['stage_ms'].items()})"
done
