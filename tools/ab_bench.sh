#!/bin/bash
# A/B: run bench.py once per env-variant string given as arguments, e.g.
#   tools/ab_bench.sh "KGE_ENT_SLICES=4" "KGE_ENT_SLICES=8" "KGE_X=1 -- --hidden-dim 1024"
# Each line of gpurun_out/ab.jsonl = {"env": ..., bench JSON}.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-200}
for v in "$@"; do
  # "K=V ... -- --bench-arg ...": environment, then extra bench.py arguments
  envs=${v%% -- *}; extra=""
  [ "$envs" != "$v" ] && extra=${v#* -- }
  env $envs timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-rank ${BENCH_ARGS:-} $extra > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant '$v' rc=$rc"; tail -20 gpurun_out/ab_one.err; exit $rc; fi
  python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
d = {"env": sys.argv[1], **d}
open("gpurun_out/ab.jsonl", "a").write(json.dumps(d) + "\n")
print(sys.argv[1], round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms", {k: round(v, 4) for k, v in d.get("stage_ms", {}).items()})
PY
done
