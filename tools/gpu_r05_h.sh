# round 5: entity gradient pass timed repeated / after the row pass / after a cache flush
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05h"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 300 python -u tools/entity_gather_probe.py > "$O/entity_gather_probe.json" 2> "$O/probe.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 "$ROOT/tools/entity_gather_probe.py" --reps 10 > "$O/probe_under_prof.json" 2> "$O/prof.err" || exit $?
