# round 5: the cross-CU entity-pass probe (validated gradient, CU scaling, chunked pipeline)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05e"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 300 python -u tools/cu_split_probe.py > "$O/cu_split_probe.json" 2> "$O/cu_split_probe.err" || exit $?
