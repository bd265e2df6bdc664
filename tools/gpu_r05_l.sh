# round 5 validation, part 2: smoke, the default bench line (with the CPU
# baseline), the driver's 20/5 window, then tools/profile.sh (kernel trace +
# FETCH_SIZE / WRITE_SIZE passes) for the roofline traffic of this tree
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05l"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_driver_window.json" 2> "$O/bench_driver_window.err" || exit $?
bash tools/profile.sh > "$O/profile.log" 2>&1 || exit $?
