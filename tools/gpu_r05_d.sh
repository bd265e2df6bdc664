# round 5: the GPU suite from the config-5 tests on (the rest passed in r05d's
# first call), smoke, the cross-CU entity-pass probe, the bench line
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05d"
mkdir -p "$O"
cd "$ROOT"
( while true; do date >> "$O/heartbeat2.txt"; sleep 30; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest tests/test_partition_gpu.py tests/test_rank_parity_gpu.py tests/test_rccl_gpu.py \
  tests/test_run_gpu.py tests/test_sampler.py tests/test_ship_gpu.py tests/test_torch_ops_gpu.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations=15 > "$O/gpu_tests2.log" 2>&1
rc=$?
kill $HB
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python -u tools/cu_split_probe.py > "$O/cu_split_probe.json" 2> "$O/cu_split_probe.err" || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || exit $?
