# round 4 final tree: the whole GPU suite (verbose, heartbeat), smoke(), the default bench line and the driver's short window, the kernel-trace profile
set -o pipefail
mkdir -p gpurun_out
( while true; do date >> gpurun_out/r04z_heartbeat.txt; sleep 30; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider --durations=10 > gpurun_out/r04z_gpu_tests.log 2>&1
rc=$?
kill $HB
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04z_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r04z_bench_default.json 2> gpurun_out/r04z_bench.err || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04z_bench_20.json 2>> gpurun_out/r04z_bench.err || exit $?
PMC=0 bash tools/profile.sh > gpurun_out/r04z_profile.log 2>&1 || exit $?
