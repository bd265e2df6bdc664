# round 4: the training-side GPU suite, verbose, with a heartbeat (a hung test is reported by pytest's own timeout)
set -o pipefail
mkdir -p gpurun_out
( while true; do date >> gpurun_out/r04s_heartbeat.txt; sleep 30; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "not rank" --durations=15 > gpurun_out/r04s_tests.log 2>&1
rc=$?
kill $HB
echo "rc=$rc"
exit $rc
