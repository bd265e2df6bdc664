# round 4: the countries run.py test alone, verbose, with the single-workgroup scan and with rocPRIM's
set -o pipefail
mkdir -p gpurun_out
( while true; do date >> gpurun_out/r04r_heartbeat.txt; sleep 30; done ) &
HB=$!
timeout -k 10 400 python -u -m pytest tests/test_run_gpu.py -x -v -s --timeout 380 --timeout-method thread -p no:cacheprovider -k "countries" --durations=0 > gpurun_out/r04r_countries.log 2>&1
rc=$?
KGE_CSR_ROCPRIM=1 timeout -k 10 400 python -u -m pytest tests/test_run_gpu.py -x -v -s --timeout 380 --timeout-method thread -p no:cacheprovider -k "countries" --durations=0 > gpurun_out/r04r_countries_rocprim.log 2>&1
rc2=$?
kill $HB
echo "rc=$rc rc2=$rc2"
exit $rc
