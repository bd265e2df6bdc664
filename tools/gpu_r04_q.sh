# round 4: single-workgroup CSR scan: training parity suites, then the step's kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not rank" > gpurun_out/r04q_tests.log 2>&1 || exit $?
PMC=0 STEPS=30 bash tools/profile.sh > gpurun_out/r04q_profile.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank > gpurun_out/r04q_bench200.json 2> gpurun_out/r04q_bench.err || exit $?
KGE_CSR_ROCPRIM=1 timeout -k 10 200 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank > gpurun_out/r04q_bench200_rocprim.json 2>> gpurun_out/r04q_bench.err || exit $?
timeout -k 10 200 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank > gpurun_out/r04q_bench200_b.json 2>> gpurun_out/r04q_bench.err || exit $?
