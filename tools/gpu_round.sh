#!/bin/bash
# GPU box routine: parity tests, then a short bench. Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest $TESTS -m gpu -q -p no:cacheprovider -rs ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --steps ${STEPS:-30} --warmup 3 --cpu-budget ${CPU_BUDGET:-8} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?
  echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
  exit $rc
fi
