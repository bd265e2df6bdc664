# round 4: the filter index looked up on the device (KGE_RANK_FILTER_TABLE): ranks, whole-pass time
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04u_rank.log 2>&1 || exit $?
for k in 1 2; do
  for v in 1 0; do
    KGE_RANK_FILTER_TABLE=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stage-timer > gpurun_out/r04u_b_${v}_$k.json 2>> gpurun_out/r04u_bench.err || exit $?
  done
done
