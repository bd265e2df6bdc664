# round 4: single-workgroup CSR scan against rocPRIM's: 200-step windows and the step's kernel trace
set -o pipefail
mkdir -p gpurun_out
PMC=0 STEPS=30 bash tools/profile.sh > gpurun_out/r04q_profile.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank > gpurun_out/r04q_b1_$k.json 2>> gpurun_out/r04q_bench.err || exit $?
  KGE_CSR_ROCPRIM=1 timeout -k 10 200 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank > gpurun_out/r04q_b0_$k.json 2>> gpurun_out/r04q_bench.err || exit $?
done
