# round 4 final tree: the whole GPU suite, smoke(), the default bench line, the
# kernel-trace profile + PMC traffic of the training step, the entity pass's
# stall counters for the default pass and the wave-specialised variant
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04d_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r04d_bench_default.json 2> gpurun_out/r04d_bench.err || exit $?
bash tools/profile.sh > gpurun_out/r04d_profile.log 2>&1 || exit $?
for V in csr ws; do
  if [ $V = csr ]; then E="KGE_ENT_BUCKETS=0"; else E="KGE_ENT_BUCKETS=1 KGE_ENT_VARIANT=5"; fi
  TAG=ent_${V}_a COUNTERS="TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" ENVS="$E" bash tools/pmc_kernel.sh > gpurun_out/r04d_pmc_${V}_a.txt 2>&1 || exit $?
  TAG=ent_${V}_f COUNTERS="FETCH_SIZE" ENVS="$E" bash tools/pmc_kernel.sh > gpurun_out/r04d_pmc_${V}_f.txt 2>&1 || exit $?
  TAG=ent_${V}_w COUNTERS="WRITE_SIZE" ENVS="$E" bash tools/pmc_kernel.sh > gpurun_out/r04d_pmc_${V}_w.txt 2>&1 || exit $?
done
