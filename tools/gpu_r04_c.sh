# round 4: the persistent ranking tile A/B, the pure-stream early-step test, the rank tests with lo·lo dropped, a long buckets A/B, the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/dbg/stream_hump > gpurun_out/r04c_stream_hump.jsonl 2> gpurun_out/r04c_stream_hump.err || exit $?
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c_rank.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "bucket or column_slices or fused_adam" > gpurun_out/r04c_parity_ent.log 2>&1 || exit $?
MODELS="DistMult ComplEx" bash tools/ab_rank.sh "KGE_XTILE_PERSIST=0" "KGE_XTILE_PERSIST=1" "KGE_XTILE_PERSIST=0" "KGE_XTILE_PERSIST=1" > gpurun_out/r04c_ab_persist.txt 2>&1 || exit $?
bash tools/ab_entity.sh KGE_ENT_VARIANT=0 KGE_ENT_VARIANT=1 KGE_ENT_VARIANT=5 KGE_ENT_VARIANT=2 KGE_ENT_VARIANT=4 KGE_ENT_VARIANT=0 KGE_ENT_VARIANT=1 KGE_ENT_VARIANT=5 > gpurun_out/r04c_ab_entity.txt 2>&1 || exit $?
for k in 1 2 3; do
  KGE_ENT_BUCKETS=1 timeout -k 10 100 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank >> gpurun_out/r04c_ab_buckets.jsonl 2>> gpurun_out/r04c_bench.err || exit $?
  KGE_ENT_BUCKETS=0 timeout -k 10 100 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank >> gpurun_out/r04c_ab_csr.jsonl 2>> gpurun_out/r04c_bench.err || exit $?
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04c_bench_default.json 2>> gpurun_out/r04c_bench.err || exit $?
timeout -k 10 200 python -u tools/bench_rank.py --models pRotatE --reps 2 --rank-trig reference > gpurun_out/r04c_rank_protate_host.jsonl 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/r04c_pmc_list.txt" 2>&1 || true
