# round 4: the pure-stream early-step test, the rank tests with lo·lo dropped, a long buckets A/B, the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/dbg/stream_hump > gpurun_out/r04c_stream_hump.jsonl 2> gpurun_out/r04c_stream_hump.err || exit $?
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c_rank.log 2>&1 || exit $?
for k in 1 2 3; do
  KGE_ENT_BUCKETS=1 timeout -k 10 100 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank >> gpurun_out/r04c_ab_buckets.jsonl 2>> gpurun_out/r04c_bench.err || exit $?
  KGE_ENT_BUCKETS=0 timeout -k 10 100 python -u bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-rank >> gpurun_out/r04c_ab_csr.jsonl 2>> gpurun_out/r04c_bench.err || exit $?
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04c_bench_default.json 2>> gpurun_out/r04c_bench.err || exit $?
timeout -k 10 200 python -u tools/bench_rank.py --models pRotatE --reps 2 --rank-trig reference > gpurun_out/r04c_rank_protate_host.jsonl 2>&1 || exit $?
