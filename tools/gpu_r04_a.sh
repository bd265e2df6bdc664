set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py tests/test_capi.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r04_rccl.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "bucket or column_slices or fused_epilogue or finalize" > gpurun_out/r04_parity.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_rank_parity_gpu.py tests/test_torch_ops_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04_rank.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rank > gpurun_out/r04_bench_buckets.json 2> gpurun_out/r04_bench_buckets.err || exit $?
KGE_ENT_BUCKETS=0 timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rank > gpurun_out/r04_bench_csr.json 2>> gpurun_out/r04_bench_buckets.err || exit $?
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rank > gpurun_out/r04_bench_buckets2.json 2>> gpurun_out/r04_bench_buckets.err || exit $?
timeout -k 10 400 python -u -m pytest tests/test_dp_config4_gpu.py tests/test_partition_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04_dp.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/hump_trace.py --steps 150 --warmup 5 > gpurun_out/r04_hump.jsonl 2> gpurun_out/r04_hump.err || exit $?
