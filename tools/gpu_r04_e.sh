# round 4: the bucket path with the unrolled sort and the queued relation scan against the CSR; bucket tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "bucket or column_slices or fused_adam or relation" > gpurun_out/r04e_parity.log 2>&1 || exit $?
bash tools/ab_entity.sh KGE_ENT_BUCKETS=0 KGE_ENT_BUCKETS=1 KGE_ENT_BUCKETS=0 KGE_ENT_BUCKETS=1 > gpurun_out/r04e_ab_buckets3.txt 2>&1 || exit $?
timeout -k 10 120 ./tools/dbg/stream_hump > gpurun_out/r04e_stream_hump.jsonl 2> gpurun_out/r04e_stream_hump.err || exit $?
