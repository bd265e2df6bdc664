# round 4: ranking tile A/B (128- vs 256-candidate split-bf16 tiles, lo·lo dropped), the early-step trace, buckets A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "bucket or column_slices" > gpurun_out/r04_parity_b.log 2>&1 || exit $?
timeout -k 10 100 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rank > gpurun_out/r04b_bench_bk1.json 2> gpurun_out/r04b_bench.err || exit $?
KGE_ENT_BUCKETS=0 timeout -k 10 100 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rank > gpurun_out/r04b_bench_bk0.json 2>> gpurun_out/r04b_bench.err || exit $?
timeout -k 10 100 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rank > gpurun_out/r04b_bench_bk1b.json 2>> gpurun_out/r04b_bench.err || exit $?
KGE_ENT_BUCKETS=0 timeout -k 10 100 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rank > gpurun_out/r04b_bench_bk0b.json 2>> gpurun_out/r04b_bench.err || exit $?
timeout -k 10 120 python -u tools/hump_trace.py --bursts 0:150,1000:60,50:60,5000:60 > gpurun_out/r04b_hump.jsonl 2> gpurun_out/r04b_hump.err || exit $?
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_rank_wm.log 2>&1 || exit $?
MODELS="DistMult ComplEx" bash tools/ab_rank.sh "KGE_XTILE_WM=2" "KGE_XTILE_WM=4" "KGE_XTILE_WM=4 KGE_XTILE_LOLO=0" "KGE_XTILE_WM=2 KGE_XTILE_LOLO=0" "KGE_XTILE_WM=2" "KGE_XTILE_WM=4" > gpurun_out/r04_ab_wm.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_rank.py --models pRotatE --reps 2 --rank-trig reference > gpurun_out/r04_rank_protate_host.jsonl 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_rank.py --models pRotatE --reps 2 --rank-trig device >> gpurun_out/r04_rank_protate_host.jsonl 2>&1 || exit $?
