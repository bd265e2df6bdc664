# round 4: the 256-candidate split tile with a deeper LDS ring (5 slabs in flight) against the default
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q --timeout 300 --timeout-method thread -k "split_bf16 or full_size" > gpurun_out/r04h_rank.log 2>&1 || exit $?
MODELS="DistMult ComplEx" bash tools/ab_rank.sh "KGE_XTILE_WM=2" "KGE_XTILE_WM=4 KGE_XTILE_NST=6" "KGE_XTILE_WM=4 KGE_XTILE_NST=5" "KGE_XTILE_WM=2" "KGE_XTILE_WM=4 KGE_XTILE_NST=6" > gpurun_out/r04h_ab_nst.txt 2>&1 || exit $?
