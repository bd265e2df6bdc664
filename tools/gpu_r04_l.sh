# round 4: the 64x32-per-wave split tile (3 workgroups per CU) against the default after the bank swap
set -o pipefail
mkdir -p gpurun_out
MODELS="DistMult ComplEx" bash tools/ab_rank.sh "KGE_XTILE_TQ=2" "KGE_XTILE_TQ=1" "KGE_XTILE_TQ=2" "KGE_XTILE_TQ=1" > gpurun_out/r04l_ab_tq.txt 2>&1 || exit $?
