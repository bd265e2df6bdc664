# round 4: split tile with the next slab's DMA issued after the fragment reads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rank_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04p_rank.log 2>&1 || exit $?
MODELS="DistMult ComplEx" bash tools/ab_rank.sh "KGE_XTILE_TQ=2" "KGE_XTILE_TQ=2" > gpurun_out/r04p_ab.txt 2>&1 || exit $?
TAG=tileA4 COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" bash tools/pmc_rank.sh > gpurun_out/r04p_tileA.txt 2>&1 || exit $?
