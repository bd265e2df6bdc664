# round 4: where the split ranking tile's cycles go (SQ wave-state counters, two passes)
set -o pipefail
mkdir -p gpurun_out
TAG=tileA COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" bash tools/pmc_rank.sh > gpurun_out/r04i_tileA.txt 2>&1 || exit $?
TAG=tileB COUNTERS="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA" bash tools/pmc_rank.sh > gpurun_out/r04i_tileB.txt 2>&1 || exit $?
