# round 4: wave states and LDS bank conflicts of the training kernels
set -o pipefail
mkdir -p gpurun_out
TAG=trainA COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" bash tools/pmc_kernel.sh > gpurun_out/r04k_trainA.txt 2>&1 || exit $?
TAG=trainB COUNTERS="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" bash tools/pmc_kernel.sh > gpurun_out/r04k_trainB.txt 2>&1 || exit $?
