# round 5: counters of the RotatE register tile at the FB15k shape (is it VALU-issue bound?) — two SQ passes
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
X="--shape fb15k -d 1000 --gamma 24"
TAG=rotA MODELS=RotatE EXTRA="$X" COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  bash tools/pmc_rank.sh > gpurun_out/r05af_rotA.txt 2>&1 || exit $?
TAG=rotB MODELS=RotatE EXTRA="$X" COUNTERS="SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  bash tools/pmc_rank.sh > gpurun_out/r05af_rotB.txt 2>&1 || exit $?
