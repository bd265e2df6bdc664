# round 5: counters of the pRotatE and TransE register tiles (wn18rr / FB15k shapes) (is it VALU-issue bound?) — two SQ passes
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
X="--shape fb15k -d 1000 --gamma 24"
TAG=protA MODELS=pRotatE EXTRA="--shape wn18rr -d 500 --gamma 6" COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  bash tools/pmc_rank.sh > gpurun_out/r05ag_protA.txt 2>&1 || exit $?
TAG=traA MODELS=TransE EXTRA="$X" COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  bash tools/pmc_rank.sh > gpurun_out/r05ag_traA.txt 2>&1 || exit $?
