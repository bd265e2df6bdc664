// Instantiates the model-templated kernels (kge_kernels.inc) for DISTMULT.
#include "kge_kernels.inc"
KGE_INSTANTIATE_MODEL(kge::DISTMULT, distmult)
