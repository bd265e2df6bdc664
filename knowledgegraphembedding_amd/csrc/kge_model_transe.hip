// Instantiates the model-templated kernels (kge_kernels.inc) for TRANSE.
#include "kge_kernels.inc"
KGE_INSTANTIATE_MODEL(kge::TRANSE, transe)
