// Instantiates the model-templated kernels (kge_kernels.inc) for PROTATE.
#include "kge_kernels.inc"
KGE_INSTANTIATE_MODEL(kge::PROTATE, protate)
