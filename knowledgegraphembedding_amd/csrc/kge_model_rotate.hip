// Instantiates the model-templated kernels (kge_kernels.inc) for ROTATE.
#include "kge_kernels.inc"
KGE_INSTANTIATE_MODEL(kge::ROTATE, rotate)
