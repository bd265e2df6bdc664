// Instantiates the model-templated kernels (kge_kernels.inc) for COMPLEX.
#include "kge_kernels.inc"
KGE_INSTANTIATE_MODEL(kge::COMPLEX, complex)
