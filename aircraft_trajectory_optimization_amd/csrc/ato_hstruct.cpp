// ato_hstruct.cpp -- host-only part of libato.so: Hessian structure analysis and colouring
// (HessLayout::build, ato_hessian.hpp). Compiled with the host C++ compiler.
#define ATO_HESS_ANALYSIS_IMPL
#include "ato_hessian.hpp"
