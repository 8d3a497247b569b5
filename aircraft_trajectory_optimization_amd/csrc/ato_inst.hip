// ato_inst.hip -- explicit instantiation of the evaluation launchers for ONE model variant.
// Compiled once per variant with -DATO_INST=<0..11> (see build_native.py).
#define ATO_DEFINE_LAUNCHERS
#include "ato_kernels.hpp"

#ifndef ATO_INST
#error "compile with -DATO_INST=<model index>"
#endif

namespace ato {
#if ATO_INST == 0
using Model = DroneModel<ESP, GLOBAL>;
#elif ATO_INST == 1
using Model = DroneModel<ESP, PARAM_GR>;
#elif ATO_INST == 2
using Model = DroneModel<ESP, PARAM_REL>;
#elif ATO_INST == 3
using Model = DroneModel<YPR, GLOBAL>;
#elif ATO_INST == 4
using Model = DroneModel<YPR, PARAM_GR>;
#elif ATO_INST == 5
using Model = DroneModel<YPR, PARAM_REL>;
#elif ATO_INST == 6
using Model = PointModel<GLOBAL>;
#elif ATO_INST == 7
using Model = PointModel<PARAM_GR>;
#elif ATO_INST == 8
using Model = PointModel<PARAM_REL>;
#elif ATO_INST == 9
using Model = DroneModel<DCM, GLOBAL>;
#elif ATO_INST == 10
using Model = DroneModel<DCM, PARAM_GR>;
#elif ATO_INST == 11
using Model = DroneModel<DCM, PARAM_REL>;
#endif
template hipError_t launch_eval<Model, double>(const ProbD&, int, int, const double*, double*, double*, double*,
                                              double*, double*, hipStream_t, hipEvent_t*, int);
template hipError_t launch_hess<Model>(const ProbD&, const HessDev&, int, int, const double*, const double*,
                                       const double*, double*, double*, double*, hipStream_t);
template hipError_t launch_eval<Model, float>(const ProbD&, int, int, const float*, float*, float*, float*,
                                             float*, float*, hipStream_t, hipEvent_t*, int);
}  // namespace ato
