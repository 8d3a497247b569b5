// diag_stamps.hip -- DIAGNOSTIC ONLY (never part of libato.so): s_memtime stamps inside the
// ODE work units to see where a wave spends its time (cdna_hip_programming.md §7 In-kernel
// stamps). Built with the library objects into tools/diag/libato_diag.so by diag_stamps.py.
//   stamp 0: unit start   1: after all decision-vector loads consumed
//   2: after every store of the unit was issued   3: after s_waitcnt vmcnt(0) (stores done)
#define ATO_DEFINE_LAUNCHERS
#include "../../aircraft_trajectory_optimization_amd/csrc/ato_kernels.hpp"
#include "../../aircraft_trajectory_optimization_amd/csrc/ato_handle.hpp"
// (ato_handle.hpp includes the kernels header)

namespace {
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

using M = ato::DroneModel<ato::ESP, ato::PARAM_GR>;

template <int KIND>
__global__ __launch_bounds__(64) void k_stamped(ato::ProbD p, int B, const double* __restrict__ w,
                                               double* __restrict__ g, double* __restrict__ J,
                                               unsigned long long* __restrict__ st) {
    using namespace ato;
    const int l = threadIdx.x;
    const int chunk = blockIdx.x * 64;
    const int own = 2 * (l & 31) + (l >> 5);
    const int32_t* ut = p.units + 4 * blockIdx.y;
    const long Bb = (long)B * 8;
    const DevWPaired<double> W{reinterpret_cast<const char*>(w + chunk), Bb, (uint32_t)(own * 8)};
    DevSinkPaired<double, true, true, true> s;
    s.Jc = reinterpret_cast<const char*>(J + chunk);
    s.gc = reinterpret_cast<const char*>(g + chunk);
    s.Bb = Bb;
    s.pair_off = (uint32_t)(((l >= 32 ? (long)B : 0L) + 2 * (l & 31)) * 8);
    s.self_off = own * 8;
    s.pend = 0;
    s.odd = false;
    unsigned long long t0 = stamp();
    const int n = ut[1], k = ut[2];
    if (ut[0] != KIND) return;
    const int32_t* sg = p.seg + (long)(n * p.K1 + k) * NSEG * 2;
    const int sk = KIND == UNIT_ODE_A ? SEG_ODE_A : SEG_ODE_B;
    s.begin(sg[2 * sk], sg[2 * sk + 1]);
    // loads: h and the model inputs, consumed into a value the compiler must wait for
    const Cols<M> c{p.N, p.K1};
    double acc = W(n);
    for (int i = 0; i < M::NZ; ++i) acc += W(c.z(n, k, i));
    for (int j = 0; j < p.K1; ++j) acc += W(c.z(n, j, 0));
    asm volatile("" ::"v"(acc));
    unsigned long long t1 = stamp();
    if (KIND == UNIT_ODE_A) seg_ode<M, double, 0, 0, ode_split<M>()>(p, n, k, W, s);
    else seg_ode<M, double, 0, ode_split<M>(), M::NZ>(p, n, k, W, s);
    s.finish();
    unsigned long long t2 = stamp();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t3 = stamp();
    if (l == 0) {
        unsigned long long* o = st + ((long)blockIdx.y * gridDim.x + blockIdx.x) * 4;
        o[0] = t0;
        o[1] = t1;
        o[2] = t2;
        o[3] = t3 + (acc == 12345.678 ? 1 : 0);
    }
}
}  // namespace

extern "C" int atodiag_stamps(ato_handle* h, int B, int kind, const double* w, double* g, double* J,
                              unsigned long long* stamps, void* stream) {
    const dim3 grid((B + 63) / 64, h->pd.n_units);
    if (kind == ato::UNIT_ODE_A)
        hipLaunchKernelGGL(k_stamped<ato::UNIT_ODE_A>, grid, dim3(64), 0, (hipStream_t)stream, h->pd, B, w, g, J, stamps);
    else
        hipLaunchKernelGGL(k_stamped<ato::UNIT_ODE_B>, grid, dim3(64), 0, (hipStream_t)stream, h->pd, B, w, g, J, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
