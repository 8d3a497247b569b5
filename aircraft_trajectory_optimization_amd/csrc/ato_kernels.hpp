// ato_kernels.hpp -- batched NLP evaluation kernels for gfx950 (templates).
//
// Work decomposition ("SIMT over the batch"): every instance of a batch shares the
// problem structure, so a wave holds 64 INSTANCES of the same collocation node. Every
// lane runs identical control flow (no divergence); with the interleaved batch layout
// ([element][instance]) each Jacobian entry a wave writes is one 512-byte contiguous
// store (8 B x 64 lanes), and every decision-variable read is a coalesced 512-byte load.
// The node-uniform problem data (coefficients, Darboux frame of the node, segment
// offsets) is wave-uniform and comes through the scalar path.
//
//   grid.x = ceil(B / 64) instance chunks, grid.y = work units (ProbD::units, built by
//   ato_layout.hpp): the tail (gates, closure, f), the two ODE row groups of every
//   collocation node, the s-dot / dU / regularity rows of every node, the continuity rows
//   of every interval (which also write the interval's cost partial). k_cost_reduce then
//   sums the partials into f in a fixed order.
#pragma once
#include <hip/hip_runtime.h>
#include "ato_layout.hpp"

namespace ato {

template <class T, bool WJ, bool WG>
struct DevSink {
    T* J;
    T* g;
    long je, ge;
    long e, r;
    __device__ __forceinline__ void begin(int row0, int nnz0) {
        r = (long)row0 * ge;
        e = (long)nnz0 * je;
    }
    __device__ __forceinline__ void jac(int, T v) {
        if (WJ) J[e] = v;
        e += je;
    }
    __device__ __forceinline__ void row(T gv, double, double) {
        if (WG) g[r] = gv;
        r += ge;
    }
};

template <class T>
struct DevW {
    const T* __restrict__ w;
    long ws;
    __device__ __forceinline__ T operator()(int col) const { return w[(long)col * ws]; }
};

constexpr int WAVE = 64;

template <class M, class T, bool WJ, bool WG, bool WF>
__global__ __launch_bounds__(WAVE) void k_eval(ProbD p, int B, int layout, const T* __restrict__ w,
                                               T* __restrict__ g, T* __restrict__ J,
                                               T* __restrict__ gf, T* __restrict__ fpart) {
    const int b = blockIdx.x * WAVE + threadIdx.x;
    if (b >= B) return;
    const int32_t* ut = p.units + 4 * blockIdx.y;      // wave-uniform: scalar loads
    long st;
    const T* wb;
    T *gb = nullptr, *Jb = nullptr, *gfb = nullptr;
    if (layout == ATO_LAYOUT_INTERLEAVED) {
        st = B;
        wb = w + b;
        if (WG) gb = g + b;
        if (WJ) Jb = J + b;
        if (WF) gfb = gf + b;
    } else {
        st = 1;
        wb = w + (long)b * p.nw;
        if (WG) gb = g + (long)b * p.ng;
        if (WJ) Jb = J + (long)b * p.nnz;
        if (WF) gfb = gf + (long)b * p.nw;
    }
    const DevW<T> W{wb, st};
    DevSink<T, WJ, WG> s{Jb, gb, st, st, 0, 0};
    const GradOut<T> go{gfb, st, WF ? fpart + b : nullptr, B};
    run_unit<M, T, WJ || WG, WF>(p, ut[0], ut[1], ut[2], W, s, go);
}

// f[b] = sum_n fpart[n][b]  (fixed order, loads issued in batches)
template <class T>
__global__ __launch_bounds__(256) void k_cost_reduce(int N, int B, const T* __restrict__ fpart,
                                                    T* __restrict__ f) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    f[b] = reduce_cost(fpart + b, (long)B, N);
}

// Host-side launcher, explicitly instantiated per model in ato_inst.hip (one translation unit
// per model variant so the library builds in parallel).
// ev (optional): events recorded before and after k_eval (ev[2] == end as well)
template <class M, class T>
hipError_t launch_eval(const ProbD& p, int B, int layout, const T* w, T* g, T* J, T* gf, T* f, T* fpart,
                       hipStream_t st, hipEvent_t* ev);

#ifdef ATO_DEFINE_LAUNCHERS
template <class M, class T>
hipError_t launch_eval(const ProbD& p, int B, int layout, const T* w, T* g, T* J, T* gf, T* f, T* fpart,
                       hipStream_t st, hipEvent_t* ev) {
    const dim3 block(WAVE);
    if (ev) (void)hipEventRecord(ev[0], st);
    const dim3 grid((B + WAVE - 1) / WAVE, p.n_units);
    const bool wj = J != nullptr, wg = g != nullptr, wf = gf != nullptr;
    auto go = [&]<bool WJ, bool WG, bool WF>() {
        hipLaunchKernelGGL((k_eval<M, T, WJ, WG, WF>), grid, block, 0, st, p, B, layout, w, g, J, gf, fpart);
    };
    if (wj && wg && wf) go.template operator()<true, true, true>();
    else if (wj && wg) go.template operator()<true, true, false>();
    else if (wg && wf) go.template operator()<false, true, true>();
    else if (wg) go.template operator()<false, true, false>();
    else if (wj && wf) go.template operator()<true, false, true>();
    else if (wj) go.template operator()<true, false, false>();
    else if (wf) go.template operator()<false, false, true>();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[1], st);
    if (wf) {
        hipLaunchKernelGGL((k_cost_reduce<T>), dim3((B + 255) / 256), dim3(256), 0, st, p.N, B, (const T*)fpart, f);
        e = hipGetLastError();
    }
    if (ev) (void)hipEventRecord(ev[2], st);
    return e;
}
#endif

}  // namespace ato
