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
//   grid.x = ceil(B / 64) instance chunks, grid.y = P node units (+1 tail unit)
//   node unit (n, k): collocation rows of (n, k), its regularity / stage / sphere row,
//                     the continuity + fixed-s rows of interval n (k == 0), cost gradient
//   tail unit:        equal-h rows, gates, loop closure
//   k_cost_reduce:    f = sum_n partial(n)   (deterministic order)
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
    const int unit = blockIdx.y;
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

    if (unit < p.P) {
        const int n = unit / p.K1, k = unit - n * p.K1;
        const int32_t* sg = p.seg + (long)unit * NSEG * 2;
        if (WJ || WG) {
            for (int kind = 0; kind < NSEG; ++kind) {
                const int r0 = sg[2 * kind];
                if (r0 < 0) continue;
                s.begin(r0, sg[2 * kind + 1]);
                run_node_seg<M, T>(p, kind, n, k, W, s);
            }
        }
        if (WF) {
            constexpr int NZ = M::NZ, NU = M::NU;
            const Cols<M> c{p.N, p.K1};
            T gu[NU], gdu[NU];
            stage_cost<M, T>(p, n, k, W, gu, gdu);
            const T h = W(n);
            const T hB = h * T(p.Bq[k]);
            const long base = (long)c.node(n, k) * st;
#pragma unroll
            for (int i = 0; i < NZ; ++i) gfb[base + i * st] = T(0);
#pragma unroll
            for (int i = 0; i < NU; ++i) gfb[base + (NZ + i) * st] = hB * gu[i];
#pragma unroll
            for (int i = 0; i < NU; ++i) gfb[base + (NZ + NU + i) * st] = hB * gdu[i];
            if (k == 0) {
                T acc = T(0);
                for (int j = 0; j < p.K1; ++j)
                    acc += T(p.Bq[j]) * stage_cost<M, T>(p, n, j, W, (T*)nullptr, (T*)nullptr);
                gfb[(long)n * st] = acc;
                fpart[(long)n * B + b] = h * acc;
            }
        }
    } else if (WJ || WG) {
        for (int t = 0; t < p.n_tail; ++t) {
            const int32_t* tl = p.tail + 4 * t;
            s.begin(tl[2], tl[3]);
            run_tail_seg<M, T>(p, tl[0], tl[1], W, s);
        }
    }
}

template <class T>
__global__ __launch_bounds__(256) void k_cost_reduce(int N, int B, const T* __restrict__ fpart,
                                                    T* __restrict__ f) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    T acc = T(0);
    for (int n = 0; n < N; ++n) acc += fpart[(long)n * B + b];
    f[b] = acc;
}


// Host-side launcher, explicitly instantiated per model in ato_inst.hip (one translation unit
// per model variant so the library builds in parallel).
// ev (optional): three events recorded before k_eval, between the kernels and after k_cost_reduce
template <class M, class T>
hipError_t launch_eval(const ProbD& p, int B, int layout, const T* w, T* g, T* J, T* gf, T* fpart, T* f,
                       hipStream_t st, hipEvent_t* ev);

#ifdef ATO_DEFINE_LAUNCHERS
template <class M, class T>
hipError_t launch_eval(const ProbD& p, int B, int layout, const T* w, T* g, T* J, T* gf, T* fpart, T* f,
                       hipStream_t st, hipEvent_t* ev) {
    const dim3 block(WAVE);
    if (ev) (void)hipEventRecord(ev[0], st);
    const dim3 grid((B + WAVE - 1) / WAVE, p.P + (p.n_tail > 0 ? 1 : 0));
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
