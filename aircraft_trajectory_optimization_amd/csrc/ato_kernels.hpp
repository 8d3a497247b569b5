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
#include <vector>
#include <type_traits>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include "ato_layout.hpp"
#include "ato_hessian.hpp"

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
    __device__ __forceinline__ void skip() { e += je; }
    __device__ __forceinline__ void row_skip() { r += ge; }
    __device__ __forceinline__ void finish() {}
};

// Paired Jacobian writer (interleaved layout, even B). Lane l holds instance
// 2 (l mod 32) + (l >= 32) of its 64-instance chunk, so lanes l and l + 32 hold adjacent
// instances. Two consecutive entries (e, e+1) are exchanged with v_permlane32_swap (lanes
// 32-63 of the first value trade with lanes 0-31 of the second): afterwards lanes 0-31 hold
// entry e of instances (2l, 2l+1) and lanes 32-63 entry e+1 of the same instance pairs, and
// one 16-byte store per lane (8 bytes in fp32) writes both entries: half the store
// instructions of one store per entry, same bytes (cdna_hip_programming.md T21).
template <class T>
__device__ __forceinline__ void swap_halves(T& a, T& b);

template <>
__device__ __forceinline__ void swap_halves<double>(double& a, double& b) {
    uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
    auto lo = __builtin_amdgcn_permlane32_swap(ua.x, ub.x, false, false);
    auto hi = __builtin_amdgcn_permlane32_swap(ua.y, ub.y, false, false);
    ua.x = lo[0];
    ub.x = lo[1];
    ua.y = hi[0];
    ub.y = hi[1];
    a = __builtin_bit_cast(double, ua);
    b = __builtin_bit_cast(double, ub);
}

template <>
__device__ __forceinline__ void swap_halves<float>(float& a, float& b) {
    auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                              false, false);
    a = __builtin_bit_cast(float, (unsigned)r[0]);
    b = __builtin_bit_cast(float, (unsigned)r[1]);
}

template <class T>
struct Pair2 { T x, y; };

#ifdef ATO_EVAL_NT       // DIAGNOSTIC (tools/diag/kkt_variants.py): streaming (nontemporal) J / g stores
template <class T>
__device__ __forceinline__ void st_pair(char* p, T a, T b) {
    typedef T v2 __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(v2{a, b}, reinterpret_cast<v2*>(p));
}
template <class T>
__device__ __forceinline__ void st_one(char* p, T a) { __builtin_nontemporal_store(a, reinterpret_cast<T*>(p)); }
#else
template <class T>
__device__ __forceinline__ void st_pair(char* p, T a, T b) { *reinterpret_cast<Pair2<T>*>(p) = Pair2<T>{a, b}; }
template <class T>
__device__ __forceinline__ void st_one(char* p, T a) { *reinterpret_cast<T*>(p) = a; }
#endif

template <class T, bool WJ, bool WG, bool FULL>
struct DevSinkPaired {
    const char* Jc;     // (char*) (J + chunk base): uniform
    const char* gc;     // (char*) (g + chunk base): uniform
    char* Jr;           // byte address of entry e's 64-instance row: uniform
    char* gr;           // byte address of row r's 64-instance row: uniform
    long Bb;            // entry stride in bytes (B * sizeof(T))
    uint32_t pair_off;  // this lane's byte offset in a pair store: (l >= 32 ? B : 0) + 2 (l mod 32) elements
    uint32_t self_off;  // this lane's own instance byte offset inside the chunk
    bool pvalid, svalid;
    T pend;
    bool odd;
    __device__ __forceinline__ void flush() {
        if (WJ && odd && (FULL || svalid)) st_one(Jr - Bb + self_off, pend);
        odd = false;
    }
    __device__ __forceinline__ void begin(int row0, int nnz0) {
        flush();
        Jr = const_cast<char*>(Jc) + (long)nnz0 * Bb;
        gr = const_cast<char*>(gc) + (long)row0 * Bb;
    }
    __device__ __forceinline__ void finish() { flush(); }
    __device__ __forceinline__ void jac(int, T v) {
        if (WJ) {
            if (!odd) {
                pend = v;
                odd = true;
            } else {
                T a = pend, b2 = v;
                swap_halves(a, b2);
                if (FULL || pvalid) st_pair(Jr - Bb + pair_off, a, b2);
                odd = false;
            }
        }
        Jr += Bb;
    }
    __device__ __forceinline__ void row(T gv, double, double) {
        if (WG && (FULL || svalid)) st_one(gr + self_off, gv);
        gr += Bb;
    }
    // an entry another work unit writes: the pending entry (if any) is stored alone
    __device__ __forceinline__ void skip() {
        flush();
        Jr += Bb;
    }
    __device__ __forceinline__ void row_skip() { gr += Bb; }
};

// fp32 quad writer (interleaved layout, B % 64 == 0). Lane l holds instance 4 (l mod 16) + l / 16
// of its 64-instance chunk, so the four 16-lane rows of the wave hold four consecutive instances.
// Four consecutive entries e .. e+3 are transposed across the rows (v_permlane32_swap, then
// v_permlane16_swap): row m then holds entry e+m of instances 4j .. 4j+3 in lane j + 16 m, and one
// 16-byte store per lane writes four entries of all 64 instances -- half the store instructions of
// the paired writer, which in fp32 stores only 8 bytes per lane. Entries left over at a segment end
// are stored one per instruction.
// DIAGNOSTIC, rejected (tools/r03h.sh, profiles/r03/eval_ab_r03h/): fig-8 fp32 B = 8192 681 vs 638 us with
// the paired writer, racetrack fp32 B = 512 39.0 vs 32.7 us -- the two permlane stages cost more than
// the store instructions they save. Build with -DATO_EVAL_F32_QUAD=1 to select it.
#ifndef ATO_EVAL_F32_QUAD
#define ATO_EVAL_F32_QUAD 0
#endif
__device__ __forceinline__ void swap_rows16(float& a, float& b) {
    auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                              false, false);
    a = __builtin_bit_cast(float, (unsigned)r[0]);
    b = __builtin_bit_cast(float, (unsigned)r[1]);
}

__device__ __forceinline__ void st_quad(char* p, float a, float b, float c, float d) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<v4*>(p) = v4{a, b, c, d};
}

template <bool WJ, bool WG>
struct DevSinkQuad {
    const char* Jc;     // (char*) (J + chunk base): uniform
    const char* gc;     // (char*) (g + chunk base): uniform
    char* Jr;           // byte address of the next entry's 64-instance row: uniform
    char* gr;           // byte address of the next row's 64-instance row: uniform
    long Bb;            // entry stride in bytes (B * 4)
    long quad_off;      // this lane's byte offset in a quad store: (l / 16) B + 16 (l mod 16) bytes
    uint32_t self_off;  // this lane's own instance byte offset inside the chunk
    float p0, p1, p2;   // pending entries (shifted in from p2)
    int n;              // number pending (wave-uniform)
    __device__ __forceinline__ void flush() {
        if (WJ) {
            if (n >= 1) st_one(Jr - Bb + self_off, p2);
            if (n >= 2) st_one(Jr - 2 * Bb + self_off, p1);
            if (n >= 3) st_one(Jr - 3 * Bb + self_off, p0);
        }
        n = 0;
    }
    __device__ __forceinline__ void begin(int row0, int nnz0) {
        flush();
        Jr = const_cast<char*>(Jc) + (long)nnz0 * Bb;
        gr = const_cast<char*>(gc) + (long)row0 * Bb;
    }
    __device__ __forceinline__ void finish() { flush(); }
    __device__ __forceinline__ void jac(int, float v) {
        if (WJ) {
            if (n < 3) {
                p0 = p1;
                p1 = p2;
                p2 = v;
                ++n;
            } else {
                float a = p0, b = p1, c = p2, d = v;     // entries e .. e+3 of this lane's instance
                swap_halves(a, c);
                swap_halves(b, d);
                swap_rows16(a, b);
                swap_rows16(c, d);
                st_quad(Jr - 3 * Bb + quad_off, a, b, c, d);
                n = 0;
            }
        }
        Jr += Bb;
    }
    __device__ __forceinline__ void row(float gv, double, double) {
        if (WG) st_one(gr + self_off, gv);
        gr += Bb;
    }
    __device__ __forceinline__ void skip() {
        flush();
        Jr += Bb;
    }
    __device__ __forceinline__ void row_skip() { gr += Bb; }
};

// decision-vector reads for the paired kernel: uniform row base + 32-bit lane byte offset
template <class T>
struct DevWPaired {
    const char* w0;     // (char*) (w + chunk base)
    long Bb;
    uint32_t off;       // this lane's (clamped) instance byte offset
    const double* pb;   // this lane's column of the per-instance constants (ProbD::isph), or NULL
    long ps;
    __device__ __forceinline__ T operator()(int col) const {
        return *reinterpret_cast<const T*>(w0 + (long)col * Bb + off);
    }
    __device__ __forceinline__ double par(long i) const { return pb[i * ps]; }
};

template <class T>
struct DevW {
    const T* __restrict__ w;
    long ws;
    const double* pb;   // this instance's column of the per-instance constants, or NULL
    long ps;
    __device__ __forceinline__ T operator()(int col) const { return w[(long)col * ws]; }
    __device__ __forceinline__ double par(long i) const { return pb[i * ps]; }
};

constexpr int WAVE = 64;

template <class M, class T, int KS, bool WJ, bool WG, bool WF, int UMASK>
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
    const DevW<T> W{wb, st, p.isph ? p.isph + b : nullptr, (long)p.isph_stride};
    DevSink<T, WJ, WG> s{Jb, gb, st, st, 0, 0};
    const GradOut<T> go{gfb, st, WF ? fpart + b : nullptr, B};
    run_unit<M, T, KS, WJ || WG, WF, UMASK>(p, ut[0], ut[1], ut[2], W, s, go);
}

// One work unit of the paired / quad kernels: the gradient pass (grad f, cost partials) and the row
// pass (g, J; whole wave). The gradient pass runs FIRST: its loads would otherwise queue behind the
// row pass's ~100 stores (vmcnt counts loads and stores in order, so waiting for a load waits for
// every store issued before it): B = 4096 527.5 -> 482 us, B = 512 48.2 -> 47.7 us (tools/r03h.sh;
// ATO_EVAL_GRAD_FIRST=0 restores rows first). Rejected diagnostic: ATO_EVAL_LIN_KS=K1 (node /
// interval units with a compile-time node count, so their loads hoist ahead of the stores): 218 us
// at B = 512, the hoisted loads' registers and code size cost far more.
#ifndef ATO_EVAL_GRAD_FIRST
#define ATO_EVAL_GRAD_FIRST 1
#endif
#ifndef ATO_EVAL_LIN_KS
#define ATO_EVAL_LIN_KS 0
#endif
template <class M, class T, int KS, bool ROWS, bool GRAD, int UMASK, class W, class S, class GO>
__device__ __forceinline__ void eval_unit(const ProbD& p, const int32_t* ut, const W& w, S& s, const GO& go) {
    const int kind = ut[0], n = ut[1], k = ut[2];
    auto run = [&]<bool R, bool G>() {
        if constexpr (ATO_EVAL_LIN_KS > 0 && KS == 0) {
            if (p.K1 == ATO_EVAL_LIN_KS && (kind == UNIT_NODE || kind == UNIT_INTERVAL)) {
                run_unit<M, T, ATO_EVAL_LIN_KS, R, G, UMASK & UMASK_LIN>(p, kind, n, k, w, s, go);
                return;
            }
        }
        run_unit<M, T, KS, R, G, UMASK>(p, kind, n, k, w, s, go);
    };
    if (ATO_EVAL_GRAD_FIRST && GRAD) run.template operator()<false, true>();
    if (ROWS) run.template operator()<true, false>();     // whole wave
    if (!ATO_EVAL_GRAD_FIRST && GRAD) run.template operator()<false, true>();
}

// Interleaved layout, even B: every lane stays active (permlane swaps need the whole wave);
// lanes past the end of the batch compute on the last instance and store nothing.
#ifdef ATO_EVAL_WPE      // DIAGNOSTIC (tools/diag/kkt_variants.py): force an occupancy target
#define ATO_EVAL_ATTR __attribute__((amdgpu_waves_per_eu(ATO_EVAL_WPE, ATO_EVAL_WPE)))
#else
#define ATO_EVAL_ATTR
#endif
// TILED: grid (tile, units, tiles) of launch_eval's instance tiles (a separate instantiation, so that
// the untiled kernel's code -- and its floating-point contraction -- is not touched by the tiling)
template <class M, class T, int KS, bool WJ, bool WG, bool WF, bool FULL, int UMASK, bool TILED = false>
__global__ __launch_bounds__(WAVE) ATO_EVAL_ATTR void k_eval_paired(ProbD p, int B, int unit0, const T* __restrict__ w,
                                                      T* __restrict__ g, T* __restrict__ J,
                                                      T* __restrict__ gf, T* __restrict__ fpart) {
    constexpr bool QUAD = FULL && ATO_EVAL_F32_QUAD && std::is_same_v<T, float>;
    const int l = threadIdx.x;
    const int chunk = TILED ? (blockIdx.z * gridDim.x + blockIdx.x) * WAVE : blockIdx.x * WAVE;
    if (TILED && chunk >= B) return;                                   // past the end of the last tile
    // instance of this lane inside the chunk
    const int own = QUAD ? 4 * (l & 15) + (l >> 4) : 2 * (l & 31) + (l >> 5);
    const int b = chunk + own;
    const int bl = (FULL || b < B) ? b : B - 1;     // clamped instance for loads
    const int32_t* ut = p.units + 4 * (unit0 + blockIdx.y);   // wave-uniform: scalar loads
    const long Bb = (long)B * sizeof(T);
    const DevWPaired<T> W{reinterpret_cast<const char*>(w + chunk), Bb, (uint32_t)((bl - chunk) * sizeof(T)),
                          p.isph ? p.isph + bl : nullptr, (long)p.isph_stride};
    const GradOut<T> go{WF ? gf + bl : nullptr, (long)B, WF ? fpart + bl : nullptr, B};
    if constexpr (QUAD) {
        DevSinkQuad<WJ, WG> s;
        s.Jc = reinterpret_cast<const char*>(J + chunk);
        s.gc = reinterpret_cast<const char*>(g + chunk);
        s.Jr = nullptr;
        s.gr = nullptr;
        s.Bb = Bb;
        s.quad_off = (long)(l >> 4) * Bb + 16 * (l & 15);
        s.self_off = (uint32_t)(own * sizeof(T));
        s.p0 = s.p1 = s.p2 = 0.0f;
        s.n = 0;
        eval_unit<M, T, KS, WJ || WG, WF, UMASK>(p, ut, W, s, go);
    } else {
        DevSinkPaired<T, WJ, WG, FULL> s;
        s.Jc = reinterpret_cast<const char*>(J + chunk);
        s.gc = reinterpret_cast<const char*>(g + chunk);
        s.Jr = nullptr;
        s.gr = nullptr;
        s.Bb = Bb;
        s.pair_off = (uint32_t)(((l >= 32 ? (long)B : 0L) + 2 * (l & 31)) * sizeof(T));
        s.self_off = (uint32_t)(own * sizeof(T));
        s.pvalid = chunk + 2 * (l & 31) < B;
        s.svalid = b < B;
        s.pend = T(0);
        s.odd = false;
        eval_unit<M, T, KS, WJ || WG, WF && FULL, UMASK>(p, ut, W, s, go);
        if (WF && !FULL && b < B) run_unit<M, T, KS, false, true, UMASK>(p, ut[0], ut[1], ut[2], W, s, go);
    }
}

// f[b] = sum_n fpart[n][b]  (fixed order, loads issued in batches)
template <class T>
__global__ __launch_bounds__(256) void k_cost_reduce(int N, int B, const T* __restrict__ fpart,
                                                    T* __restrict__ f) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    f[b] = reduce_cost(fpart + b, (long)B, N);
}

// ------------------------------------------------------------------ Hessian of the Lagrangian
// Tangents of the Jacobian entries of a seeded pass (see ato_hessian.hpp); g rows are ignored.
template <class T>
struct DevTangentSink {
    T* J;
    long je, e;
    __device__ __forceinline__ void begin(int, int nnz0) { e = (long)nnz0 * je; }
    __device__ __forceinline__ void jac(int, const Dual<T, 1>& v) {
        J[e] = v.d[0];
        e += je;
    }
    __device__ __forceinline__ void row(const Dual<T, 1>&, double, double) {}
    __device__ __forceinline__ void skip() { e += je; }
    __device__ __forceinline__ void row_skip() {}
    __device__ __forceinline__ void finish() {}
};

// Masked pass (ATO_HESS_MASK=1): only the entries that the colour changes are stored
// (HessLayout::amask, this colour's row); the masked take lists read no others, and the rest of the
// tangents are exact zeros. Same H, 22 % less time at B = 512 -- but the conditional store changes
// how the compiler contracts the tangent arithmetic into FMAs, so H rounds differently from the
// default pass (Hessian).
template <class T>
struct DevTangentSinkMasked {
    T* J;
    long je, e;
    const uint32_t* mask;
    int ei;                                   // entry index (wave-uniform)
    __device__ __forceinline__ void begin(int, int nnz0) {
        e = (long)nnz0 * je;
        ei = nnz0;
    }
    __device__ __forceinline__ void jac(int, const Dual<T, 1>& v) {
        if (mask[ei >> 5] >> (ei & 31) & 1u) J[e] = v.d[0];
        e += je;
        ++ei;
    }
    __device__ __forceinline__ void row(const Dual<T, 1>&, double, double) {}
    __device__ __forceinline__ void skip() {
        e += je;
        ++ei;
    }
    __device__ __forceinline__ void row_skip() {}
    __device__ __forceinline__ void finish() {}
};

// seeded passes for colours c0 + z (z = blockIdx.z): dJ = d J / d eps, dgf = d grad f / d eps along v_c,
// colour z's tangents at dJ + z sJ, dgf + z sG (outputs interleaved [entry][B]; w in either layout)
template <class M, int UMASK, bool MASKED = false>
__global__ __launch_bounds__(WAVE) void k_hess_dual(ProbD p, int B, int layout, const double* __restrict__ w,
                                                   const int32_t* __restrict__ color, int c0,
                                                   const uint32_t* __restrict__ amask, int mask_words,
                                                   double* __restrict__ dJ, double* __restrict__ dgf, long sJ,
                                                   long sG) {
    const int b = blockIdx.x * WAVE + threadIdx.x;
    if (b >= B) return;
    const int c = c0 + (int)blockIdx.z;
    dJ += (long)blockIdx.z * sJ;
    dgf += (long)blockIdx.z * sG;
    const int32_t* ut = p.units + 4 * blockIdx.y;
    const bool il = layout == ATO_LAYOUT_INTERLEAVED;
    const ColorW<double, DevW<double>> W{DevW<double>{il ? w + b : w + (long)b * p.nw, il ? (long)B : 1L,
                                                      p.isph ? p.isph + b : nullptr, (long)p.isph_stride},
                                         color, c};
    const TangentGrad<double> go{dgf + b, (long)B};
    if constexpr (MASKED) {
        DevTangentSinkMasked<double> s{dJ + b, (long)B, 0, amask + (long)c * mask_words, 0};
        run_unit<M, Dual<double, 1>, 0, true, true, UMASK>(p, ut[0], ut[1], ut[2], W, s, go);
    } else {
        DevTangentSink<double> s{dJ + b, (long)B, 0};
        run_unit<M, Dual<double, 1>, 0, true, true, UMASK>(p, ut[0], ut[1], ut[2], W, s, go);
    }
}

// Hessian entries recovered from colours c0 .. c1 - 1: one wave = one take for 64 instances; the take's
// colour from the take offsets (a template only so that every translation unit may instantiate it)
template <int UNUSED = 0>
__global__ __launch_bounds__(WAVE) void k_hess_take(int B, int layout, int ng, int nnzh, int t0, int c0, int c1,
                                                   const int32_t* __restrict__ take_off,
                                                   const int32_t* __restrict__ take_e,
                                                   const int32_t* __restrict__ take_r,
                                                   const int32_t* __restrict__ tk_ptr,
                                                   const int32_t* __restrict__ tk_ent,
                                                   const int32_t* __restrict__ tk_row,
                                                   const double* __restrict__ lam, const double* __restrict__ sigma,
                                                   const double* __restrict__ dJ, const double* __restrict__ dgf,
                                                   long sJ, long sG, double* __restrict__ H) {
    const int b = blockIdx.x * WAVE + threadIdx.x;
    if (b >= B) return;
    const int t = t0 + blockIdx.y;
    int c = c0;
    while (c + 1 < c1 && take_off[c + 1] <= t) ++c;          // (uniform across the wave)
    dJ += (long)(c - c0) * sJ;
    dgf += (long)(c - c0) * sG;
    const int e = take_e[t], r = take_r[t];
    const bool il = layout == ATO_LAYOUT_INTERLEAVED;
    const double* lb = il ? lam + b : lam + (long)b * ng;
    const long ls = il ? (long)B : 1L;
    const double v = hess_take(tk_ptr, tk_ent, tk_row, t, r, sigma[b], lb, ls, dJ + b, (long)B, dgf + b, (long)B);
    if (il) H[(long)e * B + b] = v;
    else H[(long)b * nnzh + e] = v;
}

// device copies of the HessLayout tables
struct HessDev {
    const int32_t *color, *take_e, *take_r, *tk_ptr, *tk_ent, *tk_row;   // take lists (masked or full)
    const uint32_t* amask;          // [n_colors][mask_words]; NULL: the full (default) pass
    int mask_words;
    const int32_t* take_off_host;   // host array [n_colors + 1]
    int n_colors, nnzh;
    const int32_t* take_off;        // device copy
    int group;                      // colours per launch (their scratch side by side)
};

template <class M>
hipError_t launch_hess(const ProbD& p, const HessDev& hd, int B, int layout, const double* w, const double* lam,
                       const double* sigma, double* H, double* dJ, double* dgf, hipStream_t st);

// Host-side launcher, explicitly instantiated per model in ato_inst.hip (one translation unit
// per model variant so the library builds in parallel).
// ev (optional): events recorded before / after the g, J kernels and after the cost reduction
// tile > 0: instance-tiled workgroup order -- grid (tile, units, tiles), so the dispatcher (x fastest,
// z slowest) runs tile 64-instance chunks through every unit before the next tile starts
template <class M, class T>
hipError_t launch_eval(const ProbD& p, int B, int layout, const T* w, T* g, T* J, T* gf, T* f, T* fpart,
                       hipStream_t st, hipEvent_t* ev, int tile = 0);

#ifdef ATO_DEFINE_LAUNCHERS
template <class M, class T>
hipError_t launch_eval(const ProbD& p, int B, int layout, const T* w, T* g, T* J, T* gf, T* f, T* fpart,
                       hipStream_t st, hipEvent_t* ev, int tile) {
    const dim3 block(WAVE);
    const int chunks = (B + WAVE - 1) / WAVE;
    const bool wj = J != nullptr, wg = g != nullptr, wf = gf != nullptr;
    // Paired 16-byte stores need the interleaved layout and whole 64-instance chunks.
    // (Measured and rejected: separate kernels per unit class on fork / join side streams --
    // the cross-stream waits cost more than the per-class register allocation gained at
    // B = 512, and nothing at B = 4096; compile-time K everywhere -- the hoisted loads cut
    // occupancy to one wave per SIMD.)
    const bool paired = layout == ATO_LAYOUT_INTERLEAVED && (B % WAVE) == 0 && wg;
    // timing (ev != nullptr): the evaluation kernel is launched with start / stop events that the
    // runtime stamps at the kernel's own start and end (hipExtLaunchKernel), i.e. its execution
    // time as a kernel trace reports it, without the dispatch gaps of separately recorded events
    hipEvent_t e0 = ev ? ev[0] : nullptr, e1 = ev ? ev[1] : nullptr;
    // Collocation and RK4 problems get separate instantiations so neither pays the other's
    // register allocation (the RK4 dual-number step vs the collocation ODE units).
    auto launch = [&]<int UM>() {
        const dim3 grid(chunks, p.n_units);
        if (paired) {
            if (tile > 0 && chunks > tile && wj && wg) {     // instance tiles (the J-producing passes)
                const dim3 tgrid(tile, p.n_units, (chunks + tile - 1) / tile);
                if (wf)
                    hipExtLaunchKernelGGL((k_eval_paired<M, T, 0, true, true, true, true, UM, true>), tgrid, block, 0, st, e0, e1, 0, p, B, 0, w, g, J, gf, fpart);
                else
                    hipExtLaunchKernelGGL((k_eval_paired<M, T, 0, true, true, false, true, UM, true>), tgrid, block, 0, st, e0, e1, 0, p, B, 0, w, g, J, gf, fpart);
                return;
            }
            if (wj && wg && wf)
                hipExtLaunchKernelGGL((k_eval_paired<M, T, 0, true, true, true, true, UM>), grid, block, 0, st, e0, e1, 0, p, B, 0, w, g, J, gf, fpart);
            else if (wj && wg)
                hipExtLaunchKernelGGL((k_eval_paired<M, T, 0, true, true, false, true, UM>), grid, block, 0, st, e0, e1, 0, p, B, 0, w, g, J, gf, fpart);
            else if (wg && wf)
                hipExtLaunchKernelGGL((k_eval_paired<M, T, 0, false, true, true, true, UM>), grid, block, 0, st, e0, e1, 0, p, B, 0, w, g, J, gf, fpart);
            else
                hipExtLaunchKernelGGL((k_eval_paired<M, T, 0, false, true, false, true, UM>), grid, block, 0, st, e0, e1, 0, p, B, 0, w, g, J, gf, fpart);
            return;
        }
        auto go = [&]<bool WJ, bool WG, bool WF>() {
            hipExtLaunchKernelGGL((k_eval<M, T, 0, WJ, WG, WF, UM>), grid, block, 0, st, e0, e1, 0, p, B, layout, w, g, J, gf, fpart);
        };
        if (wj && wg && wf) go.template operator()<true, true, true>();
        else if (wj && wg) go.template operator()<true, true, false>();
        else if (wg && wf) go.template operator()<false, true, true>();
        else if (wg) go.template operator()<false, true, false>();
        else if (wj && wf) go.template operator()<true, false, true>();
        else if (wj) go.template operator()<true, false, false>();
        else if (wf) go.template operator()<false, false, true>();
    };
    if (p.trans == ATO_TRANS_RK4) launch.template operator()<UMASK_RK4>();
    else launch.template operator()<UMASK_COLLOC>();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (wf) {
        hipExtLaunchKernelGGL((k_cost_reduce<T>), dim3((B + 255) / 256), dim3(256), 0, st, nullptr,
                              ev ? ev[2] : nullptr, 0, p.N, B, (const T*)fpart, f);
        e = hipGetLastError();
    } else if (ev) {
        (void)hipEventRecord(ev[2], st);
    }
    return e;
}

template <class M>
hipError_t launch_hess(const ProbD& p, const HessDev& hd, int B, int layout, const double* w, const double* lam,
                       const double* sigma, double* H, double* dJ, double* dgf, hipStream_t st) {
    const int chunks = (B + WAVE - 1) / WAVE;
    const long sJ = (long)p.nnz * B, sG = (long)p.nw * B;
    const int G = hd.group > 0 ? hd.group : 1;
    for (int c0 = 0; c0 < hd.n_colors; c0 += G) {
        const int c1 = c0 + G < hd.n_colors ? c0 + G : hd.n_colors;
        {
            const dim3 grid(chunks, p.n_units, c1 - c0);
            const uint32_t* am = hd.amask;
            if (p.trans == ATO_TRANS_RK4) {
                if (am) hipLaunchKernelGGL((k_hess_dual<M, UMASK_RK4, true>), grid, dim3(WAVE), 0, st, p, B, layout, w, hd.color, c0, am, hd.mask_words, dJ, dgf, sJ, sG);
                else hipLaunchKernelGGL((k_hess_dual<M, UMASK_RK4>), grid, dim3(WAVE), 0, st, p, B, layout, w, hd.color, c0, am, hd.mask_words, dJ, dgf, sJ, sG);
            } else {
                if (am) hipLaunchKernelGGL((k_hess_dual<M, UMASK_COLLOC, true>), grid, dim3(WAVE), 0, st, p, B, layout, w, hd.color, c0, am, hd.mask_words, dJ, dgf, sJ, sG);
                else hipLaunchKernelGGL((k_hess_dual<M, UMASK_COLLOC>), grid, dim3(WAVE), 0, st, p, B, layout, w, hd.color, c0, am, hd.mask_words, dJ, dgf, sJ, sG);
            }
        }
        const int t0 = hd.take_off_host[c0], nt = hd.take_off_host[c1] - t0;
        if (nt > 0)
            hipLaunchKernelGGL(k_hess_take<0>, dim3(chunks, nt), dim3(WAVE), 0, st, B, layout, p.ng, hd.nnzh, t0, c0,
                               c1, hd.take_off, hd.take_e, hd.take_r, hd.tk_ptr, hd.tk_ent, hd.tk_row, lam, sigma,
                               (const double*)dJ, (const double*)dgf, sJ, sG, H);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
#endif

}  // namespace ato
