// ato_kkt.hip -- batched multifrontal LDL^T factorisation and solve of the interior-point KKT
// system (include/ato_kkt.h). Replaces IPOPT's MUMPS / MA97 factorisation (ref:
// drone3d/raceline/base_raceline.py:752-799, the `ipopt_time` of :182-189) for a batch of
// independent instances; the plan tables (fronts, levels, extend-add maps) come from
// solver/kkt_plan.py.
//
// Factor (k_front_factor_w<T, W>): one 512-thread workgroup per (front, instance) of a level. The
// front's block (<= 32*T positions) lives in REGISTERS: thread (ti, tj) = (tid % 32, tid / 32)
// holds A[32 I + ti][32 J + tj] and A[32 I + ti][32 J + 16 + tj] for every lower tile J <= I
// (T(T+1) doubles). The original entries are assembled through a 32-row LDS strip per tile
// row; the children's contribution blocks are then added in registers (extend-add through an
// LDS position map, children in a fixed order). Own positions are eliminated by Bunch-Kaufman
// pivoting (1x1 or 2x2; candidates and the pivot search restricted to own positions): the
// pivot column(s) are copied to LDS by their owners, every wave reduces the same max /
// argmax, and every thread applies the rank-1 / rank-2 update to its tiles (tiles without
// live rows are skipped). The factor columns are written compactly (live positions only,
// physical order) into the front's slice of the instance's stream, with a pivot record and
// the inverse pivot block per step. The trailing block (the Schur complement) is the front's
// contribution block, written to HBM for the parent's launch.
//
// Solve: k_front_fwd<T> (levels upwards: L y = b and the D solve of the own positions; the
// trailing part of y is the front's contribution to its parent's right-hand side) and
// k_front_bwd<T> (levels downwards: L^T x = z; the trailing values are final already). One
// 256-thread workgroup per (front, instance): wave 0 sweeps with the front vector in
// registers (4 positions per lane), all four waves stream the factor columns through a
// two-slot LDS ring so that the sweep reads LDS only.
#include <exception>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <string>
#include <vector>
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include "../../include/ato_kkt.h"
#include "../../include/ato.h"

void ato_internal_set_error(const std::string& msg);   // ato_capi.hip: ato_last_error()

struct ato_kkt {
    int n = 0, m = 0, dim = 0, F = 0, L = 0, max_ent = 0;
    int64_t l_size = 0, cb_size = 0;
    int32_t sc_size = 0;
    std::vector<int32_t> level_ptr, level_tiles;
    int32_t *d_pos_ptr = nullptr, *d_n_own = nullptr, *d_pos_index = nullptr, *d_parent_pos = nullptr;
    int32_t *d_child_ptr = nullptr, *d_child_list = nullptr, *d_ent_ptr = nullptr, *d_ent_pos = nullptr;
    int32_t *d_ent_src = nullptr, *d_piv_off = nullptr, *d_sc_off = nullptr;
    int32_t *d_kres_ptr = nullptr, *d_kres_col = nullptr, *d_kres_src = nullptr;
    int64_t *d_l_off = nullptr, *d_cb_off = nullptr;
    int32_t* d_forder = nullptr;     // [F] fronts of every level grouped by kernel class (factor launches)
    int32_t* d_n_sad = nullptr;      // [F] saddle fronts: nS, else 0 (NULL: the plan has none)
    int32_t* d_sad_txy = nullptr;    // [F][2] saddle fronts: (tx, ty)
    double sad_tau = 0.0;            // saddle fallback on the barrier diagonal (Plan::sad_tau; ATO_KKT_SADDLE_TAU)
    // cls: kernel class; saddle segments (cls SADDLE_CLS): nsm = the k_front_saddle variant, lds its
    // shared-memory bytes, cls2 the Bunch-Kaufman class of the fallback launch
    struct Seg { int start, count, cls, nsm = 0, cls2 = 0; size_t lds = 0; };
    std::vector<char> level_sad;     // per level: holds saddle fronts
    std::vector<std::vector<Seg>> segs;   // per level: contiguous runs of d_forder of one class
    hipStream_t side = nullptr;      // second stream for the other classes of a level
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int32_t cap = 0;                 // instances with factor storage
    double* d_L = nullptr;           // [cap][l_size]
    double* d_cb = nullptr;          // [cap][cb_size] contribution blocks
    double* d_sc = nullptr;          // [cap][sc_size] solve contributions
    int2* d_piv = nullptr;           // [cap][dim] {p | type << 16, r}
    double* d_dinv = nullptr;        // [cap][dim][3]
    int2* d_sinfo = nullptr;         // [cap][F] {steps, used stream length of the front}
    int32_t* d_spec = nullptr;       // [cap][dim] second column Bunch-Kaufman took for an own position last time
    int device = 0;                  // HIP device of the handle (ato_kkt_create's current device)
};

#ifdef ATO_KKT_STAMPS
// DIAGNOSTIC build only (tools/diag/kkt_phase.py): shader-clock phase totals of the workgroup
// (front ATO_KKT_STAMP_FRONT, instance 0) of the factorisation, thread 0
#ifndef ATO_KKT_STAMP_FRONT
#define ATO_KKT_STAMP_FRONT 0
#endif
__device__ unsigned long long g_kkt_stamps[16];
#endif

namespace {

int fail(int code, const std::string& m) {
    ato_internal_set_error(m);
    return code;
}

#define KKT_HIP(call)                                                                               \
    do {                                                                                            \
        hipError_t e_ = (call);                                                                     \
        if (e_ != hipSuccess) return fail(ATO_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int FT = 512;                   // factor threads per (front, instance) (16 x 32 grid)
constexpr int ST = 128;                   // solve threads per (front, instance): two waves (256: B = 512 solve 3.02 ms, 128: 2.63 ms)
constexpr int EPT = 8;                    // entries per thread and front (<= 4096 per front)
#ifndef ATO_KKT_W_JSKIP
#define ATO_KKT_W_JSKIP 1
#endif
#ifndef ATO_KKT_S16_JSKIP
#define ATO_KKT_S16_JSKIP 0    // 1: skip the tile columns left of the pivot's tile in the leaf update. Off: the
                               // per-tile guards cost more scalar issue than the FMAs they save (B = 512
                               // factor 15.16 -> 13.74 ms with two row groups; profiles/r03/kkt_leaf16/r03z_*)
#endif
#ifndef ATO_KKT_S16_NG
#define ATO_KKT_S16_NG 2      // row groups of the 16-wide-tile Schur update (with tile guards: 2 groups 18.46 ms,
                              // 3: 18.22, 4: 18.57; without: 2: 13.74, 3: 14.07)
#endif
#ifndef ATO_KKT_PRIO
#define ATO_KKT_PRIO 0        // wave priority of the pivot search and decision (s_setprio), 0 before the Schur
                              // update: the fronts sharing a CU issue their chain ahead of another's FMAs
#endif
#define KKT_PRIO_CHAIN() do { if (ATO_KKT_PRIO) __builtin_amdgcn_s_setprio(ATO_KKT_PRIO); } while (0)
#define KKT_PRIO_UPDATE() do { if (ATO_KKT_PRIO) __builtin_amdgcn_s_setprio(0); } while (0)
#ifndef ATO_KKT_CH
#define ATO_KKT_CH 512      // 8 KB ring: B = 512 solve 3.28 -> 3.01 ms against 16 KB (64 KB: 11.1 ms); B = 1 0.37 -> 0.38 ms
#endif
constexpr int CH = ATO_KKT_CH;            // doubles per ring chunk of the solve (2 x CH x 8 B LDS ring)
constexpr int CPT = CH / ST;              // chunk doubles per thread
// a factor column (two for a 2x2 pivot: 2 x 32 T doubles) must fit in the two resident chunks
static_assert(CH >= 2 * 32 * 8, "solve ring chunk smaller than the largest column pair");
constexpr int MAX_FRONT_TILES = 9;        // fronts up to 288 positions
constexpr int MAXT = MAX_FRONT_TILES;     // strips per front in ent_ptr
constexpr double BK_ALPHA = 0.64038820320220756872767623199676;   // (1 + sqrt(17)) / 8
constexpr int SRC_SHIFT = 29;
constexpr int SAD_DONE = -1;              // sinfo.x of a saddle front factorised by k_front_saddle
constexpr int SAD_FALLBACK = -2;          // ... left to the Bunch-Kaufman launch that follows
constexpr int SADDLE_CLS = 200;           // kernel class of the saddle fronts
constexpr double SAD_PIVOT_TOL = 1e-12;   // LU pivot of J_YX against max |J_YX| (tests/kkt_emulation.py)

struct Plan {
    int n, m, dim, F;
    const int* pos_ptr;
    const int* n_own;
    const int* pos_index;
    const int* parent_pos;
    const int* child_ptr;
    const int* child_list;
    const int* ent_ptr;
    const int* ent_pos;
    const int2* ent_src;
    const long long* l_off;
    const int* piv_off;
    const long long* cb_off;
    const int* sc_off;
    const int* forder;            // factor launches: front = forder[f0 + blockIdx.x]
    const int* n_sad;             // [F] saddle fronts: nS (NULL: none)
    const int2* sad_txy;          // [F] saddle fronts: trailing rows [0, tx) coupled to X, [T - ty, T) to Y
    long long l_size, cb_size;
    int sc_size;
    int cap;                      // reserved storage slots: listed instances at or past it are skipped
    // saddle fronts fall back to Bunch-Kaufman when max |H_XX diagonal| > sad_tau max|J_YX|^2 (0: never):
    // G = -E^T H E carries the barrier diagonal (up to 1e10 near active bounds) through J^-1, where
    // Bunch-Kaufman would take those entries first as 1 x 1 pivots
    double sad_tau;
};

struct Vals {
    const double* H;
    const double* J;
    const double* dx;
    const double* dr;
    long long se, sb;
};

__device__ __forceinline__ double src_value(const Vals& v, int code, int b) {
    if (code < 0) return 0.0;
    const int kind = code >> SRC_SHIFT;
    const long long idx = code & ((1 << SRC_SHIFT) - 1);
    const double* p = kind == 0 ? v.H : kind == 1 ? v.J : kind == 2 ? v.dx : v.dr;
    if (!p) return 0.0;
    return p[idx * v.se + (long long)b * v.sb];
}

// bit blend a = m ? b : a on doubles through integer ops (a select of two array loads would be
// folded into a variable-index load and push the whole register array to scratch)
__device__ __forceinline__ double blend(double a, double b, unsigned long long m) {
    return __longlong_as_double((__double_as_longlong(a) & ~m) | (__double_as_longlong(b) & m));
}

// live-position bit mask; every word access uses a compile-time index (no scratch)
template <int NW>
struct Mask {
    unsigned long long w[NW];
    __device__ __forceinline__ bool get(int i) const {
        unsigned long long r = 0ull;
#pragma unroll
        for (int k = 0; k < NW; ++k) r |= (((i >> 6) == k) ? ~0ull : 0ull) & w[k];
        return (r >> (i & 63)) & 1ull;
    }
    __device__ __forceinline__ void clear(int i) {
#pragma unroll
        for (int k = 0; k < NW; ++k) w[k] &= ~((((i >> 6) == k) ? 1ull : 0ull) << (i & 63));
    }
    __device__ __forceinline__ int count() const {
        int c = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) c += __popcll(w[k]);
        return c;
    }
    __device__ __forceinline__ bool any_in_tile(int I) const {   // positions 32I .. 32I+31
        return ((w[I >> 1] >> ((I & 1) * 32)) & 0xffffffffull) != 0ull;
    }
    __device__ __forceinline__ void set_range(int lo, int hi) {   // [lo, hi)
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int l = min(max(lo - 64 * k, 0), 64), h = min(max(hi - 64 * k, 0), 64);
            const unsigned long long mh = h >= 64 ? ~0ull : ((1ull << h) - 1ull);
            const unsigned long long ml = l >= 64 ? ~0ull : ((1ull << l) - 1ull);
            w[k] = mh & ~ml;
        }
    }
};

#ifdef ATO_KKT_STAMPS
__device__ __forceinline__ unsigned long long kstamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define KST_DECL(on_) unsigned long long kst_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, kst_last = kstamp(); const bool kst_on = (on_);
#define KST(i) do { if (kst_on) { const unsigned long long t_ = kstamp(); kst_acc[i] += t_ - kst_last; kst_last = t_; } } while (0)
#define KST_DUMP(n_) do { if (kst_on && threadIdx.x == 0) { for (int i_ = 0; i_ < 10; ++i_) g_kkt_stamps[i_] = kst_acc[i_]; g_kkt_stamps[15] = (n_); } } while (0)
#else
#define KST_DECL(on_)
#define KST(i)
#define KST_DUMP(n_)
#endif

// LDS-only workgroup barrier: waits for this wave's LDS operations, not for its global stores
// (the factor columns written every step are read only by later launches)
__device__ __forceinline__ void lds_barrier() { __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}

// max over the 64 lanes (all lanes active), returned as a scalar: DPP within each 16-lane row,
// then the four row results by readlane
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
    v = max(v, dpp_u32<0xB1>(v));    // quad_perm [1,0,3,2]
    v = max(v, dpp_u32<0x4E>(v));    // quad_perm [2,3,0,1]
    v = max(v, dpp_u32<0x141>(v));   // row_half_mirror
    v = max(v, dpp_u32<0x140>(v));   // row_mirror
    const unsigned r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const unsigned r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return max(max(r0, r1), max(r2, r3));
}

// sum over the 64 lanes in a fixed order (deterministic), returned wave-uniform
__device__ __forceinline__ double wave_sum(double v) {
    v += dpp_f64<0xB1>(v);
    v += dpp_f64<0x4E>(v);
    v += dpp_f64<0x141>(v);
    v += dpp_f64<0x140>(v);
    return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// ordering key of |v| at position i (< 512): float magnitude with the low 9 mantissa bits
// replaced by (511 - i), so the max key is a (near-)largest entry, ties to the smallest index;
// 0 = no candidate. The pivot tests then use the exact double value at the chosen index.
__device__ __forceinline__ unsigned mag_key(double v, int i) {
    return (__float_as_uint((float)fabs(v)) & 0xFFFFFE00u) | (unsigned)(511 - i);
}

constexpr int slot(int I, int J) { return I * (I + 1) / 2 + J; }

// 1 / d by the hardware reciprocal and two Newton steps (a few ulp; four dependent ops instead of
// the ten of an IEEE division on the pivot chain). d is never 0 here: Bunch-Kaufman takes a 1x1
// pivot only with |d| >= alpha lambda > 0, and a 2x2 only with det <= (alpha^2 - 1) lambda^2 < 0.
__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    return fma(fma(-d, r, 1.0), r, r);
}

// value of position p (= lane p % 64, register p / 64) of a per-lane array, wave-uniform
template <int NQ>
__device__ __forceinline__ double lane_pick(const double (&v)[NQ], int p) {
    const int q = p >> 6;
    double x = v[0];
#pragma unroll
    for (int k = 1; k < NQ; ++k) x = blend(x, v[k], q == k ? ~0ull : 0ull);
    return readlane_f64(x, p & 63);
}

template <int NQ>
__device__ __forceinline__ void lane_set(double (&y)[NQ], int p, double v, int lane) {
#pragma unroll
    for (int k = 0; k < NQ; ++k) y[k] = blend(y[k], v, ((p & 63) == lane && (p >> 6) == k) ? ~0ull : 0ull);
}

// ------------------------------------------------------------------------------------------
// factorisation
// ------------------------------------------------------------------------------------------
// entry h of a per-thread register row, h wave-uniform (a select chain: no indexed registers)
template <int NC>
__device__ __forceinline__ double pick(const double (&v)[NC], int h) {
    double x = v[0];
#pragma unroll
    for (int q = 1; q < NC; ++q) x = blend(x, v[q], h == q ? ~0ull : 0ull);
    return x;
}

// column k of the block into c[0 .. 32T): thread (ti, tj) of a workgroup of 32 NTJ threads owns
// rows 32I+ti and the NC = 32 / NTJ columns 32J + h NTJ + tj (h < NC) of every lower tile (I, J).
// Only lower-triangle entries are read: A[i][k] for i >= k, A[k][i] for i < k. The diagonal
// tiles also carry upper copies, which round differently from the lower entries (l_i c_j
// against l_j c_i); reading only lower entries makes the factors independent of the tiling, so
// every kernel variant (32- or 16-wide tiles) produces the same factors bit for bit.
template <int T, int NC>
__device__ __forceinline__ void extract_column(const double (&a)[T * (T + 1) / 2][NC], int k, int ti, int tj,
                                               double* __restrict__ c) {
    constexpr int NTJ = 32 / NC;
    const int K = k >> 5, kk = k & 31, kt = kk % NTJ, h = kk / NTJ;
#pragma unroll
    for (int KK = 0; KK < T; ++KK) {
        if (K == KK) {
            if (tj == kt) {
#pragma unroll
                for (int I = KK; I < T; ++I)
                    if (I != KK || ti >= kk) c[32 * I + ti] = pick<NC>(a[slot(I, KK)], h);
            }
            if (ti == kk) {
#pragma unroll
                for (int J = 0; J < KK; ++J) {
#pragma unroll
                    for (int q = 0; q < NC; ++q) c[32 * J + q * NTJ + tj] = a[slot(KK, J)][q];
                }
#pragma unroll
                for (int q = 0; q < NC; ++q)
                    if (q * NTJ + tj < kk) c[32 * KK + q * NTJ + tj] = a[slot(KK, KK)][q];
            }
        }
    }
}

__global__ void k_inertia_zero(int batch, int cap, const int* __restrict__ list, int* __restrict__ inertia) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= batch) return;
    const int b = list ? list[i] : i;
    if (b < 0 || b >= cap) return;
    inertia[3 * b + 0] = 0;
    inertia[3 * b + 1] = 0;
    inertia[3 * b + 2] = 0;
}

// W: waves per SIMD the register allocation targets; FTT: threads per (front, instance) --
// 512 (16 column owners per tile row, two columns each) or, for fronts of at most two tiles,
// one wave (2 column owners, 16 columns each: no workgroup barrier is more than a wave's)
template <int T, int W, int FTT>
__global__ __launch_bounds__(FTT) __attribute__((amdgpu_waves_per_eu(W))) void k_front_factor_w(Plan P, Vals V, int f0, int batch, const int* __restrict__ list,
                                                     double* __restrict__ Lst, int2* __restrict__ piv,
                                                     double* __restrict__ dinv, int2* __restrict__ sinfo,
                                                     double* __restrict__ CB, int* __restrict__ inertia,
                                                     int* __restrict__ spec) {
    constexpr int NP = 32 * T;
    constexpr int NW = (NP + 63) / 64;
    constexpr int NQ = (NP + 63) / 64;
    constexpr int NS = T * (T + 1) / 2;
    constexpr int SR = NP + 1;                   // strip row stride (odd: conflict-free reads)
    constexpr int NTJ = FTT / 32;                // column owners per tile row
    constexpr int NC = 32 / NTJ;                 // columns per thread and tile
    static_assert(NP <= FTT, "factor-column stores: one position per thread");
    constexpr int SRW = FTT == 64 ? 16 : 32;     // assembly strip rows (one wave: half a tile row, so
                                                 // more fronts share a CU's LDS)
    extern __shared__ double smem[];
    double* strip = smem;                        // [SRW][SR]
    double* colb = strip + SRW * SR;             // [2 parity][2 (k, r)][NP]
    int* inv = reinterpret_cast<int*>(colb + 4 * NP);   // [NP] position -> child trailing index

    const int f = P.forder[f0 + blockIdx.x];
    const int bi = blockIdx.y;
    if (bi >= batch) return;
    const int b = list ? __builtin_amdgcn_readfirstlane(list[bi]) : bi;
    if (list && b >= P.cap) return;            // a listed slot past the reserved storage: nothing is touched
    if (P.n_sad && P.n_sad[f] > 0 && sinfo[(long long)b * P.F + f].x != SAD_FALLBACK) return;
    const int tid = threadIdx.x;
    const int ti = tid & 31, tj = tid >> 5;
    const int lane = tid & 63;

    const int p0 = P.pos_ptr[f];
    const int A = P.pos_ptr[f + 1] - p0;
    const int own = P.n_own[f];
    double a[NS][NC];
    double* Lb = Lst + (long long)b * P.l_size + P.l_off[f];
    int2* pv = piv + (long long)b * P.dim + P.piv_off[f];
    double* dv = dinv + ((long long)b * P.dim + P.piv_off[f]) * 3;
    int npos = 0, nneg = 0, nzero = 0;
    long long loff = 0;                          // running offset in the front's column stream
    KST_DECL(f == ATO_KKT_STAMP_FRONT && blockIdx.y == 0)

    // ---- original entries (positions and values) into registers (512 threads: all at once;
    // one wave: strip by strip from the per-strip entry ranges)
    int epos[FTT == FT ? EPT : 1];
    double eval[FTT == FT ? EPT : 1];
    if constexpr (FTT == FT) {
        const int e0 = P.ent_ptr[f * MAXT], e1 = P.ent_ptr[(f + 1) * MAXT];
#pragma unroll
        for (int q = 0; q < EPT; ++q) {
            const int e = e0 + tid + q * FT;
            epos[q] = -1;
            eval[q] = 0.0;
            if (e < e1) {
                epos[q] = P.ent_pos[e];
                const int2 sc = P.ent_src[e];
                eval[q] = src_value(V, sc.x, b) + src_value(V, sc.y, b);
            }
        }
    }
    // ---- assemble strip by strip (SRW rows of tile row I at a time)
#pragma unroll
    for (int I = 0; I < T; ++I) {
        if (32 * I < A) {
#pragma unroll
            for (int hh = 0; hh < 32 / SRW; ++hh) {
                for (int i = tid; i < SRW * SR; i += FTT) strip[i] = 0.0;
                __syncthreads();
                auto in_strip = [&](int p) { return (p >> 5) == I && ((p & 31) / SRW) == hh; };
                auto put = [&](int ep, double ev) {
                    const int pa = ep >> 16, pb = ep & 0xffff;
                    if (ep >= 0 && in_strip(pa)) strip[(pa % SRW) * SR + pb] = ev;
                    if (ep >= 0 && in_strip(pb) && (pa >> 5) == I && pa != pb) strip[(pb % SRW) * SR + pa] = ev;
                };
                if constexpr (FTT == FT) {
#pragma unroll
                    for (int q = 0; q < EPT; ++q) put(epos[q], eval[q]);
                } else {
                    for (int e = P.ent_ptr[f * MAXT + I] + tid; e < P.ent_ptr[f * MAXT + I + 1]; e += FTT) {
                        const int ep = P.ent_pos[e];
                        if (in_strip(ep >> 16) || in_strip(ep & 0xffff)) {
                            const int2 sc = P.ent_src[e];
                            put(ep, src_value(V, sc.x, b) + src_value(V, sc.y, b));
                        }
                    }
                }
                __syncthreads();
                if (ti / SRW == hh) {
#pragma unroll
                    for (int J = 0; J <= I; ++J) {
#pragma unroll
                        for (int q = 0; q < NC; ++q) a[slot(I, J)][q] = strip[(ti % SRW) * SR + 32 * J + q * NTJ + tj];
                    }
                }
                __syncthreads();
            }
        } else {
#pragma unroll
            for (int J = 0; J <= I; ++J) {
#pragma unroll
                for (int q = 0; q < NC; ++q) a[slot(I, J)][q] = 0.0;
            }
        }
    }
    // ---- extend-add of the children's contribution blocks (fixed child order: deterministic)
    for (int ci = P.child_ptr[f]; ci < P.child_ptr[f + 1]; ++ci) {
        const int c = P.child_list[ci];
        const int pc = P.pos_ptr[c], oc = P.n_own[c];
        const int tqc = P.pos_ptr[c + 1] - pc - oc;
        const int* pm = P.parent_pos + pc + oc;
        const double* cbc = CB + (long long)b * P.cb_size + P.cb_off[c];
        for (int i = tid; i < NP; i += FTT) inv[i] = -1;
        __syncthreads();
        for (int q = tid; q < tqc; q += FTT) inv[pm[q]] = q;
        __syncthreads();
        int qr[T];
#pragma unroll
        for (int I = 0; I < T; ++I) qr[I] = inv[32 * I + ti];
#pragma unroll
        for (int J = 0; J < T; ++J) {
#pragma unroll
            for (int h = 0; h < NC; ++h) {
                const int qc = inv[32 * J + h * NTJ + tj];
#pragma unroll
                for (int I = J; I < T; ++I)
                    if (qr[I] >= 0 && qc >= 0) a[slot(I, J)][h] += cbc[(long long)qr[I] * tqc + qc];
            }
        }
        __syncthreads();
    }
    // ---- restricted Bunch-Kaufman elimination of the own positions (all decisions scalar; the
    // next candidate by a find-first-set over the ballot of the lanes' live flags at the end of
    // the step, as in k_front_factor_s; tiles left of the pivot's tile are skipped in the update)
    bool lvq[NQ];                 // per lane: position lane + 64 q live
#pragma unroll
    for (int q = 0; q < NQ; ++q) lvq[q] = lane + 64 * q < A;
    bool lvt = tid < A;           // per thread: its factor-column position tid live ...
    int cit = tid;                // ... and its index among the live positions
    int kc = 0, steps = 0, par = 0, nlive = A;
    KST(0);                      // assembly
    {   // first live own position >= kc: find-first-set over the ballot of the lanes' live flags
        int nk = own;
#pragma unroll
        for (int q = NQ - 1; q >= 0; --q) {
            const int lo = kc - 64 * q, hi = own - 64 * q;
            unsigned long long m = lo <= 0 ? ~0ull : (lo >= 64 ? 0ull : (~0ull << lo));
            m &= hi >= 64 ? ~0ull : (hi <= 0 ? 0ull : ((1ull << hi) - 1ull));
            const unsigned long long w = __ballot(lvq[q]) & m;
            nk = w ? 64 * q + (int)__builtin_ctzll(w) : nk;
        }
        kc = nk;
    }
    while (kc < own) {
        const int k = kc;
        double* ck = colb + (par * 2 + 0) * NP;
        double* cr = colb + (par * 2 + 1) * NP;
        KKT_PRIO_CHAIN();
        extract_column<T, NC>(a, k, ti, tj, ck);
        lds_barrier();
        KST(1);                  // extract + barrier (waits for the slowest wave's update)
        // lambda = max_{i eligible, i != k} |A_ik| and its index r
        // every lane keeps its column values: A_kk and lambda come back by readlane, not LDS
        unsigned key = 0u;
        double cv[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = lane + 64 * q;
            cv[q] = ck[i];
            if (i < own && i != k && lvq[q]) key = max(key, mag_key(cv[q], i));
        }
        key = wave_max_u32(key);
        KST(5);                  // column read, magnitude keys, DPP max
        const int r = key ? 511 - (int)(key & 0x1FFu) : -1;
        const double akk = lane_pick<NQ>(cv, k);
        const double lam = r >= 0 ? fabs(lane_pick<NQ>(cv, r)) : 0.0;
        int type;            // 0: 1x1 at p, 1: 2x2 (k, r), 2: zero column
        double arr = 0.0;    // A_rr (when column r was extracted)
        int p = k;
        bool use_r = false;
        double cw[NQ];       // column r (when extracted), same lane layout as cv
#pragma unroll
        for (int q = 0; q < NQ; ++q) cw[q] = 0.0;
        if (r < 0 || lam == 0.0) {
            type = akk == 0.0 ? 2 : 0;
        } else if (fabs(akk) >= BK_ALPHA * lam) {
            type = 0;
        } else {
            extract_column<T, NC>(a, r, ti, tj, cr);
            lds_barrier();
            unsigned key2 = 0u;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int i = lane + 64 * q;
                cw[q] = cr[i];
                if (i < own && i != r && lvq[q]) key2 = max(key2, mag_key(cw[q], i));
            }
            key2 = wave_max_u32(key2);
            const int j2 = key2 ? 511 - (int)(key2 & 0x1FFu) : -1;
            const double sig = j2 >= 0 ? fabs(lane_pick<NQ>(cw, j2)) : 0.0;
            arr = lane_pick<NQ>(cw, r);
            if (fabs(akk) * sig >= BK_ALPHA * lam * lam) {
                type = 0;
            } else if (fabs(arr) >= BK_ALPHA * sig) {
                type = 0;
                p = r;
                use_r = true;
            } else {
                type = 1;
            }
        }
        KST(2);                  // pivot search and decision
        // ---- pivot record, inertia, factor columns, Schur update
        double i00 = 0.0, i01 = 0.0, i11 = 0.0;
        if (type == 2) {
            ++nzero;
        } else if (type == 0) {
            const double d = use_r ? arr : akk;
            i00 = rcp_nr(d);
            if (d > 0.0) ++npos; else ++nneg;
        } else {
            const double A00 = akk, A01 = lane_pick<NQ>(cv, r), A11 = arr;
            const double det = A00 * A11 - A01 * A01;
            const double rdet = rcp_nr(det);
            i00 = A11 * rdet;
            i01 = -A01 * rdet;
            i11 = A00 * rdet;
            if (det < 0.0) { ++npos; ++nneg; }
            else if (A00 + A11 > 0.0) npos += 2;
            else nneg += 2;
        }
        KST(6);                  // pivot inverse, inertia
        const int ncol = type == 1 ? 2 : 1;
        nlive -= ncol;
        {
            const int e1p = type == 1 ? k : (type == 2 ? k : p);
            const int e2p = type == 1 ? r : -1;
            lvt = lvt && tid != e1p && tid != e2p;
            cit -= (tid > e1p ? 1 : 0) + (e2p >= 0 && tid > e2p ? 1 : 0);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int i = lane + 64 * q;
                lvq[q] = lvq[q] && i != e1p && i != e2p;
            }
        }
        KST(7);                  // live-set bookkeeping
        if (tid == 0) {
            pv[steps] = make_int2((type == 1 ? k : p) | (type << 16), type == 1 ? r : -1);
            dv[3 * steps + 0] = i00;
            dv[3 * steps + 1] = i01;
            dv[3 * steps + 2] = i11;
        }
        // L's column(s) of this step from the pivot columns in LDS: row i of the first column is
        // c0[i] i00 (+ cr[i] i01 for a 2x2 pivot), of the second cr[i] i11 + c0[i] i01. Re-read
        // from LDS rather than held in registers across the decision (frees the registers for a
        // second workgroup per CU).
        const double* c0p = use_r ? cr : ck;     // column p (1x1) or k (2x2)
        if (lvt) {
            const int ci = cit;
            const double x0 = c0p[tid];
            if (type == 0) {
                Lb[loff + ci] = x0 * i00;
            } else if (type == 1) {
                const double x1 = cr[tid];
                Lb[loff + 2 * ci] = fma(x0, i00, x1 * i01);
                Lb[loff + 2 * ci + 1] = fma(x0, i01, x1 * i11);
            } else {
                Lb[loff + ci] = 0.0;
            }
        }
        loff += (long long)nlive * ncol;
        KST(3);                  // pivot inverse, record, factor-column stores
        // Schur update: one rank-1 pass (1x1 pivot) or two (2x2 pivot), A -= l c^T with c the
        // pivot column (pass 0: c0, pass 1: cr)
        const int npass = type == 0 ? 1 : type == 1 ? 2 : 0;
        KKT_PRIO_UPDATE();
        for (int pass = 0; pass < npass; ++pass) {
            const double* cc = pass == 1 ? cr : c0p;
            const double f0 = pass == 1 ? i01 : i00, f1 = pass == 1 ? i11 : i01;
            // column-tile outer loop: column tiles without a live position are skipped (a uniform branch
            // around a whole tile column; B = 512 24.8 -> 23.2 ms). Dead entries are never read again.
            double li[T];
#pragma unroll
            for (int I = 0; I < T; ++I) {
                const double x0 = c0p[32 * I + ti];
                li[I] = type == 1 ? fma(x0, f0, cr[32 * I + ti] * f1) : x0 * i00;
            }
#pragma unroll
            for (int J = 0; J < T; ++J) {
                if (!ATO_KKT_W_JSKIP || J >= (k >> 5)) {   // tiles left of the pivot's tile: eliminated positions
                    double cj[NC];
#pragma unroll
                    for (int h = 0; h < NC; ++h) cj[h] = cc[32 * J + h * NTJ + tj];
#pragma unroll
                    for (int I = J; I < T; ++I) {
#pragma unroll
                        for (int h = 0; h < NC; ++h) a[slot(I, J)][h] = fma(-li[I], cj[h], a[slot(I, J)][h]);
                    }
                }
            }
        }
        ++steps;
        par ^= 1;
        KST(4);                  // Schur update
        {   // first live own position >= kc: find-first-set over the ballot of the lanes' live flags
            int nk = own;
#pragma unroll
            for (int q = NQ - 1; q >= 0; --q) {
                const int lo = kc - 64 * q, hi = own - 64 * q;
                unsigned long long m = lo <= 0 ? ~0ull : (lo >= 64 ? 0ull : (~0ull << lo));
                m &= hi >= 64 ? ~0ull : (hi <= 0 ? 0ull : ((1ull << hi) - 1ull));
                const unsigned long long w = __ballot(lvq[q]) & m;
                nk = w ? 64 * q + (int)__builtin_ctzll(w) : nk;
            }
            kc = nk;
        }
    }
    KST_DUMP(steps);
    if (tid == 0) {
        sinfo[(long long)b * P.F + f] = make_int2(steps, (int)loff);
        atomicAdd(&inertia[3 * b + 0], npos);
        atomicAdd(&inertia[3 * b + 1], nneg);
        atomicAdd(&inertia[3 * b + 2], nzero);
    }
    // ---- trailing Schur complement -> contribution block of the parent (HBM)
    const int tq = A - own;
    if (tq > 0) {
        double* cb = CB + (long long)b * P.cb_size + P.cb_off[f];
#pragma unroll
        for (int I = 0; I < T; ++I) {
#pragma unroll
            for (int J = 0; J <= I; ++J) {
#pragma unroll
                for (int h = 0; h < NC; ++h) {
                    const int i = 32 * I + ti, j = 32 * J + h * NTJ + tj;
                    // diagonal tiles hold both (i, j) and (j, i), which differ by rounding:
                    // only the lower one writes (one writer per entry, deterministic)
                    if (i >= own && i < A && j >= own && j < A && (I != J || i >= j)) {
                        cb[(long long)(i - own) * tq + (j - own)] = a[slot(I, J)][h];
                        cb[(long long)(j - own) * tq + (i - own)] = a[slot(I, J)][h];
                    }
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// 16-wide tiles for fronts of 161-192 positions (the interval leaves, 161-182 on the racetrack):
// the same restricted Bunch-Kaufman elimination as k_front_factor_w, with thread (ti, tj) =
// (tid % 16, tid / 16) of 256 holding A[16 I + ti][16 J + tj] of every lower tile J <= I (one
// double per tile). Against six 32-wide tiles (192 positions, 21 tiles of 1024 entries) a
// 161-176-position front keeps 66 tiles of 256 entries: 21 % fewer register entries and Schur
// FMAs per step, dead tile columns are skipped at 16 positions instead of 32, and the assembly
// strip is 16 rows, so the LDS (30 KB instead of 57 KB) no longer limits a CU to two fronts.
// Operations per entry and their order are those of k_front_factor_w, and both read only the
// lower-triangle entries, so the factors are bit for bit those of k_front_factor_w.
// ------------------------------------------------------------------------------------------
template <int TT>
__device__ __forceinline__ void extract_column16(const double (&a)[TT * (TT + 1) / 2], int k, int ti, int tj,
                                                 double* __restrict__ c) {
    const int K = k >> 4, kk = k & 15;
    // one case per tile column (a switch: a branch tree instead of a compare per tile)
    auto one = [&](auto KC) {
        constexpr int KK = decltype(KC)::value;
        if (tj == kk) {
#pragma unroll
            for (int I = KK; I < TT; ++I)
                if (I != KK || ti >= kk) c[16 * I + ti] = a[slot(I, KK)];
        }
        if (ti == kk) {
#pragma unroll
            for (int J = 0; J <= KK; ++J)
                if (J != KK || tj < kk) c[16 * J + tj] = a[slot(KK, J)];
        }
    };
    static_assert(TT <= 12, "extract_column16: tile-column cases");
    switch (K) {
        case 0: one(std::integral_constant<int, 0>{}); break;
        case 1: one(std::integral_constant<int, 1>{}); break;
        case 2: one(std::integral_constant<int, 2>{}); break;
        case 3: one(std::integral_constant<int, 3>{}); break;
        case 4: one(std::integral_constant<int, 4>{}); break;
        case 5: one(std::integral_constant<int, 5>{}); break;
        case 6: if constexpr (TT > 6) one(std::integral_constant<int, 6>{}); break;
        case 7: if constexpr (TT > 7) one(std::integral_constant<int, 7>{}); break;
        case 8: if constexpr (TT > 8) one(std::integral_constant<int, 8>{}); break;
        case 9: if constexpr (TT > 9) one(std::integral_constant<int, 9>{}); break;
        case 10: if constexpr (TT > 10) one(std::integral_constant<int, 10>{}); break;
        case 11: if constexpr (TT > 11) one(std::integral_constant<int, 11>{}); break;
        default: break;
    }
}

template <int NW>
__device__ __forceinline__ bool any_in_tile16(const Mask<NW>& m, int J) {   // positions 16J .. 16J+15
    return ((m.w[J >> 2] >> ((J & 3) * 16)) & 0xffffull) != 0ull;
}

template <int TT, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void k_front_factor_s(
    Plan P, Vals V, int f0, int batch, const int* __restrict__ list, double* __restrict__ Lst,
    int2* __restrict__ piv, double* __restrict__ dinv, int2* __restrict__ sinfo, double* __restrict__ CB,
    int* __restrict__ inertia) {
    constexpr int FTT = 256;
    constexpr int NP = 16 * TT;
    static_assert(NP <= FTT, "one factor-column position per thread");
    constexpr int NW = (NP + 63) / 64;
    constexpr int NQ = NW;
    constexpr int NS = TT * (TT + 1) / 2;
    constexpr int SR = NP + 1;                   // strip row stride (odd: conflict-free reads)
    extern __shared__ double smem[];
    double* strip = smem;                        // [16][SR]
    double* colb = strip + 16 * SR;              // [2 parity][2 (k, r)][NP]
    int* inv = reinterpret_cast<int*>(colb + 4 * NP);   // [NP] position -> child trailing index

    const int f = P.forder[f0 + blockIdx.x];
    const int bi = blockIdx.y;
    if (bi >= batch) return;
    const int b = list ? __builtin_amdgcn_readfirstlane(list[bi]) : bi;
    if (list && b >= P.cap) return;            // a listed slot past the reserved storage: nothing is touched
    if (P.n_sad && P.n_sad[f] > 0 && sinfo[(long long)b * P.F + f].x != SAD_FALLBACK) return;
    const int tid = threadIdx.x;
    const int ti = tid & 15, tj = tid >> 4;
    const int lane = tid & 63;

    const int p0 = P.pos_ptr[f];
    const int A = P.pos_ptr[f + 1] - p0;
    const int own = P.n_own[f];
    double a[NS];
    double* Lb = Lst + (long long)b * P.l_size + P.l_off[f];
    int2* pv = piv + (long long)b * P.dim + P.piv_off[f];
    double* dv = dinv + ((long long)b * P.dim + P.piv_off[f]) * 3;
    int npos = 0, nneg = 0, nzero = 0;
    long long loff = 0;

    // ---- assemble 16-row strip by strip (entries of the plan's 32-row strip I / 2)
#pragma unroll
    for (int I = 0; I < TT; ++I) {
        if (16 * I < A) {
            for (int i = tid; i < 16 * SR; i += FTT) strip[i] = 0.0;
            __syncthreads();
            for (int e = P.ent_ptr[f * MAXT + (I >> 1)] + tid; e < P.ent_ptr[f * MAXT + (I >> 1) + 1]; e += FTT) {
                const int ep = P.ent_pos[e];
                const int pa = ep >> 16, pb = ep & 0xffff;
                if ((pa >> 4) == I) {
                    const int2 sc = P.ent_src[e];
                    const double ev = src_value(V, sc.x, b) + src_value(V, sc.y, b);
                    strip[(pa & 15) * SR + pb] = ev;
                    if ((pb >> 4) == I && pa != pb) strip[(pb & 15) * SR + pa] = ev;
                }
            }
            __syncthreads();
#pragma unroll
            for (int J = 0; J <= I; ++J) a[slot(I, J)] = strip[ti * SR + 16 * J + tj];
            __syncthreads();
        } else {
#pragma unroll
            for (int J = 0; J <= I; ++J) a[slot(I, J)] = 0.0;
        }
    }
    // ---- extend-add of the children's contribution blocks (fixed child order: deterministic)
    for (int ci = P.child_ptr[f]; ci < P.child_ptr[f + 1]; ++ci) {
        const int c = P.child_list[ci];
        const int pc = P.pos_ptr[c], oc = P.n_own[c];
        const int tqc = P.pos_ptr[c + 1] - pc - oc;
        const int* pm = P.parent_pos + pc + oc;
        const double* cbc = CB + (long long)b * P.cb_size + P.cb_off[c];
        for (int i = tid; i < NP; i += FTT) inv[i] = -1;
        __syncthreads();
        for (int q = tid; q < tqc; q += FTT) inv[pm[q]] = q;
        __syncthreads();
        int qr[TT];
#pragma unroll
        for (int I = 0; I < TT; ++I) qr[I] = inv[16 * I + ti];
#pragma unroll
        for (int J = 0; J < TT; ++J) {
            const int qc = inv[16 * J + tj];
#pragma unroll
            for (int I = J; I < TT; ++I)
                if (qr[I] >= 0 && qc >= 0) a[slot(I, J)] += cbc[(long long)qr[I] * tqc + qc];
        }
        __syncthreads();
    }
    // ---- restricted Bunch-Kaufman elimination of the own positions (all decisions scalar).
    // Scalar work is kept short: every wave runs it, and the CU's one scalar unit serves the
    // waves of up to three fronts (SQ counters: ~340 scalar instructions per pivot step and wave
    // against ~240 vector ones before). The next candidate is a find-first-set over the ballot of
    // the lanes' live flags, evaluated at the END of the step (with the scan at the loop head the
    // register allocator copied the whole register block on every iteration); tiles left of the
    // pivot's tile hold only eliminated positions, so the update starts there; the live count is a
    // counter.
    bool lvq[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) lvq[q] = lane + 64 * q < A;
    bool lvt = tid < A;
    int cit = tid;
    int kc = 0, steps = 0, par = 0, nlive = A;
    {   // first live own position >= kc: find-first-set over the ballot of the lanes' live flags
        int nk = own;
#pragma unroll
        for (int q = NQ - 1; q >= 0; --q) {
            const int lo = kc - 64 * q, hi = own - 64 * q;
            unsigned long long m = lo <= 0 ? ~0ull : (lo >= 64 ? 0ull : (~0ull << lo));
            m &= hi >= 64 ? ~0ull : (hi <= 0 ? 0ull : ((1ull << hi) - 1ull));
            const unsigned long long w = __ballot(lvq[q]) & m;
            nk = w ? 64 * q + (int)__builtin_ctzll(w) : nk;
        }
        kc = nk;
    }
    while (kc < own) {
        const int k = kc;
        double* ck = colb + (par * 2 + 0) * NP;
        double* cr = colb + (par * 2 + 1) * NP;
        KKT_PRIO_CHAIN();
        extract_column16<TT>(a, k, ti, tj, ck);
        lds_barrier();
        unsigned key = 0u;
        double cv[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = lane + 64 * q;
            cv[q] = ck[i];
            if (i < own && i != k && lvq[q]) key = max(key, mag_key(cv[q], i));
        }
        key = wave_max_u32(key);
        const int r = key ? 511 - (int)(key & 0x1FFu) : -1;
        const double akk = lane_pick<NQ>(cv, k);
        const double lam = r >= 0 ? fabs(lane_pick<NQ>(cv, r)) : 0.0;
        int type;            // 0: 1x1 at p, 1: 2x2 (k, r), 2: zero column
        double arr = 0.0;
        int p = k;
        bool use_r = false;
        if (r < 0 || lam == 0.0) {
            type = akk == 0.0 ? 2 : 0;
        } else if (fabs(akk) >= BK_ALPHA * lam) {
            type = 0;
        } else {
            extract_column16<TT>(a, r, ti, tj, cr);
            lds_barrier();
            unsigned key2 = 0u;
            double cw[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int i = lane + 64 * q;
                cw[q] = cr[i];
                if (i < own && i != r && lvq[q]) key2 = max(key2, mag_key(cw[q], i));
            }
            key2 = wave_max_u32(key2);
            const int j2 = key2 ? 511 - (int)(key2 & 0x1FFu) : -1;
            const double sig = j2 >= 0 ? fabs(lane_pick<NQ>(cw, j2)) : 0.0;
            arr = lane_pick<NQ>(cw, r);
            if (fabs(akk) * sig >= BK_ALPHA * lam * lam) {
                type = 0;
            } else if (fabs(arr) >= BK_ALPHA * sig) {
                type = 0;
                p = r;
                use_r = true;
            } else {
                type = 1;
            }
        }
        // ---- pivot record, inertia, factor columns, Schur update
        double i00 = 0.0, i01 = 0.0, i11 = 0.0;
        if (type == 2) {
            ++nzero;
        } else if (type == 0) {
            const double d = use_r ? arr : akk;
            i00 = rcp_nr(d);
            if (d > 0.0) ++npos; else ++nneg;
        } else {
            const double A00 = akk, A01 = lane_pick<NQ>(cv, r), A11 = arr;
            const double det = A00 * A11 - A01 * A01;
            const double rdet = rcp_nr(det);
            i00 = A11 * rdet;
            i01 = -A01 * rdet;
            i11 = A00 * rdet;
            if (det < 0.0) { ++npos; ++nneg; }
            else if (A00 + A11 > 0.0) npos += 2;
            else nneg += 2;
        }
        const int ncol = type == 1 ? 2 : 1;
        nlive -= type == 1 ? 2 : 1;
        {
            const int e1p = type == 1 ? k : (type == 2 ? k : p);
            const int e2p = type == 1 ? r : -1;
            lvt = lvt && tid != e1p && tid != e2p;
            cit -= (tid > e1p ? 1 : 0) + (e2p >= 0 && tid > e2p ? 1 : 0);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int i = lane + 64 * q;
                lvq[q] = lvq[q] && i != e1p && i != e2p;
            }
        }
        if (tid == 0) {
            pv[steps] = make_int2((type == 1 ? k : p) | (type << 16), type == 1 ? r : -1);
            dv[3 * steps + 0] = i00;
            dv[3 * steps + 1] = i01;
            dv[3 * steps + 2] = i11;
        }
        const double* c0p = use_r ? cr : ck;     // column p (1x1) or k (2x2)
        if (lvt) {
            const int ci = cit;
            const double x0 = c0p[tid];
            if (type == 0) {
                Lb[loff + ci] = x0 * i00;
            } else if (type == 1) {
                const double x1 = cr[tid];
                Lb[loff + 2 * ci] = fma(x0, i00, x1 * i01);
                Lb[loff + 2 * ci + 1] = fma(x0, i01, x1 * i11);
            } else {
                Lb[loff + ci] = 0.0;
            }
        }
        loff += (long long)nlive * ncol;
        const int npass = type == 0 ? 1 : type == 1 ? 2 : 0;
        const int J0 = k >> 4;                   // tiles left of k's tile hold only eliminated positions
        KKT_PRIO_UPDATE();
#pragma unroll 1
        for (int pass = 0; pass < npass; ++pass) {
            const double* cc = pass == 1 ? cr : c0p;
            const double g0 = pass == 1 ? i01 : i00, g1 = pass == 1 ? i11 : i01;
            // rows in NG groups (fewer row factors live at once: VGPR pressure)
            constexpr int NG = ATO_KKT_S16_NG;
#pragma unroll
            for (int G = 0; G < NG; ++G) {
                const int I0 = (G * TT) / NG, I1 = ((G + 1) * TT) / NG;
                if (I1 <= J0) continue;              // rows of eliminated tiles only
                double li[TT];
#pragma unroll
                for (int I = 0; I < TT; ++I) {
                    if (I >= I0 && I < I1) {
                        const double x0 = c0p[16 * I + ti];
                        li[I] = type == 1 ? fma(x0, g0, cr[16 * I + ti] * g1) : x0 * i00;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int J = 0; J < I1; ++J) {
                    if (ATO_KKT_S16_JSKIP == 0 || J >= J0) {
                        const double cj = cc[16 * J + tj];
#pragma unroll
                        for (int I = (J > I0 ? J : I0); I < I1; ++I) a[slot(I, J)] = fma(-li[I], cj, a[slot(I, J)]);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        ++steps;
        par ^= 1;
        {   // first live own position >= kc: find-first-set over the ballot of the lanes' live flags
            int nk = own;
#pragma unroll
            for (int q = NQ - 1; q >= 0; --q) {
                const int lo = kc - 64 * q, hi = own - 64 * q;
                unsigned long long m = lo <= 0 ? ~0ull : (lo >= 64 ? 0ull : (~0ull << lo));
                m &= hi >= 64 ? ~0ull : (hi <= 0 ? 0ull : ((1ull << hi) - 1ull));
                const unsigned long long w = __ballot(lvq[q]) & m;
                nk = w ? 64 * q + (int)__builtin_ctzll(w) : nk;
            }
            kc = nk;
        }
    }
    if (tid == 0) {
        sinfo[(long long)b * P.F + f] = make_int2(steps, (int)loff);
        atomicAdd(&inertia[3 * b + 0], npos);
        atomicAdd(&inertia[3 * b + 1], nneg);
        atomicAdd(&inertia[3 * b + 2], nzero);
    }
    // ---- trailing Schur complement -> contribution block of the parent (HBM)
    const int tq = A - own;
    if (tq > 0) {
        double* cb = CB + (long long)b * P.cb_size + P.cb_off[f];
#pragma unroll
        for (int I = 0; I < TT; ++I) {
#pragma unroll
            for (int J = 0; J <= I; ++J) {
                const int i = 16 * I + ti, j = 16 * J + tj;
                if (i >= own && i < A && j >= own && j < A && (I != J || i >= j)) {
                    cb[(long long)(i - own) * tq + (j - own)] = a[slot(I, J)];
                    cb[(long long)(j - own) * tq + (i - own)] = a[slot(I, J)];
                }
            }
        }
    }
}

template <int TT>
size_t factor_s_lds() {
    constexpr int NP = 16 * TT;
    return sizeof(double) * (16 * (NP + 1) + 4 * NP) + sizeof(int) * NP;
}


// ------------------------------------------------------------------------------------------
// Saddle fronts (solver/kkt_plan.py collocation_saddle): own = nS states X of nodes 1..K of an
// interval, then their nS ODE defect rows Y; trailing T (controls, h, the anchor node, continuity
// and path rows). With no row diagonal on Y (delta_c = 0) the block
//     K_SS = [[H, J^T], [J, 0]]     (H = H_XX + diag_x, J = J_YX square)
// has the inverse [[0, E], [E^T, G]], E = J^-1, G = -E^T H E, and the inertia (nS, nS, 0) whatever
// H is; so it is eliminated without the Bunch-Kaufman pivot chain over 2 nS positions:
//   E:   Gauss-Jordan inversion of J with partial pivoting, held in REGISTERS (lane = row, the eight
//        waves own the columns j = wave mod 8): the wave owning column k picks the pivot and
//        publishes the column, one barrier per step, every thread updates its entries (the pivot
//        row by readlane). No row swaps: the result is E with permuted rows and columns,
//        E[k][c] = M[p_k][j : p_j = c], written unscrambled to LDS;
//   all: HE = H E, G = -E^T (HE), W = K_TS K_SS^-1 = [B_y E^T, B_x E + B_y G] and the contribution
//        block S = -W K_ST (lower tiles, mirrored: one writer per entry) as 16 x 16 fp64 MFMA
//        tiles (v_mfma_f64_16x16x4_f64) from LDS operands.
// Stored for the solve (the front's factor-column slice): K_SS^-1 (2nS x 2nS, symmetric) and W
// (T x 2nS), sinfo = {SAD_DONE, doubles}. A pivot below SAD_PIVOT_TOL max|J_YX| or a nonzero Y
// diagonal marks the (front, instance) SAD_FALLBACK instead, and the Bunch-Kaufman launch that
// follows factorises exactly those (tests/kkt_emulation.py restates both paths).
// ------------------------------------------------------------------------------------------
constexpr int SAD_NT = 512;           // threads per (saddle front, instance): eight waves
constexpr int SAD_NW = SAD_NT / 64;

typedef double sad_v4d __attribute__((ext_vector_type(4)));

// C[i][j] = sum_k a(i, k) b(k, j) over an M x N output in 16 x 16 tiles, one wave per tile, K in
// steps of 4 (v_mfma_f64_16x16x4_f64: lane l holds A[l & 15][k + l / 16] and B[k + l / 16][l & 15],
// result row l / 16 + 4 q, column l & 15 in register q). Out-of-range operands are zero.
template <class FA, class FB, class FC>
__device__ __forceinline__ void sad_mfma(int M, int N, int K, FA a, FB b, FC c, int wave, int lane,
                                         bool lower = false) {
    const int tm = (M + 15) >> 4, tn = (N + 15) >> 4;
    for (int tile = wave; tile < tm * tn; tile += SAD_NW) {
        const int i0 = (tile / tn) * 16, j0 = (tile % tn) * 16;
        if (lower && j0 > i0) continue;
        const int ai = i0 + (lane & 15), bj = j0 + (lane & 15), kk = lane >> 4;
        sad_v4d acc = {0.0, 0.0, 0.0, 0.0};
        for (int k0 = 0; k0 < K; k0 += 32) {     // eight k-steps of operands in flight, then the MFMAs
            double av[8], bv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int k = k0 + 4 * q + kk;
                av[q] = (ai < M && k < K) ? a(ai, k) : 0.0;
                bv[q] = (k < K && bj < N) ? b(k, bj) : 0.0;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], bv[q], acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = i0 + (lane >> 4) + 4 * q, j = j0 + (lane & 15);
            if (i < M && j < N) c(i, j, acc[q]);
        }
    }
}

struct SadLds {      // shared-memory carve of one saddle front (runtime sizes)
    double *E, *H, *Bx, *By, *col, *dv, *mx, *prow;
    int *piv, *pp, *flag, *hkey;
    int ldn;
};

// E and H / G (nS x nS), K_TX rows [0, tx) and K_TY rows [T - ty, T) (the others are zero), the
// published pivot columns: 68 KB on the racetrack (nS 52, tx <= 27, ty 30), two fronts per CU
__device__ __forceinline__ SadLds sad_lds(double* smem, int nS, int tx, int ty) {
    SadLds L;
    L.ldn = nS + 1;
    L.E = smem;                                  // J (assembly) -> E
    L.H = L.E + nS * L.ldn;                      // H -> G
    L.Bx = L.H + nS * L.ldn;                     // [tx][X]
    L.By = L.Bx + tx * L.ldn;                    // [ty][Y]
    L.col = L.By + ty * L.ldn;                   // [2][64] published pivot columns
    L.dv = L.col + 128;                          // [2] pivots
    L.mx = L.dv + 2;                             // [SAD_NW] max |J| per wave
    L.prow = L.mx + SAD_NW;                      // [64] the pivot row (each wave its own columns)
    L.piv = reinterpret_cast<int*>(L.prow + 64);     // [nS] pivot row of every step
    L.pp = L.piv + nS;                           // [2]
    L.flag = L.pp + 2;
    L.hkey = L.flag + 1;                         // max |H diagonal| (float bits)
    return L;
}

inline size_t sad_lds_bytes(int nS, int tx, int ty) {
    const size_t d = (size_t)(2 * nS + tx + ty) * (nS + 1) + 128 + 2 + SAD_NW + 64;
    return d * sizeof(double) + sizeof(int) * (nS + 4);
}

template <int NSM>
__global__ __launch_bounds__(SAD_NT) void k_front_saddle(Plan P, Vals V, int f0, int batch, const int* __restrict__ list,
                                                         double* __restrict__ Lst, int2* __restrict__ sinfo,
                                                         double* __restrict__ CB, int* __restrict__ inertia) {
    static_assert(NSM <= 64, "one Gauss-Jordan row per lane");
    constexpr int CM = (NSM + SAD_NW - 1) / SAD_NW;          // columns per thread
    extern __shared__ double smem[];
    const int f = P.forder[f0 + blockIdx.x];
    const int bi = blockIdx.y;
    if (bi >= batch) return;
    const int b = list ? __builtin_amdgcn_readfirstlane(list[bi]) : bi;
    if (list && b >= P.cap) return;            // a listed slot past the reserved storage: nothing is touched
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int p0 = P.pos_ptr[f];
    const int A = P.pos_ptr[f + 1] - p0;
    const int nS = P.n_sad[f], n2 = 2 * nS, T = A - n2;
    const int2 txy = P.sad_txy[f];
    const int tx = txy.x, ty0 = T - txy.y;        // K_TX rows [0, tx), K_TY rows [ty0, T)
    const SadLds L = sad_lds(smem, nS, tx, txy.y);
    const int ldn = L.ldn;
    KST_DECL(f == ATO_KKT_STAMP_FRONT && blockIdx.y == 0)

    // ---- assembly: J (Y x X) into E, H (X x X), K_TX, K_TY; a Y diagonal -> fallback
    for (int i = tid; i < (2 * nS + tx + txy.y) * ldn; i += SAD_NT) L.E[i] = 0.0;
    if (tid == 0) {
        *L.flag = 0;
        *L.hkey = 0;
    }
    __syncthreads();
    {
        const int e0 = P.ent_ptr[f * MAXT], e1 = P.ent_ptr[(f + 1) * MAXT];
        for (int e = e0 + tid; e < e1; e += SAD_NT) {
            const int ep = P.ent_pos[e];
            const int pa = ep >> 16, pb = ep & 0xffff;
            const int2 sc = P.ent_src[e];
            const double v = src_value(V, sc.x, b) + src_value(V, sc.y, b);
            if (pa < nS) {
                L.H[pa * ldn + pb] = v;
                L.H[pb * ldn + pa] = v;
                if (pa == pb) atomicMax(reinterpret_cast<unsigned*>(L.hkey), __float_as_uint((float)fabs(v)));
            } else if (pa < n2) {
                if (pb < nS) L.E[(pa - nS) * ldn + pb] = v;
                else if (v != 0.0) *L.flag = 1;
            } else if (pb < nS) {
                L.Bx[(pa - n2) * ldn + pb] = v;
            } else if (pb < n2) {
                L.By[(pa - n2 - ty0) * ldn + (pb - nS)] = v;
            }
        }
    }
    __syncthreads();
    KST(0);                      // assembly

    // ---- Gauss-Jordan inversion of J in registers: row `lane`, columns wave + 8 m
    double Mr[CM];
    double lmx = 0.0;
#pragma unroll
    for (int m = 0; m < CM; ++m) {
        const int j = wave + SAD_NW * m;
        Mr[m] = (lane < nS && j < nS) ? L.E[lane * ldn + j] : 0.0;
        lmx = fmax(lmx, fabs(Mr[m]));
    }
    {
        const unsigned km = wave_max_u32(__float_as_uint((float)lmx));
        if (lane == 0) L.mx[wave] = (double)__uint_as_float(km);
    }
    __syncthreads();
    double mx = 0.0;
#pragma unroll
    for (int w = 0; w < SAD_NW; ++w) mx = fmax(mx, L.mx[w]);
    // a nonzero Y diagonal, or a barrier diagonal too large for the structured elimination: fall back
    // before the Gauss-Jordan sweep (uniform: every thread reads the same shared values)
    if (*L.flag || (P.sad_tau > 0.0 && (double)__uint_as_float(*reinterpret_cast<unsigned*>(L.hkey)) >
                                          P.sad_tau * mx * mx)) {
        if (tid == 0) sinfo[(long long)b * P.F + f] = make_int2(SAD_FALLBACK, 0);
        return;
    }
    bool used = false;
    int mystep = -1;
    for (int k = 0; k < nS; ++k) {
        const int par = k & 1;
        if (wave == (k & (SAD_NW - 1))) {        // owner of column k: pivot search, publish the column
            const int mk = k / SAD_NW;
            double v = Mr[0];
#pragma unroll
            for (int m = 1; m < CM; ++m) v = blend(v, Mr[m], m == mk ? ~0ull : 0ull);
            const unsigned key = wave_max_u32(lane < nS && !used ? mag_key(v, lane) : 0u);
            const int p = key ? 511 - (int)(key & 0x1FFu) : 0;
            const double d = readlane_f64(v, p);
            L.col[par * 64 + lane] = v;
            if (lane == 0) {
                L.piv[k] = p;
                L.pp[par] = p;
                L.dv[par] = 1.0 / d;
                if (key == 0u || !(fabs(d) > SAD_PIVOT_TOL * mx)) *L.flag = 1;
            }
        }
        KST(7);                  // owner: search and publish (wave 0 owns every eighth column)
        __syncthreads();
        const int p = __builtin_amdgcn_readfirstlane(L.pp[par]);
        const double inv = L.dv[par];
        const double fr = L.col[par * 64 + lane];
        if (lane == p) {
            used = true;
            mystep = k;
#pragma unroll
            for (int m = 0; m < CM; ++m) L.prow[wave + SAD_NW * m] = Mr[m];   // this wave's columns of row p
        }
        KST(8);                  // barrier, published pivot read
#pragma unroll
        for (int m = 0; m < CM; ++m) {
            const int j = wave + SAD_NW * m;
            const double pr = j == k ? inv : L.prow[j] * inv;
            Mr[m] = lane == p ? pr : fma(-fr, pr, j == k ? 0.0 : Mr[m]);
        }
        KST(9);                  // update
    }
    KST(1);                      // Gauss-Jordan
    int2* si = sinfo + (long long)b * P.F + f;
    if (*L.flag) {
        if (tid == 0) *si = make_int2(SAD_FALLBACK, 0);
#ifdef ATO_KKT_STAMPS
        if (tid == 0) atomicAdd(&g_kkt_stamps[14], 1ull);
#endif
        return;
    }
    // E[k][c] = M[p_k][j] with p_j = c: row `lane` was the pivot of step mystep
    if (lane < nS) {
#pragma unroll
        for (int m = 0; m < CM; ++m) {
            const int j = wave + SAD_NW * m;
            if (j < nS) L.E[mystep * ldn + L.piv[j]] = Mr[m];
        }
    }
    __syncthreads();
    KST(2);                      // unscramble
    // ---- HE = H E (scratch: the front's factor slice, rewritten below), G = -E^T (HE) (over H)
    const double* E = L.E;
    double* Hm = L.H;
    const double* Bx = L.Bx;
    const double* By = L.By;
    double* Lb = Lst + (long long)b * P.l_size + P.l_off[f];
    double* Wg = Lb + (long long)n2 * n2;         // W [T][2 nS] in the factor slice
    double* HE = Lb;
    // K_TS (t, k): k < nS from K_TX, k >= nS from K_TY (zero outside their row ranges)
    auto kts = [&](int t, int k) {
        return k < nS ? (t < tx ? Bx[t * ldn + k] : 0.0) : (t >= ty0 ? By[(t - ty0) * ldn + (k - nS)] : 0.0);
    };
    sad_mfma(nS, nS, nS, [&](int i, int k) { return Hm[i * ldn + k]; }, [&](int k, int j) { return E[k * ldn + j]; },
             [&](int i, int j, double v) { HE[i * nS + j] = v; }, wave, lane);
    __syncthreads();
    sad_mfma(nS, nS, nS, [&](int i, int k) { return E[k * ldn + i]; }, [&](int k, int j) { return HE[k * nS + j]; },
             [&](int i, int j, double v) { Hm[i * ldn + j] = -v; }, wave, lane);
    __syncthreads();
    KST(3);                      // H E, G
    // ---- W = [K_TY E^T, K_TX E + K_TY G] into the factor slice
    sad_mfma(T, nS, nS, [&](int t, int k) { return kts(t, nS + k); }, [&](int k, int i) { return E[i * ldn + k]; },
             [&](int t, int i, double v) { Wg[(long long)t * n2 + i] = v; }, wave, lane);
    sad_mfma(T, nS, n2, [&](int t, int k) { return kts(t, k); },
             [&](int k, int i) { return k < nS ? E[k * ldn + i] : Hm[(k - nS) * ldn + i]; },
             [&](int t, int i, double v) { Wg[(long long)t * n2 + nS + i] = v; }, wave, lane);
    __syncthreads();
    KST(4);                      // W
    // ---- contribution block S = -W K_ST (lower tiles, mirrored), then K_SS^-1 to the factor slice
    if (T > 0) {
        double* cb = CB + (long long)b * P.cb_size + P.cb_off[f];
        sad_mfma(T, T, n2, [&](int s, int k) { return Wg[(long long)s * n2 + k]; }, [&](int k, int t) { return kts(t, k); },
                 [&](int s, int t, double v) {
                     if (s >= t) {
                         cb[(long long)s * T + t] = -v;
                         cb[(long long)t * T + s] = -v;
                     }
                 }, wave, lane, true);
    }
    __syncthreads();             // the H E scratch is read by the other waves until here
    KST(5);                      // S
    for (int q = tid; q < n2 * n2; q += SAD_NT) {
        const int i = q / n2, j = q - i * n2;
        double v;
        if (i < nS) v = j < nS ? 0.0 : E[i * ldn + (j - nS)];
        else v = j < nS ? E[j * ldn + (i - nS)] : Hm[(i - nS) * ldn + (j - nS)];
        Lb[q] = v;
    }
    KST(6);                      // stores
    KST_DUMP(1);
    if (tid == 0) {
        *si = make_int2(SAD_DONE, n2 * n2 + T * n2);
        atomicAdd(&inertia[3 * b + 0], nS);
        atomicAdd(&inertia[3 * b + 1], nS);
    }
}

// solve of a saddle front: forward u = K_SS^-1 b_S (into x), contribution -W b_S to the parent;
// backward x_S = u - W^T x_T. 128 threads; thread r < 2 nS owns row r of K_SS^-1 (symmetric, so
// column r: coalesced reads), thread t < T row t of W
__device__ void saddle_fwd(const Plan& P, int f, int b, const double* Lb, double* scf, double* xb, long long se,
                           double* sbuf, int tid) {
    const int p0 = P.pos_ptr[f], A = P.pos_ptr[f + 1] - p0, nS = P.n_sad[f], n2 = 2 * nS, T = A - n2;
    for (int i = tid; i < n2; i += ST) sbuf[i] = xb[(long long)P.pos_index[p0 + i] * se];
    __syncthreads();
    double u = 0.0;
    if (tid < n2) {
        for (int k = tid < nS ? nS : 0; k < n2; ++k) u = fma(Lb[(long long)k * n2 + tid], sbuf[k], u);
    }
    const double* W = Lb + (long long)n2 * n2;
    for (int t = tid; t < T; t += ST) {
        double acc = 0.0;
        for (int k = 0; k < n2; ++k) acc = fma(W[(long long)t * n2 + k], sbuf[k], acc);
        scf[t] = -acc;
    }
    if (tid < n2) xb[(long long)P.pos_index[p0 + tid] * se] = u;
}

__device__ void saddle_bwd(const Plan& P, int f, int b, const double* Lb, double* xb, long long se, double* sbuf,
                           int tid) {
    const int p0 = P.pos_ptr[f], A = P.pos_ptr[f + 1] - p0, nS = P.n_sad[f], n2 = 2 * nS, T = A - n2;
    for (int t = tid; t < T; t += ST) sbuf[t] = xb[(long long)P.pos_index[p0 + n2 + t] * se];
    __syncthreads();
    const double* W = Lb + (long long)n2 * n2;
    for (int k = tid; k < n2; k += ST) {
        double acc = 0.0;
        for (int t = 0; t < T; ++t) acc = fma(W[(long long)t * n2 + k], sbuf[t], acc);
        const long long o = (long long)P.pos_index[p0 + k] * se;
        xb[o] = xb[o] - acc;
    }
}

// ------------------------------------------------------------------------------------------
// solve
// ------------------------------------------------------------------------------------------
// Stream of the front's factor columns through a two-slot LDS ring. Forward: chunks 0, 1, 2,
// ... of [0, total); backward: the same chunks in reverse. Chunk c lives in slot c & 1.
// C: doubles per chunk (a power of two holding the front's largest column pair: CH up to eight tiles,
// 2 CH for nine, ring_chunk<T>)
template <int T>
constexpr int ring_chunk() { return T > 8 ? 2 * CH : CH; }
static_assert(2 * CH >= 2 * 32 * MAX_FRONT_TILES, "solve ring chunk smaller than the largest column pair");

template <int C>
struct Ring {
    double* buf;           // [2][C]
    __device__ __forceinline__ double at(long long off) const { return buf[off & (2 * C - 1)]; }
};

template <int C>
__device__ __forceinline__ void ring_load(const double* __restrict__ src, long long total, long long c,
                                          double (&r)[C / ST], int tid) {
#pragma unroll
    for (int q = 0; q < C / ST; ++q) {
        const long long o = c * C + q * ST + tid;
        r[q] = (c >= 0 && o < total) ? src[o] : 0.0;
    }
}

template <int C>
__device__ __forceinline__ void ring_store(double* buf, long long c, const double (&r)[C / ST], int tid) {
    double* dst = buf + (c & 1) * C;
#pragma unroll
    for (int q = 0; q < C / ST; ++q) dst[q * ST + tid] = r[q];
}

template <int NQ>
__device__ __forceinline__ double lane_get(const double (&y)[NQ], int p) {
    const int q = p >> 6;
    double v = y[0];
#pragma unroll
    for (int k = 1; k < NQ; ++k) v = blend(v, y[k], q == k ? ~0ull : 0ull);
    return readlane_f64(v, p & 63);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the front's pivot records and inverse pivot blocks into LDS (all threads), then a barrier
__device__ __forceinline__ void stage_records(const int2* __restrict__ pv, const double* __restrict__ dvp,
                                              int steps, int tid, int2* s_piv, double* s_dinv) {
    for (int u = tid; u < steps; u += ST) {
        s_piv[u] = pv[u];
        s_dinv[3 * u + 0] = dvp[3 * u + 0];
        s_dinv[3 * u + 1] = dvp[3 * u + 1];
        s_dinv[3 * u + 2] = dvp[3 * u + 2];
    }
}

struct FrontSolve {
    int f, b, p0, A, own, steps;
    long long total;
    const double* Lb;
    const int2* pv;
    const double* dvp;
    double* xb;
};

__device__ __forceinline__ FrontSolve front_solve_setup(const Plan& P, int f, int b, const double* Lst,
                                                        const int2* piv, const double* dinv,
                                                        const int2* sinfo, double* x, long long sb) {
    FrontSolve s;
    s.f = f;
    s.b = b;
    s.p0 = P.pos_ptr[f];
    s.A = P.pos_ptr[f + 1] - s.p0;
    s.own = P.n_own[f];
    const int2 inf = sinfo[(long long)b * P.F + f];
    s.steps = min(max(inf.x, 0), s.own);
    const long long cap = (long long)s.own * s.A - (long long)s.own * (s.own + 1) / 2;
    s.total = min(max((long long)inf.y, 0ll), cap);
    s.Lb = Lst + (long long)b * P.l_size + P.l_off[f];
    s.pv = piv + (long long)b * P.dim + P.piv_off[f];
    s.dvp = dinv + ((long long)b * P.dim + P.piv_off[f]) * 3;
    s.xb = x + (long long)b * sb;
    return s;
}

template <int T>
__global__ __launch_bounds__(ST) void k_front_fwd(Plan P, int f0, int batch, const int* __restrict__ list,
                                                  const double* __restrict__ Lst, const int2* __restrict__ piv,
                                                  const double* __restrict__ dinv, const int2* __restrict__ sinfo,
                                                  double* __restrict__ SC, double* __restrict__ x, long long se,
                                                  long long sb) {
    constexpr int NP = 32 * T;
    constexpr int NQ = (NP + 63) / 64;
    constexpr int CHT = ring_chunk<T>();
    __shared__ double ring_buf[2 * CHT];
    __shared__ double cvec[NP];
    __shared__ int2 s_piv[NP];
    __shared__ double s_dinv[3 * NP];
    __shared__ int s_done;

    const int bi = blockIdx.y;
    if (bi >= batch) return;
    const int b = list ? __builtin_amdgcn_readfirstlane(list[bi]) : bi;
    if (list && b >= P.cap) return;            // a listed slot past the reserved storage: nothing is touched
    const FrontSolve F = front_solve_setup(P, f0 + blockIdx.x, b, Lst, piv, dinv, sinfo, x, sb);
    const int tid = threadIdx.x;
    if (P.n_sad && P.n_sad[F.f] > 0 && sinfo[(long long)b * P.F + F.f].x == SAD_DONE) {
        saddle_fwd(P, F.f, b, F.Lb, SC + (long long)b * P.sc_size + P.sc_off[F.f], F.xb, se, cvec, tid);
        return;
    }
    const int lane = tid & 63;
    const bool w0 = tid < 64;
    Ring<CHT> ring{ring_buf};
    double stage_r[CHT / ST];

    // ---- right-hand side: own entries of b, zero trailing, plus the children's contributions
    for (int i = tid; i < NP; i += ST) cvec[i] = i < F.own ? F.xb[(long long)P.pos_index[F.p0 + i] * se] : 0.0;
    stage_records(F.pv, F.dvp, F.steps, tid, s_piv, s_dinv);
    ring_load<CHT>(F.Lb, F.total, 0, stage_r, tid);
    ring_store<CHT>(ring.buf, 0, stage_r, tid);
    ring_load<CHT>(F.Lb, F.total, 1, stage_r, tid);
    ring_store<CHT>(ring.buf, 1, stage_r, tid);
    __syncthreads();
    for (int ci = P.child_ptr[F.f]; ci < P.child_ptr[F.f + 1]; ++ci) {
        const int c = P.child_list[ci];
        const int pc = P.pos_ptr[c], oc = P.n_own[c];
        const int tqc = P.pos_ptr[c + 1] - pc - oc;
        const double* scc = SC + (long long)b * P.sc_size + P.sc_off[c];
        for (int q = tid; q < tqc; q += ST) cvec[P.parent_pos[pc + oc + q]] += scc[q];
        __syncthreads();
    }

    // ---- forward sweep L y = b (wave 0), factor columns streamed through the ring
    double y[NQ];
    bool lv[NQ];          // position lane + 64 q live
    int ci[NQ];           // live positions below it (its index in a compact factor column)
    if (w0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = lane + 64 * q;
            y[q] = i < NP ? cvec[i] : 0.0;
            lv[q] = i < F.A;
            ci[q] = min(i, F.A);
        }
    }
    int nlive = F.A, t = 0;
    long long off = 0;
    int2 rec_nx = F.steps > 0 ? s_piv[0] : make_int2(0, -1);   // record of step t, read one step ahead
    const long long nchunks = (F.total + CHT - 1) / CHT;
    if (tid == 0) s_done = 0;
    for (long long c = 0;; ++c) {
        ring_load<CHT>(F.Lb, F.total, c + 2, stage_r, tid);     // in flight while wave 0 sweeps
        if (w0) {
            const long long limit = (c + 2) * CHT;
            while (t < F.steps) {
                const int2 rec = rec_nx;
                const int type = __builtin_amdgcn_readfirstlane(rec.x >> 16);
                const int pp = __builtin_amdgcn_readfirstlane(min(rec.x & 0xffff, NP - 1));
                const int rr = __builtin_amdgcn_readfirstlane(min(max(rec.y, 0), NP - 1));
                const int ncol = type == 1 ? 2 : 1;
                const int nl_after = nlive - ncol;
                if (off + (long long)nl_after * ncol > limit) break;     // column not resident yet
                rec_nx = s_piv[min(t + 1, NP - 1)];
                // branch-free: every lane reads (dead positions read a harmless ring word, and their
                // update is discarded by the blend); all the column reads are issued before y is
                // touched, so one LDS round trip per step
                const bool two = type == 1;
                double c0[NQ], c1[NQ];
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int i = lane + 64 * q;
                    lv[q] = lv[q] && i != pp && !(two && i == rr);
                    ci[q] -= (i > pp ? 1 : 0) + (two && i > rr ? 1 : 0);
                    const int idx = two ? 2 * ci[q] : ci[q];
                    c0[q] = ring.at(off + idx);
                    c1[q] = ring.at(off + idx + 1);
                }
                const double zp = lane_get<NQ>(y, pp);
                const double zr = two ? lane_get<NQ>(y, rr) : 0.0;
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const double upd = two ? c0[q] * zp + c1[q] * zr : c0[q] * zp;
                    y[q] = blend(y[q], y[q] - upd, lv[q] ? ~0ull : 0ull);
                }
                off += (long long)nl_after * ncol;
                nlive = nl_after;
                ++t;
            }
            if (lane == 0) s_done = t >= F.steps ? 1 : 0;
        }
        __syncthreads();
        if (s_done != 0) break;
        ring_store<CHT>(ring.buf, c + 2, stage_r, tid);
        __syncthreads();
        if (c + 2 > nchunks + 2) break;               // safety: never loop past the stream
    }
    if (!w0) return;
    // ---- D solve of the own positions, own values out, trailing values to the parent
    for (int u = 0; u < F.steps; ++u) {
        const int2 rec = s_piv[u];
        const int type = __builtin_amdgcn_readfirstlane(rec.x >> 16);
        const int pp = __builtin_amdgcn_readfirstlane(min(rec.x & 0xffff, NP - 1));
        const double d0 = s_dinv[3 * u], d1 = s_dinv[3 * u + 1], d2 = s_dinv[3 * u + 2];
        if (type == 1) {
            const int rr = __builtin_amdgcn_readfirstlane(min(max(rec.y, 0), NP - 1));
            const double yp = lane_get<NQ>(y, pp), yr = lane_get<NQ>(y, rr);
            lane_set<NQ>(y, pp, d0 * yp + d1 * yr, lane);
            lane_set<NQ>(y, rr, d1 * yp + d2 * yr, lane);
        } else {
            lane_set<NQ>(y, pp, d0 * lane_get<NQ>(y, pp), lane);
        }
    }
    double* scf = SC + (long long)b * P.sc_size + P.sc_off[F.f];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int i = lane + 64 * q;
        if (i < F.own) F.xb[(long long)P.pos_index[F.p0 + i] * se] = y[q];
        else if (i < F.A) scf[i - F.own] = y[q];
    }
}

template <int T>
__global__ __launch_bounds__(ST) void k_front_bwd(Plan P, int f0, int batch, const int* __restrict__ list,
                                                  const double* __restrict__ Lst, const int2* __restrict__ piv,
                                                  const double* __restrict__ dinv, const int2* __restrict__ sinfo,
                                                  double* __restrict__ x, long long se, long long sb) {
    constexpr int NP = 32 * T;
    constexpr int NQ = (NP + 63) / 64;
    constexpr int CHT = ring_chunk<T>();
    __shared__ double ring_buf[2 * CHT];
    __shared__ double cvec[NP];
    __shared__ int2 s_piv[NP];     // (the backward sweep needs no inverse pivot blocks: 4.6 KB less LDS)
    __shared__ int s_done;

    const int bi = blockIdx.y;
    if (bi >= batch) return;
    const int b = list ? __builtin_amdgcn_readfirstlane(list[bi]) : bi;
    if (list && b >= P.cap) return;            // a listed slot past the reserved storage: nothing is touched
    const FrontSolve F = front_solve_setup(P, f0 + blockIdx.x, b, Lst, piv, dinv, sinfo, x, sb);
    const int tid = threadIdx.x;
    if (P.n_sad && P.n_sad[F.f] > 0 && sinfo[(long long)b * P.F + F.f].x == SAD_DONE) {
        saddle_bwd(P, F.f, b, F.Lb, F.xb, se, cvec, tid);
        return;
    }
    const int lane = tid & 63;
    const bool w0 = tid < 64;
    Ring<CHT> ring{ring_buf};
    double stage_r[CHT / ST];
    const long long nchunks = (F.total + CHT - 1) / CHT;
    const long long clast = nchunks - 1;

    // own: the forward (D-scaled) values; trailing: final values of the ancestors' positions
    for (int i = tid; i < NP; i += ST) cvec[i] = i < F.A ? F.xb[(long long)P.pos_index[F.p0 + i] * se] : 0.0;
    for (int u = tid; u < F.steps; u += ST) s_piv[u] = F.pv[u];
    ring_load<CHT>(F.Lb, F.total, clast, stage_r, tid);
    ring_store<CHT>(ring.buf, clast, stage_r, tid);
    ring_load<CHT>(F.Lb, F.total, clast - 1, stage_r, tid);
    ring_store<CHT>(ring.buf, clast - 1, stage_r, tid);
    if (tid == 0) s_done = 0;
    __syncthreads();

    double y[NQ];
    bool lv[NQ];
    int ci[NQ];
    if (w0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = lane + 64 * q;
            y[q] = i < NP ? cvec[i] : 0.0;
            lv[q] = i >= F.own && i < F.A;
            ci[q] = min(max(i - F.own, 0), F.A - F.own);
        }
    }
    int nlive = F.A - F.own, t = F.steps - 1;
    long long off = F.total;                                  // stream end of this front
    int2 rec_nx = s_piv[max(t, 0)];
    for (long long c = clast;; --c) {
        ring_load<CHT>(F.Lb, F.total, c - 2, stage_r, tid);
        if (w0) {
            const long long lower = (c - 1) * CHT;          // chunks c-1 and c are resident
            while (t >= 0) {
                const int2 rec = rec_nx;
                const int type = __builtin_amdgcn_readfirstlane(rec.x >> 16);
                const int pp = __builtin_amdgcn_readfirstlane(min(rec.x & 0xffff, NP - 1));
                const int rr = __builtin_amdgcn_readfirstlane(min(max(rec.y, 0), NP - 1));
                const int ncol = type == 1 ? 2 : 1;
                const long long o = off - (long long)nlive * ncol;
                if (o < lower) break;                             // column not resident yet
                rec_nx = s_piv[max(t - 1, 0)];
                const bool two = type == 1;
                double c0[NQ], c1[NQ];     // all column reads first: one LDS round trip per step
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int idx = two ? 2 * ci[q] : ci[q];
                    c0[q] = ring.at(o + idx);
                    c1[q] = ring.at(o + idx + 1);
                }
                // the PRODUCT is masked, not the operand: a dead lane reads an arbitrary ring word
                // (possibly Inf / NaN), and 0 * Inf would poison the sum
                double sp = 0.0, sr = 0.0;
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const unsigned long long mq = lv[q] ? ~0ull : 0ull;
                    sp += blend(0.0, c0[q] * y[q], mq);
                    sr += two ? blend(0.0, c1[q] * y[q], mq) : 0.0;
                }
                sp = wave_sum(sp);
                lane_set<NQ>(y, pp, lane_get<NQ>(y, pp) - sp, lane);
                if (two) {
                    sr = wave_sum(sr);
                    lane_set<NQ>(y, rr, lane_get<NQ>(y, rr) - sr, lane);
                }
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int i = lane + 64 * q;
                    lv[q] = lv[q] || i == pp || (two && i == rr);
                    ci[q] += (i > pp ? 1 : 0) + (two && i > rr ? 1 : 0);
                }
                nlive += ncol;
                off = o;
                --t;
            }
            if (lane == 0) s_done = t < 0 ? 1 : 0;
        }
        __syncthreads();
        if (s_done != 0) break;
        ring_store<CHT>(ring.buf, c - 2, stage_r, tid);
        __syncthreads();
        if (c < -2) break;                                // safety
    }
    if (!w0) return;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int i = lane + 64 * q;
        if (i < F.own) F.xb[(long long)P.pos_index[F.p0 + i] * se] = y[q];
    }
}

// ------------------------------------------------------------------------------------------
// residual out = rhs - K x (iterative refinement): 4 KKT rows per 256-thread workgroup, one wave
// per row, lanes = 64 instances (coalesced in the interleaved layout), the row's entries in
// their fixed CSR order
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_kkt_residual(int dim, int batch, const int* __restrict__ list,
                                                      const int* __restrict__ rp,
                                                      const int* __restrict__ col, const int* __restrict__ src,
                                                      Vals V, const double* __restrict__ x,
                                                      const double* __restrict__ rhs, double* __restrict__ out) {
    const int r = __builtin_amdgcn_readfirstlane(blockIdx.y * 4 + (threadIdx.x >> 6));
    const int bi = blockIdx.x * 64 + (threadIdx.x & 63);
    if (r >= dim || bi >= batch) return;
    const int b = list ? list[bi] : bi;
    const int e0 = rp[r], e1 = rp[r + 1];
    double acc = 0.0;
    for (int e = e0; e < e1; ++e) {
        const int c = col[e];
        acc = fma(src_value(V, src[e], b), x[(long long)c * V.se + (long long)b * V.sb], acc);
    }
    const long long o = (long long)r * V.se + (long long)b * V.sb;
    out[o] = rhs[o] - acc;
}

template <int T, int FTT = FT>
size_t factor_lds() {
    constexpr int NP = 32 * T;
    constexpr int SRW = FTT == 64 ? 16 : 32;
    return sizeof(double) * (SRW * (NP + 1) + 4 * NP) + sizeof(int) * 2 * NP;
}

// Six-tile fronts hold 138 VGPRs: one 512-thread workgroup per CU. Allocated for four waves per
// SIMD (a few spilled registers, reloaded from scratch a few times per pivot step), two workgroups
// share a CU and overlap their pivot chains: B = 512 factorisation 37.3 -> 28.1 ms, B = 1 0.77 ->
// 0.80 ms. So the four-wave variant runs when the level has more workgroups than the chip has CUs.
constexpr int CUS = 256;
#ifndef ATO_KKT_LEAF_FTT
#define ATO_KKT_LEAF_FTT 256
#endif
#ifndef ATO_KKT_SMALL_FTT
#define ATO_KKT_SMALL_FTT 256
#endif

template <int T>
int launch_factor_level(const ato_kkt* h, const Plan& P, const Vals& V, int f0, int nf, int batch, const int* list,
                        int* inertia, hipStream_t st) {
    // fronts of at most two tiles in a level of many workgroups: one wave each (throughput; B = 512
    // factorisation 27.0 -> 24.8 ms); few workgroups (small batches): 512 threads each, whose
    // shorter pivot steps set the latency (B = 1: 0.76 ms vs 0.87 ms with one wave)
    bool one_wave = false;
    if constexpr (T <= 2) {
        one_wave = (long long)nf * batch >= 4 * CUS;
        if (one_wave)
            hipLaunchKernelGGL((k_front_factor_w<T, 1, 64>), dim3(nf, batch), dim3(64), (factor_lds<T, 64>()), st, P, V,
                               f0, batch, list, h->d_L, h->d_piv, h->d_dinv, h->d_sinfo, h->d_cb, inertia,
                               h->d_spec);
    }
#if ATO_KKT_LEAF_FTT == 256
    // Six-tile fronts (the interval leaves): 256 threads, one wave per SIMD, four columns per thread
    // and tile (about 220 VGPRs). Every wave runs the pivot search and decision, so four waves do
    // that work instead of eight, and no SIMD interleaves two waves of the same front's chain.
    if constexpr (T == 6) {
        if (!one_wave) {
            hipLaunchKernelGGL((k_front_factor_w<T, 2, 256>), dim3(nf, batch), dim3(256), factor_lds<T>(), st, P, V,
                               f0, batch, list, h->d_L, h->d_piv, h->d_dinv, h->d_sinfo, h->d_cb, inertia,
                               h->d_spec);
            one_wave = true;
        }
    }
#endif
#if ATO_KKT_SMALL_FTT == 256
    // fronts of at most two tiles in levels of few workgroups (small batches, restoration phases):
    // 256 threads, one wave per SIMD (the same reasoning as the leaves)
    if constexpr (T <= 2) {
        if (!one_wave) {
            hipLaunchKernelGGL((k_front_factor_w<T, 1, 256>), dim3(nf, batch), dim3(256), factor_lds<T>(), st, P, V,
                               f0, batch, list, h->d_L, h->d_piv, h->d_dinv, h->d_sinfo, h->d_cb, inertia,
                               h->d_spec);
            one_wave = true;
        }
    }
#endif
    if (!one_wave) {
        auto k = k_front_factor_w<T, 1, FT>;
        if constexpr (T == 6)
            if ((long long)nf * batch > CUS) k = k_front_factor_w<T, 4, FT>;
        hipLaunchKernelGGL(k, dim3(nf, batch), dim3(FT), factor_lds<T>(), st, P, V, f0, batch, list,
                           h->d_L, h->d_piv, h->d_dinv, h->d_sinfo, h->d_cb, inertia, h->d_spec);
    }
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

template <int T>
int launch_fwd_level(const ato_kkt* h, const Plan& P, int f0, int nf, int batch, const int* list, double* x,
                     long long se, long long sb, hipStream_t st) {
    hipLaunchKernelGGL(k_front_fwd<T>, dim3(nf, batch), dim3(ST), 0, st, P, f0, batch, list, h->d_L, h->d_piv,
                       h->d_dinv, h->d_sinfo, h->d_sc, x, se, sb);
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

template <int T>
int launch_bwd_level(const ato_kkt* h, const Plan& P, int f0, int nf, int batch, const int* list, double* x,
                     long long se, long long sb, hipStream_t st) {
    hipLaunchKernelGGL(k_front_bwd<T>, dim3(nf, batch), dim3(ST), 0, st, P, f0, batch, list, h->d_L, h->d_piv,
                       h->d_dinv, h->d_sinfo, x, se, sb);
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

#ifndef ATO_KKT_S16_W
#define ATO_KKT_S16_W 3
#endif
template <int TT>
int launch_factor_s(const ato_kkt* h, const Plan& P, const Vals& V, int f0, int nf, int batch, const int* list,
                    int* inertia, hipStream_t st) {
    hipLaunchKernelGGL((k_front_factor_s<TT, ATO_KKT_S16_W>), dim3(nf, batch), dim3(256), factor_s_lds<TT>(), st, P, V,
                       f0, batch, list, h->d_L, h->d_piv, h->d_dinv, h->d_sinfo, h->d_cb, inertia);
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

// Kernel class of a front of A positions: 16-wide tiles (111) for 161-176 positions, otherwise
// the number of 32-wide tiles. A level's fronts are launched class by class (ato_kkt::segs), so
// one 65-position separator no longer moves its whole level to three tiles.
int front_class(int A, bool s16) {
    if (s16 && A > 160 && A <= 176) return 111;
    return std::max(1, (A + 31) / 32);
}

// the 16-wide-tile kernel pays off once about four fronts share every CU; below that many
// workgroups the six-tile kernel's shorter pivot steps set the time (both give the same factors
// bit for bit). Racetrack leaves (50 per instance), factor ms six-tile / 16-wide: B = 8 0.78 / 0.80,
// B = 16 1.08 / 1.09, B = 24 1.36 / 1.21, B = 30 1.47 / 1.30 (profiles/r03/kkt_leaf16/r03am)
int s16_min_workgroups() {
    static const int v = [] {
        const char* e = getenv("ATO_KKT_S16_MIN");
        return e ? atoi(e) : 4 * CUS;
    }();
    return v;
}

int launch_saddle(const ato_kkt* h, const Plan& P, const Vals& V, const ato_kkt::Seg& sg, int batch,
                  const int* list, int* inertia, hipStream_t st) {
    const dim3 grid(sg.count, batch);
#define ATO_SAD(N_) hipLaunchKernelGGL((k_front_saddle<N_>), grid, dim3(SAD_NT), sg.lds, st, P, V, sg.start, batch, list, \
                                       h->d_L, h->d_sinfo, h->d_cb, inertia)
    switch (sg.nsm) {
        case 32: ATO_SAD(32); break;
        case 48: ATO_SAD(48); break;
        case 56: ATO_SAD(56); break;
        case 64: ATO_SAD(64); break;
        default: return fail(ATO_ERR_UNSUPPORTED, "KKT saddle front size");
    }
#undef ATO_SAD
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

int launch_segment(const ato_kkt* h, const Plan& P, const Vals& V, const ato_kkt::Seg& sg, int batch,
                   const int* list, int* inertia, hipStream_t st) {
    const int f0 = sg.start, nf = sg.count;
    if (sg.cls == SADDLE_CLS) {
        // the structured elimination, then Bunch-Kaufman for the (front, instance) pairs it left
        // (SAD_FALLBACK); the other workgroups of that launch return at once
        if (int rc = launch_saddle(h, P, V, sg, batch, list, inertia, st)) return rc;
        return launch_segment(h, P, V, ato_kkt::Seg{sg.start, sg.count, sg.cls2}, batch, list, inertia, st);
    }
#define ATO_CALL(T_) launch_factor_level<T_>(h, P, V, f0, nf, batch, list, inertia, st)
    switch (sg.cls) {
        case 1: return ATO_CALL(1);
        case 2: return ATO_CALL(2);
        case 3: return ATO_CALL(3);
        case 4: return ATO_CALL(4);
        case 5: return ATO_CALL(5);
        case 6: return ATO_CALL(6);
        case 7: return ATO_CALL(7);
        case 8: return ATO_CALL(8);
        case 9: return ATO_CALL(9);
        case 111:
            if ((long long)nf * batch >= s16_min_workgroups())
                return launch_factor_s<11>(h, P, V, f0, nf, batch, list, inertia, st);
            return ATO_CALL(6);
        default: return fail(ATO_ERR_UNSUPPORTED, "KKT tiles");
    }
#undef ATO_CALL
}

// Fronts of one level are independent: with more than one class the first class runs on the
// caller's stream and the others on the handle's side stream (fork / join through events), so a
// class of a few fronts overlaps the large one instead of trailing it.
int factor_level(ato_kkt* h, const Plan& P, const Vals& V, int l, int batch, const int* list, int* inertia,
                 hipStream_t st) {
    const std::vector<ato_kkt::Seg>& sg = h->segs[l];
    const int nfl = h->level_ptr[l + 1] - h->level_ptr[l];
    // few workgroups (small batches): one launch at the level's tile count -- the level's time is
    // one front's latency, which a second launch and the stream fork / join only add to
    // (the kernel variant never changes the factors)
    if (sg.size() > 1 && (long long)nfl * batch < 4 * CUS && !h->level_sad[l])
        return launch_segment(h, P, V, ato_kkt::Seg{h->level_ptr[l], nfl, h->level_tiles[l]}, batch, list, inertia, st);
    if (sg.size() == 1) return launch_segment(h, P, V, sg[0], batch, list, inertia, st);
    if (!h->side) {
        // created on the handle's device, whatever device is current on the calling thread
        int cur = 0;
        KKT_HIP(hipGetDevice(&cur));
        if (cur != h->device) KKT_HIP(hipSetDevice(h->device));
        const hipError_t e1 = hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking);
        const hipError_t e2 = e1 == hipSuccess ? hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) : e1;
        const hipError_t e3 = e2 == hipSuccess ? hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) : e2;
        if (cur != h->device) KKT_HIP(hipSetDevice(cur));
        KKT_HIP(e3);
    }
    KKT_HIP(hipEventRecord(h->ev_fork, st));
    KKT_HIP(hipStreamWaitEvent(h->side, h->ev_fork, 0));
    for (size_t i = 1; i < sg.size(); ++i) {
        const int rc = launch_segment(h, P, V, sg[i], batch, list, inertia, h->side);
        if (rc != ATO_OK) return rc;
    }
    const int rc = launch_segment(h, P, V, sg[0], batch, list, inertia, st);
    if (rc != ATO_OK) return rc;
    KKT_HIP(hipEventRecord(h->ev_join, h->side));
    KKT_HIP(hipStreamWaitEvent(st, h->ev_join, 0));
    return ATO_OK;
}

int solve_level(const ato_kkt* h, const Plan& P, int l, bool fwd, int batch, const int* list, double* x,
                long long se, long long sb, hipStream_t st) {
    const int f0 = h->level_ptr[l], nf = h->level_ptr[l + 1] - f0;
#define ATO_CALL(T_) (fwd ? launch_fwd_level<T_>(h, P, f0, nf, batch, list, x, se, sb, st) \
                          : launch_bwd_level<T_>(h, P, f0, nf, batch, list, x, se, sb, st))
    switch (h->level_tiles[l]) {
        case 1: return ATO_CALL(1);
        case 2: return ATO_CALL(2);
        case 3: return ATO_CALL(3);
        case 4: return ATO_CALL(4);
        case 5: return ATO_CALL(5);
        case 6: return ATO_CALL(6);
        case 7: return ATO_CALL(7);
        case 8: return ATO_CALL(8);
        case 9: return ATO_CALL(9);
        default: return fail(ATO_ERR_UNSUPPORTED, "KKT tiles");
    }
#undef ATO_CALL
}

Plan make_plan(const ato_kkt* h) {
    Plan P;
    P.n = h->n;
    P.m = h->m;
    P.dim = h->dim;
    P.F = h->F;
    P.pos_ptr = h->d_pos_ptr;
    P.n_own = h->d_n_own;
    P.pos_index = h->d_pos_index;
    P.parent_pos = h->d_parent_pos;
    P.child_ptr = h->d_child_ptr;
    P.child_list = h->d_child_list;
    P.ent_ptr = h->d_ent_ptr;
    P.ent_pos = h->d_ent_pos;
    P.ent_src = reinterpret_cast<const int2*>(h->d_ent_src);
    P.l_off = reinterpret_cast<const long long*>(h->d_l_off);
    P.piv_off = h->d_piv_off;
    P.cb_off = reinterpret_cast<const long long*>(h->d_cb_off);
    P.sc_off = h->d_sc_off;
    P.forder = h->d_forder;
    P.n_sad = h->d_n_sad;
    P.cap = h->cap;
    P.sad_txy = reinterpret_cast<const int2*>(h->d_sad_txy);
    P.l_size = h->l_size;
    P.cb_size = h->cb_size;
    P.sc_size = h->sc_size;
    P.sad_tau = h->sad_tau;
    return P;
}

template <class V>
int upload(const V* host, size_t n, V** dev) {
    *dev = nullptr;
    if (n == 0) return ATO_OK;
    KKT_HIP(hipMalloc((void**)dev, n * sizeof(V)));
    KKT_HIP(hipMemcpy(*dev, host, n * sizeof(V), hipMemcpyHostToDevice));
    return ATO_OK;
}

void free_storage(ato_kkt* h) {
    for (void* p : {(void*)h->d_L, (void*)h->d_cb, (void*)h->d_sc, (void*)h->d_piv, (void*)h->d_dinv,
                    (void*)h->d_sinfo, (void*)h->d_spec})
        (void)hipFree(p);
    h->d_spec = nullptr;
    h->d_L = nullptr;
    h->d_cb = nullptr;
    h->d_sc = nullptr;
    h->d_piv = nullptr;
    h->d_dinv = nullptr;
    h->d_sinfo = nullptr;
    h->cap = 0;
}

}  // namespace

extern "C" {

#ifdef ATO_KKT_STAMPS
int ato_kkt_diag_stamps(unsigned long long* out) {
    KKT_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kkt_stamps), sizeof(unsigned long long) * 16));
    return ATO_OK;
}
#endif

static int kkt_create_impl(const ato_kkt_plan_desc* d, ato_kkt** out);

// host exceptions of the plan set-up must not cross the C ABI (std::terminate would abort the process)
int ato_kkt_create(const ato_kkt_plan_desc* d, ato_kkt** out) {
    try {
        return kkt_create_impl(d, out);
    } catch (const std::exception& e) {
        return fail(ATO_ERR_ARG, std::string("host exception: ") + e.what());
    } catch (...) {
        return fail(ATO_ERR_ARG, "host exception");
    }
}

static int kkt_create_impl(const ato_kkt_plan_desc* d, ato_kkt** out) {
    if (!d || !out) return fail(ATO_ERR_ARG, "null argument");
    *out = nullptr;
    if (d->n_fronts < 1 || d->n_levels < 1 || d->n < 0 || d->m < 0) return fail(ATO_ERR_ARG, "bad KKT plan sizes");
    const int F = d->n_fronts, L = d->n_levels;
    if (d->level_ptr[0] != 0 || d->level_ptr[L] != F) return fail(ATO_ERR_ARG, "KKT plan: levels do not cover the fronts");
    ato_kkt* h = new ato_kkt();
    if (hipGetDevice(&h->device) != hipSuccess) {
        delete h;
        return fail(ATO_ERR_HIP, "hipGetDevice failed");
    }
    h->n = d->n;
    h->m = d->m;
    h->dim = d->n + d->m;
    h->F = F;
    h->L = L;
    h->l_size = d->l_size;
    h->cb_size = d->cb_size;
    h->sc_size = d->sc_size;
    h->level_ptr.assign(d->level_ptr, d->level_ptr + L + 1);
    h->level_tiles.assign(d->level_tiles, d->level_tiles + L);
    const int P = d->pos_ptr[F];
    const int E = d->ent_ptr[F * MAXT];
    const int C = d->child_ptr[F];
    int own_total = 0;
    for (int l = 0; l < L; ++l) {
        const int T = d->level_tiles[l];
        if (T < 1 || T > MAX_FRONT_TILES) {
            delete h;
            return fail(ATO_ERR_UNSUPPORTED, "KKT fronts wider than 288 positions");
        }
        for (int f = d->level_ptr[l]; f < d->level_ptr[l + 1]; ++f) {
            const int A = d->pos_ptr[f + 1] - d->pos_ptr[f];
            const int es = d->ent_ptr[(f + 1) * MAXT] - d->ent_ptr[f * MAXT];
            h->max_ent = std::max(h->max_ent, es);
            own_total += d->n_own[f];
            bool children_below = true;
            for (int c = d->child_ptr[f]; c < d->child_ptr[f + 1]; ++c)
                children_below = children_below && d->child_list[c] < d->level_ptr[l];
            if (A > 32 * T || d->n_own[f] > A || !children_below) {
                delete h;
                return fail(ATO_ERR_ARG, "KKT plan: front larger than its level's tiles, or a child not below it");
            }
            for (int q = d->n_own[f]; q < A; ++q) {
                const int pp = d->parent_pos[d->pos_ptr[f] + q];
                if (pp < 0 || pp >= 32 * MAX_FRONT_TILES) {
                    delete h;
                    return fail(ATO_ERR_ARG, "KKT plan: trailing position without a parent position");
                }
            }
        }
    }
    if (own_total != h->dim) {
        delete h;
        return fail(ATO_ERR_ARG, "KKT plan: own positions do not cover the KKT dimension");
    }
    // factor launch order: the fronts of every level grouped by kernel class, larger classes first
    // (ATO_KKT_SPLIT=0: one launch per level at the level's tile count; ATO_KKT_S16=0: no
    // 16-wide-tile class), each group in plan order
    {
        if (const char* e_tau = getenv("ATO_KKT_SADDLE_TAU")) h->sad_tau = atof(e_tau);
        const char* e_split = getenv("ATO_KKT_SPLIT");
        const char* e_s16 = getenv("ATO_KKT_S16");
        const bool split = !(e_split && e_split[0] == '0');
        const bool s16 = split && !(e_s16 && e_s16[0] == '0');
        std::vector<int32_t> order;
        order.reserve(F);
        h->segs.assign(L, {});
        h->level_sad.assign(L, 0);
        // saddle fronts the kernel takes: own = 2 nS <= 128, no children, blocks within the LDS;
        // any other front the plan marks is factorised by Bunch-Kaufman like the rest
        std::vector<int32_t> nsad(F, 0), txy(2 * (size_t)F, 0);
        bool any_sad = false;
        for (int f = 0; f < F && d->n_sad; ++f) {
            const int nS = d->n_sad[f], A = d->pos_ptr[f + 1] - d->pos_ptr[f], T = A - 2 * nS;
            if (nS <= 0 || nS > 64 || d->n_own[f] != 2 * nS || d->child_ptr[f + 1] != d->child_ptr[f]) continue;
            // trailing rows coupled to X end at tx, those coupled to Y start at T - ty (the plan orders them)
            int tx = 0, ty = 0;
            for (int e = d->ent_ptr[f * MAXT]; e < d->ent_ptr[(f + 1) * MAXT]; ++e) {
                const int pa = d->ent_pos[e] >> 16, pb = d->ent_pos[e] & 0xffff;
                if (pa < 2 * nS) continue;
                if (pb < nS) tx = std::max(tx, pa - 2 * nS + 1);
                else if (pb < 2 * nS) ty = std::max(ty, T - (pa - 2 * nS));
            }
            if (sad_lds_bytes(nS, tx, ty) <= 160 * 1024) {
                nsad[f] = nS;
                txy[2 * f] = tx;
                txy[2 * f + 1] = ty;
                any_sad = true;
            }
        }
        auto is_sad = [&](int f) { return nsad[f] > 0; };
        for (int l = 0; l < L; ++l) {
            std::vector<std::pair<int, int>> fc;   // (-class, front)
            for (int f = d->level_ptr[l]; f < d->level_ptr[l + 1]; ++f)
                fc.push_back({is_sad(f) ? -SADDLE_CLS
                                        : split ? -front_class(d->pos_ptr[f + 1] - d->pos_ptr[f], s16) : -d->level_tiles[l], f});
            std::stable_sort(fc.begin(), fc.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
            for (size_t i = 0; i < fc.size(); ++i) {
                if (i == 0 || fc[i].first != fc[i - 1].first)
                    h->segs[l].push_back({(int)order.size(), 0, -fc[i].first});
                ato_kkt::Seg& sg = h->segs[l].back();
                ++sg.count;
                order.push_back(fc[i].second);
                if (sg.cls == SADDLE_CLS) {
                    const int f = fc[i].second;
                    const int A = d->pos_ptr[f + 1] - d->pos_ptr[f], nS = nsad[f];
                    h->level_sad[l] = 1;
                    sg.nsm = std::max(sg.nsm, nS <= 32 ? 32 : nS <= 48 ? 48 : nS <= 56 ? 56 : 64);
                    sg.cls2 = std::max(sg.cls2, front_class(A, false));
                    (void)A;
                    sg.lds = std::max(sg.lds, sad_lds_bytes(nS, txy[2 * f], txy[2 * f + 1]));
                }
            }
        }
        if (any_sad) {
            int rc = upload(nsad.data(), nsad.size(), &h->d_n_sad);
            if (rc == ATO_OK) rc = upload(txy.data(), txy.size(), &h->d_sad_txy);
            if (rc != ATO_OK) {
                ato_kkt_destroy(h);
                return rc;
            }
        }
        if (int rc = upload(order.data(), order.size(), &h->d_forder)) {
            ato_kkt_destroy(h);
            return rc;
        }
    }
    if (h->max_ent > EPT * FT) {
        delete h;
        return fail(ATO_ERR_UNSUPPORTED, "KKT plan: more than 4096 entries in one front");
    }
    int rc = ATO_OK;
    if ((rc = upload(d->pos_ptr, F + 1, &h->d_pos_ptr)) || (rc = upload(d->n_own, F, &h->d_n_own)) ||
        (rc = upload(d->pos_index, P, &h->d_pos_index)) || (rc = upload(d->parent_pos, P, &h->d_parent_pos)) ||
        (rc = upload(d->child_ptr, F + 1, &h->d_child_ptr)) || (rc = upload(d->child_list, C, &h->d_child_list)) ||
        (rc = upload(d->ent_ptr, F * MAXT + 1, &h->d_ent_ptr)) || (rc = upload(d->ent_pos, E, &h->d_ent_pos)) ||
        (rc = upload(d->ent_src, 2 * (size_t)E, &h->d_ent_src)) || (rc = upload(d->piv_off, F, &h->d_piv_off)) ||
        (rc = upload(d->l_off, F, &h->d_l_off)) || (rc = upload(d->cb_off, F, &h->d_cb_off)) ||
        (rc = upload(d->sc_off, F, &h->d_sc_off)) || (rc = upload(d->kres_ptr, h->dim + 1, &h->d_kres_ptr)) ||
        (rc = upload(d->kres_col, (size_t)d->kres_ptr[h->dim], &h->d_kres_col)) ||
        (rc = upload(d->kres_src, (size_t)d->kres_ptr[h->dim], &h->d_kres_src))) {
        ato_kkt_destroy(h);
        return rc;
    }
    *out = h;
    return ATO_OK;
}

int ato_kkt_destroy(ato_kkt* h) {
    if (!h) return ATO_OK;
    if (h->side) {
        (void)hipStreamSynchronize(h->side);
        (void)hipStreamDestroy(h->side);
        (void)hipEventDestroy(h->ev_fork);
        (void)hipEventDestroy(h->ev_join);
    }
    free_storage(h);
    for (void* p : {(void*)h->d_pos_ptr, (void*)h->d_n_own, (void*)h->d_pos_index, (void*)h->d_parent_pos,
                    (void*)h->d_child_ptr, (void*)h->d_child_list, (void*)h->d_ent_ptr, (void*)h->d_ent_pos,
                    (void*)h->d_ent_src, (void*)h->d_piv_off, (void*)h->d_l_off, (void*)h->d_cb_off,
                    (void*)h->d_sc_off, (void*)h->d_kres_ptr, (void*)h->d_kres_col, (void*)h->d_kres_src,
                    (void*)h->d_forder, (void*)h->d_n_sad, (void*)h->d_sad_txy})
        (void)hipFree(p);
    delete h;
    return ATO_OK;
}

int ato_kkt_reserve(ato_kkt* h, int32_t max_batch) {
    if (!h || max_batch < 0) return fail(ATO_ERR_ARG, "bad argument");
    if (max_batch <= h->cap) return ATO_OK;
    if (h->d_L) KKT_HIP(hipDeviceSynchronize());    // queued factor / solve kernels may still use the old storage
    free_storage(h);
    // transactional: either every buffer of the new capacity is allocated, or none is kept and the
    // handle is left without storage (d_L == nullptr, cap == 0), which factor / solve refuse. (A
    // failure part-way through used to leave d_L set with later buffers null and cap 0, which a
    // listed factorisation did not catch.)
    const size_t B = (size_t)max_batch;
    const size_t bytes[7] = {sizeof(double) * std::max<size_t>(1, (size_t)h->l_size * B),
                             sizeof(double) * std::max<size_t>(1, (size_t)h->cb_size * B),
                             sizeof(double) * std::max<size_t>(1, (size_t)h->sc_size * B),
                             sizeof(int2) * std::max<size_t>(1, (size_t)h->dim * B),
                             sizeof(double) * 3 * std::max<size_t>(1, (size_t)h->dim * B),
                             sizeof(int2) * std::max<size_t>(1, (size_t)h->F * B),
                             sizeof(int32_t) * std::max<size_t>(1, (size_t)h->dim * B)};
    void* p[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    hipError_t e = hipSuccess;
    for (int i = 0; i < 7 && e == hipSuccess; ++i) e = hipMalloc(&p[i], bytes[i]);
    if (e == hipSuccess) e = hipMemset(p[6], 0xFF, bytes[6]);     // -1: no guess
    if (e != hipSuccess) {
        for (void* q : p) (void)hipFree(q);
        (void)hipGetLastError();
        return fail(ATO_ERR_HIP, std::string("ato_kkt_reserve: ") + hipGetErrorString(e) + " (" +
                                     std::to_string(max_batch) + " instances; the handle keeps no storage)");
    }
    h->d_L = static_cast<double*>(p[0]);
    h->d_cb = static_cast<double*>(p[1]);
    h->d_sc = static_cast<double*>(p[2]);
    h->d_piv = static_cast<int2*>(p[3]);
    h->d_dinv = static_cast<double*>(p[4]);
    h->d_sinfo = static_cast<int2*>(p[5]);
    h->d_spec = static_cast<int32_t*>(p[6]);
    h->cap = max_batch;
    return ATO_OK;
}

int ato_kkt_factor(ato_kkt* h, int32_t batch, const int32_t* list, int64_t se, int64_t sb, const double* H,
                   const double* J, const double* dx, const double* dr, int32_t* inertia, void* stream) {
    if (!h || !inertia || batch < 0) return fail(ATO_ERR_ARG, "bad argument");
    if (batch == 0) return ATO_OK;
    if (!h->d_L || h->cap == 0) return fail(ATO_ERR_STATE, "call ato_kkt_reserve() first");
    if (batch > h->cap) return fail(ATO_ERR_STATE, "ato_kkt_reserve() too small for this batch");
    if (batch > 65535) return fail(ATO_ERR_UNSUPPORTED, "KKT batch above 65535 instances per call");
    const Plan P = make_plan(h);
    const Vals V{H, J, dx, dr, se, sb};
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_inertia_zero, dim3((batch + 255) / 256), dim3(256), 0, st, batch, h->cap, list, inertia);
    KKT_HIP(hipGetLastError());
    for (int l = 0; l < h->L; ++l) {
        const int rc = factor_level(h, P, V, l, batch, list, inertia, st);
        if (rc != ATO_OK) return rc;
    }
    return ATO_OK;
}

int ato_kkt_solve(ato_kkt* h, int32_t batch, const int32_t* list, int64_t se, int64_t sb, double* x,
                  void* stream) {
    if (!h || !x || batch < 0) return fail(ATO_ERR_ARG, "bad argument");
    if (batch == 0) return ATO_OK;
    if (!h->d_L || h->cap == 0) return fail(ATO_ERR_STATE, "call ato_kkt_reserve() first");
    if (batch > h->cap) return fail(ATO_ERR_STATE, "ato_kkt_reserve() too small for this batch");
    if (batch > 65535) return fail(ATO_ERR_UNSUPPORTED, "KKT batch above 65535 instances per call");
    const Plan P = make_plan(h);
    hipStream_t st = static_cast<hipStream_t>(stream);
    for (int l = 0; l < h->L; ++l) {
        const int rc = solve_level(h, P, l, true, batch, list, x, se, sb, st);
        if (rc != ATO_OK) return rc;
    }
    for (int l = h->L - 1; l >= 0; --l) {
        const int rc = solve_level(h, P, l, false, batch, list, x, se, sb, st);
        if (rc != ATO_OK) return rc;
    }
    return ATO_OK;
}

int ato_kkt_residual(ato_kkt* h, int32_t batch, int64_t se, int64_t sb, const double* H, const double* J,
                     const double* dx, const double* dr, const double* x, const double* rhs, double* out,
                     void* stream) {
    if (!h || !x || !rhs || !out || !J || !dx || !dr || batch < 0) return fail(ATO_ERR_ARG, "bad argument");
    if (batch == 0) return ATO_OK;
    if (h->dim > 4 * 65535) return fail(ATO_ERR_UNSUPPORTED, "KKT residual: dimension above 262140");
    const Vals V{H, J, dx, dr, se, sb};
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_kkt_residual, dim3((batch + 63) / 64, (h->dim + 3) / 4), dim3(256), 0, st, h->dim, batch,
                       nullptr, h->d_kres_ptr, h->d_kres_col, h->d_kres_src, V, x, rhs, out);
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

int ato_kkt_residual_list(ato_kkt* h, int32_t count, const int32_t* list, int64_t se, int64_t sb, const double* H,
                          const double* J, const double* dx, const double* dr, const double* x, const double* rhs,
                          double* out, void* stream) {
    if (!list) return ato_kkt_residual(h, count, se, sb, H, J, dx, dr, x, rhs, out, stream);
    if (!h || !x || !rhs || !out || !J || !dx || !dr || count < 0) return fail(ATO_ERR_ARG, "bad argument");
    if (count == 0) return ATO_OK;
    if (h->dim > 4 * 65535) return fail(ATO_ERR_UNSUPPORTED, "KKT residual: dimension above 262140");
    const Vals V{H, J, dx, dr, se, sb};
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_kkt_residual, dim3((count + 63) / 64, (h->dim + 3) / 4), dim3(256), 0, st, h->dim, count,
                       list, h->d_kres_ptr, h->d_kres_col, h->d_kres_src, V, x, rhs, out);
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

}  // extern "C"
