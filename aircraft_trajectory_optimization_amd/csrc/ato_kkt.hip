// ato_kkt.hip -- batched staged LDL^T factorisation and solve of the interior-point KKT system
// (include/ato_kkt.h). Replaces IPOPT's MUMPS / MA97 factorisation (ref:
// drone3d/raceline/base_raceline.py:752-799, the `ipopt_time` of :182-189) for a batch of
// independent instances; the plan tables come from solver/kkt_plan.py.
//
// Factor (k_kkt_factor<T>): one 512-thread workgroup per instance walks the stages. The
// augmented block of a stage (<= 32*T positions) lives in REGISTERS: thread (ti, tj) = (tid % 32,
// tid / 32) holds A[32 I + ti][32 J + tj] and A[32 I + ti][32 J + 16 + tj] for every lower tile
// J <= I (T(T+1) doubles; 2 waves per SIMD leave 256 VGPRs per lane).
// Assembly goes through a 32-row LDS strip per tile row (entries scattered from the H / J /
// diagonal arrays, plus the Schur complement carried from the previous stage). Own positions
// are then eliminated by Bunch-Kaufman pivoting (1x1 or 2x2; candidates and the pivot search
// restricted to own positions): the pivot column(s) are copied to LDS by their owners, every
// wave reduces the same max / argmax, and every thread applies the rank-1 / rank-2 update to
// its tiles (tiles without live rows are skipped). The factor columns are written compactly
// (live positions only, physical order) into one contiguous stream per instance, with a pivot
// record and the inverse pivot block per step. The trailing block (next stage's coupling rows +
// border) goes to LDS and is added into the next stage's assembly.
//
// Solve (k_kkt_solve<T>): one 256-thread workgroup per instance. Wave 0 runs the forward
// (L y = b), D and backward (L^T x = z) sweeps with the stage vector in registers (4 positions
// per lane); all four waves stream the factor columns through a two-slot LDS ring so that
// the sweep reads LDS only.
#include <hip/hip_runtime.h>
#include <string>
#include <vector>
#include <cstdint>
#include "../../include/ato_kkt.h"
#include "../../include/ato.h"

void ato_internal_set_error(const std::string& msg);   // ato_capi.hip: ato_last_error()

struct ato_kkt {
    int n = 0, m = 0, dim = 0, S = 0, T = 0, max_tq = 0, max_ent = 0;
    int64_t l_size = 0;
    int32_t *d_stage_ptr = nullptr, *d_n_own = nullptr, *d_pos_index = nullptr, *d_carry_dst = nullptr;
    int32_t *d_ent_ptr = nullptr, *d_ent_pos = nullptr, *d_ent_src = nullptr, *d_piv_off = nullptr;
    int32_t cap = 0;                 // instances with factor storage
    double* d_L = nullptr;           // [cap][l_size]
    int2* d_piv = nullptr;           // [cap][dim] {p | type << 16, r}
    double* d_dinv = nullptr;        // [cap][dim][3]
    int2* d_sinfo = nullptr;         // [cap][S+1] {steps, stream offset of the stage}; [S] = {total, 0}
};

#ifdef ATO_KKT_STAMPS
// DIAGNOSTIC build only (tools/diag/kkt_stamps.py): shader-clock phase totals of block 0
__device__ unsigned long long g_kkt_stamps[16];
#endif

namespace {

#ifdef ATO_KKT_STAMPS
__device__ __forceinline__ unsigned long long kstamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define KST_DECL unsigned long long kst_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, kst_last = kstamp(); \
    const bool kst_on = blockIdx.x == 0;
#define KST(i) do { if (kst_on) { const unsigned long long t_ = kstamp(); kst_acc[i] += t_ - kst_last; kst_last = t_; } } while (0)
#define KST_DUMP(nsteps) do { if (kst_on && threadIdx.x == 0) { for (int i_ = 0; i_ < 8; ++i_) g_kkt_stamps[i_] = kst_acc[i_]; g_kkt_stamps[8] = (nsteps); } } while (0)
#define KST_DUMP2(nsteps) do { if (kst_on && threadIdx.x == 0) { for (int i_ = 0; i_ < 4; ++i_) g_kkt_stamps[10 + i_] = kst_acc[i_]; g_kkt_stamps[14] = (nsteps); } } while (0)
#else
#define KST_DECL
#define KST(i)
#define KST_DUMP(nsteps)
#define KST_DUMP2(nsteps)
#endif

int fail(int code, const std::string& m) {
    ato_internal_set_error(m);
    return code;
}

#define KKT_HIP(call)                                                                               \
    do {                                                                                            \
        hipError_t e_ = (call);                                                                     \
        if (e_ != hipSuccess) return fail(ATO_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int FT = 512;                   // factor threads per instance (16 x 32 grid)
constexpr int ST = 256;                   // solve threads per instance
constexpr int EPT = 8;                    // entries per thread and stage (<= 4096 per stage)
constexpr int CH = 4096;                  // doubles per ring chunk of the solve (2 x 32 KB LDS ring)
constexpr int CPT = CH / ST;              // chunk doubles per thread
constexpr double BK_ALPHA = 0.64038820320220756872767623199676;   // (1 + sqrt(17)) / 8
constexpr int SRC_SHIFT = 29;

struct Plan {
    int n, m, dim, S, max_tq;
    const int* stage_ptr;
    const int* n_own;
    const int* pos_index;
    const int* carry_dst;
    const int* ent_ptr;
    const int* ent_pos;
    const int2* ent_src;
    const int* piv_off;
    long long l_size;
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
    __device__ __forceinline__ void set(int i) {
#pragma unroll
        for (int k = 0; k < NW; ++k) w[k] |= (((i >> 6) == k) ? 1ull : 0ull) << (i & 63);
    }
    __device__ __forceinline__ int count() const {
        int c = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) c += __popcll(w[k]);
        return c;
    }
    // live positions strictly below i
    __device__ __forceinline__ int below(int i) const {
        int c = 0;
        const int wi = i >> 6;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            if (k < wi) c += __popcll(w[k]);
            else if (k == wi) c += __popcll(w[k] & ((1ull << (i & 63)) - 1ull));
        }
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

// LDS-only workgroup barrier: waits for this wave's LDS operations, not for its global stores
// (the factor columns written every step are read only by the solve launch)
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

__device__ __forceinline__ double uni(double v) {   // wave-uniform copy (SGPRs)
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
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

// rows 32I + ti (I < T) of a column held as v[q] = c[lane + 64q]: lanes 0-31 of v[q] hold tile 2q,
// lanes 32-63 tile 2q + 1, and a self v_permlane32_swap broadcasts each half to the whole wave
// (no LDS round trip for the row factors of the Schur update)
template <int T, int NQ>
__device__ __forceinline__ void column_rows(const double (&v)[NQ], double (&x)[T]) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const uint2 u = __builtin_bit_cast(uint2, v[q]);
        const auto lo = __builtin_amdgcn_permlane32_swap(u.x, u.x, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(u.y, u.y, false, false);
        if (2 * q < T) x[2 * q] = __builtin_bit_cast(double, make_uint2(lo[0], hi[0]));
        if (2 * q + 1 < T) x[2 * q + 1] = __builtin_bit_cast(double, make_uint2(lo[1], hi[1]));
    }
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

// ------------------------------------------------------------------------------------------
// factorisation
// ------------------------------------------------------------------------------------------
// column k of the block into c[0 .. 32T): thread (ti, tj) owns rows 32I+ti and columns 32J+tj,
// 32J+16+tj of every lower tile (I, J)
template <int T>
__device__ __forceinline__ void extract_column(const double (&a)[T * (T + 1) / 2][2], int k, int ti, int tj,
                                               double* __restrict__ c) {
    const int K = k >> 5, kk = k & 31, kt = k & 15;
    const unsigned long long hm = (k & 16) ? ~0ull : 0ull;
#pragma unroll
    for (int KK = 0; KK < T; ++KK) {
        if (K == KK) {
            if (tj == kt) {
#pragma unroll
                for (int I = KK; I < T; ++I) c[32 * I + ti] = blend(a[slot(I, KK)][0], a[slot(I, KK)][1], hm);
            }
            if (ti == kk) {
#pragma unroll
                for (int J = 0; J < KK; ++J) {
                    c[32 * J + tj] = a[slot(KK, J)][0];
                    c[32 * J + 16 + tj] = a[slot(KK, J)][1];
                }
            }
        }
    }
}

template <int T>
__global__ __launch_bounds__(FT) void k_kkt_factor(Plan P, Vals V, int batch, const int* __restrict__ list,
                                                   double* __restrict__ Lst, int2* __restrict__ piv,
                                                   double* __restrict__ dinv, int2* __restrict__ sinfo,
                                                   int* __restrict__ inertia) {
    constexpr int NP = 32 * T;
    constexpr int NW = (NP + 63) / 64;
    constexpr int NQ = (NP + 63) / 64;
    constexpr int NS = T * (T + 1) / 2;
    constexpr int SR = NP + 1;                   // strip row stride (odd: conflict-free reads)
    extern __shared__ double smem[];
    double* strip = smem;                        // [32][SR]
    double* colb = strip + 32 * SR;              // [2 parity][2 (k, r)][NP]
    double* carry = colb + 4 * NP;               // [max_tq][max_tq]
    int* cdst = reinterpret_cast<int*>(carry + P.max_tq * P.max_tq);   // [max_tq]

    const int bi = blockIdx.x;
    if (bi >= batch) return;
    const int b = list ? __builtin_amdgcn_readfirstlane(list[bi]) : bi;
    const int tid = threadIdx.x;
    const int ti = tid & 31, tj = tid >> 5;
    const int lane = tid & 63;

    double a[NS][2];
    double* Lb = Lst + (long long)b * P.l_size;
    int2* pv = piv + (long long)b * P.dim;
    double* dv = dinv + (long long)b * P.dim * 3;
    int npos = 0, nneg = 0, nzero = 0;
    long long loff = 0;                          // running offset in the instance's column stream
    int tq_in = 0;
    int kst_steps = 0;
    KST_DECL

    for (int s = 0; s < P.S; ++s) {
        const int p0 = P.stage_ptr[s];
        const int A = P.stage_ptr[s + 1] - p0;
        const int own = P.n_own[s];
        // ---- this stage's entries (positions and values) into registers
        const int e0 = P.ent_ptr[s * T], e1 = P.ent_ptr[(s + 1) * T];
        int epos[EPT];
        double eval[EPT];
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
        // ---- assemble strip by strip
#pragma unroll
        for (int I = 0; I < T; ++I) {
            if (32 * I < A) {
                for (int i = tid; i < 32 * SR; i += FT) strip[i] = 0.0;
                __syncthreads();
#pragma unroll
                for (int q = 0; q < EPT; ++q) {
                    const int pa = epos[q] >> 16, pb = epos[q] & 0xffff;
                    if (epos[q] >= 0 && (pa >> 5) == I) {
                        strip[(pa & 31) * SR + pb] = eval[q];
                        if ((pb >> 5) == I && pa != pb) strip[(pb & 31) * SR + pa] = eval[q];
                    }
                }
                __syncthreads();
                // carry-in: Schur complement of the previous stage (full symmetric tq x tq)
                for (int e = tid; e < tq_in * tq_in; e += FT) {
                    const int q1 = e / tq_in, q2 = e - q1 * tq_in;
                    const int d1 = cdst[q1], d2 = cdst[q2];
                    if ((d1 >> 5) == I) strip[(d1 & 31) * SR + d2] += carry[q1 * P.max_tq + q2];
                }
                __syncthreads();
#pragma unroll
                for (int J = 0; J <= I; ++J) {
                    a[slot(I, J)][0] = strip[ti * SR + 32 * J + tj];
                    a[slot(I, J)][1] = strip[ti * SR + 32 * J + 16 + tj];
                }
                __syncthreads();
            } else {
#pragma unroll
                for (int J = 0; J <= I; ++J) a[slot(I, J)][0] = a[slot(I, J)][1] = 0.0;
            }
        }
        KST(0);     // assembly
        // ---- restricted Bunch-Kaufman elimination of the own positions (all decisions scalar)
        Mask<NW> live;                // scalar copy: candidate scan, tile skipping
        live.set_range(0, A);
        bool lvq[NQ];                 // per lane: position lane + 64 q live
#pragma unroll
        for (int q = 0; q < NQ; ++q) lvq[q] = lane + 64 * q < A;
        bool lvt = tid < A;           // per thread: its factor-column position tid live ...
        int cit = tid;                // ... and its index among the live positions
        int kc = 0, steps = 0, par = 0;
        const int g0 = P.piv_off[s];
        const long long lstart = loff;
        while (true) {
            while (kc < own && !live.get(kc)) ++kc;
            if (kc >= own) break;
            const int k = kc;
            double* ck = colb + (par * 2 + 0) * NP;
            double* cr = colb + (par * 2 + 1) * NP;
            KST(7);
            extract_column<T>(a, k, ti, tj, ck);
            lds_barrier();
            KST(1);     // extract + barrier
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
                extract_column<T>(a, r, ti, tj, cr);
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
            KST(2);     // pivot search
            // ---- pivot record, inertia, factor columns, Schur update
            double i00 = 0.0, i01 = 0.0, i11 = 0.0;
            if (type == 2) {
                live.clear(k);
                ++nzero;
            } else if (type == 0) {
                const double d = use_r ? arr : akk;
                i00 = 1.0 / d;
                live.clear(p);
                if (d > 0.0) ++npos; else ++nneg;
            } else {
                const double A00 = akk, A01 = lane_pick<NQ>(cv, r), A11 = arr;
                const double det = A00 * A11 - A01 * A01;
                const double rdet = 1.0 / det;
                i00 = A11 * rdet;
                i01 = -A01 * rdet;
                i11 = A00 * rdet;
                live.clear(k);
                live.clear(r);
                if (det < 0.0) { ++npos; ++nneg; }
                else if (A00 + A11 > 0.0) npos += 2;
                else nneg += 2;
            }
            const int nlive = live.count();
            const int ncol = type == 1 ? 2 : 1;
            {
                const int e1 = type == 1 ? k : (type == 2 ? k : p);
                const int e2 = type == 1 ? r : -1;
                lvt = lvt && tid != e1 && tid != e2;
                cit -= (tid > e1 ? 1 : 0) + (e2 >= 0 && tid > e2 ? 1 : 0);
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int i = lane + 64 * q;
                    lvq[q] = lvq[q] && i != e1 && i != e2;
                }
            }
            if (tid == 0) {
                pv[g0 + steps] = make_int2((type == 1 ? k : p) | (type << 16), type == 1 ? r : -1);
                dv[3 * (g0 + steps) + 0] = i00;
                dv[3 * (g0 + steps) + 1] = i01;
                dv[3 * (g0 + steps) + 2] = i11;
            }
            // row factors of the thread's rows 32I + ti: l0 = rows of L's first column, l1 of the
            // second (2x2 pivot); A -= l0 c0^T (+ l1 cr^T), c0 = column p (1x1) or k (2x2)
            double l0[T], l1[T];
            {
                double xk[T], xr[T];
                column_rows<T, NQ>(cv, xk);
                column_rows<T, NQ>(cw, xr);
                if (type == 1) {
#pragma unroll
                    for (int I = 0; I < T; ++I) {
                        l0[I] = xk[I] * i00 + xr[I] * i01;
                        l1[I] = xk[I] * i01 + xr[I] * i11;
                    }
                } else {
#pragma unroll
                    for (int I = 0; I < T; ++I) {
                        l0[I] = (use_r ? xr[I] : xk[I]) * i00;
                        l1[I] = 0.0;
                    }
                }
            }
#ifdef ATO_KKT_EXP_NOSTORE
            if (false) {              // DIAGNOSTIC experiment: no factor-column stores
#else
            if (lvt) {
#endif
                // position tid = row 32 tj + ti of the thread: its factor entries are l0[tj], l1[tj]
                double v0 = l0[0];
#pragma unroll
                for (int I = 1; I < T; ++I) v0 = blend(v0, l0[I], tj == I ? ~0ull : 0ull);
                const int ci = cit;
                if (type == 0) {
                    Lb[loff + ci] = v0;
                } else if (type == 1) {
                    double v1 = l1[0];
#pragma unroll
                    for (int I = 1; I < T; ++I) v1 = blend(v1, l1[I], tj == I ? ~0ull : 0ull);
                    Lb[loff + 2 * ci] = v0;
                    Lb[loff + 2 * ci + 1] = v1;
                } else {
                    Lb[loff + ci] = 0.0;
                }
            }
            loff += (long long)nlive * ncol;
            KST(3);     // record + factor column stores
            // Schur update: one rank-1 pass (1x1 pivot) or two (2x2 pivot); tiles of dead rows are
            // skipped, dead column tiles are updated too (harmless, no per-tile branches)
#ifdef ATO_KKT_EXP_NOUPD
            const int npass = 0;      // DIAGNOSTIC experiment: no Schur update (wrong results)
#else
            const int npass = type == 0 ? 1 : type == 1 ? 2 : 0;
#endif
            for (int pass = 0; pass < npass; ++pass) {
                const double* cc = pass == 1 ? cr : (use_r ? cr : ck);
                double cj[T][2];
#pragma unroll
                for (int J = 0; J < T; ++J) {
                    cj[J][0] = cc[32 * J + tj];
                    cj[J][1] = cc[32 * J + 16 + tj];
                }
                double li[T];
#pragma unroll
                for (int I = 0; I < T; ++I) li[I] = pass == 1 ? l1[I] : l0[I];
#pragma unroll
                for (int I = 0; I < T; ++I) {
                    if (live.any_in_tile(I)) {
#pragma unroll
                        for (int J = 0; J <= I; ++J) {
                            a[slot(I, J)][0] = fma(-li[I], cj[J][0], a[slot(I, J)][0]);
                            a[slot(I, J)][1] = fma(-li[I], cj[J][1], a[slot(I, J)][1]);
                        }
                    }
                }
            }
            ++steps;
            ++kst_steps;
            par ^= 1;
            KST(4);     // Schur update
        }
        if (tid == 0) sinfo[(long long)b * (P.S + 1) + s] = make_int2(steps, (int)lstart);
        // ---- trailing Schur complement -> carry for the next stage
        const int tq = A - own;
        if (s + 1 < P.S) {
#pragma unroll
            for (int I = 0; I < T; ++I) {
#pragma unroll
                for (int J = 0; J <= I; ++J) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int i = 32 * I + ti, j = 32 * J + 16 * h + tj;
                        // diagonal tiles hold both (i, j) and (j, i), which differ by rounding:
                        // only the lower one writes (one writer per carry entry, deterministic)
                        if (i >= own && i < A && j >= own && j < A && (I != J || i >= j)) {
                            carry[(i - own) * P.max_tq + (j - own)] = a[slot(I, J)][h];
                            carry[(j - own) * P.max_tq + (i - own)] = a[slot(I, J)][h];
                        }
                    }
                }
            }
            if (tid < tq) cdst[tid] = P.carry_dst[p0 + own + tid];
            tq_in = tq;
        }
        __syncthreads();
    }
    KST(5);
    KST_DUMP(kst_steps);
    (void)kst_steps;
    if (tid == 0) {
        sinfo[(long long)b * (P.S + 1) + P.S] = make_int2((int)loff, 0);
        inertia[3 * b + 0] = npos;
        inertia[3 * b + 1] = nneg;
        inertia[3 * b + 2] = nzero;
    }
}

// ------------------------------------------------------------------------------------------
// solve
// ------------------------------------------------------------------------------------------
// Stream of factor columns through a two-slot LDS ring. Forward: chunks 0, 1, 2, ... of
// [0, total); backward: the same chunks in reverse. Chunk c lives in slot c & 1.
struct Ring {
    double* buf;           // [2][CH]
    __device__ __forceinline__ double at(long long off) const { return buf[off & (2 * CH - 1)]; }
};

__device__ __forceinline__ void ring_load(const double* __restrict__ src, long long total, long long c,
                                          double (&r)[CPT], int tid) {
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
        const long long o = c * CH + q * ST + tid;
        r[q] = (c >= 0 && o < total) ? src[o] : 0.0;
    }
}

__device__ __forceinline__ void ring_store(double* buf, long long c, const double (&r)[CPT], int tid) {
    double* dst = buf + (c & 1) * CH;
#pragma unroll
    for (int q = 0; q < CPT; ++q) dst[q * ST + tid] = r[q];
}

template <int NQ>
__device__ __forceinline__ double lane_get(const double (&y)[NQ], int p) {
    const int q = p >> 6;
    double v = y[0];
#pragma unroll
    for (int k = 1; k < NQ; ++k) v = blend(v, y[k], q == k ? ~0ull : 0ull);
    return readlane_f64(v, p & 63);
}

template <int NQ>
__device__ __forceinline__ void lane_set(double (&y)[NQ], int p, double v, int lane) {
#pragma unroll
    for (int k = 0; k < NQ; ++k) y[k] = blend(y[k], v, ((p & 63) == lane && (p >> 6) == k) ? ~0ull : 0ull);
}

// wave 0: stage the pivot records and inverse pivot blocks of a stage into LDS
__device__ __forceinline__ void stage_records(const int2* __restrict__ pv, const double* __restrict__ dvp, int g0,
                                              int steps, int lane, int2* s_piv, double* s_dinv) {
    for (int u = lane; u < steps; u += 64) {
        s_piv[u] = pv[g0 + u];
        s_dinv[3 * u + 0] = dvp[3 * (g0 + u) + 0];
        s_dinv[3 * u + 1] = dvp[3 * (g0 + u) + 1];
        s_dinv[3 * u + 2] = dvp[3 * (g0 + u) + 2];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int T>
__global__ __launch_bounds__(ST) void k_kkt_solve(Plan P, int batch, const int* __restrict__ list,
                                                  const double* __restrict__ Lst, const int2* __restrict__ piv,
                                                  const double* __restrict__ dinv, const int2* __restrict__ sinfo,
                                                  double* __restrict__ x, long long se, long long sb) {
    constexpr int NP = 32 * T;
    constexpr int NW = (NP + 63) / 64;
    constexpr int NQ = (NP + 63) / 64;
    __shared__ double ring_buf[2 * CH];
    __shared__ double cvec[2][NP];            // carried trailing values (forward) / stage vector (backward)
    __shared__ int2 s_piv[NP];
    __shared__ double s_dinv[3 * NP];
    __shared__ int s_done;

    const int bi = blockIdx.x;
    if (bi >= batch) return;
    const int b = list ? __builtin_amdgcn_readfirstlane(list[bi]) : bi;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const bool w0 = tid < 64;
    const double* Lb = Lst + (long long)b * P.l_size;
    const int2* pv = piv + (long long)b * P.dim;
    const double* dvp = dinv + (long long)b * P.dim * 3;
    const int2* si = sinfo + (long long)b * (P.S + 1);
    double* xb = x + (long long)b * sb;
    Ring ring{ring_buf};
    double stage_r[CPT];

    const long long total = min((long long)si[P.S].x, P.l_size);
    int kst_steps = 0;
    KST_DECL
    const long long nchunks = (total + CH - 1) / CH;

    // ===================== forward: L y = b, then y <- D^{-1} y per stage =====================
    double y[NQ];
    bool lv[NQ];          // position lane + 64 q live (wave 0)
    int ci[NQ];           // live positions below it (its index in a compact factor column)
    int nlive = 0;
    int s = -1, t = 0, steps = 0, A = 0, own = 0, p0 = 0, g0 = 0;
    int2 rec_nx = make_int2(0, -1);   // pivot record of step t, read one step ahead (off the y chain)
    long long off = 0;
    bool finished = false;
    if (tid == 0) s_done = 0;
    for (int i = tid; i < 2 * NP; i += ST) (&cvec[0][0])[i] = 0.0;
    ring_load(Lb, total, 0, stage_r, tid);
    ring_store(ring.buf, 0, stage_r, tid);
    ring_load(Lb, total, 1, stage_r, tid);
    ring_store(ring.buf, 1, stage_r, tid);
    __syncthreads();
    for (long long c = 0;; ++c) {
        ring_load(Lb, total, c + 2, stage_r, tid);     // in flight while wave 0 sweeps
        if (w0 && !finished) {
            const long long limit = (c + 2) * CH;
            while (true) {
                if (s < 0 || t >= steps) {
                    // ---- close the current stage: D solve, write own, carry trailing
                    if (s >= 0) {
                        for (int u = 0; u < steps; ++u) {
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
                        const int nb = (s + 1) & 1;
#pragma unroll
                        for (int q = 0; q < NQ; ++q) {
                            const int i = lane + 64 * q;
                            if (i < own) xb[(long long)P.pos_index[p0 + i] * se] = y[q];
                        }
                        for (int i = lane; i < NP; i += 64) cvec[nb][i] = 0.0;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                        for (int q = 0; q < NQ; ++q) {
                            const int i = lane + 64 * q;
                            if (i >= own && i < A && s + 1 < P.S) cvec[nb][P.carry_dst[p0 + i]] = y[q];
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                    ++s;
                    if (s >= P.S) {
                        finished = true;
                        break;
                    }
                    // ---- open stage s
                    p0 = P.stage_ptr[s];
                    A = P.stage_ptr[s + 1] - p0;
                    own = P.n_own[s];
                    g0 = P.piv_off[s];
                    const int2 inf = si[s];
                    steps = min(max(inf.x, 0), own);
                    off = inf.y;
                    t = 0;
                    stage_records(pv, dvp, g0, steps, lane, s_piv, s_dinv);
                    rec_nx = s_piv[0];
                    const int cb = s & 1;
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const int i = lane + 64 * q;
                        double v = 0.0;
                        if (i < own) v = xb[(long long)P.pos_index[p0 + i] * se];
                        if (i < A) v += cvec[cb][i];
                        y[q] = v;
                    }
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const int i = lane + 64 * q;
                        lv[q] = i < A;
                        ci[q] = min(i, A);
                    }
                    nlive = A;
                    KST(0);
                    continue;
                }
                const int2 rec = rec_nx;
                const int type = __builtin_amdgcn_readfirstlane(rec.x >> 16);
                const int pp = __builtin_amdgcn_readfirstlane(min(rec.x & 0xffff, NP - 1));
                const int rr = __builtin_amdgcn_readfirstlane(min(max(rec.y, 0), NP - 1));
                const int ncol = type == 1 ? 2 : 1;
                const int nl_after = nlive - ncol;
                if (off + (long long)nl_after * ncol > limit) break;     // column not resident yet
                rec_nx = s_piv[min(t + 1, NP - 1)];
                // branch-free: every lane reads (dead positions read a harmless ring word); all the
                // column reads are issued before y is touched, so one LDS round trip per step
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
                ++kst_steps;
                KST(1);
            }
            if (finished && lane == 0) s_done = 1;
        }
        __syncthreads();
        const bool done = s_done != 0;
        if (done) break;
        ring_store(ring.buf, c + 2, stage_r, tid);
        __syncthreads();
        KST(2);
        if (c + 2 > nchunks + 2) break;               // safety: never loop past the stream
    }
    __syncthreads();

    // ===================== backward: L^T x = z, stages and steps in reverse =====================
    if (tid == 0) s_done = 0;
    const long long clast = nchunks - 1;
    ring_load(Lb, total, clast, stage_r, tid);
    ring_store(ring.buf, clast, stage_r, tid);
    ring_load(Lb, total, clast - 1, stage_r, tid);
    ring_store(ring.buf, clast - 1, stage_r, tid);
    __syncthreads();
    s = P.S;
    t = -1;
    finished = false;
    for (long long c = clast;; --c) {
        ring_load(Lb, total, c - 2, stage_r, tid);
        if (w0 && !finished) {
            const long long lower = (c - 1) * CH;          // chunks c-1 and c are resident
            while (true) {
                if (s >= P.S || t < 0) {
                    if (s < P.S) {
                        // ---- close stage s: write own positions, keep the stage vector for s-1
#pragma unroll
                        for (int q = 0; q < NQ; ++q) {
                            const int i = lane + 64 * q;
                            if (i < own) xb[(long long)P.pos_index[p0 + i] * se] = y[q];
                            if (i < A) cvec[s & 1][i] = y[q];
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                    --s;
                    if (s < 0) {
                        finished = true;
                        break;
                    }
                    p0 = P.stage_ptr[s];
                    A = P.stage_ptr[s + 1] - p0;
                    own = P.n_own[s];
                    g0 = P.piv_off[s];
                    const int2 inf = si[s];
                    steps = min(max(inf.x, 0), own);
                    off = s + 1 < P.S ? (long long)si[s + 1].y : total;   // stream end of this stage
                    t = steps - 1;
                    stage_records(pv, dvp, g0, steps, lane, s_piv, s_dinv);
                    rec_nx = s_piv[max(t, 0)];
                    const int nb = (s + 1) & 1;
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const int i = lane + 64 * q;
                        double v = 0.0;
                        if (i < own) v = xb[(long long)P.pos_index[p0 + i] * se];
                        else if (i < A) v = cvec[nb][P.carry_dst[p0 + i]];
                        y[q] = v;
                    }
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const int i = lane + 64 * q;
                        lv[q] = i >= own && i < A;
                        ci[q] = min(max(i - own, 0), A - own);
                    }
                    nlive = A - own;
                    KST(0);
                    continue;
                }
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
                ++kst_steps;
                KST(1);
            }
            if (finished && lane == 0) s_done = 1;
        }
        __syncthreads();
        if (s_done != 0) break;
        ring_store(ring.buf, c - 2, stage_r, tid);
        __syncthreads();
        KST(2);
        if (c < -2) break;                                // safety
    }
    KST(3);
    KST_DUMP2(kst_steps);
    (void)kst_steps;
}

template <int T>
int launch_factor(const ato_kkt* h, const Plan& P, const Vals& V, int batch, const int* list, int* inertia,
                  hipStream_t st) {
    constexpr int NP = 32 * T;
    const size_t lds = sizeof(double) * (32 * (NP + 1) + 4 * NP + (size_t)h->max_tq * h->max_tq) +
                       sizeof(int) * h->max_tq;
    if (lds > 160 * 1024) return fail(ATO_ERR_UNSUPPORTED, "KKT factor: LDS need exceeds 160 KB");
    hipLaunchKernelGGL(k_kkt_factor<T>, dim3(batch), dim3(FT), lds, st, P, V, batch, list, h->d_L, h->d_piv,
                       h->d_dinv, h->d_sinfo, inertia);
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

template <int T>
int launch_solve(const ato_kkt* h, const Plan& P, int batch, const int* list, double* x, long long se,
                 long long sb, hipStream_t st) {
    hipLaunchKernelGGL(k_kkt_solve<T>, dim3(batch), dim3(ST), 0, st, P, batch, list, h->d_L, h->d_piv, h->d_dinv,
                       h->d_sinfo, x, se, sb);
    KKT_HIP(hipGetLastError());
    return ATO_OK;
}

Plan make_plan(const ato_kkt* h) {
    Plan P;
    P.n = h->n;
    P.m = h->m;
    P.dim = h->dim;
    P.S = h->S;
    P.max_tq = h->max_tq;
    P.stage_ptr = h->d_stage_ptr;
    P.n_own = h->d_n_own;
    P.pos_index = h->d_pos_index;
    P.carry_dst = h->d_carry_dst;
    P.ent_ptr = h->d_ent_ptr;
    P.ent_pos = h->d_ent_pos;
    P.ent_src = reinterpret_cast<const int2*>(h->d_ent_src);
    P.piv_off = h->d_piv_off;
    P.l_size = h->l_size;
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
    (void)hipFree(h->d_L);
    (void)hipFree(h->d_piv);
    (void)hipFree(h->d_dinv);
    (void)hipFree(h->d_sinfo);
    h->d_L = nullptr;
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

int ato_kkt_create(const ato_kkt_plan_desc* d, ato_kkt** out) {
    if (!d || !out) return fail(ATO_ERR_ARG, "null argument");
    *out = nullptr;
    if (d->tiles < 1 || d->tiles > 8) return fail(ATO_ERR_UNSUPPORTED, "KKT blocks wider than 256 positions");
    if (d->n_stages < 1 || d->n < 0 || d->m < 0) return fail(ATO_ERR_ARG, "bad KKT plan sizes");
    ato_kkt* h = new ato_kkt();
    h->n = d->n;
    h->m = d->m;
    h->dim = d->n + d->m;
    h->S = d->n_stages;
    h->T = d->tiles;
    h->l_size = d->l_size;
    const int S = d->n_stages;
    const int P = d->stage_ptr[S];
    const int E = d->ent_ptr[S * d->tiles];
    for (int s = 0; s < S; ++s) {
        const int A = d->stage_ptr[s + 1] - d->stage_ptr[s];
        if (A > 32 * d->tiles || d->n_own[s] > A) {
            delete h;
            return fail(ATO_ERR_ARG, "KKT plan: stage larger than its tiles");
        }
        h->max_tq = std::max(h->max_tq, A - d->n_own[s]);
        const int es = d->ent_ptr[(s + 1) * d->tiles] - d->ent_ptr[s * d->tiles];
        h->max_ent = std::max(h->max_ent, es);
    }
    if (h->max_ent > EPT * FT) {
        delete h;
        return fail(ATO_ERR_UNSUPPORTED, "KKT plan: more than 4096 entries in one stage");
    }
    int rc = ATO_OK;
    if ((rc = upload(d->stage_ptr, S + 1, &h->d_stage_ptr)) || (rc = upload(d->n_own, S, &h->d_n_own)) ||
        (rc = upload(d->pos_index, P, &h->d_pos_index)) || (rc = upload(d->carry_dst, P, &h->d_carry_dst)) ||
        (rc = upload(d->ent_ptr, S * d->tiles + 1, &h->d_ent_ptr)) || (rc = upload(d->ent_pos, E, &h->d_ent_pos)) ||
        (rc = upload(d->ent_src, 2 * (size_t)E, &h->d_ent_src)) || (rc = upload(d->piv_off, S, &h->d_piv_off))) {
        ato_kkt_destroy(h);
        return rc;
    }
    *out = h;
    return ATO_OK;
}

int ato_kkt_destroy(ato_kkt* h) {
    if (!h) return ATO_OK;
    free_storage(h);
    for (int32_t* p : {h->d_stage_ptr, h->d_n_own, h->d_pos_index, h->d_carry_dst, h->d_ent_ptr, h->d_ent_pos,
                       h->d_ent_src, h->d_piv_off})
        (void)hipFree(p);
    delete h;
    return ATO_OK;
}

int ato_kkt_reserve(ato_kkt* h, int32_t max_batch) {
    if (!h || max_batch < 0) return fail(ATO_ERR_ARG, "bad argument");
    if (max_batch <= h->cap) return ATO_OK;
    free_storage(h);
    KKT_HIP(hipMalloc((void**)&h->d_L, sizeof(double) * (size_t)h->l_size * max_batch));
    KKT_HIP(hipMalloc((void**)&h->d_piv, sizeof(int2) * (size_t)h->dim * max_batch));
    KKT_HIP(hipMalloc((void**)&h->d_dinv, sizeof(double) * 3 * (size_t)h->dim * max_batch));
    KKT_HIP(hipMalloc((void**)&h->d_sinfo, sizeof(int2) * (size_t)(h->S + 1) * max_batch));
    h->cap = max_batch;
    return ATO_OK;
}

int ato_kkt_factor(ato_kkt* h, int32_t batch, const int32_t* list, int64_t se, int64_t sb, const double* H,
                   const double* J, const double* dx, const double* dr, int32_t* inertia, void* stream) {
    if (!h || !inertia || batch < 0) return fail(ATO_ERR_ARG, "bad argument");
    if (batch == 0) return ATO_OK;
    if (!list && batch > h->cap) return fail(ATO_ERR_STATE, "ato_kkt_reserve() too small for this batch");
    if (!h->d_L) return fail(ATO_ERR_STATE, "call ato_kkt_reserve() first");
    const Plan P = make_plan(h);
    const Vals V{H, J, dx, dr, se, sb};
    hipStream_t st = static_cast<hipStream_t>(stream);
    switch (h->T) {
        case 1: return launch_factor<1>(h, P, V, batch, list, inertia, st);
        case 2: return launch_factor<2>(h, P, V, batch, list, inertia, st);
        case 3: return launch_factor<3>(h, P, V, batch, list, inertia, st);
        case 4: return launch_factor<4>(h, P, V, batch, list, inertia, st);
        case 5: return launch_factor<5>(h, P, V, batch, list, inertia, st);
        case 6: return launch_factor<6>(h, P, V, batch, list, inertia, st);
        case 7: return launch_factor<7>(h, P, V, batch, list, inertia, st);
        case 8: return launch_factor<8>(h, P, V, batch, list, inertia, st);
        default: return fail(ATO_ERR_UNSUPPORTED, "KKT tiles");
    }
}

int ato_kkt_solve(ato_kkt* h, int32_t batch, const int32_t* list, int64_t se, int64_t sb, double* x,
                  void* stream) {
    if (!h || !x || batch < 0) return fail(ATO_ERR_ARG, "bad argument");
    if (batch == 0) return ATO_OK;
    if (!h->d_L) return fail(ATO_ERR_STATE, "call ato_kkt_reserve() first");
    if (!list && batch > h->cap) return fail(ATO_ERR_STATE, "ato_kkt_reserve() too small for this batch");
    const Plan P = make_plan(h);
    hipStream_t st = static_cast<hipStream_t>(stream);
    switch (h->T) {
        case 1: return launch_solve<1>(h, P, batch, list, x, se, sb, st);
        case 2: return launch_solve<2>(h, P, batch, list, x, se, sb, st);
        case 3: return launch_solve<3>(h, P, batch, list, x, se, sb, st);
        case 4: return launch_solve<4>(h, P, batch, list, x, se, sb, st);
        case 5: return launch_solve<5>(h, P, batch, list, x, se, sb, st);
        case 6: return launch_solve<6>(h, P, batch, list, x, se, sb, st);
        case 7: return launch_solve<7>(h, P, batch, list, x, se, sb, st);
        case 8: return launch_solve<8>(h, P, batch, list, x, se, sb, st);
        default: return fail(ATO_ERR_UNSUPPORTED, "KKT tiles");
    }
}

}  // extern "C"
