// ato_ipm.hip -- fused column kernels of the batched interior-point iteration (include/ato_ipm.h).
//
// The batched solver (solver/batched_ipm.py) restates IPOPT's iteration (ref:
// drone3d/raceline/base_raceline.py:752-799, the solver behind ca.nlpsol) on [element][W]
// device tensors. Each of its vector steps -- optimality errors, barrier right-hand side,
// fraction to the boundary, filter measures, multiplier safeguard -- was tens of elementwise
// tensor operations (one launch each, most of an iteration's launches once the batch has
// shrunk). Here each step is one launch (plus one for per-column reductions).
//
// Layout: element e of column b at e * W + b; thread b of a 64-wide column block reads
// consecutive columns (coalesced 512-byte rows). Reductions: stage 1 = one workgroup per
// (column block, chunk of CH elements of one part), partial results to the workspace
// [quantity][chunk][W]; stage 2 = one thread per column folds the chunks in order. Maxima and
// minima propagate NaN like torch.maximum / amax. Compiled with -ffp-contract=off: no fused
// multiply-adds, so elementwise results equal the host formulas bit for bit.
#include <hip/hip_runtime.h>
#include <cmath>
#include <string>
#include "../../include/ato_ipm.h"
#include "../../include/ato.h"

void ato_internal_set_error(const std::string& msg);   // ato_capi.hip: ato_last_error()

namespace {

constexpr int CH = 32;          // elements per reduction chunk
constexpr int CB = 64;          // columns per workgroup
constexpr int QMAX = 9;         // partial quantities per chunk (errors)

__device__ __forceinline__ double nmax(double a, double b) {
    return (a != a || b != b) ? __builtin_nan("") : (a > b ? a : b);
}
__device__ __forceinline__ double nmin(double a, double b) {
    return (a != a || b != b) ? __builtin_nan("") : (a < b ? a : b);
}
__device__ __forceinline__ bool fin(double v) { return fabs(v) < INFINITY; }

// chunking of up to four parts of different lengths
struct Parts {
    int len[4];
    int c0[5];                  // first chunk of every part; c0[4] = total
};

Parts make_parts(int a, int b, int c, int d) {
    Parts p;
    const int l[4] = {a, b, c, d};
    p.c0[0] = 0;
    for (int i = 0; i < 4; ++i) {
        p.len[i] = l[i];
        p.c0[i + 1] = p.c0[i] + (l[i] + CH - 1) / CH;
    }
    return p;
}

__device__ __forceinline__ void chunk_of(const Parts& p, int c, int& part, int& e0, int& e1) {
    part = c < p.c0[1] ? 0 : c < p.c0[2] ? 1 : c < p.c0[3] ? 2 : 3;
    e0 = (c - p.c0[part]) * CH;
    e1 = min(e0 + CH, p.len[part]);
}

struct Dev {
    int n, m, mi, meq, W;
    const int* iin;
    const int* ieq;
    const double *xL, *xU, *dL, *dU;
};

__device__ __forceinline__ long long at(const Dev& d, int e, int b) { return (long long)e * d.W + b; }

// slacks of the bounds (batched_ipm.py _slacks): 1 where the bound is absent
__device__ __forceinline__ void xslacks(const Dev& d, const double* x, int e, int b, double& a, double& bb,
                                        bool& hl, bool& hu) {
    const long long i = at(d, e, b);
    const double lo = d.xL[i], hi = d.xU[i], v = x[i];
    hl = fin(lo);
    hu = fin(hi);
    a = hl ? v - lo : 1.0;
    bb = hu ? hi - v : 1.0;
}

__device__ __forceinline__ void sslacks(const Dev& d, const double* s, int i0, int b, double& c, double& dd,
                                        bool& hl, bool& hu) {
    const long long i = at(d, i0, b);
    const double lo = d.dL[i], hi = d.dU[i], v = s[i];
    hl = fin(lo);
    hu = fin(hi);
    c = hl ? v - lo : 1.0;
    dd = hu ? hi - v : 1.0;
}

// ------------------------------------------------------------------------------------------
// errors: q = 0 du, 1 pr, 2 co, 3 pr_uns (max); 4 |zl|, 5 |zu|, 6 |vl|, 7 |vu|, 8 |y| (sums)
// parts: variables, slack rows, equality rows, all rows (for |y|)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(CB) void k_errors(Dev d, Parts P, const double* __restrict__ x,
                                               const double* __restrict__ s, const double* __restrict__ g,
                                               const double* __restrict__ c_rhs, const double* __restrict__ sg,
                                               const double* __restrict__ y, const double* __restrict__ zl,
                                               const double* __restrict__ zu, const double* __restrict__ vl,
                                               const double* __restrict__ vu, const double* __restrict__ dual_x,
                                               const double* __restrict__ mu, double* __restrict__ work) {
    const int b = blockIdx.x * CB + threadIdx.x;
    const int c = blockIdx.y;
    if (b >= d.W) return;
    int part, e0, e1;
    chunk_of(P, c, part, e0, e1);
    const double m_ = mu[b];
    double q[QMAX] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (part == 0) {
        for (int e = e0; e < e1; ++e) {
            double a, bb;
            bool hl, hu;
            xslacks(d, x, e, b, a, bb, hl, hu);
            const long long i = at(d, e, b);
            q[0] = nmax(q[0], fabs(dual_x[i]));
            if (hl) q[2] = nmax(q[2], fabs(a * zl[i] - m_));
            if (hu) q[2] = nmax(q[2], fabs(bb * zu[i] - m_));
            q[4] += fabs(zl[i]);
            q[5] += fabs(zu[i]);
        }
    } else if (part == 1) {
        for (int k = e0; k < e1; ++k) {
            double cc, dd;
            bool hl, hu;
            sslacks(d, s, k, b, cc, dd, hl, hu);
            const long long i = at(d, k, b);
            const int row = d.iin[k];
            const long long ir = at(d, row, b);
            const double ds = (-y[ir] - vl[i]) + vu[i];
            q[0] = nmax(q[0], fabs(ds));
            if (hl) q[2] = nmax(q[2], fabs(cc * vl[i] - m_));
            if (hu) q[2] = nmax(q[2], fabs(dd * vu[i] - m_));
            q[6] += fabs(vl[i]);
            q[7] += fabs(vu[i]);
            const double r = g[ir] - s[i];
            q[1] = nmax(q[1], fabs(r));
            q[3] = nmax(q[3], fabs(r / sg[ir]));
        }
    } else if (part == 2) {
        for (int k = e0; k < e1; ++k) {
            const long long ir = at(d, d.ieq[k], b);
            const double r = g[ir] - c_rhs[at(d, k, b)];
            q[1] = nmax(q[1], fabs(r));
            q[3] = nmax(q[3], fabs(r / sg[ir]));
        }
    } else {
        for (int k = e0; k < e1; ++k) q[8] += fabs(y[at(d, k, b)]);
    }
    const int NC = P.c0[4];
#pragma unroll
    for (int k = 0; k < QMAX; ++k) work[((long long)k * NC + c) * d.W + b] = q[k];
}

// Stage 2 of the reductions: FG thread groups per column; group g folds quantities 0..NQ-1 of its
// contiguous chunk range [c0, c1) in chunk order, and the FG partial results are merged in group
// order (fixed shape: deterministic). Within a range the loads of U chunks are issued together
// before the U folds (the fold is a chain of dependent operations, its loads are not). W = 512
// keeps only 8 column blocks busy, so the groups are what fills the memory pipeline:
// k_errors_fold 388 -> 213 us with batched loads alone, k_measures_fold 122 -> 33 us.
constexpr int FG = 8;
__device__ __forceinline__ void fold_range(int NC, int g, int& c0, int& c1) {
    c0 = (int)((long long)NC * g / FG);
    c1 = (int)((long long)NC * (g + 1) / FG);
}

template <int NQ, int U, class F>
__device__ __forceinline__ void fold_chunks(const double* __restrict__ work, int NC, int W, int b, int c0, int c1,
                                            F&& fold) {
    int c = c0;
    for (; c + U <= c1; c += U) {
        double v[U][NQ];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int k = 0; k < NQ; ++k) v[u][k] = work[((long long)k * NC + c + u) * W + b];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) fold(v[u]);
    }
    for (; c < c1; ++c) {
        double v[NQ];
#pragma unroll
        for (int k = 0; k < NQ; ++k) v[k] = work[((long long)k * NC + c) * W + b];
        fold(v);
    }
}

// The errors fold in two launches (k_errors_fold above kept 8 workgroups busy at W = 512 and ran
// 368 us, gpurun_out r05l): EG chunk ranges per column in parallel, then the EG partials of every
// column in range order (deterministic).
constexpr int EG = 32;
__device__ __forceinline__ void errors_fold_q(double (&q)[QMAX], const double (&v)[QMAX]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = nmax(q[k], v[k]);
#pragma unroll
    for (int k = 4; k < QMAX; ++k) q[k] += v[k];
}

__global__ __launch_bounds__(CB) void k_errors_fold1(int W, int NC, const double* __restrict__ work,
                                                     double* __restrict__ part) {
    const int b = blockIdx.x * CB + threadIdx.x, g = blockIdx.y;
    if (b >= W) return;
    const int c0 = (int)((long long)NC * g / EG), c1 = (int)((long long)NC * (g + 1) / EG);
    double q[QMAX] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    fold_chunks<QMAX, 2>(work, NC, W, b, c0, c1, [&](const double (&v)[QMAX]) { errors_fold_q(q, v); });
#pragma unroll
    for (int k = 0; k < QMAX; ++k) part[((long long)k * EG + g) * W + b] = q[k];
}

__global__ __launch_bounds__(CB) void k_errors_fold2(int W, int m, double s_max, const double* __restrict__ n_bounds,
                                                     const double* __restrict__ part, double* __restrict__ out) {
    const int b = blockIdx.x * CB + threadIdx.x;
    if (b >= W) return;
    double q[QMAX] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int g = 0; g < EG; ++g) {
        double v[QMAX];
#pragma unroll
        for (int k = 0; k < QMAX; ++k) v[k] = part[((long long)k * EG + g) * W + b];
        errors_fold_q(q, v);
    }
    const double nz = n_bounds[b];
    const double zsum = ((q[4] + q[5]) + q[6]) + q[7];
    const double s_d = nmax((q[8] + zsum) / fmax((double)m + nz, 1.0), s_max) / s_max;
    const double s_c = nmax(zsum / fmax(nz, 1.0), s_max) / s_max;
    const double du = q[0], pr = q[1], co = q[2];
    out[0 * W + b] = nmax(nmax(du / s_d, pr), co / s_c);
    out[1 * W + b] = du;
    out[2 * W + b] = pr;
    out[3 * W + b] = co;
    out[4 * W + b] = q[3];
}

// ------------------------------------------------------------------------------------------
// right-hand side: one thread per (element, column) of variables | slacks | rows
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rhs(Dev d, const double* __restrict__ x, const double* __restrict__ s,
                                             const double* __restrict__ g, const double* __restrict__ c_rhs,
                                             const double* __restrict__ gf, const double* __restrict__ jty,
                                             const double* __restrict__ y, const double* __restrict__ zl,
                                             const double* __restrict__ zu, const double* __restrict__ vl,
                                             const double* __restrict__ vu, const double* __restrict__ mu,
                                             double kd, double* __restrict__ Sx, double* __restrict__ Ss,
                                             double* __restrict__ gx, double* __restrict__ gs,
                                             double* __restrict__ rhs_x, double* __restrict__ rhs_s,
                                             double* __restrict__ rhs_y) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long nx = (long long)d.n * d.W, ns = (long long)d.mi * d.W;
    if (t < nx) {
        const int e = (int)(t / d.W), b = (int)(t - (long long)e * d.W);
        double a, bb;
        bool hl, hu;
        xslacks(d, x, e, b, a, bb, hl, hu);
        const double m_ = mu[b];
        Sx[t] = (hl ? zl[t] / a : 0.0) + (hu ? zu[t] / bb : 0.0);
        double v = (gf[t] - m_ * (hl ? 1.0 / a : 0.0)) + m_ * (hu ? 1.0 / bb : 0.0);
        v = v + (kd * m_) * ((hl && !hu ? 1.0 : 0.0) - (hu && !hl ? 1.0 : 0.0));
        gx[t] = v;
        rhs_x[t] = -(v + jty[t]);
    } else if (t < nx + ns) {
        const long long u = t - nx;
        const int k = (int)(u / d.W), b = (int)(u - (long long)k * d.W);
        double cc, dd;
        bool hl, hu;
        sslacks(d, s, k, b, cc, dd, hl, hu);
        const double m_ = mu[b];
        Ss[u] = (hl ? vl[u] / cc : 0.0) + (hu ? vu[u] / dd : 0.0);
        double v = (-m_) * (hl ? 1.0 / cc : 0.0) + m_ * (hu ? 1.0 / dd : 0.0);
        v = v + (kd * m_) * ((hl && !hu ? 1.0 : 0.0) - (hu && !hl ? 1.0 : 0.0));
        gs[u] = v;
        rhs_s[u] = -(v - y[at(d, d.iin[k], b)]);
    }
}

// rhs_y = -r: slack rows -(g - s), equality rows -(g - c_rhs)
__global__ __launch_bounds__(256) void k_resid_rows(Dev d, const double* __restrict__ g, const double* __restrict__ s,
                                                    const double* __restrict__ c_rhs, double* __restrict__ out) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long ns = (long long)d.mi * d.W, ne = (long long)d.meq * d.W;
    if (t < ns) {
        const int k = (int)(t / d.W), b = (int)(t - (long long)k * d.W);
        const long long ir = at(d, d.iin[k], b);
        out[ir] = -(g[ir] - s[t]);
    } else if (t < ns + ne) {
        const long long u = t - ns;
        const int k = (int)(u / d.W), b = (int)(u - (long long)k * d.W);
        const long long ir = at(d, d.ieq[k], b);
        out[ir] = -(g[ir] - c_rhs[u]);
    }
}

// ------------------------------------------------------------------------------------------
// direction: multiplier steps (elementwise) and per-column minima / dot products
// q = 0 alpha_max candidates (min), 1 alpha_z candidates (min), 2 gx.dx, 3 gs.ds (sums)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double ftb_ratio(double v, double dv, bool mask, double ntau) {
    return (mask && dv < 0.0) ? (ntau * v) / dv : INFINITY;
}

__global__ __launch_bounds__(CB) void k_direction(Dev d, Parts P, const double* __restrict__ x,
                                                  const double* __restrict__ s, const double* __restrict__ dx,
                                                  const double* __restrict__ ds, const double* __restrict__ zl,
                                                  const double* __restrict__ zu, const double* __restrict__ vl,
                                                  const double* __restrict__ vu, const double* __restrict__ gx,
                                                  const double* __restrict__ gs, const double* __restrict__ mu,
                                                  const double* __restrict__ tau, double* __restrict__ dzl,
                                                  double* __restrict__ dzu, double* __restrict__ dvl,
                                                  double* __restrict__ dvu, double* __restrict__ work) {
    const int b = blockIdx.x * CB + threadIdx.x;
    const int c = blockIdx.y;
    if (b >= d.W) return;
    int part, e0, e1;
    chunk_of(P, c, part, e0, e1);
    const double m_ = mu[b], nt = -tau[b];
    double q0 = INFINITY, q1 = INFINITY, q2 = 0.0, q3 = 0.0;
    if (part == 0) {
        for (int e = e0; e < e1; ++e) {
            double a, bb;
            bool hl, hu;
            xslacks(d, x, e, b, a, bb, hl, hu);
            const long long i = at(d, e, b);
            const double dxi = dx[i], zli = zl[i], zui = zu[i];
            const double l = hl ? ((m_ / a) - zli) - ((zli / a) * dxi) : 0.0;
            const double u = hu ? ((m_ / bb) - zui) + ((zui / bb) * dxi) : 0.0;
            dzl[i] = l;
            dzu[i] = u;
            q0 = nmin(q0, nmin(ftb_ratio(a, dxi, hl, nt), ftb_ratio(bb, -dxi, hu, nt)));
            q1 = nmin(q1, nmin(ftb_ratio(zli, l, hl, nt), ftb_ratio(zui, u, hu, nt)));
            q2 += gx[i] * dxi;
        }
    } else {
        for (int k = e0; k < e1; ++k) {
            double cc, dd;
            bool hl, hu;
            sslacks(d, s, k, b, cc, dd, hl, hu);
            const long long i = at(d, k, b);
            const double dsi = ds[i], vli = vl[i], vui = vu[i];
            const double l = hl ? ((m_ / cc) - vli) - ((vli / cc) * dsi) : 0.0;
            const double u = hu ? ((m_ / dd) - vui) + ((vui / dd) * dsi) : 0.0;
            dvl[i] = l;
            dvu[i] = u;
            q0 = nmin(q0, nmin(ftb_ratio(cc, dsi, hl, nt), ftb_ratio(dd, -dsi, hu, nt)));
            q1 = nmin(q1, nmin(ftb_ratio(vli, l, hl, nt), ftb_ratio(vui, u, hu, nt)));
            q3 += gs[i] * dsi;
        }
    }
    const int NC = P.c0[4];
    work[((long long)0 * NC + c) * d.W + b] = q0;
    work[((long long)1 * NC + c) * d.W + b] = q1;
    work[((long long)2 * NC + c) * d.W + b] = q2;
    work[((long long)3 * NC + c) * d.W + b] = q3;
}

__global__ __launch_bounds__(CB * FG) void k_direction_fold(int W, int NC, const double* __restrict__ work,
                                                            double* __restrict__ out) {
    __shared__ double part[FG][4][CB];
    const int lane = threadIdx.x % CB, grp = threadIdx.x / CB;
    const int b = blockIdx.x * CB + lane;
    double q0 = INFINITY, q1 = INFINITY, q2 = 0.0, q3 = 0.0;
    auto fold = [&](const double (&v)[4]) {
        q0 = nmin(q0, v[0]);
        q1 = nmin(q1, v[1]);
        q2 += v[2];
        q3 += v[3];
    };
    if (b < W) {
        int c0, c1;
        fold_range(NC, grp, c0, c1);
        fold_chunks<4, 8>(work, NC, W, b, c0, c1, fold);
    }
    part[grp][0][lane] = q0;
    part[grp][1][lane] = q1;
    part[grp][2][lane] = q2;
    part[grp][3][lane] = q3;
    __syncthreads();
    if (grp != 0 || b >= W) return;
    for (int g = 1; g < FG; ++g) {
        const double v[4] = {part[g][0][lane], part[g][1][lane], part[g][2][lane], part[g][3][lane]};
        fold(v);
    }
    out[0 * W + b] = nmin(q0, 1.0);
    out[1 * W + b] = nmin(q1, 1.0);
    out[2 * W + b] = q2 + q3;
}

// ------------------------------------------------------------------------------------------
// measures: q = 0 sum |r|, 1 sum log(slacks), 2 sum of one-sided slacks
// parts: variables, slack rows, equality rows
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(CB) void k_measures(Dev d, Parts P, const double* __restrict__ x,
                                                 const double* __restrict__ s, const double* __restrict__ g,
                                                 const double* __restrict__ c_rhs, double* __restrict__ work) {
    const int b = blockIdx.x * CB + threadIdx.x;
    const int c = blockIdx.y;
    if (b >= d.W) return;
    int part, e0, e1;
    chunk_of(P, c, part, e0, e1);
    double th = 0.0, lg = 0.0, lin = 0.0;
    if (part == 0) {
        for (int e = e0; e < e1; ++e) {
            double a, bb;
            bool hl, hu;
            xslacks(d, x, e, b, a, bb, hl, hu);
            if (hl) lg += log(a);
            if (hu) lg += log(bb);
            if (hl && !hu) lin += a;
            if (hu && !hl) lin += bb;
        }
    } else if (part == 1) {
        for (int k = e0; k < e1; ++k) {
            double cc, dd;
            bool hl, hu;
            sslacks(d, s, k, b, cc, dd, hl, hu);
            if (hl) lg += log(cc);
            if (hu) lg += log(dd);
            if (hl && !hu) lin += cc;
            if (hu && !hl) lin += dd;
            th += fabs(g[at(d, d.iin[k], b)] - s[at(d, k, b)]);
        }
    } else {
        for (int k = e0; k < e1; ++k) th += fabs(g[at(d, d.ieq[k], b)] - c_rhs[at(d, k, b)]);
    }
    const int NC = P.c0[4];
    work[((long long)0 * NC + c) * d.W + b] = th;
    work[((long long)1 * NC + c) * d.W + b] = lg;
    work[((long long)2 * NC + c) * d.W + b] = lin;
}

__global__ __launch_bounds__(CB * FG) void k_measures_fold(int W, int NC, const double* __restrict__ f,
                                                           const double* __restrict__ mu, double kd,
                                                           const double* __restrict__ work, double* __restrict__ out) {
    __shared__ double part[FG][3][CB];
    const int lane = threadIdx.x % CB, grp = threadIdx.x / CB;
    const int b = blockIdx.x * CB + lane;
    double th = 0.0, lg = 0.0, lin = 0.0;
    auto fold = [&](const double (&v)[3]) {
        th += v[0];
        lg += v[1];
        lin += v[2];
    };
    if (b < W) {
        int c0, c1;
        fold_range(NC, grp, c0, c1);
        fold_chunks<3, 8>(work, NC, W, b, c0, c1, fold);
    }
    part[grp][0][lane] = th;
    part[grp][1][lane] = lg;
    part[grp][2][lane] = lin;
    __syncthreads();
    if (grp != 0 || b >= W) return;
    for (int g = 1; g < FG; ++g) {
        const double v[3] = {part[g][0][lane], part[g][1][lane], part[g][2][lane]};
        fold(v);
    }
    const double m_ = mu[b];
    out[0 * W + b] = th;
    out[1 * W + b] = (f[b] - m_ * lg) + (kd * m_) * lin;
}

// ------------------------------------------------------------------------------------------
// multipliers: z += az dz, then the kappa_sigma safeguard at the accepted slacks
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double safeguard(double z, double m_, double ks, double sl) {
    return nmin(nmax(z, m_ / (ks * sl)), (ks * m_) / sl);
}

__global__ __launch_bounds__(256) void k_multipliers(Dev d, const double* __restrict__ x, const double* __restrict__ s,
                                                     const double* __restrict__ mu, const double* __restrict__ az,
                                                     double ks, double* __restrict__ zl, double* __restrict__ zu,
                                                     double* __restrict__ vl, double* __restrict__ vu,
                                                     const double* __restrict__ dzl, const double* __restrict__ dzu,
                                                     const double* __restrict__ dvl, const double* __restrict__ dvu) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long nx = (long long)d.n * d.W, ns = (long long)d.mi * d.W;
    if (t < nx) {
        const int e = (int)(t / d.W), b = (int)(t - (long long)e * d.W);
        double a, bb;
        bool hl, hu;
        xslacks(d, x, e, b, a, bb, hl, hu);
        const double m_ = mu[b], al = az[b];
        const double l = zl[t] + al * dzl[t], u = zu[t] + al * dzu[t];
        zl[t] = hl ? safeguard(l, m_, ks, a) : 0.0;
        zu[t] = hu ? safeguard(u, m_, ks, bb) : 0.0;
    } else if (t < nx + ns) {
        const long long u0 = t - nx;
        const int k = (int)(u0 / d.W), b = (int)(u0 - (long long)k * d.W);
        double cc, dd;
        bool hl, hu;
        sslacks(d, s, k, b, cc, dd, hl, hu);
        const double m_ = mu[b], al = az[b];
        const double l = vl[u0] + al * dvl[u0], u = vu[u0] + al * dvu[u0];
        vl[u0] = hl ? safeguard(l, m_, ks, cc) : 0.0;
        vu[u0] = hu ? safeguard(u, m_, ks, dd) : 0.0;
    }
}

int fail(int code, const std::string& m) {
    ato_internal_set_error(m);
    return code;
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ATO_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return ATO_OK;
}

bool make_dev(const ato_ipm_dims* d, const ato_ipm_bounds* bd, Dev& v) {
    if (!d || !bd || d->n < 0 || d->m < 0 || d->mi < 0 || d->meq < 0 || d->mi + d->meq != d->m || d->W <= 0 ||
        (d->mi && !d->iin) || (d->meq && !d->ieq) || (d->n && (!bd->xL || !bd->xU)) ||
        (d->mi && (!bd->dL || !bd->dU)))
        return false;
    v = Dev{d->n, d->m, d->mi, d->meq, d->W, d->iin, d->ieq, bd->xL, bd->xU, bd->dL, bd->dU};
    return true;
}

dim3 col_grid(int W, int NC) { return dim3((W + CB - 1) / CB, NC); }
unsigned lin_blocks(long long cnt) { return (unsigned)((cnt + 255) / 256); }

// ------------------------------------------------------------------------------------------
// filter acceptance of a trial point (batched_ipm.py _accept), one thread per column
// ------------------------------------------------------------------------------------------
// torch.pow(tensor, scalar) on the device: its special exponents, std::pow otherwise
__device__ __forceinline__ double tpow(double x, double e) {
    if (e == 2.0) return x * x;
    if (e == 3.0) return x * x * x;
    if (e == 0.5) return sqrt(x);
    if (e == 1.0) return x;
    return pow(x, e);
}

struct FilterPrm {
    double s_phi, s_theta, delta, eta_phi, gamma_theta, gamma_phi, obj_max_inc, compare_tol;
    long long max_filter_resets, filter_reset_trigger;
};

// one trial's FilterLSAcceptor::CheckAcceptabilityOfTrialPoint: rejected by theta_max, the
// current-iterate test (Armijo in the f-type case, else sufficient decrease; Compare_le tolerance;
// obj_max_inc) or the filter
struct TrialTest {
    bool ok, arm_case, rej, it_ok, in_f;
};

__device__ __forceinline__ TrialTest filter_trial(const FilterPrm& o, double th, double ph, double gd, double al,
                                                  double tt, double pt, const double* Fb, long long k1, int fmax,
                                                  double tmax, double tmin) {
    TrialTest r;
    r.rej = !(tt <= tmax);
    r.in_f = false;
    const int kn = (int)(k1 < fmax ? k1 : fmax);
    for (int k = 0; k < kn; ++k)
        if (tt >= Fb[2 * k] && pt >= Fb[2 * k + 1]) r.in_f = true;
    const double ngd = -gd;
    const double mgd = ngd != ngd ? ngd : (ngd < 0.0 ? 0.0 : ngd);      // torch.clamp(min=0): NaN stays
    const bool switching = (gd < 0.0) && (al * tpow(mgd, o.s_phi) > o.delta * tpow(th, o.s_theta));
    r.arm_case = (th <= tmin) && switching;
    // IpUtils Compare_le(lhs, rhs, base): lhs - rhs <= compare_tol |base| (ArmijoHolds,
    // IsAcceptableToCurrentIterate)
    const double dp = pt - ph;
    const bool ok_arm = dp - (o.eta_phi * al) * gd <= o.compare_tol * fabs(ph);
    const bool ok_suf = (tt - (1.0 - o.gamma_theta) * th <= o.compare_tol * fabs(th)) ||
                        (dp - (-o.gamma_phi * th) <= o.compare_tol * fabs(ph));
    // obj_max_inc (FilterLSAcceptor::CheckAcceptabilityOfTrialPoint): the barrier objective may not
    // grow by more than 10^obj_max_inc of its magnitude
    bool inc = false;
    if (pt > ph) {
        const double base = fabs(ph) > 10.0 ? log10(fabs(ph)) : 1.0;
        inc = log10(pt - ph) > o.obj_max_inc + base;
    }
    r.it_ok = !inc && (r.arm_case ? ok_arm : ok_suf);
    r.ok = !r.rej && r.it_ok && !r.in_f;
    return r;
}

// the filter reset heuristic of CheckAcceptabilityOfTrialPoint for one tested trial: a rejection by
// the current-iterate test clears "last rejection due to the filter", a rejection by the filter sets
// it (theta_max leaves it); an acceptance after filter_reset_trigger successive iterations whose last
// rejection was the filter's clears the filter (at most max_filter_resets times)
__device__ __forceinline__ void filter_reset_step(const FilterPrm& o, const TrialTest& t, long long& n, long long& c,
                                                  bool& last, long long& nf) {
    if (t.rej) return;
    if (!t.it_ok) {
        last = false;
    } else if (t.in_f) {
        last = true;
    } else {
        if (o.max_filter_resets > 0 && n < o.max_filter_resets) {
            if (last) {
                ++c;
                if (c >= o.filter_reset_trigger) {
                    nf = 0;
                    ++n;
                    c = 0;
                }
            } else {
                c = 0;
            }
        }
        last = false;
    }
}

__global__ __launch_bounds__(CB) void k_filter_accept(int W, int fmax, const double* __restrict__ theta,
                                                      const double* __restrict__ phi,
                                                      const double* __restrict__ gphi_d,
                                                      const double* __restrict__ alpha,
                                                      const double* __restrict__ tht, const double* __restrict__ pht,
                                                      const double* __restrict__ F, int64_t* __restrict__ nf,
                                                      const double* __restrict__ theta_max,
                                                      const double* __restrict__ theta_min,
                                                      const uint8_t* __restrict__ pend,
                                                      const uint8_t* __restrict__ first, FilterPrm o,
                                                      int64_t* __restrict__ fr_n, int64_t* __restrict__ fr_cnt,
                                                      uint8_t* __restrict__ fr_last,
                                                      uint8_t* __restrict__ ok_out, uint8_t* __restrict__ arm_out,
                                                      uint8_t* __restrict__ soc_out) {
    const int b = blockIdx.x * CB + threadIdx.x;
    if (b >= W) return;
    const double th = theta[b], tt = tht[b];
    const TrialTest t = filter_trial(o, th, phi[b], gphi_d[b], alpha[b], tt, pht[b], F + (long long)b * fmax * 2,
                                     nf[b], fmax, theta_max[b], theta_min[b]);
    const bool pd = pend[b] != 0;
    const bool ok = pd && t.ok;
    ok_out[b] = ok ? 1 : 0;
    arm_out[b] = (ok && t.arm_case) ? 1 : 0;
    soc_out[b] = (pd && !ok && first[b] != 0 && tt >= th) ? 1 : 0;
    if (fr_n && pd) {
        long long n = fr_n[b], c = fr_cnt[b], k = nf[b];
        bool last = fr_last[b] != 0;
        filter_reset_step(o, t, n, c, last, k);
        fr_n[b] = n;
        fr_cnt[b] = c;
        fr_last[b] = last ? 1 : 0;
        nf[b] = k;
    }
}

// K successive backtracking trials of each of P columns, evaluated together (trial k of column p at
// alpha0[p] / 2^k; tht, pht [K][P]) and tested in order, exactly as K rounds of the lockstep line
// search would (batched_ipm.py _multi_trials): a column stops at its first trial with alpha <= alpha_min
// (failed) or at its first accepted trial (kacc = k, arm); the reset heuristic runs on every tested trial
__global__ __launch_bounds__(CB) void k_filter_multi(int P, int K, int fmax, const double* __restrict__ theta,
                                                     const double* __restrict__ phi,
                                                     const double* __restrict__ gphi_d,
                                                     const double* __restrict__ alpha0,
                                                     const double* __restrict__ alpha_min,
                                                     const double* __restrict__ tht, const double* __restrict__ pht,
                                                     const double* __restrict__ F, int64_t* __restrict__ nf,
                                                     const double* __restrict__ theta_max,
                                                     const double* __restrict__ theta_min, FilterPrm o,
                                                     int64_t* __restrict__ fr_n, int64_t* __restrict__ fr_cnt,
                                                     uint8_t* __restrict__ fr_last, int32_t* __restrict__ kacc,
                                                     uint8_t* __restrict__ fail_out, uint8_t* __restrict__ arm_out) {
    const int p = blockIdx.x * CB + threadIdx.x;
    if (p >= P) return;
    const double th = theta[p], ph = phi[p], gd = gphi_d[p], amin = alpha_min[p];
    const double tmax = theta_max[p], tmin = theta_min[p];
    const double* Fb = F + (long long)p * fmax * 2;
    long long n = fr_n[p], c = fr_cnt[p], k1 = nf[p];
    bool last = fr_last[p] != 0;
    int ka = -1;
    bool fl = false, arm = false;
    double al = alpha0[p];
    for (int k = 0; k < K; ++k) {
        if (!(al > amin)) {
            fl = true;
            break;
        }
        const TrialTest t = filter_trial(o, th, ph, gd, al, tht[(long long)k * P + p], pht[(long long)k * P + p], Fb,
                                         k1, fmax, tmax, tmin);
        filter_reset_step(o, t, n, c, last, k1);
        if (t.ok) {
            ka = k;
            arm = t.arm_case;
            break;
        }
        al = al * 0.5;
    }
    fr_n[p] = n;
    fr_cnt[p] = c;
    fr_last[p] = last ? 1 : 0;
    nf[p] = k1;
    kacc[p] = ka;
    fail_out[p] = fl ? 1 : 0;
    arm_out[p] = arm ? 1 : 0;
}

// ------------------------------------------------------------------------------------------
// KKT diagonals of one inertia-correction pass (batched_ipm.py _kkt_step): dx = Sx + dw,
// Ds = Ss + dw, dr = -dc on every row and -dc - 1 / Ds on the slack rows; one thread per element
// of [variables | slack rows | equality rows] x column
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_kkt_diag(Dev d, const double* __restrict__ Sx, const double* __restrict__ Ss,
                                                  const double* __restrict__ dw, const double* __restrict__ dc,
                                                  double* __restrict__ dx, double* __restrict__ dr,
                                                  double* __restrict__ Ds) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long nW = (long long)d.n * d.W, iW = (long long)d.mi * d.W, eW = (long long)d.meq * d.W;
    if (t < nW) {
        const int b = (int)(t % d.W);
        dx[t] = Sx[t] + dw[b];
    } else if (t < nW + iW) {
        const long long u = t - nW;
        const int r = (int)(u / d.W), b = (int)(u - (long long)r * d.W);
        const double ds = Ss[u] + dw[b];
        Ds[u] = ds;
        dr[at(d, d.iin[r], b)] = -dc[b] - 1.0 / ds;
    } else if (t < nW + iW + eW) {
        const long long u = t - nW - iW;
        const int r = (int)(u / d.W), b = (int)(u - (long long)r * d.W);
        dr[at(d, d.ieq[r], b)] = -dc[b];
    }
}

// ------------------------------------------------------------------------------------------
// IPOPT's PDPerturbationHandler per column (batched_ipm.py BatchedPerturbation, solver/ipm.py
// PerturbationHandler) and the bookkeeping of one inertia-correction pass of _kkt_step, one
// thread per column: the whole per-pass state machine in one launch instead of ~40 masked
// torch operations per call.
// ------------------------------------------------------------------------------------------
enum { DEG_UNK = 0, DEG_NO = 1, DEG_YES = 2 };
enum { T_NONE = 0, T_C0X0 = 1, T_CPX0 = 2, T_C0XP = 3, T_CPXP = 4 };

struct PertPrm {
    double delta_w_0, delta_w_min, delta_w_max, kappa_w_minus, kappa_w_plus, kappa_w_plus_bar, delta_c_base, kappa_c;
    long long degen_iters_max;
};

struct PertCol {           // one column's handler state (registers)
    long long hdeg, jdeg, diters, test;
    double dx, dc, dx_last, dc_last;
};

__device__ inline double cmax(double a, double b) { return a != a ? a : (a < b ? b : a); }   // torch.clamp(min=b)

__device__ inline void pert_finalize(PertCol& c, const PertPrm& o) {
    const bool uh = c.hdeg == DEG_UNK, uj = c.jdeg == DEG_UNK;
    const long long t = c.test;
    if ((t == T_CPX0 && uj) || (t == T_C0XP && uh) || t == T_CPXP) c.diters += 1;
    const bool reach = c.diters >= o.degen_iters_max;
    if ((t == T_C0X0 || t == T_CPX0) && uh) c.hdeg = DEG_NO;
    else if (((t == T_C0XP && uh) || t == T_CPXP) && reach) c.hdeg = DEG_YES;
    if ((t == T_C0X0 || t == T_C0XP) && uj) c.jdeg = DEG_NO;
    else if (((t == T_CPX0 && uj) || t == T_CPXP) && reach) c.jdeg = DEG_YES;
}

__device__ inline bool pert_wrong_inertia(PertCol& c, const PertPrm& o) {   // get_deltas_for_wrong_inertia
    const double last = c.dx_last;
    const double first = last == 0.0 ? o.delta_w_0 : cmax(last * o.kappa_w_minus, o.delta_w_min);
    const double grow = (last == 0.0 || 1e5 * last < c.dx) ? c.dx * o.kappa_w_plus_bar : c.dx * o.kappa_w_plus;
    c.dx = c.dx == 0.0 ? first : grow;
    return c.dx <= o.delta_w_max;
}

__device__ inline double pert_cd(double mu, const PertPrm& o) { return o.delta_c_base * tpow(mu, o.kappa_c); }

__device__ inline bool pert_consider(PertCol& c, double mu, const PertPrm& o) {       // returns: failed
    pert_finalize(c, o);
    if (c.dx > 0.0) c.dx_last = c.dx;
    if (c.dc > 0.0) c.dc_last = c.dc;
    c.test = (c.hdeg == DEG_UNK || c.jdeg == DEG_UNK) ? T_C0X0 : T_NONE;
    c.dc = c.jdeg == DEG_YES ? pert_cd(mu, o) : 0.0;
    c.dx = 0.0;
    return c.hdeg == DEG_YES && !pert_wrong_inertia(c, o);
}

__device__ inline bool pert_singular(PertCol& c, double mu, const PertPrm& o) {
    bool wi;
    if (c.hdeg == DEG_UNK || c.jdeg == DEG_UNK) {
        if (c.test == T_C0X0) {
            if (c.jdeg == DEG_UNK) { c.dc = pert_cd(mu, o); c.test = T_CPX0; wi = false; }
            else { c.test = T_C0XP; wi = true; }
        } else if (c.test == T_CPX0) { c.dc = 0.0; c.test = T_C0XP; wi = true; }
        else if (c.test == T_C0XP) { c.dc = pert_cd(mu, o); c.test = T_CPXP; wi = true; }
        else wi = true;
    } else if (c.dc > 0.0 || c.jdeg == DEG_YES) wi = true;
    else { c.dc = pert_cd(mu, o); wi = false; }
    return wi && !pert_wrong_inertia(c, o);
}

__device__ inline bool pert_wrong(PertCol& c, double mu, const PertPrm& o) {
    pert_finalize(c, o);
    if (pert_wrong_inertia(c, o)) return false;
    if (c.dc != 0.0) return true;
    // fallback: delta_c > 0 and a fresh delta_w, with the Hessian's degeneracy unknown again
    c.dc = pert_cd(mu, o);
    c.dx = 0.0;
    c.test = T_NONE;
    if (c.hdeg == DEG_YES) c.hdeg = DEG_UNK;
    return !pert_wrong_inertia(c, o);
}

__global__ __launch_bounds__(CB) void k_perturb(int op, int W, int m, PertPrm o, long long* __restrict__ hdeg,
                                                long long* __restrict__ jdeg, long long* __restrict__ diters,
                                                long long* __restrict__ test, double* __restrict__ pdx,
                                                double* __restrict__ pdc, double* __restrict__ pdxl,
                                                double* __restrict__ pdcl, const double* __restrict__ mu,
                                                uint8_t* __restrict__ pend, const int32_t* __restrict__ inertia,
                                                double* __restrict__ dw_out, double* __restrict__ dc_out,
                                                uint8_t* __restrict__ tosolve, const uint8_t* __restrict__ fin) {
    const int b = blockIdx.x * CB + threadIdx.x;
    if (b >= W) return;
    bool p = pend[b] != 0;
    if (op == 2) {                              // after the solves: unrefinable ones count as singular
        p = tosolve[b] != 0 && fin[b] == 0;
        tosolve[b] = 0;
    }
    if (!p) {
        pend[b] = 0;
        return;
    }
    PertCol c{hdeg[b], jdeg[b], diters[b], test[b], pdx[b], pdc[b], pdxl[b], pdcl[b]};
    const double u = mu[b];
    if (op == 0) {
        p = !pert_consider(c, u, o);
    } else if (op == 1) {                       // one factorisation pass: classify the inertia
        const int* in = inertia + 3 * (long long)b;
        const bool sing = in[2] > 0 || in[1] < m;
        const bool wrong = !sing && in[1] > m;
        if (!sing && !wrong) {
            dw_out[b] = c.dx;
            dc_out[b] = c.dc;
            tosolve[b] = 1;
            p = false;
        } else {
            p = !(sing ? pert_singular(c, u, o) : pert_wrong(c, u, o));
        }
    } else {
        p = !pert_singular(c, u, o);
    }
    hdeg[b] = c.hdeg; jdeg[b] = c.jdeg; diters[b] = c.diters; test[b] = c.test;
    pdx[b] = c.dx; pdc[b] = c.dc; pdxl[b] = c.dx_last; pdcl[b] = c.dc_last;
    pend[b] = p ? 1 : 0;
}


// ------------------------------------------------------------------------------------------
// Termination tests of a lockstep iteration (batched_ipm.py solve, the `check` block) and the
// monotone barrier update (MonotoneMuUpdate, the `barrier` loop), one thread per column.
// ------------------------------------------------------------------------------------------
enum { ST_OPTIMAL = 1, ST_ACCEPTABLE = 2, ST_MAX_ITER = 3, ST_TINY_STEP = 8 };

struct StatusPrm {
    double tol, dual_inf_tol, constr_viol_tol, compl_inf_tol, acceptable_tol;
    long long acceptable_iter;
    double acceptable_dual_inf_tol, acceptable_constr_viol_tol, acceptable_compl_inf_tol;
};

__global__ __launch_bounds__(CB) void k_status(int W, StatusPrm o, const double* __restrict__ E0,
                                               const double* __restrict__ du, const double* __restrict__ pr_uns,
                                               const double* __restrict__ co, const double* __restrict__ sf,
                                               const long long* __restrict__ own, const long long* __restrict__ lim,
                                               uint8_t* __restrict__ act, long long* __restrict__ n_acc,
                                               long long* __restrict__ status) {
    const int b = blockIdx.x * CB + threadIdx.x;
    if (b >= W) return;
    bool a = act[b] != 0;
    long long st = status[b], na = n_acc[b];
    const double e = E0[b];
    // OptimalityErrorConvergenceCheck: the dual and complementarity tests on unscaled quantities (/ sf)
    const double du_u = du[b] / sf[b], co_u = co[b] / sf[b], pu = pr_uns[b];
    if (a && e <= o.tol && du_u <= o.dual_inf_tol && pu <= o.constr_viol_tol && co_u <= o.compl_inf_tol) {
        st = ST_OPTIMAL;
        a = false;
    }
    // CurrentIsAcceptable
    const bool acc = e <= o.acceptable_tol && du_u <= o.acceptable_dual_inf_tol && pu <= o.acceptable_constr_viol_tol &&
                     co_u <= o.acceptable_compl_inf_tol;
    na = (a && acc) ? na + 1 : 0;
    if (a && na >= o.acceptable_iter) {
        st = ST_ACCEPTABLE;
        a = false;
    }
    if (a && own[b] >= lim[b]) {
        st = ST_MAX_ITER;
        a = false;
    }
    act[b] = a ? 1 : 0;
    n_acc[b] = na;
    status[b] = st;
}

struct BarrierPrm {
    double kappa_eps, kappa_mu, theta_mu, mu_min, tau_min;
};

__global__ __launch_bounds__(CB) void k_barrier(int W, BarrierPrm o, const double* __restrict__ Emu,
                                                uint8_t* __restrict__ mu_act, uint8_t* __restrict__ force,
                                                uint8_t* __restrict__ act, long long* __restrict__ status,
                                                double* __restrict__ mu, double* __restrict__ tau,
                                                long long* __restrict__ nf, uint8_t* __restrict__ upd) {
    const int b = blockIdx.x * CB + threadIdx.x;
    if (b >= W) return;
    const double m = mu[b];
    const bool fo = force[b] != 0;
    bool ma = mu_act[b] != 0;
    const bool want = ma && ((Emu[b] <= o.kappa_eps * m) || fo);
    const double a = o.kappa_mu * m, c = tpow(m, o.theta_mu);
    const double mn = cmax(nmin(a, c), o.mu_min);             // torch.clamp(torch.minimum(.), min=)
    const bool same = mn == m;
    if (want && fo && same) {                                  // tiny step with mu at its floor
        status[b] = ST_TINY_STEP;
        act[b] = 0;
        ma = false;
    }
    const bool u = want && !same;
    if (u) {
        mu[b] = mn;
        tau[b] = cmax(1.0 - mn, o.tau_min);
        nf[b] = 0;
    }
    mu_act[b] = ma ? 1 : 0;
    force[b] = 0;
    upd[b] = u ? 1 : 0;
}


// ------------------------------------------------------------------------------------------
// Iterative refinement of the KKT solves (batched_ipm.py _refine, IPOPT's PDFullSpaceSolver):
// k_refine_pass = one pass over the [N][W] vectors of a step (the update a += b of the refining
// columns, column maxima of |a| and |c|: partials per row chunk), k_refine_decide = one workgroup
// folding the partials into IPOPT's residual ratio and the per-column decisions, with the ordered
// list of the columns that refine next (what torch.nonzero gave the host). Maxima are exact and
// propagate NaN as torch.amax does, so the fold order does not matter.
// ------------------------------------------------------------------------------------------
constexpr int RF_THREADS = 256;                  // 4 waves: 64 columns x 4 row strides
constexpr int RD_THREADS = 1024;                 // the decision workgroup

__global__ __launch_bounds__(RF_THREADS) void k_refine_pass(int N, int W, int rows, double* __restrict__ a,
                                                           const double* __restrict__ b,
                                                           const uint8_t* __restrict__ upd,
                                                           const double* __restrict__ c,
                                                           const uint8_t* __restrict__ sel,
                                                           double* __restrict__ pa, double* __restrict__ pc) {
    __shared__ double sa[4][64], sc[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int col = blockIdx.x * 64 + lane;
    const int r0 = blockIdx.y * rows, r1 = min(N, r0 + rows);
    const bool on = col < W && (!sel || sel[col] != 0);
    const bool up = on && b && upd && upd[col] != 0;
    double ma = 0.0, mc = 0.0;
    if (on) {
        for (int r = r0 + wv; r < r1; r += 4) {
            const long long i = (long long)r * W + col;
            double v = a[i];
            if (up) {
                v = v + b[i];
                a[i] = v;
            }
            ma = nmax(ma, fabs(v));
            if (c) mc = nmax(mc, fabs(c[i]));
        }
    }
    sa[wv][lane] = ma;
    sc[wv][lane] = mc;
    __syncthreads();
    if (wv == 0 && col < W) {
        const long long o = (long long)blockIdx.y * W + col;
        pa[o] = nmax(nmax(sa[0][lane], sa[1][lane]), nmax(sa[2][lane], sa[3][lane]));
        if (pc) pc[o] = nmax(nmax(sc[0][lane], sc[1][lane]), nmax(sc[2][lane], sc[3][lane]));
    }
}

struct RefinePrm {
    double ratio_max, ratio_singular;
    int min_steps, max_steps;
};

// IPOPT's residual ratio |r| / (min(|x|, 1e6 |rhs|) + |rhs|) (|r| where |x| + |rhs| = 0)
__device__ __forceinline__ double refine_ratio(double nres, double nx, double nr) {
    return nr + nx == 0.0 ? nres : nres / (nmin(nx, 1e6 * nr) + nr);
}

// mode 0: out0 = column maxima of the partials pa; mode 1: the first residual of the solve (sel = the
// solved columns); mode 2: after refinement step k (k counted from 1; sel = the columns that refined)
__global__ __launch_bounds__(RD_THREADS) void k_refine_decide(int W, int nch, int mode, int k, RefinePrm o,
                                                              const double* __restrict__ pa,
                                                              const double* __restrict__ pc,
                                                              const uint8_t* __restrict__ sel,
                                                              const double* __restrict__ nr, double* __restrict__ rr,
                                                              double* __restrict__ old, uint8_t* __restrict__ bad,
                                                              uint8_t* __restrict__ refine, uint8_t* __restrict__ need,
                                                              int32_t* __restrict__ list, uint8_t* __restrict__ ok) {
    __shared__ int wcount[RD_THREADS / 64];
    __shared__ int total;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) total = 0;
    __syncthreads();
    for (int base = 0; base < W; base += RD_THREADS) {
        const int col = base + tid;
        bool flag = false;
        if (col < W) {
            double nx = 0.0, nres = 0.0;
            for (int q = 0; q < nch; ++q) {
                nx = nmax(nx, pa[(long long)q * W + col]);
                if (pc) nres = nmax(nres, pc[(long long)q * W + col]);
            }
            if (mode == 0) {
                rr[col] = nx;
            } else {
                const bool s = sel[col] != 0;
                double r = rr[col];
                bool rf, bd;
                if (mode == 1) {
                    r = s ? refine_ratio(nres, nx, nr[col]) : 0.0;
                    old[col] = r;
                    bd = false;
                    rf = s;
                } else {
                    bd = bad[col] != 0;
                    rf = false;
                    if (s) {
                        r = refine_ratio(nres, nx, nr[col]);
                        const bool quit = (r > o.ratio_max && k > o.max_steps) || (r > old[col] && k > o.min_steps);
                        bd = bd || (quit && r > o.ratio_singular);
                        rf = !quit;
                        old[col] = r;
                    }
                }
                rr[col] = r;
                bad[col] = bd ? 1 : 0;
                refine[col] = rf ? 1 : 0;
                flag = rf && fin(r) && (k >= o.min_steps ? r > o.ratio_max : true);
                need[col] = flag ? 1 : 0;
                ok[col] = (fin(r) && !bd) ? 1 : 0;
            }
        }
        if (mode != 0) {   // ordered compaction of the flags: wave ballots, then the waves in order
            const unsigned long long bal = __ballot(flag);
            if (lane == 0) wcount[wv] = __popcll(bal);
            __syncthreads();
            int off = total;
            for (int w = 0; w < wv; ++w) off += wcount[w];
            if (flag) list[1 + off + __popcll(bal & ((1ull << lane) - 1ull))] = col;
            __syncthreads();
            if (tid == 0) {
                int t = total;
                for (int w = 0; w < RD_THREADS / 64; ++w) t += wcount[w];
                total = t;
            }
            __syncthreads();
        }
    }
    if (mode != 0 && tid == 0) list[0] = total;
}


// ------------------------------------------------------------------------------------------
// Scaled Jacobian and its transpose product (batched_ipm.py, the optimality check and the soft
// restoration's primal-dual error): Js = jv * sg[row] entry by entry and jty = Js^T y, one thread per
// (column i, instance) walking column i's entries in the structure's column order (the stable argsort
// of the entries by column), so the sum runs in the order torch's segment_reduce adds them, from 0.
// Products and sums are rounded one at a time (no contraction into FMAs): bit for bit the torch
// formulation (a gather, a product, a gather, a product, a segment sum), in one pass over jv instead
// of five over [nnz][W].
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_js_jty(int n, int W, const int32_t* __restrict__ col_ptr,
                                                const int32_t* __restrict__ src, const int32_t* __restrict__ row,
                                                const double* __restrict__ jv, const double* __restrict__ sg,
                                                const double* __restrict__ y, double* __restrict__ js,
                                                double* __restrict__ jty) {
#pragma clang fp contract(off)
    const int b = blockIdx.x * 64 + (threadIdx.x & 63);
    const int i = blockIdx.y * 4 + (threadIdx.x >> 6);          // one wave per column: uniform entry loop
    if (i >= n || b >= W) return;
    const int e0 = col_ptr[i], e1 = col_ptr[i + 1];
    double acc = 0.0;
    for (int k = e0; k < e1; ++k) {
        const long long e = (long long)src[k] * W + b;
        const long long r = (long long)row[k] * W + b;
        double v = jv[e];
        if (sg) {
            v = v * sg[r];
            if (js) js[e] = v;
        }
        const double t = v * y[r];
        acc = acc + t;
    }
    jty[(long long)i * W + b] = acc;
}

// ------------------------------------------------------------------------------------------
// Rows of the restoration phase's reduced KKT system (batched_ipm.py _RestorationKKT.factor): the
// p and n variables of row i are eliminated, so the row diagonal becomes dr - 1/dp - 1/dn (the same
// operations in the same order as the torch formulation), and their diagonals' signs add to the
// inertia: cnt[b] = (#dp > 0 + #dn > 0, #dp < 0 + #dn < 0) over the rows (integer atomics: exact).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_resto_rows(int m, int W, int rows, const double* __restrict__ dr,
                                                    const double* __restrict__ dp, const double* __restrict__ dn,
                                                    double* __restrict__ drow, int* __restrict__ cnt) {
    __shared__ int sp[4][64], sn[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int col = blockIdx.x * 64 + lane;
    const int r0 = blockIdx.y * rows, r1 = min(m, r0 + rows);
    int np = 0, nn = 0;
    if (col < W) {
        for (int r = r0 + wv; r < r1; r += 4) {
            const long long i = (long long)r * W + col;
            const double a = dp[i], c = dn[i];
            drow[i] = (dr[i] - 1.0 / a) - 1.0 / c;
            np += (a > 0.0) + (c > 0.0);
            nn += (a < 0.0) + (c < 0.0);
        }
    }
    sp[wv][lane] = np;
    sn[wv][lane] = nn;
    __syncthreads();
    if (wv == 0 && col < W) {
        const int tp = sp[0][lane] + sp[1][lane] + sp[2][lane] + sp[3][lane];
        const int tn = sn[0][lane] + sn[1][lane] + sn[2][lane] + sn[3][lane];
        if (tp) atomicAdd(&cnt[2 * col + 0], tp);
        if (tn) atomicAdd(&cnt[2 * col + 1], tn);
    }
}

}  // namespace

extern "C" {

int ato_ipm_perturb(int32_t op, int32_t W, int32_t m, const double* prm, int64_t* hdeg, int64_t* jdeg,
                    int64_t* diters, int64_t* test, double* dx, double* dc, double* dx_last, double* dc_last,
                    const double* mu, uint8_t* pend, const int32_t* inertia, double* dw_out, double* dc_out,
                    uint8_t* tosolve, const uint8_t* fin, void* stream) {
    if (op < 0 || op > 2 || W < 0 || !prm) return fail(ATO_ERR_ARG, "ato_ipm_perturb: arguments");
    if (W == 0) return 0;
    if (!hdeg || !jdeg || !diters || !test || !dx || !dc || !dx_last || !dc_last || !mu || !pend ||
        (op == 1 && (!inertia || !dw_out || !dc_out || !tosolve)) || (op == 2 && (!tosolve || !fin)))
        return fail(ATO_ERR_ARG, "ato_ipm_perturb: arguments");
    const PertPrm o{prm[0], prm[1], prm[2], prm[3], prm[4], prm[5], prm[6], prm[7], (long long)prm[8]};
    hipLaunchKernelGGL(k_perturb, dim3((W + CB - 1) / CB), dim3(CB), 0, static_cast<hipStream_t>(stream), (int)op, W,
                       m, o, reinterpret_cast<long long*>(hdeg), reinterpret_cast<long long*>(jdeg),
                       reinterpret_cast<long long*>(diters), reinterpret_cast<long long*>(test), dx, dc, dx_last,
                       dc_last, mu, pend, inertia, dw_out, dc_out, tosolve, fin);
    return check_launch("ato_ipm_perturb");
}

int ato_ipm_kkt_diag(const ato_ipm_dims* d, const double* Sx, const double* Ss, const double* dw, const double* dc,
                     double* dx, double* dr, double* Ds, void* stream) {
    if (!d || d->n < 0 || d->mi < 0 || d->meq < 0 || d->mi + d->meq != d->m || d->W <= 0 || !Sx || !dw || !dc ||
        !dx || !dr || (d->mi && (!Ss || !Ds || !d->iin)) || (d->meq && !d->ieq))
        return fail(ATO_ERR_ARG, "ato_ipm_kkt_diag: arguments");
    const Dev v{d->n, d->m, d->mi, d->meq, d->W, d->iin, d->ieq, nullptr, nullptr, nullptr, nullptr};
    const long long cnt = (long long)(d->n + d->m) * d->W;
    if (cnt)
        hipLaunchKernelGGL(k_kkt_diag, dim3(lin_blocks(cnt)), dim3(256), 0, static_cast<hipStream_t>(stream), v, Sx,
                           Ss, dw, dc, dx, dr, Ds);
    return check_launch("ato_ipm_kkt_diag");
}

size_t ato_ipm_work_size(const ato_ipm_dims* d) {
    if (!d || d->W <= 0) return 0;
    const Parts P = make_parts(d->n, d->mi, d->meq, d->m);
    return (size_t)QMAX * (P.c0[4] + EG) * d->W;      // chunk partials + the errors fold's range partials
}

int ato_ipm_errors(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                   const double* g, const double* c_rhs, const double* sg, const double* y, const double* zl,
                   const double* zu, const double* vl, const double* vu, const double* dual_x, const double* mu,
                   const double* n_bounds, double s_max, double* work, double* out, void* stream) {
    Dev v;
    if (!make_dev(d, bd, v) || !work || !out || !mu || !n_bounds) return fail(ATO_ERR_ARG, "ato_ipm_errors: arguments");
    const Parts P = make_parts(d->n, d->mi, d->meq, d->m);
    auto st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_errors, col_grid(d->W, P.c0[4]), dim3(CB), 0, st, v, P, x, s, g, c_rhs, sg, y, zl, zu, vl,
                       vu, dual_x, mu, work);
    double* part = work + (size_t)QMAX * P.c0[4] * d->W;
    hipLaunchKernelGGL(k_errors_fold1, col_grid(d->W, EG), dim3(CB), 0, st, d->W, P.c0[4], work, part);
    hipLaunchKernelGGL(k_errors_fold2, col_grid(d->W, 1), dim3(CB), 0, st, d->W, d->m, s_max, n_bounds, part, out);
    return check_launch("ato_ipm_errors");
}

int ato_ipm_rhs(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                const double* g, const double* c_rhs, const double* gf, const double* jty, const double* y,
                const double* zl, const double* zu, const double* vl, const double* vu, const double* mu,
                double kappa_d, double* Sx, double* Ss, double* gx, double* gs, double* rhs_x, double* rhs_s,
                double* rhs_y, void* stream) {
    Dev v;
    if (!make_dev(d, bd, v) || !mu) return fail(ATO_ERR_ARG, "ato_ipm_rhs: arguments");
    auto st = static_cast<hipStream_t>(stream);
    const long long cnt = (long long)(d->n + d->mi) * d->W;
    if (cnt)
        hipLaunchKernelGGL(k_rhs, dim3(lin_blocks(cnt)), dim3(256), 0, st, v, x, s, g, c_rhs, gf, jty, y, zl, zu, vl,
                           vu, mu, kappa_d, Sx, Ss, gx, gs, rhs_x, rhs_s, rhs_y);
    const long long cr = (long long)d->m * d->W;
    if (cr) hipLaunchKernelGGL(k_resid_rows, dim3(lin_blocks(cr)), dim3(256), 0, st, v, g, s, c_rhs, rhs_y);
    return check_launch("ato_ipm_rhs");
}

int ato_ipm_direction(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                      const double* dx, const double* ds, const double* zl, const double* zu, const double* vl,
                      const double* vu, const double* gx, const double* gs, const double* mu, const double* tau,
                      double* dzl, double* dzu, double* dvl, double* dvu, double* work, double* out, void* stream) {
    Dev v;
    if (!make_dev(d, bd, v) || !work || !out || !mu || !tau) return fail(ATO_ERR_ARG, "ato_ipm_direction: arguments");
    const Parts P = make_parts(d->n, d->mi, 0, 0);
    auto st = static_cast<hipStream_t>(stream);
    if (P.c0[4])
        hipLaunchKernelGGL(k_direction, col_grid(d->W, P.c0[4]), dim3(CB), 0, st, v, P, x, s, dx, ds, zl, zu, vl, vu,
                           gx, gs, mu, tau, dzl, dzu, dvl, dvu, work);
    hipLaunchKernelGGL(k_direction_fold, col_grid(d->W, 1), dim3(CB * FG), 0, st, d->W, P.c0[4], work, out);
    return check_launch("ato_ipm_direction");
}

int ato_ipm_measures(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                     const double* g, const double* c_rhs, const double* f, const double* mu, double kappa_d,
                     double* work, double* out, void* stream) {
    Dev v;
    if (!make_dev(d, bd, v) || !work || !out || !mu || !f) return fail(ATO_ERR_ARG, "ato_ipm_measures: arguments");
    const Parts P = make_parts(d->n, d->mi, d->meq, 0);
    auto st = static_cast<hipStream_t>(stream);
    if (P.c0[4])
        hipLaunchKernelGGL(k_measures, col_grid(d->W, P.c0[4]), dim3(CB), 0, st, v, P, x, s, g, c_rhs, work);
    hipLaunchKernelGGL(k_measures_fold, col_grid(d->W, 1), dim3(CB * FG), 0, st, d->W, P.c0[4], f, mu, kappa_d, work, out);
    return check_launch("ato_ipm_measures");
}

int ato_ipm_multipliers(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                        const double* mu, const double* az, double kappa_sigma, double* zl, double* zu, double* vl,
                        double* vu, const double* dzl, const double* dzu, const double* dvl, const double* dvu,
                        void* stream) {
    Dev v;
    if (!make_dev(d, bd, v) || !mu || !az) return fail(ATO_ERR_ARG, "ato_ipm_multipliers: arguments");
    auto st = static_cast<hipStream_t>(stream);
    const long long cnt = (long long)(d->n + d->mi) * d->W;
    if (cnt)
        hipLaunchKernelGGL(k_multipliers, dim3(lin_blocks(cnt)), dim3(256), 0, st, v, x, s, mu, az, kappa_sigma, zl,
                           zu, vl, vu, dzl, dzu, dvl, dvu);
    return check_launch("ato_ipm_multipliers");
}

int ato_ipm_filter_accept(int32_t W, int32_t fmax, const double* theta, const double* phi, const double* gphi_d,
                          const double* alpha, const double* tht, const double* pht, const double* F,
                          int64_t* nf, const double* theta_max, const double* theta_min,
                          const uint8_t* pend, const uint8_t* first, const double* prm, int64_t* fr_n,
                          int64_t* fr_cnt, uint8_t* fr_last, uint8_t* ok, uint8_t* arm, uint8_t* soc, void* stream) {
    if (W < 0 || fmax < 0 || !prm) return fail(ATO_ERR_ARG, "ato_ipm_filter_accept: arguments");
    if (W == 0) return 0;
    if (!theta || !phi || !gphi_d || !alpha || !tht || !pht || (fmax && !F) || !nf || !theta_max || !theta_min ||
        !pend || !first || !ok || !arm || !soc || (fr_n && (!fr_cnt || !fr_last)))
        return fail(ATO_ERR_ARG, "ato_ipm_filter_accept: arguments");
    // prm: host array (ato_ipm.h)
    const FilterPrm o{prm[0], prm[1], prm[2], prm[3], prm[4], prm[5], prm[6], prm[7], (long long)prm[8],
                      (long long)prm[9]};
    hipLaunchKernelGGL(k_filter_accept, dim3((W + CB - 1) / CB), dim3(CB), 0, static_cast<hipStream_t>(stream), W,
                       fmax, theta, phi, gphi_d, alpha, tht, pht, F, nf, theta_max, theta_min, pend, first, o,
                       reinterpret_cast<int64_t*>(fr_n), reinterpret_cast<int64_t*>(fr_cnt), fr_last, ok, arm, soc);
    return check_launch("ato_ipm_filter_accept");
}

int ato_ipm_filter_multi(int32_t P, int32_t K, int32_t fmax, const double* theta, const double* phi,
                         const double* gphi_d, const double* alpha0, const double* alpha_min, const double* tht,
                         const double* pht, const double* F, int64_t* nf, const double* theta_max,
                         const double* theta_min, const double* prm, int64_t* fr_n, int64_t* fr_cnt, uint8_t* fr_last,
                         int32_t* kacc, uint8_t* failed, uint8_t* arm, void* stream) {
    if (P < 0 || K < 1 || fmax < 0 || !prm) return fail(ATO_ERR_ARG, "ato_ipm_filter_multi: arguments");
    if (P == 0) return 0;
    if (!theta || !phi || !gphi_d || !alpha0 || !alpha_min || !tht || !pht || (fmax && !F) || !nf || !theta_max ||
        !theta_min || !fr_n || !fr_cnt || !fr_last || !kacc || !failed || !arm)
        return fail(ATO_ERR_ARG, "ato_ipm_filter_multi: arguments");
    const FilterPrm o{prm[0], prm[1], prm[2], prm[3], prm[4], prm[5], prm[6], prm[7], (long long)prm[8],
                      (long long)prm[9]};
    hipLaunchKernelGGL(k_filter_multi, dim3((P + CB - 1) / CB), dim3(CB), 0, static_cast<hipStream_t>(stream), P, K,
                       fmax, theta, phi, gphi_d, alpha0, alpha_min, tht, pht, F, nf, theta_max, theta_min, o, fr_n,
                       fr_cnt, fr_last, kacc, failed, arm);
    return check_launch("ato_ipm_filter_multi");
}

int ato_ipm_status(int32_t W, const double* prm, const double* E0, const double* du, const double* pr_uns,
                   const double* co, const double* sf, const int64_t* own, const int64_t* lim, uint8_t* act,
                   int64_t* n_acc, int64_t* status, void* stream) {
    if (W < 0 || !prm) return fail(ATO_ERR_ARG, "ato_ipm_status: arguments");
    if (W == 0) return 0;
    if (!E0 || !du || !pr_uns || !co || !sf || !own || !lim || !act || !n_acc || !status)
        return fail(ATO_ERR_ARG, "ato_ipm_status: arguments");
    const StatusPrm o{prm[0], prm[1], prm[2], prm[3], prm[4], (long long)prm[5], prm[6], prm[7], prm[8]};
    hipLaunchKernelGGL(k_status, dim3((W + CB - 1) / CB), dim3(CB), 0, static_cast<hipStream_t>(stream), W, o, E0, du,
                       pr_uns, co, sf, reinterpret_cast<const long long*>(own),
                       reinterpret_cast<const long long*>(lim), act, reinterpret_cast<long long*>(n_acc),
                       reinterpret_cast<long long*>(status));
    return check_launch("ato_ipm_status");
}

int ato_ipm_barrier(int32_t W, const double* prm, const double* Emu, uint8_t* mu_act, uint8_t* force, uint8_t* act,
                    int64_t* status, double* mu, double* tau, int64_t* nf, uint8_t* upd, void* stream) {
    if (W < 0 || !prm) return fail(ATO_ERR_ARG, "ato_ipm_barrier: arguments");
    if (W == 0) return 0;
    if (!Emu || !mu_act || !force || !act || !status || !mu || !tau || !nf || !upd)
        return fail(ATO_ERR_ARG, "ato_ipm_barrier: arguments");
    const BarrierPrm o{prm[0], prm[1], prm[2], prm[3], prm[4]};
    hipLaunchKernelGGL(k_barrier, dim3((W + CB - 1) / CB), dim3(CB), 0, static_cast<hipStream_t>(stream), W, o, Emu,
                       mu_act, force, act, reinterpret_cast<long long*>(status), mu, tau,
                       reinterpret_cast<long long*>(nf), upd);
    return check_launch("ato_ipm_barrier");
}


int ato_ipm_refine_work(int32_t N, int32_t W) {
    if (N < 0 || W < 1) return 0;
    const int nch = N ? (N + 63) / 64 : 1;       // row chunks of 64 (16 rows per wave)
    return nch < 64 ? nch : 64;
}

int ato_ipm_refine_pass(int32_t N, int32_t W, double* a, const double* b, const uint8_t* upd, const double* c,
                        const uint8_t* sel, double* part_a, double* part_c, void* stream) {
    if (N < 0 || W < 0 || (W && (!a || !part_a || (c && !part_c) || (b && !upd))))
        return fail(ATO_ERR_ARG, "ato_ipm_refine_pass: arguments");
    if (W == 0) return 0;
    const int nch = ato_ipm_refine_work(N, W);
    const int rows = N ? (N + nch - 1) / nch : 0;
    hipLaunchKernelGGL(k_refine_pass, dim3((W + 63) / 64, nch), dim3(RF_THREADS), 0, static_cast<hipStream_t>(stream),
                       N, W, rows, a, b, upd, c, sel, part_a, c ? part_c : nullptr);
    return check_launch("ato_ipm_refine_pass");
}

int ato_ipm_refine_decide(int32_t N, int32_t W, int32_t mode, int32_t k, const double* prm, const double* part_a,
                          const double* part_c, const uint8_t* sel, const double* nr, double* rr, double* old,
                          uint8_t* bad, uint8_t* refine, uint8_t* need, int32_t* list, uint8_t* ok, void* stream) {
    if (N < 0 || W < 0 || mode < 0 || mode > 2 || !prm) return fail(ATO_ERR_ARG, "ato_ipm_refine_decide: arguments");
    if (W == 0) return 0;
    if (!part_a || !rr || (mode && (!part_c || !sel || !nr || !old || !bad || !refine || !need || !list || !ok)))
        return fail(ATO_ERR_ARG, "ato_ipm_refine_decide: arguments");
    const RefinePrm o{prm[0], prm[1], (int)prm[2], (int)prm[3]};
    hipLaunchKernelGGL(k_refine_decide, dim3(1), dim3(RD_THREADS), 0, static_cast<hipStream_t>(stream), W,
                       ato_ipm_refine_work(N, W), mode, k, o, part_a, mode ? part_c : nullptr, sel, nr, rr, old, bad,
                       refine, need, list, ok);
    return check_launch("ato_ipm_refine_decide");
}


int ato_ipm_resto_rows(int32_t m, int32_t W, const double* dr, const double* dp, const double* dn, double* drow,
                       int32_t* cnt, void* stream) {
    if (m < 0 || W < 0 || (m && W && (!dr || !dp || !dn || !drow || !cnt)))
        return fail(ATO_ERR_ARG, "ato_ipm_resto_rows: arguments");
    if (m == 0 || W == 0) return 0;
    const int rows = 256;
    hipLaunchKernelGGL(k_resto_rows, dim3((W + 63) / 64, (m + rows - 1) / rows), dim3(256), 0,
                       static_cast<hipStream_t>(stream), m, W, rows, dr, dp, dn, drow, cnt);
    return check_launch("ato_ipm_resto_rows");
}

int ato_ipm_js_jty(int32_t n, int32_t nnz, int32_t W, const int32_t* col_ptr, const int32_t* src, const int32_t* row,
                   const double* jv, const double* sg, const double* y, double* js, double* jty, void* stream) {
    if (n < 0 || nnz < 0 || W < 0 || (n && W && (!col_ptr || !jty || (nnz && (!src || !row || !jv || !y)))) ||
        (js && !sg))
        return fail(ATO_ERR_ARG, "ato_ipm_js_jty: arguments");
    if (n == 0 || W == 0) return 0;
    hipLaunchKernelGGL(k_js_jty, dim3((W + 63) / 64, (n + 3) / 4), dim3(256), 0, static_cast<hipStream_t>(stream),
                       n, W, col_ptr, src, row, jv, sg, y, js, jty);
    return check_launch("ato_ipm_js_jty");
}

}  // extern "C"
