// ato_program.hpp -- the NLP transcription as "segment programs".
//
// A segment is a run of consecutive constraint rows of g(w) that one thread produces
// (the rows of one collocation node, the continuity block of one interval, one gate, ...).
// Each program walks its rows in the reference's order and, per row, calls
//     sink.jac(col, value)      for every structural Jacobian entry (ascending col)
//     sink.row(g, lbg, ubg)     to close the row
// The same code runs
//   * on the host with a pattern sink  -> CSR sparsity, lbg/ubg, segment offsets
//   * on the device with a value sink  -> g and J values for one problem instance
// so the sparsity pattern and the values cannot drift apart.
//
// Reference row families (drone3d/raceline/base_raceline.py):
//   collocation ODE / s-dot / input-rate rows     :398-434
//   regularity rows                               :1114-1130
//   model stage constraints (point-mass ball)     :436-451, point_model.py:122-129
//   continuity (+ quaternion normalisation)       :460-490, :1132-1181, drone_raceline.py:42-45
//   fixed-s rows                                  :1165-1181
//   gates                                         :545-595, :907-918, :986-1032
//   equal-h rows (global frame)                   :891-905
//   loop closure                                  :492-514, :1183-1227, drone_raceline.py:47-104
//   obstacle-tube sphere rows                     obstacles/mesh_obstacle.py:219-237
//   cost                                          :601-623
#pragma once
#include "ato_models.hpp"
#include "ato_dual.hpp"
#include "../../include/ato.h"

namespace ato {

// Row segments of node (n, k) in reference order: s-dot row, ODE rows (two groups), dU rows;
// then per interval: regularity rows, stage rows, continuity, fixed-s rows.
enum SegKind { SEG_SDOT = 0, SEG_ODE_A, SEG_ODE_B, SEG_DU, SEG_REG, SEG_STAGE, SEG_SPHERE, SEG_CONT,
               SEG_SROWS, SEG_RK4S, SEG_RK4, SEG_CPC_COMP, SEG_CPC_ORDER, SEG_CPC_PROG, NSEG };
enum TailKind { TAIL_HEQ = 0, TAIL_CLOSURE_BASE, TAIL_INITIAL, TAIL_TERMINAL, TAIL_GATE,
                TAIL_DRONE_CLOSURE };
// Work units of the evaluation kernel (one per grid.y index; see ato_layout.hpp)
//   UNIT_TAIL      one tail segment (equal-h rows, a gate, the closure); for RK4 closures one
//                  unit per column group of the step Jacobian
//   UNIT_ODE_A/B   ODE defect rows [0, SPLIT) / [SPLIT, NZ) of node (n, k > 0)
//   UNIT_NODE      s-dot, dU, regularity, stage, sphere and RK4 s rows of node (n, k); grad f of its inputs
//   UNIT_INTERVAL  continuity and fixed-s rows of interval n; d f / d h_n
//   UNIT_RK4       RK4 step rows of interval n, Jacobian column group k
enum UnitKind { UNIT_TAIL = 0, UNIT_ODE_A, UNIT_ODE_B, UNIT_NODE, UNIT_INTERVAL, UNIT_RK4 };

// Jacobian columns of one RK4 step Phi(z_n, u_n, h_n) handled by one work unit. The local
// columns are numbered h = 0, z_m = 1 + m, u_j = 1 + NZ + j; group g covers [g RK4_CG, (g+1) RK4_CG).
#ifndef ATO_RK4_CG
#define ATO_RK4_CG 3
#endif
constexpr int RK4_CG = ATO_RK4_CG;
template <class M>
constexpr int rk4_groups() { return (1 + M::NZ + M::NU + RK4_CG - 1) / RK4_CG; }

// sinks that only record the sparsity pattern (no values, sequential entries)
template <class S>
struct SinkTraits { static constexpr bool pattern = false; };

#ifndef ATO_INF
#define ATO_INF (__builtin_huge_val())
#endif

// Problem constants as the kernels see them (passed by value as a kernel argument).
struct ProbD {
    int32_t model, att, frame, trans;
    int32_t N, K, K1, P, NZ, NU, NV, nw, ng, nnz;
    int32_t closed, cleanly_closed, quat_flip, force_reg, n_gates, phase_len, has_spheres, n_tail;
    double euler_wraps, gamma;
    Vehicle veh;
    double Rc[16], dRc[16];
    double tau[ATO_KMAX + 1], Bq[ATO_KMAX + 1], C[(ATO_KMAX + 1) * (ATO_KMAX + 1)], D[ATO_KMAX + 1];
    double A_skew[4];
    const double* geom;        // [P][ATO_GEOM_WIDTH]
    const double* node_s;      // [P]
    const double* interval_s;  // [N+1]
    const ato_gate* gates;     // [n_gates]
    const double* spheres;     // [P][3]
    const int32_t* seg;        // [P][NSEG][2]  (row0, nnz0); -1 = absent
    const int32_t* tail;       // [n_tail][4]   (kind, index, row0, nnz0)
    const int32_t* units;      // [n_units][4]  (UnitKind, n, k, 0)
    int32_t n_units, pad_units;
    int32_t cls_off[4];        // unit classes [cls_off[c], cls_off[c+1]): tail, ODE, node/interval
    // per-instance sphere centres (config 4's perturbed tubes; ato_set_instance_spheres): device
    // [P][2][isph_stride] (dy, dn of node p for instance b at (2 p + c) isph_stride + b), read through
    // the decision-vector accessor's par(); NULL: the shared table `spheres`
    const double* isph;
    int64_t isph_stride;
    // CPC gate progress (cpc_m > 0): node q's lambda, mu, nu at cpc_off + 3 cpc_m q + [0, cpc_m),
    // [cpc_m, 2 cpc_m), [2 cpc_m, 3 cpc_m); waypoints [cpc_m][3] (a table like the spheres: in the
    // kernel argument an indexed array would be copied into registers)
    int32_t cpc_m, cpc_off;
    const double* cpc_wp;
    // 1: the gradient passes write only the structural nonzeros of grad f (h and the inputs; the
    // caller zero-fills the buffer once, ato_gradf_mode); 0: every entry (the states' zeros too)
    int32_t gf_sparse;
};

// nodes per interval: compile-time KS (specialised kernels for common K) or runtime p.K1
#define K1S(p) (KS ? KS : (p).K1)

// first row of the second ODE group (drone: body-velocity rows; point mass: none)
template <class M>
constexpr int ode_split() { return M::IS_DRONE ? M::IV : M::NZ; }

template <class T>
ATO_HD NodeGeom<T> load_geom(const ProbD& p, int node) {
    NodeGeom<T> G;
    const double* gp = p.geom + (long)node * ATO_GEOM_WIDTH;
    for (int i = 0; i < 9; ++i) G.Rp[i] = T(gp[i]);
    G.ks = T(gp[9]);
    G.ky = T(gp[10]);
    G.kn = T(gp[11]);
    G.mag = T(gp[12]);
    return G;
}

// column helpers: w = [h_0..h_{N-1}, (Z, U, dU) for every node (n, k)]
template <class M>
struct Cols {
    static constexpr int NZ = M::NZ, NU = M::NU, NV = NZ + 2 * NU;
    int N, K1;
    ATO_HD int node(int n, int k) const { return N + (n * K1 + k) * NV; }
    ATO_HD int z(int n, int k, int i) const { return node(n, k) + i; }
    ATO_HD int u(int n, int k, int i) const { return node(n, k) + NZ + i; }
    ATO_HD int du(int n, int k, int i) const { return node(n, k) + NZ + NU + i; }
};

// -------------------------------------------------------------------------- collocation node
// p_k = sum_j C[j][k] Z_j / h  (base_raceline.py:413-418): numerators for components [I0, I1)
template <class M, class T, int KS, class W>
ATO_HD void poly_num(const ProbD& p, int n, int k, int I0, int I1, int uz, const W& w, T* P) {
    const Cols<M> c{p.N, K1S(p)};
    const int K1 = K1S(p);
    for (int i = I0; i < I1; ++i) P[i - I0] = T(0);
#pragma unroll
    for (int j = 0; j < K1; ++j) {
        const T cj = T(p.C[j * K1 + k]);
        const int base = uz ? c.u(n, j, 0) : c.z(n, j, 0);
        for (int i = I0; i < I1; ++i) P[i - I0] += cj * w(base + i);
    }
}

// poly_ode[0] >= 0  (parametric; base_raceline.py:422-425)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_sdot(const ProbD& p, int n, int k, const W& w, S& s) {
    const Cols<M> c{p.N, K1S(p)};
    const T h = w(n), ih = T(1) / h;
    T P0;
    poly_num<M, T, KS>(p, n, k, 0, 1, 0, w, &P0);
    s.jac(n, -P0 * ih * ih);
    for (int j = 0; j < K1S(p); ++j) s.jac(c.z(n, j, 0), T(p.C[j * K1S(p) + k]) * ih);
    s.row(P0 * ih, 0.0, ATO_INF);
}

// f_i(Z_k, U_k) - poly_ode_i = 0 for rows i in [R0, R1), k > 0  (base_raceline.py:427-430)
template <class M, class T, int KS, int R0, int R1, class W, class S>
ATO_HD void seg_ode(const ProbD& p, int n, int k, const W& w, S& s) {
    constexpr int NZ = M::NZ, NU = M::NU;
    const Cols<M> c{p.N, K1S(p)};
    const int K1 = K1S(p);
    const T h = w(n);
    const T ih = T(1) / h, ih2 = ih * ih;
    T Pz[R1 - R0 > 0 ? R1 - R0 : 1];
    poly_num<M, T, KS>(p, n, k, R0, R1, 0, w, Pz);
    T z[NZ], u[NU];
#pragma unroll
    for (int i = 0; i < NZ; ++i) z[i] = w(c.z(n, k, i));
#pragma unroll
    for (int i = 0; i < NU; ++i) u[i] = w(c.u(n, k, i));
    const NodeGeom<T> G = load_geom<T>(p, n * K1 + k);
    const T ckk = T(p.C[k * K1 + k]) * ih;
    M::template rows<R0, R1>(z, u, G, p.veh, [&](int i, T fi, const T* dz, const T* du) {
        const T Pi = Pz[i - R0];
        s.jac(n, Pi * ih2);
        for (int j = 0; j < k; ++j) s.jac(c.z(n, j, i), -T(p.C[j * K1 + k]) * ih);
#pragma unroll
        for (int m = 0; m < NZ; ++m)
            if (M::zmask(i, m) || m == i) s.jac(c.z(n, k, m), m == i ? dz[m] - ckk : dz[m]);
#pragma unroll
        for (int m = 0; m < NU; ++m)
            if (M::umask(i, m)) s.jac(c.u(n, k, m), du[m]);
        for (int j = k + 1; j < K1; ++j) s.jac(c.z(n, j, i), -T(p.C[j * K1 + k]) * ih);
        s.row(fi - Pi * ih, 0.0, 0.0);
    });
}

// dU - poly_du = 0  (base_raceline.py:432-434)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_du(const ProbD& p, int n, int k, const W& w, S& s) {
    constexpr int NU = M::NU;
    const Cols<M> c{p.N, K1S(p)};
    const int K1 = K1S(p);
    const T h = w(n), ih = T(1) / h, ih2 = ih * ih;
    T Pu[NU];
    poly_num<M, T, KS>(p, n, k, 0, NU, 1, w, Pu);
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        s.jac(n, Pu[i] * ih2);
#pragma unroll
        for (int j = 0; j < K1; ++j) {
            s.jac(c.u(n, j, i), -T(p.C[j * K1 + k]) * ih);
            if (j == k) s.jac(c.du(n, k, i), T(1));
        }
        s.row(w(c.du(n, k, i)) - Pu[i] * ih, 0.0, 0.0);
    }
}

// regularity: k_n y - k_y n <= gamma at nodes with k_y^2 + k_n^2 > 0.1 (base_raceline.py:1121-1129)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_reg(const ProbD& p, int n, int k, const W& w, S& s) {
    const Cols<M> c{p.N, K1S(p)};
    const double* gp = p.geom + (long)(n * K1S(p) + k) * ATO_GEOM_WIDTH;
    const T ky = T(gp[10]), kn = T(gp[11]);
    s.jac(c.z(n, k, 1), kn);
    s.jac(c.z(n, k, 2), -ky);
    s.row(kn * w(c.z(n, k, 1)) - ky * w(c.z(n, k, 2)), -ATO_INF, p.gamma);
}

// point-mass thrust ball u.u / T_max^2 <= 1  (point_model.py:122-129)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_stage(const ProbD& p, int n, int k, const W& w, S& s) {
    const Cols<M> c{p.N, K1S(p)};
    const T it2 = T(1) / (T(p.veh.Tmax) * T(p.veh.Tmax));
    T uu = T(0);
#pragma unroll
    for (int i = 0; i < M::NU; ++i) {
        const T ui = w(c.u(n, k, i));
        uu += ui * ui;
        s.jac(c.u(n, k, i), T(2) * ui * it2);
    }
    s.row(uu / T(p.veh.Tmax) / T(p.veh.Tmax), -ATO_INF, 1.0);
}

// obstacle tube: (y - dy)^2 + (n - dn)^2 <= r_avail^2  (mesh_obstacle.py:219-237)
// (the upper bound is the shared table's r^2; with per-instance spheres the caller holds per-instance
// bounds, ato_sphere_rows)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_sphere(const ProbD& p, int n, int k, const W& w, S& s) {
    const Cols<M> c{p.N, K1S(p)};
    const long node = (long)n * K1S(p) + k;
    const double* sp = p.spheres + node * 3;
    const double dy = p.isph ? w.par(2 * node) : sp[0];
    const double dn = p.isph ? w.par(2 * node + 1) : sp[1];
    const T ey = w(c.z(n, k, 1)) - T(dy);
    const T en = w(c.z(n, k, 2)) - T(dn);
    s.jac(c.z(n, k, 1), T(2) * ey);
    s.jac(c.z(n, k, 2), T(2) * en);
    s.row(ey * ey + en * en, -ATO_INF, sp[2] * sp[2]);
}

// ---- CPC gate progress (build-side: Foehn et al. 2021; the reference only displays a CPC
// trajectory, cpc_utils.py:14-101). Global frame: the position is z[0:3] of the node.
// complementarity: mu_j (|p - w_j|^2 - nu_j) = 0, j < M
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_cpc_comp(const ProbD& p, int n, int k, const W& w, S& s) {
    const Cols<M> c{p.N, K1S(p)};
    const int m = p.cpc_m;
    const long base = p.cpc_off + 3L * m * ((long)n * K1S(p) + k);
    const T px = w(c.z(n, k, 0)), py = w(c.z(n, k, 1)), pz = w(c.z(n, k, 2));
    for (int j = 0; j < m; ++j) {
        const T ex = px - T(p.cpc_wp[3 * j]), ey = py - T(p.cpc_wp[3 * j + 1]), ez = pz - T(p.cpc_wp[3 * j + 2]);
        const T mu = w(base + m + j), nu = w(base + 2 * m + j);
        const T d2 = ex * ex + ey * ey + ez * ez - nu;
        s.jac(c.z(n, k, 0), T(2) * mu * ex);
        s.jac(c.z(n, k, 1), T(2) * mu * ey);
        s.jac(c.z(n, k, 2), T(2) * mu * ez);
        s.jac(base + m + j, d2);
        s.jac(base + 2 * m + j, -mu);
        s.row(mu * d2, 0.0, 0.0);
    }
}

// waypoint order: lambda_j - lambda_{j+1} <= 0, j < M - 1
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_cpc_order(const ProbD& p, int n, int k, const W& w, S& s) {
    const int m = p.cpc_m;
    const long base = p.cpc_off + 3L * m * ((long)n * K1S(p) + k);
    for (int j = 0; j + 1 < m; ++j) {
        s.jac(base + j, T(1));
        s.jac(base + j + 1, T(-1));
        s.row(w(base + j) - w(base + j + 1), -ATO_INF, 0.0);
    }
}

// progress: lambda_{q+1,j} - lambda_{q,j} + mu_{q,j} = 0 (q = the node, q + 1 the next one in time)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_cpc_prog(const ProbD& p, int n, int k, const W& w, S& s) {
    const int m = p.cpc_m;
    const long base = p.cpc_off + 3L * m * ((long)n * K1S(p) + k);
    const long next = base + 3L * m;
    for (int j = 0; j < m; ++j) {
        s.jac(base + j, T(-1));
        s.jac(base + m + j, T(1));
        s.jac(next + j, T(1));
        s.row(w(next + j) - w(base + j) + w(base + m + j), 0.0, 0.0);
    }
}

// quaternion normalisation op(q) = q / |q| and its Jacobian (drone_raceline.py:42-45)
template <class T>
ATO_HD void qnormalize(const T* q, T* qh, T& inv_norm) {
    const T nq = tsqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    inv_norm = T(1) / nq;
    for (int i = 0; i < 4; ++i) qh[i] = q[i] / nq;
}

// The continuity operator on the attitude components (applied to the extrapolated interval end
// state in continuity rows, closures and open-line terminal rows):
//   ESP (NO = 4): q / |q|                               drone_raceline.py:42-45
//   DCM (NO = 9): one Newton-Schulz step towards SO(3),  P(R) = R (3 I - R^T R) / 2
//                 (build-side: the reference has no DCM pose). P is the identity on SO(3) and
//                 contracts the orthonormality error quadratically, so the Gauss-Legendre
//                 collocation, which conserves R^T R inside an interval, keeps every interval on
//                 SO(3) -- the analogue of the quaternion's normalisation, with no extra rows.
//                 (Round 5 measured the alternative of P at the closure only, identity continuity
//                 rows: fewer DCM instances converge)
//   others (NO = 0): the identity.
// v[a] = op(r)_a, jac(a, m) = d op(r)_a / d r_m (every (a, m) is structural).
template <class M, class T, int KIND = M::HAS_QUAT ? 1 : (M::HAS_DCM ? 2 : 0)>
struct AttOp {
    static constexpr int NO = 0;
    T v[1];
    ATO_HD void apply(const T*) {}
    ATO_HD T jac(int, int) const { return T(0); }
};

template <class M, class T>
struct AttOp<M, T, 1> {
    static constexpr int NO = 4;
    T v[4], iq;
    ATO_HD void apply(const T* q) { qnormalize(q, v, iq); }
    ATO_HD T jac(int a, int m) const { return ((a == m ? T(1) : T(0)) - v[a] * v[m]) * iq; }
};

template <class M, class T>
struct AttOp<M, T, 2> {
    static constexpr int NO = 9;
    T v[9], R[9], S[9], RR[9];     // S = R^T R, RR = R R^T
    ATO_HD void apply(const T* r) {
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = r[i];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                S[i * 3 + j] = R[i] * R[j] + R[3 + i] * R[3 + j] + R[6 + i] * R[6 + j];
                RR[i * 3 + j] = R[3 * i] * R[3 * j] + R[3 * i + 1] * R[3 * j + 1] + R[3 * i + 2] * R[3 * j + 2];
            }
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                v[i * 3 + j] = T(1.5) * R[i * 3 + j] -
                               T(0.5) * (R[i * 3] * S[j] + R[i * 3 + 1] * S[3 + j] + R[i * 3 + 2] * S[6 + j]);
    }
    // d P_ij / d R_ab = 3/2 d_ia d_jb - 1/2 (d_ia S_bj + R_ib R_aj + RR_ia d_jb)
    ATO_HD T jac(int ij, int ab) const {
        const int i = ij / 3, j = ij % 3, a = ab / 3, b = ab % 3;
        T acc = R[i * 3 + b] * R[a * 3 + j];
        if (i == a) acc += S[b * 3 + j];
        if (j == b) acc += RR[i * 3 + a];
        T out = T(-0.5) * acc;
        if (i == a && j == b) out += T(1.5);
        return out;
    }
};

// continuity into interval n >= 1 (base_raceline.py:474-490, parametric :1149-1163)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_cont(const ProbD& p, int n, const W& w, S& s) {
    constexpr int NZ = M::NZ, NU = M::NU, IR = M::IR;
    const Cols<M> c{p.N, K1S(p)};
    const int K1 = K1S(p);
    T zb[NZ], ub[NU];
#pragma unroll
    for (int i = 0; i < NZ; ++i) zb[i] = T(0);
#pragma unroll
    for (int i = 0; i < NU; ++i) ub[i] = T(0);
#pragma unroll
    for (int k = 0; k < K1; ++k) {
        const T dk = T(p.D[k]);
#pragma unroll
        for (int i = 0; i < NZ; ++i) zb[i] += w(c.z(n - 1, k, i)) * dk;
#pragma unroll
        for (int i = 0; i < NU; ++i) ub[i] += w(c.u(n - 1, k, i)) * dk;
    }
    using Op = AttOp<M, T>;
    constexpr int NO = Op::NO;
    Op op;
    if constexpr (NO > 0) op.apply(zb + IR);
#pragma unroll
    for (int i = (M::PARAM ? 1 : 0); i < NZ; ++i) {
        const bool isq = NO > 0 && i >= IR && i < IR + NO;
        if (isq) {
            const int a = i - IR;
#pragma unroll
            for (int k = 0; k < K1; ++k) {
                const T dk = T(p.D[k]);
#pragma unroll
                for (int m = 0; m < NO; ++m) s.jac(c.z(n - 1, k, IR + m), -dk * op.jac(a, m));
            }
            s.jac(c.z(n, 0, i), T(1));
            s.row(w(c.z(n, 0, i)) - op.v[a], 0.0, 0.0);
        } else {
            for (int k = 0; k < K1; ++k) s.jac(c.z(n - 1, k, i), -T(p.D[k]));
            s.jac(c.z(n, 0, i), T(1));
            s.row(w(c.z(n, 0, i)) - zb[i], 0.0, 0.0);
        }
    }
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        for (int k = 0; k < K1; ++k) s.jac(c.u(n - 1, k, i), -T(p.D[k]));
        s.jac(c.u(n, 0, i), T(1));
        s.row(w(c.u(n, 0, i)) - ub[i], 0.0, 0.0);
    }
}

// fixed path length at both ends of interval n (base_raceline.py:1165-1181)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_srows(const ProbD& p, int n, const W& w, S& s) {
    const Cols<M> c{p.N, K1S(p)};
    s.jac(c.z(n, 0, 0), T(1));
    s.row(w(c.z(n, 0, 0)) - T(p.interval_s[n]), 0.0, 0.0);
    T zN = T(0);
#pragma unroll
    for (int k = 0; k < K1S(p); ++k) {
        zN += w(c.z(n, k, 0)) * T(p.D[k]);
        s.jac(c.z(n, k, 0), T(p.D[k]));
    }
    s.row(zN - T(p.interval_s[n + 1]), 0.0, 0.0);
}

// -------------------------------------------------------------------------- tail segments
// equal step sizes within each gate phase (base_raceline.py:891-905)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_heq(const ProbD& p, const W& w, S& s) {
    for (int n = 0; n < p.N; n += p.phase_len) {
        for (int n2 = n + 1; n2 < n + p.phase_len; ++n2) {
            s.jac(n, T(-1));
            s.jac(n2, T(1));
            s.row(w(n2) - w(n), 0.0, 0.0);
        }
    }
}

// gate rows (base_raceline.py:545-595). Gate state x = xoff + E zc, zc = sum_k coef_k Z[n,k][comp]
//   parametric: comps (y, n), E = [e_y e_n], xoff = x_c(s)   (:1028-1030)
//   global:     comps (x1, x2, x3), E = I, xoff = 0          (:912)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_gate(const ProbD& p, int gi, const W& w, S& s) {
    const ato_gate& gt = p.gates[gi];
    const Cols<M> c{p.N, K1S(p)};
    const int n = gt.interval;
    const int nk = gt.n_coef;
    const int nc = M::PARAM ? 2 : 3;
    const int comp0 = M::PARAM ? 1 : 0;
    T E[3][3];
    for (int a = 0; a < 3; ++a) {
        if (M::PARAM) {
            E[a][0] = T(gt.ey[a]);
            E[a][1] = T(gt.en[a]);
            E[a][2] = T(0);
        } else {
            for (int b = 0; b < 3; ++b) E[a][b] = T(a == b ? 1 : 0);
        }
    }
    T zc[3] = {T(0), T(0), T(0)};
    for (int k = 0; k < nk; ++k) {
        const T ck = T(gt.coef[k]);
        for (int q = 0; q < nc; ++q) zc[q] += w(c.z(n, k, comp0 + q)) * ck;
    }
    T x[3], dx[3];
    for (int a = 0; a < 3; ++a) {
        x[a] = M::PARAM ? T(gt.xc[a]) : T(0);
        for (int q = 0; q < nc; ++q) x[a] += zc[q] * E[a][q];
        dx[a] = x[a] - T(gt.gate_x[a]);
    }
    // emit one row whose value is linear or quadratic in zc:  dval/dzc given
    auto emit_row = [&](const T* dzc, T val, double lb, double ub) {
        for (int k = 0; k < nk; ++k) {
            const T ck = T(gt.coef[k]);
            for (int q = 0; q < nc; ++q) s.jac(c.z(n, k, comp0 + q), ck * dzc[q]);
        }
        s.row(val, lb, ub);
    };
    const double dmax = gt.d_max;
    if (gt.fix_center) {
        for (int a = 0; a < 3; ++a) {
            T d[3];
            for (int q = 0; q < 3; ++q) d[q] = E[a][q];
            emit_row(d, dx[a], 0.0, 0.0);
        }
        return;
    }
    // gate axes e1, e2, e3 = columns of R
    T e[3][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) e[b][a] = T(gt.R[a * 3 + b]);
    if (gt.shape == ATO_GATE_CIRCLE) {
        const T p2 = dx[0] * e[1][0] + dx[1] * e[1][1] + dx[2] * e[1][2];
        const T p3 = dx[0] * e[2][0] + dx[1] * e[2][1] + dx[2] * e[2][2];
        T d[3];
        for (int q = 0; q < 3; ++q) {
            const T E2 = E[0][q] * e[1][0] + E[1][q] * e[1][1] + E[2][q] * e[1][2];
            const T E3 = E[0][q] * e[2][0] + E[1][q] * e[2][1] + E[2][q] * e[2][2];
            d[q] = T(2) * p2 * E2 + T(2) * p3 * E3;
        }
        emit_row(d, p2 * p2 + p3 * p3, -ATO_INF, dmax * dmax);
        if (gt.axial) {
            T d1[3];
            for (int q = 0; q < 3; ++q) d1[q] = E[0][q] * e[0][0] + E[1][q] * e[0][1] + E[2][q] * e[0][2];
            const T xe = x[0] * e[0][0] + x[1] * e[0][1] + x[2] * e[0][2];
            const T ge = T(gt.gate_x[0]) * e[0][0] + T(gt.gate_x[1]) * e[0][1] + T(gt.gate_x[2]) * e[0][2];
            emit_row(d1, xe - ge, 0.0, 0.0);
        }
    } else {
        // delta = R^T (x - gate_x); rows 1,2 (+ row 0 when axial)
        for (int i = gt.axial ? 0 : 1; i < 3; ++i) {
            T d[3];
            for (int q = 0; q < 3; ++q) d[q] = E[0][q] * e[i][0] + E[1][q] * e[i][1] + E[2][q] * e[i][2];
            const T del = dx[0] * e[i][0] + dx[1] * e[i][1] + dx[2] * e[i][2];
            if (i == 0) emit_row(d, del, 0.0, 0.0);
            else emit_row(d, del, -dmax, dmax);
        }
    }
}

// end-of-horizon quantities for collocation: zF = op(sum_k D_k Z[N-1,k]), uF = sum_k D_k U[N-1,k]
// (base_raceline.py:322-348)

// drone loop closure (drone_raceline.py:47-104), appended after gates
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_drone_closure(const ProbD& p, const W& w, S& s) {
    constexpr int NZ = M::NZ, NU = M::NU, IR = M::IR, NR = M::NR;
    const Cols<M> c{p.N, K1S(p)};
    const int K1 = K1S(p), nl = p.N - 1;
    T zb[NZ], ub[NU];
#pragma unroll
    for (int i = 0; i < NZ; ++i) zb[i] = T(0);
#pragma unroll
    for (int i = 0; i < NU; ++i) ub[i] = T(0);
#pragma unroll
    for (int k = 0; k < K1; ++k) {
        const T dk = T(p.D[k]);
#pragma unroll
        for (int i = 0; i < NZ; ++i) zb[i] += w(c.z(nl, k, i)) * dk;
#pragma unroll
        for (int i = 0; i < NU; ++i) ub[i] += w(c.u(nl, k, i)) * dk;
    }
    using Op = AttOp<M, T>;
    constexpr int NO = Op::NO;
    Op op;
    if constexpr (NO > 0) op.apply(zb + IR);
    // uF - u0
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        s.jac(c.u(0, 0, i), T(-1));
        for (int k = 0; k < K1; ++k) s.jac(c.u(nl, k, i), T(p.D[k]));
        s.row(ub[i] - w(c.u(0, 0, i)), 0.0, 0.0);
    }
    auto plain = [&](int i, T offset) {
        s.jac(c.z(0, 0, i), T(-1));
        for (int k = 0; k < K1; ++k) s.jac(c.z(nl, k, i), T(p.D[k]));
        s.row(zb[i] - w(c.z(0, 0, i)) - offset, 0.0, 0.0);
    };
    plain(1, T(0));
    plain(2, T(0));
    // z_delta[7:] (ESP), z_delta[12:] (DCM) or z_delta[4:] (YPR): everything after the first
    // attitude slot(s)
    const int first_after = NO > 0 ? IR + NO : IR + 1;
    for (int i = first_after; i < NZ; ++i) plain(i, T(0));
    if constexpr (NO > 0) {
        // ESP: op(q_F) -/+ q_0 (the sign of the warm start's branch); DCM: op(R_F) - R_0
        const T sgn = (M::HAS_QUAT && p.quat_flip) ? T(1) : T(-1);
#pragma unroll
        for (int a = 0; a < NO; ++a) {
            s.jac(c.z(0, 0, IR + a), sgn);
#pragma unroll
            for (int k = 0; k < K1; ++k) {
                const T dk = T(p.D[k]);
#pragma unroll
                for (int m = 0; m < NO; ++m) s.jac(c.z(nl, k, IR + m), dk * op.jac(a, m));
            }
            s.row(op.v[a] + sgn * w(c.z(0, 0, IR + a)), 0.0, 0.0);
        }
    } else {
        const double two_pi = 6.283185307179586;
        plain(IR, T(two_pi * p.euler_wraps));
    }
    (void)NR;
    if (!M::PARAM) plain(0, T(0));
}

// open-line boundary rows (not closed): at the start (end = 0: Z[0,0], U[0,0]) and at the end
// (end = 1: zF = op(sum_k D_k Z[N-1,k]), uF = sum_k D_k U[N-1,k]; _zF applies the continuity
// operator), in the reference's order:
//   |v_g|^2 <= 0                      BaseRaceline._enforce_initial/terminal_constraints
//                                     (base_raceline.py:516-543), v_g = R v_b (f_vg)
//   drone: R[:, 2] = (0, 0, 1), w_b = 0   DroneRaceline (drone_raceline.py:110-148)
//   point mass: T_g[0] = T_g[1] = 0       PointRaceline (point_raceline.py:15-45), T_g = R u
// R is the global rotation of the attitude (global frame, parametric with global_r); the point
// mass has R = I there. (Parametric relative attitude, R = R_p(s) R(r), is rejected by the
// layout: its R depends on s through the centreline spline.)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_boundary(const ProbD& p, int end, const W& w, S& s) {
    constexpr int NZ = M::NZ, NU = M::NU, IR = M::IR, IV = M::IV;
    const Cols<M> c{p.N, K1S(p)};
    const int nb = end ? p.N - 1 : 0;
    const int kn = end ? K1S(p) : 1;
    T zb[NZ], u[NU];
#pragma unroll
    for (int i = 0; i < NZ; ++i) zb[i] = T(0);
#pragma unroll
    for (int i = 0; i < NU; ++i) u[i] = T(0);
    for (int k = 0; k < kn; ++k) {
        const T ck = end ? T(p.D[k]) : T(1);
#pragma unroll
        for (int i = 0; i < NZ; ++i) zb[i] += w(c.z(nb, k, i)) * ck;
#pragma unroll
        for (int i = 0; i < NU; ++i) u[i] += w(c.u(nb, k, i)) * ck;
    }
    T z[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) z[i] = zb[i];
    using Op = AttOp<M, T>;
    constexpr int NO = Op::NO;
    Op op;
    const bool opq = M::IS_DRONE && NO > 0 && end;
    if constexpr (M::IS_DRONE && NO > 0) {
        if (opq) {
            op.apply(zb + IR);
#pragma unroll
            for (int a = 0; a < NO; ++a) z[IR + a] = op.v[a];
        }
    }
    // one row: derivatives dz (after the operator, mask zm) and du (mask um), chained through
    // op and the node coefficients; columns ascend node by node (z block, then u block)
    auto emit = [&](const T* dz, const bool* zm, const T* du, const bool* um, T val, double lb, double ub) {
        T dzb[NZ];
        bool zmb[NZ];
#pragma unroll
        for (int m = 0; m < NZ; ++m) {
            dzb[m] = dz[m];
            zmb[m] = zm[m];
        }
        if constexpr (M::IS_DRONE && NO > 0) {
            if (opq) {
                bool anyq = false;
#pragma unroll
                for (int a = 0; a < NO; ++a) anyq = anyq || zm[IR + a];
#pragma unroll
                for (int m = 0; m < NO; ++m) {
                    T acc = T(0);
#pragma unroll
                    for (int a = 0; a < NO; ++a) acc += dz[IR + a] * op.jac(a, m);
                    dzb[IR + m] = acc;
                    zmb[IR + m] = anyq;
                }
            }
        }
        for (int k = 0; k < kn; ++k) {
            const T ck = end ? T(p.D[k]) : T(1);
#pragma unroll
            for (int m = 0; m < NZ; ++m)
                if (zmb[m]) s.jac(c.z(nb, k, m), dzb[m] * ck);
#pragma unroll
            for (int j = 0; j < NU; ++j)
                if (um[j]) s.jac(c.u(nb, k, j), du[j] * ck);
        }
        s.row(val, lb, ub);
    };
    T dz[NZ], du[NU];
    bool zm[NZ], um[NU];
    auto clear = [&]() {
#pragma unroll
        for (int m = 0; m < NZ; ++m) {
            dz[m] = T(0);
            zm[m] = false;
        }
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            du[j] = T(0);
            um[j] = false;
        }
    };
    if constexpr (M::IS_DRONE) {
        using A = typename M::A;
        constexpr int NR = M::NR, IW = M::IW;
        T Ra[9];
        A::R(z + IR, Ra);
        const T* v = z + IV;
        T vg[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) vg[a] = Ra[a * 3] * v[0] + Ra[a * 3 + 1] * v[1] + Ra[a * 3 + 2] * v[2];
        // |v_g|^2 <= 0
        clear();
#pragma unroll
        for (int m = 0; m < NR; ++m) {
            T dRa[9];
            A::dR(z + IR, Ra, m, dRa);
            T acc = T(0);
#pragma unroll
            for (int a = 0; a < 3; ++a)
                acc += vg[a] * (dRa[a * 3] * v[0] + dRa[a * 3 + 1] * v[1] + dRa[a * 3 + 2] * v[2]);
            dz[IR + m] = T(2) * acc;
            bool dep = false;
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) dep = dep || A::R_dep(a, b, m);
            zm[IR + m] = dep;
        }
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            dz[IV + b] = T(2) * (vg[0] * Ra[b] + vg[1] * Ra[3 + b] + vg[2] * Ra[6 + b]);
            zm[IV + b] = true;
        }
        emit(dz, zm, du, um, vg[0] * vg[0] + vg[1] * vg[1] + vg[2] * vg[2], -ATO_INF, 0.0);
        // e3 = R[:, 2] = (0, 0, 1)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            clear();
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                T dRa[9];
                A::dR(z + IR, Ra, m, dRa);
                dz[IR + m] = dRa[a * 3 + 2];
                zm[IR + m] = A::R_dep(a, 2, m);
            }
            const double tgt = a == 2 ? 1.0 : 0.0;
            emit(dz, zm, du, um, Ra[a * 3 + 2], tgt, tgt);
        }
        // w_b = 0
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            clear();
            dz[IW + j] = T(1);
            zm[IW + j] = true;
            emit(dz, zm, du, um, z[IW + j], 0.0, 0.0);
        }
    } else {
        // point mass with R = I: |v|^2 <= 0, T_g[0] = u[0], T_g[1] = u[1]
        clear();
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            dz[IV + b] = T(2) * z[IV + b];
            zm[IV + b] = true;
        }
        emit(dz, zm, du, um, z[IV] * z[IV] + z[IV + 1] * z[IV + 1] + z[IV + 2] * z[IV + 2], -ATO_INF, 0.0);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            clear();
            du[j] = T(1);
            um[j] = true;
            emit(dz, zm, du, um, u[j], 0.0, 0.0);
        }
    }
}

// base loop closure used by the point-mass racelines (base_raceline.py:492-514, :1183-1227)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_closure_base(const ProbD& p, const W& w, S& s) {
    constexpr int NZ = M::NZ, NU = M::NU;
    const Cols<M> c{p.N, K1S(p)};
    const int K1 = K1S(p), nl = p.N - 1;
    T zb[NZ], ub[NU];
#pragma unroll
    for (int i = 0; i < NZ; ++i) zb[i] = T(0);
#pragma unroll
    for (int i = 0; i < NU; ++i) ub[i] = T(0);
#pragma unroll
    for (int k = 0; k < K1; ++k) {
        const T dk = T(p.D[k]);
#pragma unroll
        for (int i = 0; i < NZ; ++i) zb[i] += w(c.z(nl, k, i)) * dk;
#pragma unroll
        for (int i = 0; i < NU; ++i) ub[i] += w(c.u(nl, k, i)) * dk;
    }
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        s.jac(c.u(0, 0, i), T(-1));
        for (int k = 0; k < K1; ++k) s.jac(c.u(nl, k, i), T(p.D[k]));
        s.row(ub[i] - w(c.u(0, 0, i)), 0.0, 0.0);
    }
    if (!M::PARAM || p.cleanly_closed) {
        for (int i = M::PARAM ? 1 : 0; i < NZ; ++i) {
            s.jac(c.z(0, 0, i), T(-1));
            for (int k = 0; k < K1; ++k) s.jac(c.z(nl, k, i), T(p.D[k]));
            s.row(zb[i] - w(c.z(0, 0, i)), 0.0, 0.0);
        }
    } else {
        // A z0[1:3] - zF[1:3] ; z0[3:] - zF[3:]
        for (int r = 0; r < 2; ++r) {
            s.jac(c.z(0, 0, 1), T(p.A_skew[r * 2 + 0]));
            s.jac(c.z(0, 0, 2), T(p.A_skew[r * 2 + 1]));
            for (int k = 0; k < K1; ++k) s.jac(c.z(nl, k, 1 + r), -T(p.D[k]));
            s.row(T(p.A_skew[r * 2]) * w(c.z(0, 0, 1)) + T(p.A_skew[r * 2 + 1]) * w(c.z(0, 0, 2)) - zb[1 + r],
                  0.0, 0.0);
        }
        for (int i = 3; i < NZ; ++i) {
            s.jac(c.z(0, 0, i), T(1));
            for (int k = 0; k < K1; ++k) s.jac(c.z(nl, k, i), -T(p.D[k]));
            s.row(w(c.z(0, 0, i)) - zb[i], 0.0, 0.0);
        }
    }
}

// -------------------------------------------------------------------------- RK4 transcription
// Multiple shooting with one fixed RK4 step per interval (use_rk4; base_raceline.py:363-391
// global, :1052-1112 parametric with the geometry frozen at s_n, dynamics_model.py:91-114):
//   Phi(z, u, h) = z + h/6 (k1 + 2 k2 + 2 k3 + k4),  k_i = f(z + c_i h k_{i-1}, u), c = (0, 1/2, 1/2, 1)
// The Jacobian of Phi is obtained exactly by forward-mode dual numbers through the model's value
// path, RK4_CG columns per work unit.

// structural dependencies of Phi_i (dep) and of op(Phi)_i (dop): bit m < NZ = z_m, bit NZ + j = u_j;
// every row also depends on h
template <class M>
struct RK4Dep {
    static constexpr int NZ = M::NZ, NU = M::NU;
    uint32_t dep[NZ] = {}, dop[NZ] = {};
    constexpr RK4Dep() {
        uint32_t ub[NZ] = {}, kd[NZ] = {}, acc[NZ] = {};
        for (int i = 0; i < NZ; ++i) {
            for (int j = 0; j < NU; ++j)
                if (M::umask(i, j)) ub[i] |= 1u << (NZ + j);
            for (int m = 0; m < NZ; ++m)
                if (M::zmask(i, m)) kd[i] |= 1u << m;
            kd[i] |= ub[i];
            acc[i] = kd[i];
        }
        for (int st = 1; st < 4; ++st) {
            uint32_t zs[NZ] = {}, kn[NZ] = {};
            for (int m = 0; m < NZ; ++m) zs[m] = (1u << m) | kd[m];
            for (int i = 0; i < NZ; ++i) {
                kn[i] = ub[i];
                for (int m = 0; m < NZ; ++m)
                    if (M::zmask(i, m)) kn[i] |= zs[m];
                acc[i] |= kn[i];
            }
            for (int i = 0; i < NZ; ++i) kd[i] = kn[i];
        }
        for (int i = 0; i < NZ; ++i) dep[i] = dop[i] = (1u << i) | acc[i];
        constexpr int NO = M::HAS_QUAT ? 4 : (M::HAS_DCM ? 9 : 0);
        if (NO > 0) {
            uint32_t q = 0;
            for (int a = 0; a < NO; ++a) q |= dep[M::IR + a];
            for (int a = 0; a < NO; ++a) dop[M::IR + a] = q;
        }
    }
};

// Phi of interval n (op applied to the quaternion if OP) with tangents along local columns
// [grp RK4_CG, (grp + 1) RK4_CG)
template <class M, class T, bool OP, class W>
ATO_HD void rk4_phi(const ProbD& p, int n, int grp, const W& w, Dual<T, RK4_CG>* phi) {
    using D = Dual<T, RK4_CG>;
    constexpr int NZ = M::NZ, NU = M::NU;
    const Cols<M> c{p.N, 1};
    const int l0 = grp * RK4_CG;
    auto ld = [&](int col, int lid) {
        const int dir = lid - l0;
        return D::seed(w(col), (dir >= 0 && dir < RK4_CG) ? dir : -1);
    };
    const D h = ld(n, 0);
    D z[NZ], u[NU];
#pragma unroll
    for (int m = 0; m < NZ; ++m) z[m] = ld(c.z(n, 0, m), 1 + m);
#pragma unroll
    for (int j = 0; j < NU; ++j) u[j] = ld(c.u(n, 0, j), 1 + NZ + j);
    const NodeGeom<D> G = load_geom<D>(p, n);
    D k[NZ], acc[NZ], zs[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
        k[i] = D(0.0);
        acc[i] = D(0.0);
    }
    const D hh = h / 2.0;
    // one model instance in a rolled loop over the 4 stages (unrolling it keeps all stages'
    // temporaries live and spills)
#pragma unroll 1
    for (int st = 0; st < 4; ++st) {
        const D cs = st == 0 ? D(0.0) : (st == 3 ? h : hh);
#pragma unroll
        for (int i = 0; i < NZ; ++i) zs[i] = z[i] + cs * k[i];
        M::template rows<0, NZ>(zs, u, G, p.veh, [&](int i, D fi, const D*, const D*) { k[i] = fi; });
        const double wt = (st == 0 || st == 3) ? 1.0 : 2.0;
#pragma unroll
        for (int i = 0; i < NZ; ++i) acc[i] += k[i] * wt;
    }
    const D h6 = h / 6.0;
#pragma unroll
    for (int i = 0; i < NZ; ++i) phi[i] = z[i] + h6 * acc[i];
    if constexpr (OP && AttOp<M, D>::NO > 0) {
        AttOp<M, D> op;
        op.apply(phi + M::IR);
#pragma unroll
        for (int a = 0; a < AttOp<M, D>::NO; ++a) phi[M::IR + a] = op.v[a];
    }
}

// Writes the entries of one RK4-dependent row for work-unit group grp:
//   lin(col, v)   an entry that does not come from Phi (written by group 0)
//   dh(sgn)       sgn dPhi_i/dh        dzu(sgn)  sgn dPhi_i/d(z_n, u_n) in mask order
//   row(g, lb, ub) closes the row (g written by group 0)
// In pattern mode (SinkTraits<S>::pattern) every entry is emitted without values.
template <class M, class T, class S>
struct RK4Row {
    using D = Dual<T, RK4_CG>;
    static constexpr bool PAT = SinkTraits<S>::pattern;
    S& s;
    int grp, n, l0;
    const Cols<M>& c;
    ATO_HD bool mine(int lid) const { return lid >= l0 && lid < l0 + RK4_CG; }
    // tangent j of x without a dynamic register-array index
    ATO_HD static T pick(const D& x, int j) {
        T r = x.d[0];
#pragma unroll
        for (int q = 1; q < RK4_CG; ++q)
            if (j == q) r = x.d[q];
        return r;
    }
    ATO_HD void lin(int col, T v) {
        if (PAT || grp == 0) s.jac(col, v);
        else s.skip();
    }
    ATO_HD void dh(const D& x, T sgn) {
        if (PAT) s.jac(n, T(0));
        else if (mine(0)) s.jac(n, sgn * pick(x, 0 - l0));
        else s.skip();
    }
    ATO_HD void dzu(const D& x, uint32_t mask, T sgn) {
        constexpr int NZ = M::NZ, NU = M::NU;
#pragma unroll
        for (int m = 0; m < NZ + NU; ++m) {
            if (!(mask & (1u << m))) continue;
            const int col = m < NZ ? c.z(n, 0, m) : c.u(n, 0, m - NZ);
            if (PAT) s.jac(col, T(0));
            else if (mine(1 + m)) s.jac(col, sgn * pick(x, 1 + m - l0));
            else s.skip();
        }
    }
    ATO_HD void row(T g, double lb, double ub) {
        if (PAT || grp == 0) s.row(g, lb, ub);
        else s.row_skip();
    }
};

// s rows of RK4 interval n: Z[n,0][0] = s_n (parametric, every interval; base_raceline.py:1059-1063)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_rk4s(const ProbD& p, int n, const W& w, S& s) {
    const Cols<M> c{p.N, 1};
    s.jac(c.z(n, 0, 0), T(1));
    s.row(w(c.z(n, 0, 0)) - T(p.interval_s[n]), 0.0, 0.0);
}

// step rows of RK4 interval n < N-1 (base_raceline.py:379-386 global, :1079-1097 parametric):
//   Z[n+1][i] - op(Phi)_i (i >= 1 parametric), U[n+1] - (U_n + dU_n h/2) (F10),
//   Phi_0 - s_{n+1} (parametric)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_rk4(const ProbD& p, int n, int grp, const W& w, S& s) {
    using D = Dual<T, RK4_CG>;
    constexpr int NZ = M::NZ, NU = M::NU;
    constexpr RK4Dep<M> dp{};
    const Cols<M> c{p.N, 1};
    D phi[NZ];
    if constexpr (!SinkTraits<S>::pattern) rk4_phi<M, T, true>(p, n, grp, w, phi);
    RK4Row<M, T, S> r{s, grp, n, grp * RK4_CG, c};
#pragma unroll
    for (int i = (M::PARAM ? 1 : 0); i < NZ; ++i) {
        r.dh(phi[i], T(-1));
        r.dzu(phi[i], dp.dop[i], T(-1));
        r.lin(c.z(n + 1, 0, i), T(1));
        r.row(w(c.z(n + 1, 0, i)) - phi[i].v, 0.0, 0.0);
    }
    const T h = w(n);
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        const T dui = w(c.du(n, 0, i));
        r.lin(n, -dui / T(2));
        r.lin(c.u(n, 0, i), T(-1));
        r.lin(c.du(n, 0, i), -h / T(2));
        r.lin(c.u(n + 1, 0, i), T(1));
        r.row(w(c.u(n + 1, 0, i)) - w(c.u(n, 0, i)) - dui * h / T(2), 0.0, 0.0);
    }
    if (M::PARAM) {
        // s at the end of the step is Phi_0 itself (no continuity operator on s)
        r.dh(phi[0], T(1));
        r.dzu(phi[0], dp.dep[0], T(1));
        r.row(phi[0].v - T(p.interval_s[n + 1]), 0.0, 0.0);
    }
}

// drone loop closure with zF = op(Phi(Z[N-1])), uF = U[N-1] + dU[N-1] h (base_raceline.py:322-348,
// :1034-1050; drone_raceline.py:47-104)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_drone_closure_rk4(const ProbD& p, int grp, const W& w, S& s) {
    using D = Dual<T, RK4_CG>;
    constexpr int NZ = M::NZ, NU = M::NU, IR = M::IR;
    constexpr RK4Dep<M> dp{};
    const Cols<M> c{p.N, 1};
    const int nl = p.N - 1;
    D phi[NZ];
    if constexpr (!SinkTraits<S>::pattern) rk4_phi<M, T, true>(p, nl, grp, w, phi);
    RK4Row<M, T, S> r{s, grp, nl, grp * RK4_CG, c};
    const T h = w(nl);
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        const T dui = w(c.du(nl, 0, i));
        r.lin(nl, dui);
        r.lin(c.u(0, 0, i), T(-1));
        r.lin(c.u(nl, 0, i), T(1));
        r.lin(c.du(nl, 0, i), h);
        r.row(w(c.u(nl, 0, i)) + dui * h - w(c.u(0, 0, i)), 0.0, 0.0);
    }
    auto plain = [&](int i, T offset) {
        r.dh(phi[i], T(1));
        r.lin(c.z(0, 0, i), T(-1));
        r.dzu(phi[i], dp.dop[i], T(1));
        r.row(phi[i].v - w(c.z(0, 0, i)) - offset, 0.0, 0.0);
    };
    plain(1, T(0));
    plain(2, T(0));
    constexpr int NO = AttOp<M, T>::NO;
    const int first_after = NO > 0 ? IR + NO : IR + 1;
    for (int i = first_after; i < NZ; ++i) plain(i, T(0));
    if constexpr (NO > 0) {
        const T sgn = (M::HAS_QUAT && p.quat_flip) ? T(1) : T(-1);
#pragma unroll
        for (int a = 0; a < NO; ++a) {
            r.dh(phi[IR + a], T(1));
            r.lin(c.z(0, 0, IR + a), sgn);
            r.dzu(phi[IR + a], dp.dop[IR + a], T(1));
            r.row(phi[IR + a].v + sgn * w(c.z(0, 0, IR + a)), 0.0, 0.0);
        }
    } else {
        plain(IR, T(6.283185307179586 * p.euler_wraps));
    }
    if (!M::PARAM) plain(0, T(0));
}

// point-mass loop closure with the RK4 end state (base_raceline.py:492-514, :1183-1227)
template <class M, class T, int KS, class W, class S>
ATO_HD void seg_closure_base_rk4(const ProbD& p, int grp, const W& w, S& s) {
    using D = Dual<T, RK4_CG>;
    constexpr int NZ = M::NZ, NU = M::NU;
    constexpr RK4Dep<M> dp{};
    const Cols<M> c{p.N, 1};
    const int nl = p.N - 1;
    D phi[NZ];
    if constexpr (!SinkTraits<S>::pattern) rk4_phi<M, T, true>(p, nl, grp, w, phi);
    RK4Row<M, T, S> r{s, grp, nl, grp * RK4_CG, c};
    const T h = w(nl);
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        const T dui = w(c.du(nl, 0, i));
        r.lin(nl, dui);
        r.lin(c.u(0, 0, i), T(-1));
        r.lin(c.u(nl, 0, i), T(1));
        r.lin(c.du(nl, 0, i), h);
        r.row(w(c.u(nl, 0, i)) + dui * h - w(c.u(0, 0, i)), 0.0, 0.0);
    }
    if (!M::PARAM || p.cleanly_closed) {
        for (int i = M::PARAM ? 1 : 0; i < NZ; ++i) {
            r.dh(phi[i], T(1));
            r.lin(c.z(0, 0, i), T(-1));
            r.dzu(phi[i], dp.dop[i], T(1));
            r.row(phi[i].v - w(c.z(0, 0, i)), 0.0, 0.0);
        }
    } else {
        // A z0[1:3] - zF[1:3] ; z0[3:] - zF[3:]
        for (int q = 0; q < 2; ++q) {
            r.dh(phi[1 + q], T(-1));
            r.lin(c.z(0, 0, 1), T(p.A_skew[q * 2 + 0]));
            r.lin(c.z(0, 0, 2), T(p.A_skew[q * 2 + 1]));
            r.dzu(phi[1 + q], dp.dop[1 + q], T(-1));
            r.row(T(p.A_skew[q * 2]) * w(c.z(0, 0, 1)) + T(p.A_skew[q * 2 + 1]) * w(c.z(0, 0, 2)) - phi[1 + q].v,
                  0.0, 0.0);
        }
        for (int i = 3; i < NZ; ++i) {
            r.dh(phi[i], T(-1));
            r.lin(c.z(0, 0, i), T(1));
            r.dzu(phi[i], dp.dop[i], T(-1));
            r.row(w(c.z(0, 0, i)) - phi[i].v, 0.0, 0.0);
        }
    }
}

// -------------------------------------------------------------------------- cost
// J = sum_{n,k} h_n B_k (u'Ru + du'dR du + 1)   (base_raceline.py:601-623)
// stage cost at node (n, k) and its input / input-rate gradient (without the h_n B_k factor)
template <class M, class T, int KS, class W>
ATO_HD T stage_cost(const ProbD& p, int n, int k, const W& w, T* gu, T* gdu) {
    constexpr int NU = M::NU;
    const Cols<M> c{p.N, K1S(p)};
    T u[NU], du[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        u[i] = w(c.u(n, k, i));
        du[i] = w(c.du(n, k, i));
    }
    T L = T(1);
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        T ru = T(0), rdu = T(0), gui = T(0), gdui = T(0);
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            ru += T(p.Rc[i * NU + j]) * u[j];
            rdu += T(p.dRc[i * NU + j]) * du[j];
            gui += (T(p.Rc[i * NU + j]) + T(p.Rc[j * NU + i])) * u[j];
            gdui += (T(p.dRc[i * NU + j]) + T(p.dRc[j * NU + i])) * du[j];
        }
        L += u[i] * ru + du[i] * rdu;
        if (gu) gu[i] = gui;
        if (gdu) gdu[i] = gdui;
    }
    return L;
}

}  // namespace ato
