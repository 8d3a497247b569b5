// ato_models.hpp -- vehicle ODEs f(z, u; node geometry) with hand-derived Jacobians.
//
// Shared by the HIP kernels (device) and the host pattern builder: every function is
// ATO_HD. A model evaluates its rows in groups and hands each row to an emitter
//     emit(i, f_i, dz[NZ], du[NU])
// with dz / du holding d f_i / d z and d f_i / d u. Only entries whose mask bit is set
// (ZM / UM tables) are structural; the caller writes exactly those.
//
// Reference equations:
//   attitude R(r), M(r)          drone3d/dynamics/rotations.py:44-102
//   drone pose / forces / state  drone3d/dynamics/drone_models.py:47-123 (global),
//                                drone_models.py:249-292 (parametric pose)
//   point mass                   drone3d/dynamics/point_model.py:28-75, 149-213
// Quaternions are (qi, qj, qk, qr); R(q) is divided by |q|^2 exactly as rotations.py:50-66.
#pragma once

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define ATO_HD __host__ __device__ __forceinline__
#else
#define ATO_HD inline
#endif
#include <stdint.h>
#include <math.h>

namespace ato {

enum Att { ESP = 0, YPR = 1, DCM = 2 };
enum Frame { GLOBAL = 0, PARAM_GR = 1, PARAM_REL = 2 };

template <class T>
ATO_HD T sq(T x) { return x * x; }

template <class T>
ATO_HD T tsqrt(T x) { return sqrt(x); }
template <class T>
ATO_HD T tsin(T x) { return sin(x); }
template <class T>
ATO_HD T tcos(T x) { return cos(x); }

// Vehicle constants (pytypes.py:357-402). Kept in double; cast to T where used.
struct Vehicle {
    double m, g, b[3], I[3], bw[3], l, kt, Tmax;
};

// Darboux-frame constants of one node: Rp row-major (Rp[a*3+c] = component a of column
// c of [e_s e_y e_n]), curvatures and |x_c'| (spline_centerline.py:279-294).
template <class T>
struct NodeGeom {
    T Rp[9];
    T ks, ky, kn, mag;
};

// --------------------------------------------------------------------- attitude
// Euler symmetric parameters. R = Rn(q) / |q|^2, rdot = M(q) w.
struct AttESP {
    static constexpr int NR = 4;

    template <class T>
    ATO_HD static void R(const T* q, T* Rm) {
        const T a = q[0], b = q[1], c = q[2], d = q[3];
        const T iQ = T(1) / (a * a + b * b + c * c + d * d);
        Rm[0] = (T(1) - T(2) * b * b - T(2) * c * c) * iQ;
        Rm[1] = T(2) * (a * b - c * d) * iQ;
        Rm[2] = T(2) * (a * c + b * d) * iQ;
        Rm[3] = T(2) * (a * b + c * d) * iQ;
        Rm[4] = (T(1) - T(2) * a * a - T(2) * c * c) * iQ;
        Rm[5] = T(2) * (b * c - a * d) * iQ;
        Rm[6] = T(2) * (a * c - b * d) * iQ;
        Rm[7] = T(2) * (b * c + a * d) * iQ;
        Rm[8] = (T(1) - T(2) * a * a - T(2) * b * b) * iQ;
    }

    // dR/dq_m given R (row-major 3x3).  dR = (dRn - 2 q_m R) / |q|^2
    template <class T>
    ATO_HD static void dR(const T* q, const T* Rm, int m, T* out) {
        const T a = q[0], b = q[1], c = q[2], d = q[3];
        const T iQ = T(1) / (a * a + b * b + c * c + d * d);
        T dn[9];
        if (m == 0) {
            const T v[9] = {T(0), 2 * b, 2 * c, 2 * b, -4 * a, -2 * d, 2 * c, 2 * d, -4 * a};
            for (int i = 0; i < 9; ++i) dn[i] = v[i];
        } else if (m == 1) {
            const T v[9] = {-4 * b, 2 * a, 2 * d, 2 * a, T(0), 2 * c, -2 * d, 2 * c, -4 * b};
            for (int i = 0; i < 9; ++i) dn[i] = v[i];
        } else if (m == 2) {
            const T v[9] = {-4 * c, -2 * d, 2 * a, 2 * d, -4 * c, 2 * b, 2 * a, 2 * b, T(0)};
            for (int i = 0; i < 9; ++i) dn[i] = v[i];
        } else {
            const T v[9] = {T(0), -2 * c, 2 * b, 2 * c, T(0), -2 * a, -2 * b, 2 * a, T(0)};
            for (int i = 0; i < 9; ++i) dn[i] = v[i];
        }
        const T qm2 = T(2) * q[m];
        for (int i = 0; i < 9; ++i) out[i] = (dn[i] - qm2 * Rm[i]) * iQ;
    }

    // rdot = M(q) w ; drq[i][m] = d rdot_i / d q_m (w fixed) ; Mm[i][j] = M_ij
    template <class T>
    ATO_HD static void kin(const T* q, const T* w, T* rdot, T drq[4][4], T Mm[4][3]) {
        const T a = q[0], b = q[1], c = q[2], d = q[3];
        const T h = T(0.5);
        Mm[0][0] = h * d;  Mm[0][1] = -h * c; Mm[0][2] = h * b;
        Mm[1][0] = h * c;  Mm[1][1] = h * d;  Mm[1][2] = -h * a;
        Mm[2][0] = -h * b; Mm[2][1] = h * a;  Mm[2][2] = h * d;
        Mm[3][0] = -h * a; Mm[3][1] = -h * b; Mm[3][2] = -h * c;
        for (int i = 0; i < 4; ++i) rdot[i] = Mm[i][0] * w[0] + Mm[i][1] * w[1] + Mm[i][2] * w[2];
        drq[0][0] = T(0);     drq[0][1] = h * w[2];  drq[0][2] = -h * w[1]; drq[0][3] = h * w[0];
        drq[1][0] = -h * w[2]; drq[1][1] = T(0);    drq[1][2] = h * w[0];  drq[1][3] = h * w[1];
        drq[2][0] = h * w[1];  drq[2][1] = -h * w[0]; drq[2][2] = T(0);    drq[2][3] = h * w[2];
        drq[3][0] = -h * w[0]; drq[3][1] = -h * w[1]; drq[3][2] = -h * w[2]; drq[3][3] = T(0);
    }

    // structural dependencies of rdot_i on r_m (w fixed) and on w_j
    static constexpr bool kin_r(int i, int m) { return i != m; }
    static constexpr bool kin_w(int, int) { return true; }
    // R (any row) depends on every q (normalisation)
    static constexpr bool R_dep(int, int, int) { return true; }
};

// Yaw-pitch-roll (a, b, c): R = Rz(a) Ry(b) Rx(c)
struct AttYPR {
    static constexpr int NR = 3;

    template <class T>
    ATO_HD static void R(const T* r, T* Rm) {
        const T ca = tcos(r[0]), sa = tsin(r[0]), cb = tcos(r[1]), sb = tsin(r[1]);
        const T cc = tcos(r[2]), sc = tsin(r[2]);
        Rm[0] = ca * cb; Rm[1] = ca * sb * sc - sa * cc; Rm[2] = ca * sb * cc + sa * sc;
        Rm[3] = sa * cb; Rm[4] = sa * sb * sc + ca * cc; Rm[5] = sa * sb * cc - ca * sc;
        Rm[6] = -sb;     Rm[7] = cb * sc;                Rm[8] = cb * cc;
    }

    template <class T>
    ATO_HD static void dR(const T* r, const T*, int m, T* o) {
        const T ca = tcos(r[0]), sa = tsin(r[0]), cb = tcos(r[1]), sb = tsin(r[1]);
        const T cc = tcos(r[2]), sc = tsin(r[2]);
        if (m == 0) {
            o[0] = -sa * cb; o[1] = -sa * sb * sc - ca * cc; o[2] = -sa * sb * cc + ca * sc;
            o[3] = ca * cb;  o[4] = ca * sb * sc - sa * cc;  o[5] = ca * sb * cc + sa * sc;
            o[6] = T(0);     o[7] = T(0);                    o[8] = T(0);
        } else if (m == 1) {
            o[0] = -ca * sb; o[1] = ca * cb * sc; o[2] = ca * cb * cc;
            o[3] = -sa * sb; o[4] = sa * cb * sc; o[5] = sa * cb * cc;
            o[6] = -cb;      o[7] = -sb * sc;     o[8] = -sb * cc;
        } else {
            o[0] = T(0); o[1] = ca * sb * cc + sa * sc; o[2] = -ca * sb * sc + sa * cc;
            o[3] = T(0); o[4] = sa * sb * cc - ca * sc; o[5] = -sa * sb * sc - ca * cc;
            o[6] = T(0); o[7] = cb * cc;                o[8] = -cb * sc;
        }
    }

    template <class T>
    ATO_HD static void kin(const T* r, const T* w, T* rdot, T drq[3][3], T Mm[3][3]) {
        const T cb = tcos(r[1]), sb = tsin(r[1]), cc = tcos(r[2]), sc = tsin(r[2]);
        const T icb = T(1) / cb, tb = sb / cb;
        Mm[0][0] = T(0); Mm[0][1] = sc * icb; Mm[0][2] = cc * icb;
        Mm[1][0] = T(0); Mm[1][1] = cc;       Mm[1][2] = -sc;
        Mm[2][0] = T(1); Mm[2][1] = sc * tb;  Mm[2][2] = cc * tb;
        for (int i = 0; i < 3; ++i) rdot[i] = Mm[i][0] * w[0] + Mm[i][1] * w[1] + Mm[i][2] * w[2];
        const T p = sc * w[1] + cc * w[2];     // d(.)/dc of (sc w1 + cc w2) is q
        const T qv = cc * w[1] - sc * w[2];
        drq[0][0] = T(0); drq[0][1] = p * sb * icb * icb; drq[0][2] = qv * icb;
        drq[1][0] = T(0); drq[1][1] = T(0);               drq[1][2] = -p;
        drq[2][0] = T(0); drq[2][1] = p * icb * icb;      drq[2][2] = qv * tb;
    }

    static constexpr bool kin_r(int i, int m) {
        return (i == 0) ? (m == 1 || m == 2) : (i == 1) ? (m == 2) : (m == 1 || m == 2);
    }
    static constexpr bool kin_w(int i, int j) { return !(i < 2 && j == 0); }
    // does R[row][col] depend on r_m ?
    static constexpr bool R_dep(int row, int col, int m) {
        return (row < 2) ? !(col == 0 && m == 2) : (col == 0 ? m == 1 : m != 0);
    }
};

// Direction-cosine matrix (config 5's "Non-Euclidean DCM / SO(3) pose"; not in the reference, whose
// rotations.py:19-24 offers ESP and YPR only): the attitude state IS R, row-major (r_{3i+j} = R_ij),
// with the kinematics R' = R [w]x. R(r) is the identity map, so every force / pose term the ESP
// model builds from R(q) is reused unchanged. Orthonormality is carried by the continuity operator
// (ato_program.hpp AttOp: the analogue of the reference's quaternion normalisation).
struct AttDCM {
    static constexpr int NR = 9;

    template <class T>
    ATO_HD static void R(const T* r, T* Rm) {
        for (int i = 0; i < 9; ++i) Rm[i] = r[i];
    }

    template <class T>
    ATO_HD static void dR(const T*, const T*, int m, T* out) {
        for (int i = 0; i < 9; ++i) out[i] = T(i == m ? 1 : 0);
    }
    static constexpr bool R_dep(int row, int col, int m) { return m == row * 3 + col; }

    // (R [w]x)_i0 = R_i1 w2 - R_i2 w1, _i1 = R_i2 w0 - R_i0 w2, _i2 = R_i0 w1 - R_i1 w0
    template <class T>
    ATO_HD static void kin(const T* r, const T* w, T* rdot, T drq[9][9], T Mm[9][3]) {
        for (int a = 0; a < 9; ++a) {
            for (int m = 0; m < 9; ++m) drq[a][m] = T(0);
            for (int c = 0; c < 3; ++c) Mm[a][c] = T(0);
        }
        for (int i = 0; i < 3; ++i) {
            const T r0 = r[3 * i], r1 = r[3 * i + 1], r2 = r[3 * i + 2];
            rdot[3 * i + 0] = r1 * w[2] - r2 * w[1];
            rdot[3 * i + 1] = r2 * w[0] - r0 * w[2];
            rdot[3 * i + 2] = r0 * w[1] - r1 * w[0];
            drq[3 * i + 0][3 * i + 1] = w[2];  drq[3 * i + 0][3 * i + 2] = -w[1];
            drq[3 * i + 1][3 * i + 2] = w[0];  drq[3 * i + 1][3 * i + 0] = -w[2];
            drq[3 * i + 2][3 * i + 0] = w[1];  drq[3 * i + 2][3 * i + 1] = -w[0];
            Mm[3 * i + 0][2] = r1;  Mm[3 * i + 0][1] = -r2;
            Mm[3 * i + 1][0] = r2;  Mm[3 * i + 1][2] = -r0;
            Mm[3 * i + 2][1] = r0;  Mm[3 * i + 2][0] = -r1;
        }
    }

    static constexpr bool kin_r(int i, int m) { return m / 3 == i / 3 && m != i; }
    static constexpr bool kin_w(int i, int c) { return c != i % 3; }
};

template <int A>
struct AttSel;
template <>
struct AttSel<ESP> { using type = AttESP; };
template <>
struct AttSel<YPR> { using type = AttYPR; };
template <>
struct AttSel<DCM> { using type = AttDCM; };

// --------------------------------------------------------------------- drone
// z = [p(3), r(NR), v_b(3), w_b(3)], u = 4 rotor thrusts.
template <int ATT, int FRAME>
struct DroneModel {
    using A = typename AttSel<ATT>::type;
    static constexpr int NR = A::NR;
    static constexpr int NZ = 9 + NR, NU = 4;
    static constexpr int IR = 3, IV = 3 + NR, IW = 6 + NR;
    static constexpr bool PARAM = FRAME != GLOBAL;
    static constexpr bool IS_DRONE = true;
    static constexpr bool HAS_QUAT = ATT == ESP;
    static constexpr bool HAS_DCM = ATT == DCM;

    // d(row of global R used for gravity, i.e. R_g[2][c]) / d r_m
    static constexpr bool grav_dep(int c, int m) {
        return FRAME == PARAM_REL ? true : A::R_dep(2, c, m);
    }
    // d(position-row velocity component i)/d r_m
    static constexpr bool pos_r_dep(int i, int m) {
        if (FRAME != GLOBAL) return true;      // Rp^T R mixes every row, or s-dot etc
        return A::R_dep(i, 0, m) || A::R_dep(i, 1, m) || A::R_dep(i, 2, m);
    }

    static constexpr bool zmask(int i, int m) {
        const bool isr = m >= IR && m < IR + NR;
        const bool isv = m >= IV && m < IV + 3;
        const bool isw = m >= IW && m < IW + 3;
        if (i < 3) {
            if (PARAM) return m == 1 || m == 2 || (isr && pos_r_dep(i, m - IR)) || isv;
            return (isr && pos_r_dep(i, m - IR)) || isv;
        }
        if (i < IV) {
            const int ri = i - IR;
            if (FRAME == PARAM_REL) return m == 1 || m == 2 || isr || isv || isw;
            return (isr && A::kin_r(ri, m - IR)) || (isw && A::kin_w(ri, m - IW));
        }
        if (i < IW) {
            const int vi = i - IV;
            if (isr) return grav_dep(vi, m - IR);
            if (isv) return true;
            if (isw) return (m - IW) != vi;
            return false;
        }
        return isw;
    }
    static constexpr bool umask(int i, int) { return i == IV + 2 || i >= IW; }

    // s-dot of the parametric pose and its derivatives (drone_models.py:261-267)
    template <class T>
    struct SDot {
        T Rrel[9], vp[3], dvp[3][NR];
        T sd, sd_y, sd_n, sd_r[NR], sd_v[3];
    };

    template <class T>
    ATO_HD static void pose_terms(const T* z, const T* Ra, const NodeGeom<T>& G, SDot<T>& o) {
        const T* r = z + IR;
        const T* v = z + IV;
        // Rrel: frame of the position rate. GLOBAL: R ; PARAM_GR: Rp^T R ; PARAM_REL: R_att
        if (FRAME == PARAM_GR) {
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j)
                    o.Rrel[i * 3 + j] = G.Rp[0 * 3 + i] * Ra[0 * 3 + j] + G.Rp[1 * 3 + i] * Ra[1 * 3 + j] +
                                        G.Rp[2 * 3 + i] * Ra[2 * 3 + j];
        } else {
            for (int i = 0; i < 9; ++i) o.Rrel[i] = Ra[i];
        }
        for (int i = 0; i < 3; ++i)
            o.vp[i] = o.Rrel[i * 3] * v[0] + o.Rrel[i * 3 + 1] * v[1] + o.Rrel[i * 3 + 2] * v[2];
        for (int m = 0; m < NR; ++m) {
            T dRa[9];
            A::dR(r, Ra, m, dRa);
            T dvg[3];
            for (int a = 0; a < 3; ++a) dvg[a] = dRa[a * 3] * v[0] + dRa[a * 3 + 1] * v[1] + dRa[a * 3 + 2] * v[2];
            if (FRAME == PARAM_GR) {
                for (int i = 0; i < 3; ++i)
                    o.dvp[i][m] = G.Rp[0 * 3 + i] * dvg[0] + G.Rp[1 * 3 + i] * dvg[1] + G.Rp[2 * 3 + i] * dvg[2];
            } else {
                for (int i = 0; i < 3; ++i) o.dvp[i][m] = dvg[i];
            }
        }
        o.sd = o.sd_y = o.sd_n = T(0);
        for (int m = 0; m < NR; ++m) o.sd_r[m] = T(0);
        for (int j = 0; j < 3; ++j) o.sd_v[j] = T(0);
        if (PARAM) {
            const T y = z[1], n = z[2];
            const T den = T(1) + G.ky * n - G.kn * y;
            const T iden = T(1) / (G.mag * den);
            o.sd = o.vp[0] * iden;
            o.sd_y = o.sd * G.kn / den;
            o.sd_n = -o.sd * G.ky / den;
            for (int m = 0; m < NR; ++m) o.sd_r[m] = o.dvp[0][m] * iden;
            for (int j = 0; j < 3; ++j) o.sd_v[j] = o.Rrel[j] * iden;
        }
    }

    // f and its Jacobian for rows [R0, R1), row by row (R0 / R1 fixed at compile time so a
    // kernel unit evaluates only the row groups it writes).
    template <int R0 = 0, int R1 = NZ, class T, class Emit>
    ATO_HD static void rows(const T* z, const T* u, const NodeGeom<T>& G, const Vehicle& V,
                            Emit&& emit) {
        const T* r = z + IR;
        const T* v = z + IV;
        const T* w = z + IW;
        T Ra[9];
        A::R(r, Ra);
        constexpr bool DO_POS = R0 < 3;
        constexpr bool DO_ATT = R0 < IV && R1 > IR;
        constexpr bool DO_VEL = R0 < IW && R1 > IV;
        constexpr bool DO_ANG = R1 > IW;

        // ---- position rows ------------------------------------------------------
        if constexpr (DO_POS) {
            SDot<T> P;
            pose_terms(z, Ra, G, P);
            if (PARAM) {
                const T y = z[1], n = z[2];
                const T km = G.ks * G.mag;
                {   // s-dot
                    T dz[NZ] = {}, du[NU] = {};
                    dz[1] = P.sd_y; dz[2] = P.sd_n;
                    for (int m = 0; m < NR; ++m) dz[IR + m] = P.sd_r[m];
                    for (int j = 0; j < 3; ++j) dz[IV + j] = P.sd_v[j];
                    emit(0, P.sd, dz, du);
                }
                {   // y-dot = vp1 + n ks |xc'| s-dot
                    T dz[NZ] = {}, du[NU] = {};
                    const T c = n * km;
                    dz[1] = c * P.sd_y;
                    dz[2] = km * P.sd + c * P.sd_n;
                    for (int m = 0; m < NR; ++m) dz[IR + m] = P.dvp[1][m] + c * P.sd_r[m];
                    for (int j = 0; j < 3; ++j) dz[IV + j] = P.Rrel[3 + j] + c * P.sd_v[j];
                    emit(1, P.vp[1] + c * P.sd, dz, du);
                }
                {   // n-dot = vp2 - y ks |xc'| s-dot
                    T dz[NZ] = {}, du[NU] = {};
                    const T c = y * km;
                    dz[1] = -km * P.sd - c * P.sd_y;
                    dz[2] = -c * P.sd_n;
                    for (int m = 0; m < NR; ++m) dz[IR + m] = P.dvp[2][m] - c * P.sd_r[m];
                    for (int j = 0; j < 3; ++j) dz[IV + j] = P.Rrel[6 + j] - c * P.sd_v[j];
                    emit(2, P.vp[2] - c * P.sd, dz, du);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    T dz[NZ] = {}, du[NU] = {};
                    for (int m = 0; m < NR; ++m) dz[IR + m] = P.dvp[i][m];
                    for (int j = 0; j < 3; ++j) dz[IV + j] = P.Rrel[i * 3 + j];
                    emit(i, P.vp[i], dz, du);
                }
            }
        }

        // ---- attitude rows -------------------------------------------------------
        if constexpr (DO_ATT) {
            T weff[3] = {w[0], w[1], w[2]};
            T wp[3] = {T(0), T(0), T(0)};
            T sd = T(0), sd_y = T(0), sd_n = T(0), sd_r[NR], sd_v[3];
            for (int m = 0; m < NR; ++m) sd_r[m] = T(0);
            for (int j = 0; j < 3; ++j) sd_v[j] = T(0);
            if (FRAME == PARAM_REL) {
                SDot<T> P;
                pose_terms(z, Ra, G, P);
                sd = P.sd;
                sd_y = P.sd_y;
                sd_n = P.sd_n;
                for (int m = 0; m < NR; ++m) sd_r[m] = P.sd_r[m];
                for (int j = 0; j < 3; ++j) sd_v[j] = P.sd_v[j];
                // w_eff = w_b - R^T k s-dot |xc'|      (drone_models.py:270-274)
                const T kk[3] = {G.ks, G.ky, G.kn};
                for (int c = 0; c < 3; ++c) wp[c] = kk[c] * sd * G.mag;
                for (int j = 0; j < 3; ++j) weff[j] -= Ra[j] * wp[0] + Ra[3 + j] * wp[1] + Ra[6 + j] * wp[2];
            }
            T rdot[NR], drq[NR][NR], Mm[NR][3];
            A::kin(r, weff, rdot, drq, Mm);
            if (FRAME != PARAM_REL) {
#pragma unroll
                for (int i = 0; i < NR; ++i) {
                    T dz[NZ] = {}, du[NU] = {};
                    for (int m = 0; m < NR; ++m) dz[IR + m] = drq[i][m];
                    for (int j = 0; j < 3; ++j) dz[IW + j] = Mm[i][j];
                    emit(IR + i, rdot[i], dz, du);
                }
            } else {
                // d w_eff / d x  for x in {y, n, r, v}: -R^T k |xc'| d(sd)/dx - (dR/dr)^T wp
                const T kk[3] = {G.ks, G.ky, G.kn};
                T Rtk[3];
                for (int j = 0; j < 3; ++j) Rtk[j] = (Ra[j] * kk[0] + Ra[3 + j] * kk[1] + Ra[6 + j] * kk[2]) * G.mag;
                T dwe_r[3][NR];
                for (int m = 0; m < NR; ++m) {
                    T dRa[9];
                    A::dR(r, Ra, m, dRa);
                    for (int j = 0; j < 3; ++j)
                        dwe_r[j][m] = -(dRa[j] * wp[0] + dRa[3 + j] * wp[1] + dRa[6 + j] * wp[2]) - Rtk[j] * sd_r[m];
                }
#pragma unroll
                for (int i = 0; i < NR; ++i) {
                    T dz[NZ] = {}, du[NU] = {};
                    T My = T(0), Mn = T(0);
                    for (int j = 0; j < 3; ++j) {
                        My -= Mm[i][j] * Rtk[j] * sd_y;
                        Mn -= Mm[i][j] * Rtk[j] * sd_n;
                    }
                    dz[1] = My;
                    dz[2] = Mn;
                    for (int m = 0; m < NR; ++m) {
                        T acc = drq[i][m];
                        for (int j = 0; j < 3; ++j) acc += Mm[i][j] * dwe_r[j][m];
                        dz[IR + m] = acc;
                    }
                    for (int c = 0; c < 3; ++c) {
                        T acc = T(0);
                        for (int j = 0; j < 3; ++j) acc -= Mm[i][j] * Rtk[j] * sd_v[c];
                        dz[IV + c] = acc;
                    }
                    for (int j = 0; j < 3; ++j) dz[IW + j] = Mm[i][j];
                    emit(IR + i, rdot[i], dz, du);
                }
            }
        }

        // ---- body linear velocity rows (drone_models.py:61-92, 114) ------------------
        if constexpr (DO_VEL) {
            // gravity uses row 3 of the global rotation: R (global / global_r) or Rp R (relative)
            T Rg2[3], dRg2[3][NR];
            if (FRAME == PARAM_REL) {
                for (int c = 0; c < 3; ++c)
                    Rg2[c] = G.Rp[6] * Ra[c] + G.Rp[7] * Ra[3 + c] + G.Rp[8] * Ra[6 + c];
            } else {
                for (int c = 0; c < 3; ++c) Rg2[c] = Ra[6 + c];
            }
            for (int m = 0; m < NR; ++m) {
                T dRa[9];
                A::dR(r, Ra, m, dRa);
                for (int c = 0; c < 3; ++c)
                    dRg2[c][m] = (FRAME == PARAM_REL)
                                     ? G.Rp[6] * dRa[c] + G.Rp[7] * dRa[3 + c] + G.Rp[8] * dRa[6 + c]
                                     : dRa[6 + c];
            }
            const T m_ = T(V.m), im = T(1) / m_;
            const T mg = -T(V.m) * T(V.g);
            const T usum = u[0] + u[1] + u[2] + u[3];
            // v_dot = F_b / m - w x v
            const T wxv[3] = {w[1] * v[2] - w[2] * v[1], w[2] * v[0] - w[0] * v[2], w[0] * v[1] - w[1] * v[0]};
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                T dz[NZ] = {}, du[NU] = {};
                const T Fb = -T(V.b[i]) * v[i] + mg * Rg2[i] + (i == 2 ? usum : T(0));
                for (int m = 0; m < NR; ++m) dz[IR + m] = mg * dRg2[i][m] * im;
                dz[IV + i] = -T(V.b[i]) * im;
                // -(w x v) derivatives
                if (i == 0) { dz[IV + 1] += w[2]; dz[IV + 2] += -w[1]; dz[IW + 1] = -v[2]; dz[IW + 2] = v[1]; }
                if (i == 1) { dz[IV + 0] += -w[2]; dz[IV + 2] += w[0]; dz[IW + 0] = v[2]; dz[IW + 2] = -v[0]; }
                if (i == 2) {
                    dz[IV + 0] += w[1]; dz[IV + 1] += -w[0]; dz[IW + 0] = -v[1]; dz[IW + 1] = v[0];
                    for (int j = 0; j < 4; ++j) du[j] = im;
                }
                emit(IV + i, Fb * im - wxv[i], dz, du);
            }
        }

        // ---- body angular velocity rows: w_dot = I^-1 (K_b - w x I w) -----------------
        if constexpr (DO_ANG) {
            const T I0 = T(V.I[0]), I1 = T(V.I[1]), I2 = T(V.I[2]);
            const T l = T(V.l), kt = T(V.kt);
            const T Ka[3] = {(u[0] + u[1] - u[2] - u[3]) * l, (-u[0] + u[1] + u[2] - u[3]) * l,
                             (u[0] - u[1] + u[2] - u[3]) * kt};
            const T dKa[3][4] = {{l, l, -l, -l}, {-l, l, l, -l}, {kt, -kt, kt, -kt}};
            const T Iw[3] = {I0 * w[0], I1 * w[1], I2 * w[2]};
            const T wxIw[3] = {w[1] * Iw[2] - w[2] * Iw[1], w[2] * Iw[0] - w[0] * Iw[2],
                               w[0] * Iw[1] - w[1] * Iw[0]};
            const T Ii[3] = {I0, I1, I2};
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                T dz[NZ] = {}, du[NU] = {};
                const T iI = T(1) / Ii[i];
                const T Kb = -T(V.bw[i]) * w[i] + Ka[i];
                dz[IW + i] = -T(V.bw[i]) * iI;
                if (i == 0) { dz[IW + 1] = -(I2 - I1) * w[2] * iI; dz[IW + 2] = -(I2 - I1) * w[1] * iI; }
                if (i == 1) { dz[IW + 0] = -(I0 - I2) * w[2] * iI; dz[IW + 2] = -(I0 - I2) * w[0] * iI; }
                if (i == 2) { dz[IW + 0] = -(I1 - I0) * w[1] * iI; dz[IW + 1] = -(I1 - I0) * w[0] * iI; }
                for (int j = 0; j < 4; ++j) du[j] = dKa[i][j] * iI;
                emit(IW + i, (Kb - wxIw[i]) * iI, dz, du);
            }
        }
    }
};

// --------------------------------------------------------------------- point mass
// z = [p(3), v(3)], u = thrust vector (3).
template <int FRAME>
struct PointModel {
    static constexpr int NZ = 6, NU = 3;
    static constexpr int NR = 0, IR = 3, IV = 3, IW = 6;
    static constexpr bool PARAM = FRAME != GLOBAL;
    static constexpr bool IS_DRONE = false;
    static constexpr bool HAS_QUAT = false;
    static constexpr bool HAS_DCM = false;

    static constexpr bool zmask(int i, int m) {
        if (i < 3) return PARAM ? (m == 1 || m == 2 || m >= 3) : (m == 3 + i);
        if (FRAME == PARAM_REL) return m == 1 || m == 2 || m >= 3;
        return m == i;
    }
    static constexpr bool umask(int i, int m) { return i >= 3 && (m == i - 3); }

    template <int R0 = 0, int R1 = NZ, class T, class Emit>
    ATO_HD static void rows(const T* z, const T* u, const NodeGeom<T>& G, const Vehicle& V,
                            Emit&& emit) {
        static_assert(R0 == 0 && R1 == NZ, "point-mass rows are evaluated as one group");
        const T* v = z + 3;
        T sd = T(0), sd_y = T(0), sd_n = T(0), sd_v[3] = {T(0), T(0), T(0)};
        if (PARAM) {
            // v_p = R_rel v with R_rel = Rp^T (global_r) or I (point_model.py:155-160)
            T Rrel[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j)
                    Rrel[i * 3 + j] = (FRAME == PARAM_GR) ? G.Rp[j * 3 + i] : T(i == j ? 1 : 0);
            T vp[3];
            for (int i = 0; i < 3; ++i) vp[i] = Rrel[i * 3] * v[0] + Rrel[i * 3 + 1] * v[1] + Rrel[i * 3 + 2] * v[2];
            const T y = z[1], n = z[2];
            const T den = T(1) + G.ky * n - G.kn * y;
            const T iden = T(1) / (G.mag * den);
            sd = vp[0] * iden;
            sd_y = sd * G.kn / den;
            sd_n = -sd * G.ky / den;
            for (int j = 0; j < 3; ++j) sd_v[j] = Rrel[j] * iden;
            const T km = G.ks * G.mag;
            {
                T dz[NZ] = {}, du[NU] = {};
                dz[1] = sd_y; dz[2] = sd_n;
                for (int j = 0; j < 3; ++j) dz[3 + j] = sd_v[j];
                emit(0, sd, dz, du);
            }
            {
                T dz[NZ] = {}, du[NU] = {};
                const T c = n * km;
                dz[1] = c * sd_y;
                dz[2] = km * sd + c * sd_n;
                for (int j = 0; j < 3; ++j) dz[3 + j] = Rrel[3 + j] + c * sd_v[j];
                emit(1, vp[1] + c * sd, dz, du);
            }
            {
                T dz[NZ] = {}, du[NU] = {};
                const T c = y * km;
                dz[1] = -km * sd - c * sd_y;
                dz[2] = -c * sd_n;
                for (int j = 0; j < 3; ++j) dz[3 + j] = Rrel[6 + j] - c * sd_v[j];
                emit(2, vp[2] - c * sd, dz, du);
            }
        } else {
            for (int i = 0; i < 3; ++i) {
                T dz[NZ] = {}, du[NU] = {};
                dz[3 + i] = T(1);
                emit(i, v[i], dz, du);
            }
        }
        // v_dot = (T_b + F_gb + F_db) / m  [- w_p x v for relative frame]
        const T m_ = T(V.m), im = T(1) / m_, mg = -T(V.m) * T(V.g);
        T Rg2[3];
        if (FRAME == PARAM_REL) { Rg2[0] = G.Rp[6]; Rg2[1] = G.Rp[7]; Rg2[2] = G.Rp[8]; }
        else { Rg2[0] = T(0); Rg2[1] = T(0); Rg2[2] = T(1); }
        T wp[3] = {T(0), T(0), T(0)};
        if (FRAME == PARAM_REL) { wp[0] = G.ks * sd * G.mag; wp[1] = G.ky * sd * G.mag; wp[2] = G.kn * sd * G.mag; }
        const T wxv[3] = {wp[1] * v[2] - wp[2] * v[1], wp[2] * v[0] - wp[0] * v[2], wp[0] * v[1] - wp[1] * v[0]};
        const T kk[3] = {G.ks * G.mag, G.ky * G.mag, G.kn * G.mag};
        for (int i = 0; i < 3; ++i) {
            T dz[NZ] = {}, du[NU] = {};
            const T Fb = u[i] + mg * Rg2[i] - T(V.b[i]) * v[i];
            dz[3 + i] = -T(V.b[i]) * im;
            du[i] = im;
            if (FRAME == PARAM_REL) {
                // d(w_p x v)_i: w_p = kk * sd, depends on y, n, v via sd
                const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
                // (w x v)_i = w_i1 v_i2 - w_i2 v_i1
                dz[1] -= (kk[i1] * v[i2] - kk[i2] * v[i1]) * sd_y;
                dz[2] -= (kk[i1] * v[i2] - kk[i2] * v[i1]) * sd_n;
                for (int j = 0; j < 3; ++j) dz[3 + j] -= (kk[i1] * v[i2] - kk[i2] * v[i1]) * sd_v[j];
                dz[3 + i2] -= wp[i1];
                dz[3 + i1] += wp[i2];
            }
            emit(3 + i, Fb * im - wxv[i], dz, du);
        }
    }
};

}  // namespace ato
