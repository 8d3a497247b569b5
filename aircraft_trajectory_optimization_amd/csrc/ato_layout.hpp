// ato_layout.hpp -- host side: problem validation, row order, CSR pattern, bounds.
//
// Runs every segment program of ato_program.hpp in pattern mode and lays the segments
// out in the reference's constraint order:
//   [equal-h rows (global)]                         base_raceline.py:891-905
//   per interval n:                                 base_raceline.py:393-396
//     collocation nodes k = 0..K                    :398-434
//     regularity rows (masked nodes)                :1114-1130
//     model stage constraints (point mass)          :436-451
//     continuity (n >= 1)                           :460-490 / :1132-1163
//     fixed-s rows (parametric)                     :1165-1181
//   base loop closure (closed point mass)           :357-358, :492-514, :1183-1227
//   open lines: initial and terminal rows           :359-361, :516-543, drone_raceline.py:110-148,
//                                                   point_raceline.py:15-45
//   gates                                           :907-918 / :986-1032
//   obstacle-tube spheres                           :1293-1310
//   drone loop closure (closed drone)               drone_raceline.py:150-156
// Header-only so the HIP library and the CPU test harness share it.
#pragma once
#include <string>
#include <vector>
#include <cstring>
#include <cstdlib>
#include <cmath>
#include "ato_program.hpp"

namespace ato {

struct SegPat {
    std::vector<int32_t> rowlen, cols;
    std::vector<double> lb, ub;
};

struct PatSink {
    SegPat* sp;
    int last = -1, cur = 0;
    bool sorted = true;
    void jac(int col, double) {
        if (col <= last) sorted = false;
        last = col;
        sp->cols.push_back(col);
        ++cur;
    }
    void row(double, double lb, double ub) {
        sp->rowlen.push_back(cur);
        sp->lb.push_back(lb);
        sp->ub.push_back(ub);
        cur = 0;
        last = -1;
    }
    // value-mode only (RK4 column groups); never reached in pattern mode
    void skip() { sorted = false; }
    void row_skip() { sorted = false; }
    void finish() {}
};

template <>
struct SinkTraits<PatSink> { static constexpr bool pattern = true; };

struct OnesW {
    double operator()(int) const { return 1.0; }
    double par(long) const { return 0.0; }
};

// model dispatch: calls f.template operator()<Model>() for the problem's model variant
template <class F>
bool with_model(const ProbD& p, F&& f) {
    if (p.model == ATO_MODEL_DRONE) {
        if (p.att == ATO_ATT_ESP) {
            if (p.frame == GLOBAL) { f.template operator()<DroneModel<ESP, GLOBAL>>(); return true; }
            if (p.frame == PARAM_GR) { f.template operator()<DroneModel<ESP, PARAM_GR>>(); return true; }
            if (p.frame == PARAM_REL) { f.template operator()<DroneModel<ESP, PARAM_REL>>(); return true; }
        } else if (p.att == ATO_ATT_YPR) {
            if (p.frame == GLOBAL) { f.template operator()<DroneModel<YPR, GLOBAL>>(); return true; }
            if (p.frame == PARAM_GR) { f.template operator()<DroneModel<YPR, PARAM_GR>>(); return true; }
            if (p.frame == PARAM_REL) { f.template operator()<DroneModel<YPR, PARAM_REL>>(); return true; }
        } else if (p.att == ATO_ATT_DCM) {
            if (p.frame == GLOBAL) { f.template operator()<DroneModel<DCM, GLOBAL>>(); return true; }
            if (p.frame == PARAM_GR) { f.template operator()<DroneModel<DCM, PARAM_GR>>(); return true; }
            if (p.frame == PARAM_REL) { f.template operator()<DroneModel<DCM, PARAM_REL>>(); return true; }
        }
    } else if (p.model == ATO_MODEL_POINT) {
        if (p.frame == GLOBAL) { f.template operator()<PointModel<GLOBAL>>(); return true; }
        if (p.frame == PARAM_GR) { f.template operator()<PointModel<PARAM_GR>>(); return true; }
        if (p.frame == PARAM_REL) { f.template operator()<PointModel<PARAM_REL>>(); return true; }
    }
    return false;
}

// Run one segment of the given kind with any sink / accessor. grp: RK4 Jacobian column group.
// RK4 = false leaves the RK4 programs out of an instantiation (collocation kernels).
template <class M, class T, int KS, class W, class S, bool RK4 = true>
ATO_HD void run_node_seg(const ProbD& p, int kind, int n, int k, const W& w, S& s, int grp = 0) {
    switch (kind) {
        case SEG_SDOT: seg_sdot<M, T, KS>(p, n, k, w, s); break;
        case SEG_ODE_A: seg_ode<M, T, KS, 0, ode_split<M>()>(p, n, k, w, s); break;
        case SEG_ODE_B:
            if constexpr (ode_split<M>() < M::NZ) seg_ode<M, T, KS, ode_split<M>(), M::NZ>(p, n, k, w, s);
            break;
        case SEG_DU: seg_du<M, T, KS>(p, n, k, w, s); break;
        case SEG_REG: seg_reg<M, T, KS>(p, n, k, w, s); break;
        case SEG_STAGE: seg_stage<M, T, KS>(p, n, k, w, s); break;
        case SEG_SPHERE: seg_sphere<M, T, KS>(p, n, k, w, s); break;
        case SEG_CONT: seg_cont<M, T, KS>(p, n, w, s); break;
        case SEG_SROWS: seg_srows<M, T, KS>(p, n, w, s); break;
        case SEG_RK4S: seg_rk4s<M, T, KS>(p, n, w, s); break;
        case SEG_RK4:
            if constexpr (RK4) seg_rk4<M, T, KS>(p, n, grp, w, s);
            break;
        case SEG_CPC_COMP: seg_cpc_comp<M, T, KS>(p, n, k, w, s); break;
        case SEG_CPC_ORDER: seg_cpc_order<M, T, KS>(p, n, k, w, s); break;
        case SEG_CPC_PROG: seg_cpc_prog<M, T, KS>(p, n, k, w, s); break;
        default: break;
    }
}

template <class M, class T, int KS, class W, class S, bool RK4 = true>
ATO_HD void run_tail_seg(const ProbD& p, int kind, int index, const W& w, S& s, int grp = 0) {
    const bool rk4 = RK4 && p.trans == ATO_TRANS_RK4;
    switch (kind) {
        case TAIL_HEQ: seg_heq<M, T, KS>(p, w, s); break;
        case TAIL_CLOSURE_BASE:
            if constexpr (RK4)
                if (rk4) { seg_closure_base_rk4<M, T, KS>(p, grp, w, s); break; }
            seg_closure_base<M, T, KS>(p, w, s);
            break;
        case TAIL_INITIAL: seg_boundary<M, T, KS>(p, 0, w, s); break;
        case TAIL_TERMINAL: seg_boundary<M, T, KS>(p, 1, w, s); break;
        case TAIL_GATE: seg_gate<M, T, KS>(p, index, w, s); break;
        case TAIL_DRONE_CLOSURE:
            if constexpr (RK4)
                if (rk4) { seg_drone_closure_rk4<M, T, KS>(p, grp, w, s); break; }
            seg_drone_closure<M, T, KS>(p, w, s);
            break;
        default: break;
    }
}

// number of work units of a tail segment (RK4 closures: one per Jacobian column group)
template <class M>
int tail_units(const ProbD& p, int kind) {
    const bool closure = kind == TAIL_CLOSURE_BASE || kind == TAIL_DRONE_CLOSURE;
    return (closure && p.trans == ATO_TRANS_RK4) ? rk4_groups<M>() : 1;
}

// where an instance's gradient / cost go (pointers already offset to the instance)
template <class T>
struct GradOut {
    T* gf;       // grad f, element stride st
    long st;
    T* fpart;    // per-interval cost partials h_n sum_k B_k L_nk, element stride pst
    long pst;
    ATO_HD void put_gf(long i, const T& v) const { gf[i * st] = v; }
    ATO_HD void put_fpart(long n, const T& v) const { fpart[n * pst] = v; }
};

// f = sum_n partial(n), fixed order (the k_cost_reduce kernel and the CPU harness)
template <class T>
ATO_HD T reduce_cost(const T* fpart, long pst, int N) {
    T acc = T(0);
    int n = 0;
    for (; n + 16 <= N; n += 16) {     // issue 16 independent loads before summing
        T v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = fpart[(long)(n + i) * pst];
#pragma unroll
        for (int i = 0; i < 16; ++i) acc += v[i];
    }
    for (; n < N; ++n) acc += fpart[(long)n * pst];
    return acc;
}

// Execute one work unit for one instance: the device kernel and the CPU test harness both
// call this, so the dispatch is identical.
// UMASK: unit kinds compiled into this instantiation (bit = 1 << UnitKind), so a kernel that
// only runs light units is not register-allocated for the heavy ones.
constexpr int UMASK_TAIL = 1 << UNIT_TAIL;
constexpr int UMASK_ODE = (1 << UNIT_ODE_A) | (1 << UNIT_ODE_B);
constexpr int UMASK_LIN = (1 << UNIT_NODE) | (1 << UNIT_INTERVAL);
constexpr int UMASK_RK4U = 1 << UNIT_RK4;
constexpr int UMASK_COLLOC = UMASK_TAIL | UMASK_ODE | UMASK_LIN;    // collocation problems
constexpr int UMASK_RK4 = UMASK_TAIL | UMASK_LIN | UMASK_RK4U;      // RK4 problems
constexpr int UMASK_ALL = UMASK_COLLOC | UMASK_RK4;

template <class M, class T, int KS, bool ROWS, bool GRAD, int UMASK = UMASK_ALL, class W, class S, class GO>
ATO_HD void run_unit(const ProbD& p, int kind, int n, int k, const W& w, S& s, const GO& go) {
    constexpr int NZ = M::NZ, NU = M::NU;
    constexpr bool RK4 = (UMASK & UMASK_RK4U) != 0;
    const int32_t* sg = p.seg + (long)(n * K1S(p) + (kind == UNIT_RK4 ? 0 : k)) * NSEG * 2;
    auto seg = [&](int sk) {
        if (sg[2 * sk] < 0) return;
        s.begin(sg[2 * sk], sg[2 * sk + 1]);
        run_node_seg<M, T, KS, W, S, RK4>(p, sk, n, k, w, s, k);
    };
    switch (kind) {
        case UNIT_TAIL:   // one tail segment: n = its index in p.tail
            if constexpr ((UMASK & UMASK_TAIL) != 0) {
                if (ROWS) {
                    const int32_t* tl = p.tail + 4 * n;
                    s.begin(tl[2], tl[3]);
                    run_tail_seg<M, T, KS, W, S, RK4>(p, tl[0], tl[1], w, s, k);
                }
            }
            break;
        case UNIT_ODE_A:
            if constexpr ((UMASK & (1 << UNIT_ODE_A)) != 0)
                if (ROWS) seg(SEG_ODE_A);
            break;
        case UNIT_ODE_B:
            if constexpr ((UMASK & (1 << UNIT_ODE_B)) != 0)
                if (ROWS) seg(SEG_ODE_B);
            break;
        case UNIT_NODE:
            if constexpr ((UMASK & (1 << UNIT_NODE)) == 0) break;
            if (ROWS) {
                seg(SEG_SDOT);
                seg(SEG_DU);
                seg(SEG_REG);
                seg(SEG_STAGE);
                seg(SEG_SPHERE);
                seg(SEG_RK4S);
                if (p.cpc_m > 0) {
                    seg(SEG_CPC_COMP);
                    seg(SEG_CPC_ORDER);
                    seg(SEG_CPC_PROG);
                }
            }
            if (GRAD) {
                const Cols<M> c{p.N, K1S(p)};
                T gu[NU], gdu[NU];
                stage_cost<M, T, KS>(p, n, k, w, gu, gdu);
                const T hB = w(n) * T(p.Bq[k]);
                const long base = c.node(n, k);
                if (!p.gf_sparse) {        // structural zeros: written only in the dense mode
#pragma unroll
                    for (int i = 0; i < NZ; ++i) go.put_gf(base + i, T(0));
                }
#pragma unroll
                for (int i = 0; i < NU; ++i) go.put_gf(base + NZ + i, hB * gu[i]);
#pragma unroll
                for (int i = 0; i < NU; ++i) go.put_gf(base + NZ + NU + i, hB * gdu[i]);
                if (p.cpc_m > 0 && !p.gf_sparse) {      // the progress variables are not in the cost
                    const long cb = p.cpc_off + 3L * p.cpc_m * ((long)n * K1S(p) + k);
                    for (int i = 0; i < 3 * p.cpc_m; ++i) go.put_gf(cb + i, T(0));
                }
            }
            break;
        case UNIT_INTERVAL:
            if constexpr ((UMASK & (1 << UNIT_INTERVAL)) == 0) break;
            if (ROWS) {
                seg(SEG_CONT);
                seg(SEG_SROWS);
            }
            if (GRAD) {
                T acc = T(0);
                for (int j = 0; j < K1S(p); ++j)
                    acc += T(p.Bq[j]) * stage_cost<M, T, KS>(p, n, j, w, (T*)nullptr, (T*)nullptr);
                go.put_gf(n, acc);
                go.put_fpart(n, w(n) * acc);
            }
            break;
        case UNIT_RK4:   // k = Jacobian column group
            if constexpr (RK4)
                if (ROWS) seg(SEG_RK4);
            break;
        default:
            break;
    }
    if (ROWS) s.finish();
}

struct Layout {
    ProbD p{};                        // host pointers into the vectors below
    std::vector<double> geom, node_s, interval_s, spheres, cpc_wp;
    std::vector<ato_gate> gates;
    std::vector<int32_t> seg, tail;   // segment tables (see ProbD)
    std::vector<int32_t> units;       // work-unit table (see ProbD)
    std::vector<int32_t> units_lf;    // the same units, long chains first (small batches)
    std::vector<int32_t> row_ptr, col;
    std::vector<double> lbg, ubg;
    int nz = 0, nu = 0;

    void rebind() {
        p.geom = geom.data();
        p.node_s = node_s.data();
        p.interval_s = interval_s.data();
        p.gates = gates.data();
        p.spheres = spheres.empty() ? nullptr : spheres.data();
        p.cpc_wp = cpc_wp.empty() ? nullptr : cpc_wp.data();
        p.seg = seg.data();
        p.tail = tail.data();
        p.units = units.data();
        p.n_units = (int32_t)(units.size() / 4);
    }

    // returns empty string on success
    std::string build(const ato_problem_desc& d) {
        if (d.abi_version != ATO_ABI_VERSION) return "abi_version mismatch";
        if (d.N < 1) return "N must be >= 1";
        if (d.transcription == ATO_TRANS_RK4) {
            if (d.K != 0) return "RK4 transcription needs K = 0 (one node per interval)";
        } else if (d.transcription == ATO_TRANS_COLLOCATION) {
            if (d.K < 1 || d.K > ATO_KMAX) return "K out of range [1, ATO_KMAX]";
        } else {
            return "unknown transcription";
        }
        if (d.closed && d.N < 2) return "closed problems need N >= 2";
        if (!d.closed && d.transcription == ATO_TRANS_RK4)
            return "open (non-periodic) RK4 racelines are not supported by this build";
        if (!d.closed && d.frame == ATO_FRAME_PARAMETRIC && !d.global_r)
            return "open parametric racelines need global_r (the relative attitude's R depends on s)";
        std::memset(&p, 0, sizeof(p));
        p.model = d.model;
        p.att = d.attitude;
        p.frame = d.frame == ATO_FRAME_GLOBAL ? GLOBAL : (d.global_r ? PARAM_GR : PARAM_REL);
        p.trans = d.transcription;
        p.N = d.N;
        p.K = d.K;
        p.K1 = d.K + 1;
        p.P = d.N * (d.K + 1);
        if (d.model == ATO_MODEL_DRONE) {
            nz = d.attitude == ATO_ATT_ESP ? 13 : (d.attitude == ATO_ATT_DCM ? 18 : 12);
            nu = 4;
        } else if (d.model == ATO_MODEL_POINT) {
            nz = 6;
            nu = 3;
        } else {
            return "unknown model";
        }
        if (d.model == ATO_MODEL_DRONE && d.attitude != ATO_ATT_ESP && d.attitude != ATO_ATT_YPR &&
            d.attitude != ATO_ATT_DCM)
            return "unknown attitude parameterisation";
        p.NZ = nz;
        p.NU = nu;
        p.NV = nz + 2 * nu;
        p.nw = p.N + p.P * p.NV;
        if (d.cpc_m < 0 || d.cpc_m > ATO_CPC_MAX) return "cpc_m out of range [0, ATO_CPC_MAX]";
        if (d.cpc_m > 0) {
            if (d.frame != ATO_FRAME_GLOBAL) return "CPC gate progress needs the global frame";
            if (d.n_gates != 0 || d.has_spheres) return "CPC gate progress replaces the gate and obstacle rows";
            p.cpc_m = d.cpc_m;
            p.cpc_off = p.nw;
            p.nw += p.P * 3 * d.cpc_m;
            cpc_wp.assign(d.cpc_wp, d.cpc_wp + 3 * d.cpc_m);
        }
        p.closed = d.closed;
        p.cleanly_closed = d.cleanly_closed;
        p.quat_flip = d.quat_flip;
        p.force_reg = d.force_regularity;
        p.n_gates = d.n_gates;
        p.phase_len = d.frame == ATO_FRAME_GLOBAL ? d.phase_len : 0;
        p.has_spheres = d.has_spheres;
        p.euler_wraps = d.euler_wraps;
        p.gamma = d.gamma;
        p.veh.m = d.m;
        p.veh.g = d.g;
        for (int i = 0; i < 3; ++i) {
            p.veh.b[i] = d.b[i];
            p.veh.I[i] = d.I[i];
            p.veh.bw[i] = d.bw[i];
        }
        p.veh.l = d.l;
        p.veh.kt = d.kt;
        p.veh.Tmax = d.T_max;
        std::memcpy(p.Rc, d.Rcost, sizeof(p.Rc));
        std::memcpy(p.dRc, d.dRcost, sizeof(p.dRc));
        std::memcpy(p.tau, d.tau, sizeof(p.tau));
        std::memcpy(p.Bq, d.Bq, sizeof(p.Bq));
        // C is stored with row stride K+1
        for (int j = 0; j < p.K1; ++j)
            for (int r = 0; r < p.K1; ++r) p.C[j * p.K1 + r] = d.C[j * p.K1 + r];
        std::memcpy(p.D, d.D, sizeof(p.D));
        std::memcpy(p.A_skew, d.A_skew, sizeof(p.A_skew));

        const bool param = d.frame == ATO_FRAME_PARAMETRIC;
        if (param && (!d.node_geom || !d.interval_s)) return "parametric frame needs node_geom and interval_s";
        if (d.n_gates < 0 || (d.n_gates > 0 && !d.gates)) return "bad gates";
        if (d.has_spheres && !d.spheres) return "has_spheres without spheres table";
        if (d.frame == ATO_FRAME_GLOBAL && d.phase_len < 0) return "bad phase_len";

        geom.assign((size_t)p.P * ATO_GEOM_WIDTH, 0.0);
        if (d.node_geom) std::memcpy(geom.data(), d.node_geom, geom.size() * sizeof(double));
        node_s.assign(p.P, 0.0);
        if (d.node_s) std::memcpy(node_s.data(), d.node_s, node_s.size() * sizeof(double));
        interval_s.assign(p.N + 1, 0.0);
        if (d.interval_s) std::memcpy(interval_s.data(), d.interval_s, interval_s.size() * sizeof(double));
        gates.assign(d.gates, d.gates + d.n_gates);
        for (const ato_gate& g : gates) {
            if (g.interval < 0 || g.interval >= p.N) return "gate interval out of range";
            if (g.shape != ATO_GATE_CIRCLE && g.shape != ATO_GATE_SQUARE) return "bad gate shape";
            if (g.n_coef < 1 || g.n_coef > ATO_KMAX + 1 || g.interval * p.K1 + g.n_coef > p.P)
                return "gate n_coef out of range";
            if (d.transcription == ATO_TRANS_RK4 && g.at_end)
                return "RK4 gate at the end of the horizon is not supported by this build";
        }
        spheres.clear();
        if (d.has_spheres) spheres.assign(d.spheres, d.spheres + (size_t)p.P * 3);
        seg.assign((size_t)p.P * NSEG * 2, -1);
        tail.clear();
        rebind();

        row_ptr.assign(1, 0);
        col.clear();
        lbg.clear();
        ubg.clear();
        std::string err;
        const bool ok = with_model(p, [&]<class M>() { err = this->assemble<M>(d); });
        if (!ok) return "unsupported model / frame combination";
        if (!err.empty()) return err;
        p.ng = (int32_t)lbg.size();
        p.nnz = (int32_t)col.size();
        p.n_tail = (int32_t)(tail.size() / 4);
        build_units();
        rebind();
        return "";
    }

    // Work units in three classes:
    //   0: tail segments (equal-h rows, gates, closure), one unit each
    //   1: the ODE row groups of every collocation node (register-heavy)
    //   2: node units (s-dot, dU, regularity, stage, sphere rows, input gradients) and
    //      interval units (continuity, fixed-s rows, h gradient, cost partial)
    // The tail units come first; the two orders of the rest follow.
    //
    // Unit orders. Interval-major (the default table): the ODE, interval and node units of interval
    // n together, so the re-reads of the interval's w hit the XCD's L2. Long-first (units_lf): the
    // interval units (the longest dependent chains) right after the tail, then interval-major ODE
    // and node units -- at small batches (few waves per slot) the kernel's end is set by the long
    // units dispatched last, at large ones by locality (tools/r03g.sh: B = 512 59.5 -> 47.4 us,
    // B = 4096 507 -> 526 us). ATO_UNIT_ORDER=class|interval|longfirst forces one order for both.
    static int forced_order() {
        const char* e = std::getenv("ATO_UNIT_ORDER");
        if (!e) return -1;
        if (std::strcmp(e, "class") == 0) return 0;
        if (std::strcmp(e, "longfirst") == 0) return 2;
        return 1;
    }

    void build_units() {
        const int f = forced_order();
        build_order(f < 0 ? 1 : f, units);
        build_order(f < 0 ? 2 : f, units_lf);
    }

    // order 0: class-major (all ODE units, then node and interval units; ProbD::cls_off delimits
    // the classes), 1: interval-major, 2: long-first
    void build_order(int order, std::vector<int32_t>& out) {
        out.clear();
        auto add = [&](int kind, int n, int k) {
            out.push_back(kind);
            out.push_back(n);
            out.push_back(k);
            out.push_back(0);
        };
        p.cls_off[0] = 0;
        for (int t = 0; t < (int)(tail.size() / 4); ++t) {
            int nu_t = 1;
            with_model(p, [&]<class M>() { nu_t = tail_units<M>(p, tail[4 * t]); });
            for (int g = 0; g < nu_t; ++g) add(UNIT_TAIL, t, g);
        }
        p.cls_off[1] = (int32_t)(out.size() / 4);
        auto add_ode = [&](int n) {
            for (int k = 1; k < p.K1; ++k) {
                const int32_t* sg = &seg[((size_t)(n * p.K1 + k) * NSEG) * 2];
                if (sg[2 * SEG_ODE_A] >= 0) add(UNIT_ODE_A, n, k);
                if (sg[2 * SEG_ODE_B] >= 0) add(UNIT_ODE_B, n, k);
            }
        };
        auto add_rk4 = [&](int n) {
            const int32_t* sg = &seg[((size_t)(n * p.K1) * NSEG) * 2];
            if (sg[2 * SEG_RK4] < 0) return;
            int ng_ = 1;
            with_model(p, [&]<class M>() { ng_ = rk4_groups<M>(); });
            for (int g = 0; g < ng_; ++g) add(UNIT_RK4, n, g);
        };
        if (order == 2) {
            for (int n = 0; n < p.N; ++n) add(UNIT_INTERVAL, n, 0);
            for (int n = 0; n < p.N; ++n) {
                add_ode(n);
                add_rk4(n);
                for (int k = 0; k < p.K1; ++k) add(UNIT_NODE, n, k);
            }
        } else if (order == 1) {
            for (int n = 0; n < p.N; ++n) {
                add_ode(n);
                add_rk4(n);
                add(UNIT_INTERVAL, n, 0);
                for (int k = 0; k < p.K1; ++k) add(UNIT_NODE, n, k);
            }
        } else {
            for (int n = 0; n < p.N; ++n) add_ode(n);
            for (int n = 0; n < p.N; ++n) add_rk4(n);
            p.cls_off[2] = (int32_t)(out.size() / 4);
            for (int n = 0; n < p.N; ++n) {
                add(UNIT_INTERVAL, n, 0);
                for (int k = 0; k < p.K1; ++k) add(UNIT_NODE, n, k);
            }
            p.cls_off[3] = (int32_t)(out.size() / 4);
            return;
        }
        p.cls_off[2] = p.cls_off[3] = (int32_t)(out.size() / 4);
    }

  private:
    // append one segment's pattern; returns its (row0, nnz0)
    std::pair<int, int> append(const SegPat& sp) {
        const int row0 = (int)lbg.size(), nnz0 = (int)col.size();
        size_t off = 0;
        for (size_t r = 0; r < sp.rowlen.size(); ++r) {
            for (int e = 0; e < sp.rowlen[r]; ++e) col.push_back(sp.cols[off + e]);
            off += sp.rowlen[r];
            row_ptr.push_back((int32_t)col.size());
            lbg.push_back(sp.lb[r]);
            ubg.push_back(sp.ub[r]);
        }
        return {row0, nnz0};
    }

    template <class M>
    std::string node_segment(int kind, int n, int k) {
        SegPat sp;
        PatSink s{&sp};
        run_node_seg<M, double, 0>(p, kind, n, k, OnesW{}, s);
        if (!s.sorted) return "internal: unsorted columns in node segment " + std::to_string(kind);
        auto [r0, e0] = append(sp);
        const size_t slot = ((size_t)(n * p.K1 + k) * NSEG + kind) * 2;
        seg[slot] = r0;
        seg[slot + 1] = e0;
        return "";
    }

    template <class M>
    std::string tail_segment(int kind, int index) {
        SegPat sp;
        PatSink s{&sp};
        run_tail_seg<M, double, 0>(p, kind, index, OnesW{}, s);
        if (!s.sorted) return "internal: unsorted columns in tail segment " + std::to_string(kind);
        auto [r0, e0] = append(sp);
        tail.push_back(kind);
        tail.push_back(index);
        tail.push_back(r0);
        tail.push_back(e0);
        return "";
    }

    template <class M>
    std::string assemble(const ato_problem_desc& d) {
        if (M::NZ != nz || M::NU != nu) return "internal: model size mismatch";
        std::string e;
#define ATO_TRY(x) do { e = (x); if (!e.empty()) return e; } while (0)
        if (p.phase_len > 0) ATO_TRY(tail_segment<M>(TAIL_HEQ, 0));
        const bool param = M::PARAM;
        for (int n = 0; n < p.N; ++n) {
            if (p.trans == ATO_TRANS_RK4) {   // base_raceline.py:363-391 / :1052-1112
                if (param) ATO_TRY(node_segment<M>(SEG_RK4S, n, 0));
                if (n == p.N - 1) continue;
                ATO_TRY(node_segment<M>(SEG_RK4, n, 0));
                if (!M::IS_DRONE) ATO_TRY(node_segment<M>(SEG_STAGE, n, 0));
                if (param && p.force_reg && geom[(size_t)n * ATO_GEOM_WIDTH + 13] != 0.0)
                    ATO_TRY(node_segment<M>(SEG_REG, n, 0));
                continue;
            }
            for (int k = 0; k < p.K1; ++k) {
                if (param) ATO_TRY(node_segment<M>(SEG_SDOT, n, k));
                if (k > 0) {
                    ATO_TRY(node_segment<M>(SEG_ODE_A, n, k));
                    if (ode_split<M>() < M::NZ) ATO_TRY(node_segment<M>(SEG_ODE_B, n, k));
                }
                ATO_TRY(node_segment<M>(SEG_DU, n, k));
            }
            if (param && p.force_reg)
                for (int k = 0; k < p.K1; ++k)
                    if (geom[(size_t)(n * p.K1 + k) * ATO_GEOM_WIDTH + 13] != 0.0)
                        ATO_TRY(node_segment<M>(SEG_REG, n, k));
            if (!M::IS_DRONE)
                for (int k = 0; k < p.K1; ++k) ATO_TRY(node_segment<M>(SEG_STAGE, n, k));
            if (n >= 1) ATO_TRY(node_segment<M>(SEG_CONT, n, 0));
            if (param) ATO_TRY(node_segment<M>(SEG_SROWS, n, 0));
        }
        if (p.closed && !M::IS_DRONE) ATO_TRY(tail_segment<M>(TAIL_CLOSURE_BASE, 0));
        if (!p.closed) {        // base_raceline.py:359-361
            ATO_TRY(tail_segment<M>(TAIL_INITIAL, 0));
            ATO_TRY(tail_segment<M>(TAIL_TERMINAL, 0));
        }
        for (int g = 0; g < p.n_gates; ++g) ATO_TRY(tail_segment<M>(TAIL_GATE, g));
        if (p.has_spheres) {
            if (!param) return "obstacle spheres need the parametric frame";
            for (int n = 0; n < p.N; ++n)
                for (int k = 0; k < p.K1; ++k) ATO_TRY(node_segment<M>(SEG_SPHERE, n, k));
        }
        if (p.cpc_m > 0) {      // CPC gate progress, node by node in time order
            for (int n = 0; n < p.N; ++n)
                for (int k = 0; k < p.K1; ++k) {
                    ATO_TRY(node_segment<M>(SEG_CPC_COMP, n, k));
                    if (p.cpc_m > 1) ATO_TRY(node_segment<M>(SEG_CPC_ORDER, n, k));
                    if (n * p.K1 + k + 1 < p.P) ATO_TRY(node_segment<M>(SEG_CPC_PROG, n, k));
                }
        }
        if (p.closed && M::IS_DRONE) ATO_TRY(tail_segment<M>(TAIL_DRONE_CLOSURE, 0));
#undef ATO_TRY
        (void)d;
        return "";
    }
};

}  // namespace ato
