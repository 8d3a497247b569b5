// hostcheck.cpp -- TEST-ONLY CPU build of the device segment programs.
//
// Compiles ato_program.hpp / ato_layout.hpp with g++ (no HIP) and evaluates the same
// programs the kernels run, one instance and one node at a time. It exists so the C++
// Jacobian derivations can be checked against the numpy oracle on a machine without a
// GPU. It is never loaded by the product package (aircraft_trajectory_optimization_amd),
// whose evaluation path is the HIP library only.
#include <string>
#include <vector>
#define ATO_HESS_ANALYSIS_IMPL
#include "../../aircraft_trajectory_optimization_amd/csrc/ato_hessian.hpp"

namespace {

template <class T>
struct HostSink {
    T* J;
    T* g;
    long je, ge, e, r;
    void begin(int row0, int nnz0) {
        r = (long)row0 * ge;
        e = (long)nnz0 * je;
    }
    void jac(int, T v) {
        if (J) J[e] = v;
        e += je;
    }
    void row(T gv, double, double) {
        if (g) g[r] = gv;
        r += ge;
    }
    void skip() { e += je; }
    void row_skip() { r += ge; }
    void finish() {}
};

template <class T>
struct HostW {
    const T* w;
    long ws;
    const double* pb = nullptr;   // per-instance sphere centres (ProbD::isph) of this instance
    long ps = 0;
    T operator()(int col) const { return w[(long)col * ws]; }
    double par(long i) const { return pb[i * ps]; }
};

thread_local std::string last_err;

}  // namespace

template <class T>
struct HostTangentSink {
    T* J;
    long e;
    void begin(int, int nnz0) { e = nnz0; }
    void jac(int, const ato::Dual<T, 1>& v) { J[e++] = v.d[0]; }
    void row(const ato::Dual<T, 1>&, double, double) {}
    void skip() { ++e; }
    void row_skip() {}
    void finish() {}
};

struct atoh_handle {
    ato::Layout L;
    ato::HessLayout HL;
    bool hess = false;
};

extern "C" {

const char* atoh_last_error() { return last_err.c_str(); }

int atoh_create(const ato_problem_desc* d, atoh_handle** out) {
    auto* h = new atoh_handle();
    std::string e = h->L.build(*d);
    if (!e.empty()) {
        last_err = e;
        delete h;
        return -1;
    }
    *out = h;
    return 0;
}

void atoh_destroy(atoh_handle* h) { delete h; }

// per-instance sphere centres (ato_set_instance_spheres): host table [P][2][stride], NULL clears
int atoh_set_instance_spheres(atoh_handle* h, const double* centres, long stride) {
    if (centres && !h->L.p.has_spheres) {
        last_err = "per-instance spheres need a problem with sphere rows";
        return -1;
    }
    h->L.p.isph = centres;
    h->L.p.isph_stride = centres ? stride : 0;
    return 0;
}

// row index of every node's sphere row (-1: none)
void atoh_sphere_rows(const atoh_handle* h, int32_t* rows) {
    for (int q = 0; q < h->L.p.P; ++q) rows[q] = h->L.seg[((size_t)q * ato::NSEG + ato::SEG_SPHERE) * 2];
}

void atoh_sizes(const atoh_handle* h, int32_t* nw, int32_t* ng, int32_t* nnz) {
    *nw = h->L.p.nw;
    *ng = h->L.p.ng;
    *nnz = h->L.p.nnz;
}

void atoh_sparsity(const atoh_handle* h, int32_t* row_ptr, int32_t* col) {
    for (size_t i = 0; i < h->L.row_ptr.size(); ++i) row_ptr[i] = h->L.row_ptr[i];
    for (size_t i = 0; i < h->L.col.size(); ++i) col[i] = h->L.col[i];
}

void atoh_bounds(const atoh_handle* h, double* lb, double* ub) {
    for (size_t i = 0; i < h->L.lbg.size(); ++i) {
        lb[i] = h->L.lbg[i];
        ub[i] = h->L.ubg[i];
    }
}

// instance-major evaluation of B instances: w [B][nw], g [B][ng], J [B][nnz], f [B], gf [B][nw]
// Walks the same work-unit table and calls the same run_unit() as the HIP kernel.
int atoh_eval(const atoh_handle* h, int B, const double* w, double* g, double* J, double* f, double* gf) {
    const ato::ProbD& p = h->L.p;
    bool ok = ato::with_model(p, [&]<class M>() {
        std::vector<double> fpart(p.N);
        for (int b = 0; b < B; ++b) {
            HostW<double> W{w + (long)b * p.nw, 1, p.isph ? p.isph + b : nullptr, (long)p.isph_stride};
            HostSink<double> s{J ? J + (long)b * p.nnz : nullptr, g ? g + (long)b * p.ng : nullptr, 1, 1, 0, 0};
            const ato::GradOut<double> go{gf + (long)b * p.nw, 1, fpart.data(), 1};
            for (int u = 0; u < p.n_units; ++u) {
                const int32_t* ut = p.units + 4 * u;
                ato::run_unit<M, double, 0, true, true>(p, ut[0], ut[1], ut[2], W, s, go);
            }
            f[b] = ato::reduce_cost(fpart.data(), 1, p.N);
        }
    });
    if (!ok) {
        last_err = "unsupported model";
        return -1;
    }
    return 0;
}

// the same evaluation with the instances spread over nthreads OpenMP threads (CPU baseline)
int atoh_eval_threads(const atoh_handle* h, int B, const double* w, double* g, double* J, double* f, double* gf,
                      int nthreads) {
    const ato::ProbD& p = h->L.p;
    bool ok = true;
#pragma omp parallel num_threads(nthreads)
    {
        std::vector<double> fpart(p.N);
        bool lok = ato::with_model(p, [&]<class M>() {
#pragma omp for schedule(static)
            for (int b = 0; b < B; ++b) {
                HostW<double> W{w + (long)b * p.nw, 1, p.isph ? p.isph + b : nullptr, (long)p.isph_stride};
                HostSink<double> s{J ? J + (long)b * p.nnz : nullptr, g ? g + (long)b * p.ng : nullptr, 1, 1, 0, 0};
                const ato::GradOut<double> go{gf + (long)b * p.nw, 1, fpart.data(), 1};
                for (int u = 0; u < p.n_units; ++u) {
                    const int32_t* ut = p.units + 4 * u;
                    ato::run_unit<M, double, 0, true, true>(p, ut[0], ut[1], ut[2], W, s, go);
                }
                f[b] = ato::reduce_cost(fpart.data(), 1, p.N);
            }
        });
        if (!lok) {
#pragma omp critical
            ok = false;
        }
    }
    if (!ok) {
        last_err = "unsupported model";
        return -1;
    }
    return 0;
}

int atoh_hess_sparsity(atoh_handle* h, int32_t* nnz, int32_t* n_colors) {
    if (!h->hess) {
        std::string e = h->HL.build(h->L);
        if (!e.empty()) {
            last_err = e;
            return -1;
        }
        h->hess = true;
    }
    *nnz = h->HL.nnz();
    *n_colors = h->HL.n_colors;
    return 0;
}

void atoh_hess_pattern(const atoh_handle* h, int32_t* row_ptr, int32_t* col) {
    for (size_t i = 0; i < h->HL.row_ptr.size(); ++i) row_ptr[i] = h->HL.row_ptr[i];
    for (size_t i = 0; i < h->HL.col.size(); ++i) col[i] = h->HL.col[i];
}

// instance-major: w [B][nw], lam [B][ng], sigma [B], H [B][nnz_h]; the same seeded passes and
// recovery as the HIP launcher
int atoh_hess_eval(atoh_handle* h, int B, const double* w, const double* lam, const double* sigma, double* H) {
    int32_t nnzh, nc;
    if (atoh_hess_sparsity(h, &nnzh, &nc)) return -1;
    const ato::ProbD& p = h->L.p;
    const ato::HessLayout& HL = h->HL;
    std::vector<double> dJ(p.nnz), dgf(p.nw);
    bool ok = ato::with_model(p, [&]<class M>() {
        for (int b = 0; b < B; ++b) {
            for (int c = 0; c < HL.n_colors; ++c) {
                ato::ColorW<double, HostW<double>> W{
                    HostW<double>{w + (long)b * p.nw, 1, p.isph ? p.isph + b : nullptr, (long)p.isph_stride},
                    HL.color.data(), c};
                HostTangentSink<double> s{dJ.data(), 0};
                const ato::TangentGrad<double> go{dgf.data(), 1};
                for (int u = 0; u < p.n_units; ++u) {
                    const int32_t* ut = p.units + 4 * u;
                    ato::run_unit<M, ato::Dual<double, 1>, 0, true, true>(p, ut[0], ut[1], ut[2], W, s, go);
                }
                for (int t = HL.take_off[c]; t < HL.take_off[c + 1]; ++t)
                    H[(long)b * nnzh + HL.take_e[t]] =
                        ato::hess_take(HL.tk_ptr.data(), HL.tk_ent.data(), HL.tk_row.data(), t, HL.take_r[t],
                                       sigma[b], lam + (long)b * p.ng, 1L, dJ.data(), 1L, dgf.data(), 1L);
            }
        }
    });
    if (!ok) {
        last_err = "unsupported model";
        return -1;
    }
    return 0;
}

// diagnostic: over every colour's seeded pass at one point w, the Jacobian tangents that the device
// pass does not store (HessLayout::amask bit clear) must be exact zeros; returns how many are not
// (and their largest magnitude in *max_abs)
int atoh_hess_mask_check(atoh_handle* h, const double* w, double* max_abs) {
    int32_t nnzh, nc;
    if (atoh_hess_sparsity(h, &nnzh, &nc)) return -1;
    const ato::ProbD& p = h->L.p;
    const ato::HessLayout& HL = h->HL;
    std::vector<double> dJ(p.nnz), dgf(p.nw);
    int bad = 0;
    *max_abs = 0.0;
    ato::with_model(p, [&]<class M>() {
        for (int c = 0; c < HL.n_colors; ++c) {
            ato::ColorW<double, HostW<double>> W{HostW<double>{w, 1, p.isph, (long)p.isph_stride}, HL.color.data(), c};
            HostTangentSink<double> s{dJ.data(), 0};
            const ato::TangentGrad<double> go{dgf.data(), 1};
            for (int u = 0; u < p.n_units; ++u) {
                const int32_t* ut = p.units + 4 * u;
                ato::run_unit<M, ato::Dual<double, 1>, 0, true, true>(p, ut[0], ut[1], ut[2], W, s, go);
            }
            for (int e = 0; e < p.nnz; ++e)
                if (!(HL.amask[(size_t)c * HL.mask_words + e / 32] >> (e % 32) & 1u) && dJ[e] != 0.0) {
                    ++bad;
                    *max_abs = std::max(*max_abs, std::abs(dJ[e]));
                }
        }
    });
    return bad;
}

}  // extern "C"
