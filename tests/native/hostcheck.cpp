// hostcheck.cpp -- TEST-ONLY CPU build of the device segment programs.
//
// Compiles ato_program.hpp / ato_layout.hpp with g++ (no HIP) and evaluates the same
// programs the kernels run, one instance and one node at a time. It exists so the C++
// Jacobian derivations can be checked against the numpy oracle on a machine without a
// GPU. It is never loaded by the product package (aircraft_trajectory_optimization_amd),
// whose evaluation path is the HIP library only.
#include <string>
#include <vector>
#include "../../aircraft_trajectory_optimization_amd/csrc/ato_layout.hpp"

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
};

template <class T>
struct HostW {
    const T* w;
    long ws;
    T operator()(int col) const { return w[(long)col * ws]; }
};

thread_local std::string last_err;

}  // namespace

struct atoh_handle {
    ato::Layout L;
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
int atoh_eval(const atoh_handle* h, int B, const double* w, double* g, double* J, double* f, double* gf) {
    const ato::ProbD& p = h->L.p;
    bool ok = ato::with_model(p, [&]<class M>() {
        constexpr int NZ = M::NZ, NU = M::NU;
        const ato::Cols<M> c{p.N, p.K1};
        for (int b = 0; b < B; ++b) {
            HostW<double> W{w + (long)b * p.nw, 1};
            HostSink<double> s{J ? J + (long)b * p.nnz : nullptr, g ? g + (long)b * p.ng : nullptr, 1, 1, 0, 0};
            double fsum = 0.0;
            for (int unit = 0; unit < p.P; ++unit) {
                const int n = unit / p.K1, k = unit % p.K1;
                for (int kind = 0; kind < ato::NSEG; ++kind) {
                    const int32_t* sg = p.seg + ((long)unit * ato::NSEG + kind) * 2;
                    if (sg[0] < 0) continue;
                    s.begin(sg[0], sg[1]);
                    ato::run_node_seg<M, double>(p, kind, n, k, W, s);
                }
                double gu[NU], gdu[NU];
                ato::stage_cost<M, double>(p, n, k, W, gu, gdu);
                const double hB = W(n) * p.Bq[k];
                if (gf) {
                    double* gb = gf + (long)b * p.nw;
                    for (int i = 0; i < NZ; ++i) gb[c.z(n, k, i)] = 0.0;
                    for (int i = 0; i < NU; ++i) gb[c.u(n, k, i)] = hB * gu[i];
                    for (int i = 0; i < NU; ++i) gb[c.du(n, k, i)] = hB * gdu[i];
                }
                if (k == 0) {
                    double acc = 0.0;
                    for (int j = 0; j < p.K1; ++j)
                        acc += p.Bq[j] * ato::stage_cost<M, double>(p, n, j, W, (double*)nullptr, (double*)nullptr);
                    if (gf) gf[(long)b * p.nw + n] = acc;
                    fsum += W(n) * acc;
                }
            }
            for (int t = 0; t < p.n_tail; ++t) {
                const int32_t* tl = p.tail + 4 * t;
                s.begin(tl[2], tl[3]);
                ato::run_tail_seg<M, double>(p, tl[0], tl[1], W, s);
            }
            if (f) f[b] = fsum;
        }
    });
    if (!ok) {
        last_err = "unsupported model";
        return -1;
    }
    return 0;
}

}  // extern "C"
