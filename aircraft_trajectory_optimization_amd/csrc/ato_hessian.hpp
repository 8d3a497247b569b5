// ato_hessian.hpp -- Hessian of the Lagrangian, sigma grad^2 f + sum_i lambda_i grad^2 g_i
// (IPOPT's nlp_hess_l, which the reference gets from CasADi AD; base_raceline.py:752-799).
//
// Values: forward-mode dual numbers over the SAME segment programs that produce g and J.
// Seeding w with the 0/1 vector v_c of a column colour c, the tangent of every Jacobian entry
// J_ij is sum_k d2 g_i / dw_j dw_k v_c[k] and the tangent of grad f is grad^2 f v_c, so
//     (H v_c)_r = sigma (grad^2 f v_c)_r + sum_i lambda_i dJ_ir
// and each Hessian entry is read from the one colour that isolates it (direct recovery).
//
// Structure (host, once per problem): the programs run with Dep, a "value" that is the set of
// decision variables it depends on. A Jacobian entry J_ij whose value depends on w_k gives the
// Hessian entry (j, k); the same for grad f. This is the exact structural second-order
// pattern of the transcription, not a conservative row-pair estimate.
//
// Colouring: the step-size columns h_n couple to every variable of their interval (they are
// "hubs"), so they are excluded from the row conflicts and their entries are recovered by
// symmetry from the hub colour instead (H[h, x] = H[x, h] read at row x).
#pragma once
#include <algorithm>
#include <iterator>
#include <string>
#include <utility>
#include <vector>
#include "ato_layout.hpp"

namespace ato {

// ------------------------------------------------------------------ dependency sets (host only)
struct Dep {
    std::vector<int32_t> s;   // sorted, unique
    Dep() = default;
    Dep(double) {}            // NOLINT: constants depend on nothing
    Dep(float) {}             // NOLINT
    Dep(int) {}               // NOLINT
    static Dep var(int col) {
        Dep d;
        d.s.push_back(col);
        return d;
    }
    Dep& operator+=(const Dep& b) { return merge(b); }
    Dep& operator-=(const Dep& b) { return merge(b); }
    Dep& operator*=(const Dep& b) { return merge(b); }
    Dep& merge(const Dep& b) {
        if (b.s.empty()) return *this;
        if (s.empty()) {
            s = b.s;
            return *this;
        }
        std::vector<int32_t> o;
        o.reserve(s.size() + b.s.size());
        std::set_union(s.begin(), s.end(), b.s.begin(), b.s.end(), std::back_inserter(o));
        s.swap(o);
        return *this;
    }
};
inline Dep dep_union(const Dep& a, const Dep& b) {
    Dep r = a;
    r.merge(b);
    return r;
}
inline Dep operator+(const Dep& a, const Dep& b) { return dep_union(a, b); }
inline Dep operator-(const Dep& a, const Dep& b) { return dep_union(a, b); }
inline Dep operator*(const Dep& a, const Dep& b) { return dep_union(a, b); }
inline Dep operator/(const Dep& a, const Dep& b) { return dep_union(a, b); }
inline Dep operator-(const Dep& a) { return a; }
inline Dep operator+(double, const Dep& b) { return b; }
inline Dep operator+(const Dep& a, double) { return a; }
inline Dep operator-(double, const Dep& b) { return b; }
inline Dep operator-(const Dep& a, double) { return a; }
inline Dep operator*(double, const Dep& b) { return b; }
inline Dep operator*(const Dep& a, double) { return a; }
inline Dep operator/(double, const Dep& b) { return b; }
inline Dep operator/(const Dep& a, double) { return a; }
inline Dep tsqrt(Dep a) { return a; }
inline Dep tsin(Dep a) { return a; }
inline Dep tcos(Dep a) { return a; }

struct DepW {
    Dep operator()(int col) const { return Dep::var(col); }
    double par(long) const { return 0.0; }     // per-instance constants depend on nothing
};

// records (column of the entry, variable its value depends on) pairs, and per Jacobian entry (in
// the sinks' entry order) its column and dependency set
struct DepSink {
    std::vector<std::pair<int32_t, int32_t>>* pairs;
    std::vector<std::vector<int32_t>>* ent_dep = nullptr;
    std::vector<int32_t>* ent_col = nullptr;
    int cur = 0;
    void begin(int, int nnz0) { cur = nnz0; }
    int overrun = 0;                           // entries past the Jacobian pattern (a program bug)
    void jac(int col, const Dep& v) {
        for (int32_t k : v.s) pairs->push_back({col, k});
        if (ent_dep) {
            if (cur >= 0 && cur < (int)ent_dep->size()) {
                (*ent_dep)[cur] = v.s;
                (*ent_col)[cur] = col;
            } else {
                ++overrun;
            }
        }
        ++cur;
    }
    void row(const Dep&, double, double) {}
    void skip() { ++cur; }
    void row_skip() {}
    void finish() {}
};

struct DepGrad {
    std::vector<std::pair<int32_t, int32_t>>* pairs;
    void put_gf(long i, const Dep& v) const {
        for (int32_t k : v.s) pairs->push_back({(int32_t)i, k});
    }
    void put_fpart(long, const Dep&) const {}
};

// ------------------------------------------------------------------ Hessian layout
struct HessLayout {
    std::vector<int32_t> row_ptr, col;     // lower triangle (col <= row) CSR, ascending cols
    std::vector<int32_t> color;            // [nw] colour of every decision variable
    int n_colors = 0;
    // recovery: Hessian entry e is (H v_c)_r with c = colour of its take list
    std::vector<int32_t> take_off;         // [n_colors + 1] offsets into take_e / take_r
    std::vector<int32_t> take_e, take_r;
    // CSC of the Jacobian: column r -> (J entry index, J row)
    std::vector<int32_t> csc_ptr, csc_ent, csc_row;
    // Colour c's seeded pass changes only the Jacobian entries that depend on a variable of colour c
    // (the tangent of every other entry is exactly 0): amask[c * mask_words + e / 32] bit e % 32 marks
    // them -- the only tangents the device pass stores -- and take t sums over just those entries of
    // its column: (J entry, J row) = (tk_ent, tk_row)[tk_ptr[t] .. tk_ptr[t + 1])
    std::vector<uint32_t> amask;
    int mask_words = 0;
    std::vector<int32_t> tk_ptr, tk_ent, tk_row;
    // the same take lists over the whole column (the default device pass, which stores every tangent)
    std::vector<int32_t> tkf_ptr, tkf_ent, tkf_row;
    int nnz() const { return (int)col.size(); }

    // structure analysis + colouring (host only; defined in ato_hstruct.cpp, compiled by the host
    // C++ compiler: running the programs on dependency sets inside hipcc's force-inlined device
    // headers would take minutes to compile)
    std::string build(const Layout& L);

    // every take (e, r) in colour c: row r of the symmetric pattern has exactly one column of
    // colour c, and it is the partner of r in entry e
    template <class HubF>
    std::string verify(const std::vector<std::vector<int32_t>>& adj, HubF is_hub) const {
        for (int c = 0; c < n_colors; ++c)
            for (int t = take_off[c]; t < take_off[c + 1]; ++t) {
                const int r = take_r[t];
                int cnt = 0;
                for (int x : adj[r]) cnt += color[x] == c;
                if (cnt != 1) return "hessian: colouring does not isolate entry " + std::to_string(take_e[t]);
                (void)is_hub;
            }
        return "";
    }
};

#ifdef ATO_HESS_ANALYSIS_IMPL
std::string HessLayout::build(const Layout& L) {
    const ProbD& p = L.p;
    const int nw = p.nw;
    std::vector<std::pair<int32_t, int32_t>> pairs;
    const int nnzJ = (int)L.col.size();
    std::vector<std::vector<int32_t>> ent_dep(nnzJ);
    std::vector<int32_t> ent_col(nnzJ, -1);
    int overrun = 0;
    const bool ok = with_model(p, [&]<class M>() {
        DepSink s{&pairs, &ent_dep, &ent_col};
        DepGrad go{&pairs};
        for (int u = 0; u < p.n_units; ++u) {
            const int32_t* ut = p.units + 4 * u;
            run_unit<M, Dep, 0, true, true, UMASK_ALL>(p, ut[0], ut[1], ut[2], DepW{}, s, go);
        }
        overrun = s.overrun;
    });
    if (!ok) return "hessian: unsupported model";
    // symmetric lower-triangular structure
    for (auto& pr : pairs)
        if (pr.first < pr.second) std::swap(pr.first, pr.second);
    std::sort(pairs.begin(), pairs.end());
    pairs.erase(std::unique(pairs.begin(), pairs.end()), pairs.end());
    row_ptr.assign(nw + 1, 0);
    col.clear();
    col.reserve(pairs.size());
    for (auto& pr : pairs) {
        ++row_ptr[pr.first + 1];
        col.push_back(pr.second);
    }
    for (int r = 0; r < nw; ++r) row_ptr[r + 1] += row_ptr[r];
    // full symmetric adjacency (including the diagonal when structural)
    std::vector<std::vector<int32_t>> adj(nw);
    for (auto& pr : pairs) {
        adj[pr.first].push_back(pr.second);
        if (pr.first != pr.second) adj[pr.second].push_back(pr.first);
    }
    for (auto& a : adj) std::sort(a.begin(), a.end());
    auto is_hub = [&](int v) { return v < p.N; };   // step sizes h_n
    for (auto& pr : pairs)
        if (pr.first != pr.second && is_hub(pr.first) && is_hub(pr.second))
            return "hessian: coupled step sizes are not supported by the hub colouring";

    // greedy colouring, largest row first. Conflicts of v:
    //   every column sharing a non-hub row with v (row r contains v: adj[v] holds r),
    //   hub rows containing v: that hub, and a hub conflicts with all its neighbours.
    color.assign(nw, -1);
    std::vector<int32_t> order(nw);
    for (int v = 0; v < nw; ++v) order[v] = v;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return adj[a].size() > adj[b].size(); });
    std::vector<int32_t> mark(8, -1);
    n_colors = 0;
    for (int v : order) {
        auto forbid = [&](int c) {
            if (c < 0) return;
            if (c >= (int)mark.size()) mark.resize(c + 1, -1);
            mark[c] = v;
        };
        for (int r : adj[v]) {
            if (is_hub(r)) {
                forbid(color[r]);
            } else {
                for (int w2 : adj[r])
                    if (w2 != v) forbid(color[w2]);
            }
        }
        if (is_hub(v))
            for (int r : adj[v])
                if (r != v) forbid(color[r]);
        int c = 0;
        while (c < (int)mark.size() && mark[c] == v) ++c;
        color[v] = c;
        n_colors = std::max(n_colors, c + 1);
    }
    // recovery lists
    std::vector<std::vector<std::pair<int32_t, int32_t>>> lists(n_colors);
    for (int j = 0; j < nw; ++j)
        for (int e = row_ptr[j]; e < row_ptr[j + 1]; ++e) {
            const int k = col[e];
            int c, r;
            if (!is_hub(j)) { c = color[k]; r = j; }
            else if (!is_hub(k)) { c = color[j]; r = k; }
            else { c = color[j]; r = j; }   // hub diagonal
            lists[c].push_back({e, r});
        }
    take_off.assign(n_colors + 1, 0);
    take_e.clear();
    take_r.clear();
    for (int c = 0; c < n_colors; ++c) {
        // verify unique recovery: in row r, colour c has exactly the one column it reads
        for (auto& er : lists[c]) {
            take_e.push_back(er.first);
            take_r.push_back(er.second);
        }
        take_off[c + 1] = (int32_t)take_e.size();
    }
    std::string err = verify(adj, is_hub);
    if (!err.empty()) return err;
    // CSC of J
    if (overrun) return "hessian: a seeded pass writes " + std::to_string(overrun) + " entries past the Jacobian";
    for (int e = 0; e < nnzJ; ++e)
        if (ent_col[e] != L.col[e]) return "hessian: seeded-pass entry order differs from the Jacobian pattern";
    csc_ptr.assign(nw + 1, 0);
    for (int e = 0; e < nnzJ; ++e) ++csc_ptr[L.col[e] + 1];
    for (int r = 0; r < nw; ++r) csc_ptr[r + 1] += csc_ptr[r];
    csc_ent.assign(nnzJ, 0);
    csc_row.assign(nnzJ, 0);
    std::vector<int32_t> fill(csc_ptr.begin(), csc_ptr.end() - 1);
    for (int i = 0; i + 1 < (int)L.row_ptr.size(); ++i)
        for (int e = L.row_ptr[i]; e < L.row_ptr[i + 1]; ++e) {
            const int t = fill[L.col[e]]++;
            csc_ent[t] = e;
            csc_row[t] = i;
        }
    // per-colour active entries and the take lists over them
    mask_words = (nnzJ + 31) / 32;
    amask.assign((size_t)n_colors * mask_words, 0u);
    for (int e = 0; e < nnzJ; ++e)
        for (int32_t k : ent_dep[e]) {
            const int c = color[k];
            amask[(size_t)c * mask_words + e / 32] |= 1u << (e % 32);
        }
    tk_ptr.assign(take_r.size() + 1, 0);
    tk_ent.clear();
    tk_row.clear();
    tkf_ptr.assign(take_r.size() + 1, 0);
    tkf_ent.clear();
    tkf_row.clear();
    for (int c = 0; c < n_colors; ++c)
        for (int t = take_off[c]; t < take_off[c + 1]; ++t) {
            const int r = take_r[t];
            for (int q = csc_ptr[r]; q < csc_ptr[r + 1]; ++q) {
                const int e = csc_ent[q];
                tkf_ent.push_back(e);
                tkf_row.push_back(csc_row[q]);
                if (amask[(size_t)c * mask_words + e / 32] >> (e % 32) & 1u) {
                    tk_ent.push_back(e);
                    tk_row.push_back(csc_row[q]);
                }
            }
            tk_ptr[t + 1] = (int32_t)tk_ent.size();
            tkf_ptr[t + 1] = (int32_t)tkf_ent.size();
        }
    return "";
}
#endif

// (H v_c)_r for take t (row r): sigma dgf[r] + sum over the entries of Jacobian column r that colour c
// changes of lambda_i dJ_e (the others add exact zeros); element strides: lam / dJ / dgf by their own
// stride, the caller offsets to the instance
template <class T>
ATO_HD T hess_take(const int32_t* tk_ptr, const int32_t* tk_ent, const int32_t* tk_row, int t, int r, T sigma,
                   const T* lam, long ls, const T* dJ, long js, const T* dgf, long gs) {
    T acc = sigma * dgf[(long)r * gs];
    for (int q = tk_ptr[t]; q < tk_ptr[t + 1]; ++q) acc += lam[(long)tk_row[q] * ls] * dJ[(long)tk_ent[q] * js];
    return acc;
}

// seeded decision-vector loader: columns of colour c carry tangent 1
template <class T, class BaseW>
struct ColorW {
    BaseW base;
    const int32_t* color;
    int c;
    ATO_HD Dual<T, 1> operator()(int col) const { return Dual<T, 1>::seed(base(col), color[col] == c ? 0 : -1); }
    ATO_HD double par(long i) const { return base.par(i); }
};

// gradient output of the seeded pass: only the tangent (grad^2 f v_c) is kept
template <class T>
struct TangentGrad {
    T* gf;
    long st;
    ATO_HD void put_gf(long i, const Dual<T, 1>& v) const { gf[i * st] = v.d[0]; }
    ATO_HD void put_fpart(long, const Dual<T, 1>&) const {}
};

}  // namespace ato
