// ato_capi.hip -- the C ABI of libato.so (include/ato.h): handle lifetime, sparsity, bounds,
// and dispatch of ato_eval to the per-model launchers (ato_inst.hip).
#include <hip/hip_runtime.h>
#include <string>
#include <exception>
#include <new>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include "ato_kernels.hpp"

#include "ato_handle.hpp"

static thread_local std::string g_last_error;

static int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

void ato_internal_set_error(const std::string& msg) { g_last_error = msg; }

#define ATO_HIP(call)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) return fail(ATO_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class V>
static int upload(const std::vector<V>& host, V** dev) {
    *dev = nullptr;
    if (host.empty()) return ATO_OK;
    ATO_HIP(hipMalloc((void**)dev, host.size() * sizeof(V)));
    ATO_HIP(hipMemcpy(*dev, host.data(), host.size() * sizeof(V), hipMemcpyHostToDevice));
    return ATO_OK;
}

static void release(ato_handle* h) {
    if (!h) return;
    (void)hipFree(h->d_geom);
    (void)hipFree(h->d_node_s);
    (void)hipFree(h->d_interval_s);
    (void)hipFree(h->d_spheres);
    (void)hipFree(h->d_cpc_wp);
    (void)hipFree(h->d_gates);
    (void)hipFree(h->d_seg);
    (void)hipFree(h->d_tail);
    (void)hipFree(h->d_units);
    (void)hipFree(h->d_units_lf);
    (void)hipFree(h->d_fpart);
    for (int32_t* d : {h->d_color, h->d_take_e, h->d_take_r, h->d_tk_ptr, h->d_tk_ent, h->d_tk_row, h->d_tkf_ptr,
                       h->d_tkf_ent, h->d_tkf_row, h->d_take_off})
        (void)hipFree(d);
    (void)hipFree(h->d_amask);
    (void)hipFree(h->d_dJ);
    (void)hipFree(h->d_dgf);
    for (hipEvent_t e : h->events) (void)hipEventDestroy(e);
    h->events.clear();
}

extern "C" {

const char* ato_last_error(void) { return g_last_error.c_str(); }

const char* ato_version(void) { return "ato 2 gfx950"; }

static int create_impl(const ato_problem_desc* desc, ato_handle** out);

// C++ exceptions (std::bad_alloc, std::length_error of the host layout / Hessian analysis) must not
// cross the C ABI: they would end the host process in std::terminate (SIGABRT)
#define ATO_NOEXCEPT_BODY(expr)                                                                   \
    try {                                                                                        \
        return (expr);                                                                           \
    } catch (const std::exception& e_) {                                                         \
        return fail(ATO_ERR_ARG, std::string("host exception: ") + e_.what());                   \
    } catch (...) {                                                                              \
        return fail(ATO_ERR_ARG, "host exception");                                              \
    }

int ato_create(const ato_problem_desc* desc, ato_handle** out) { ATO_NOEXCEPT_BODY(create_impl(desc, out)) }

static int create_impl(const ato_problem_desc* desc, ato_handle** out) {
    if (!desc || !out) return fail(ATO_ERR_ARG, "null argument");
    *out = nullptr;
    ato_handle* h = new (std::nothrow) ato_handle();
    if (!h) return fail(ATO_ERR_ARG, "out of host memory");
    std::string err = h->L.build(*desc);
    if (!err.empty()) {
        delete h;
        return fail(err.find("not supported") != std::string::npos ? ATO_ERR_UNSUPPORTED : ATO_ERR_ARG, err);
    }
    // Debug / profiling aid: ATO_DEBUG_UNITS=<digits> keeps only the listed unit kinds
    // (0 tail, 1 ODE_A, 2 ODE_B, 3 node, 4 interval). Outputs are then incomplete.
    if (const char* filt = std::getenv("ATO_DEBUG_UNITS")) {
        std::vector<int32_t> kept;
        int cnt[3] = {0, 0, 0};
        for (int c = 0; c < 3; ++c)   // keep the class ordering of the table
            for (size_t u = 0; u + 3 < h->L.units.size(); u += 4) {
                const int kind = h->L.units[u];
                const int cl = kind == ato::UNIT_TAIL ? 0 : (kind <= ato::UNIT_ODE_B ? 1 : 2);
                if (cl == c && std::strchr(filt, '0' + kind)) {
                    kept.insert(kept.end(), &h->L.units[u], &h->L.units[u] + 4);
                    ++cnt[c];
                }
            }
        h->L.units = kept;
        h->L.units_lf = kept;
        h->L.p.cls_off[0] = 0;
        h->L.p.cls_off[1] = cnt[0];
        h->L.p.cls_off[2] = cnt[0] + cnt[1];
        h->L.p.cls_off[3] = cnt[0] + cnt[1] + cnt[2];
        h->L.rebind();
    }
    int rc;
    if (hipGetDevice(&h->device) != hipSuccess) {
        delete h;
        return fail(ATO_ERR_HIP, "no HIP device");
    }
    if ((rc = upload(h->L.geom, &h->d_geom)) || (rc = upload(h->L.node_s, &h->d_node_s)) ||
        (rc = upload(h->L.interval_s, &h->d_interval_s)) || (rc = upload(h->L.spheres, &h->d_spheres)) ||
        (rc = upload(h->L.gates, &h->d_gates)) || (rc = upload(h->L.seg, &h->d_seg)) ||
        (rc = upload(h->L.tail, &h->d_tail)) || (rc = upload(h->L.units, &h->d_units)) ||
        (rc = upload(h->L.units_lf, &h->d_units_lf)) || (rc = upload(h->L.cpc_wp, &h->d_cpc_wp))) {
        release(h);
        delete h;
        return rc;
    }
    h->pd = h->L.p;
    h->pd.geom = h->d_geom;
    h->pd.node_s = h->d_node_s;
    h->pd.interval_s = h->d_interval_s;
    h->pd.spheres = h->d_spheres;
    h->pd.cpc_wp = h->d_cpc_wp;
    h->pd.gates = h->d_gates;
    h->pd.seg = h->d_seg;
    h->pd.tail = h->d_tail;
    h->pd.units = h->d_units;
    h->pd_lf = h->pd;
    h->pd_lf.units = h->d_units_lf;
    if (const char* e = std::getenv("ATO_LONGFIRST_MAX_B")) h->lf_max_batch = std::atoi(e);
    if (const char* e = std::getenv("ATO_EVAL_TILE")) h->eval_tile = std::atoi(e);
    if (const char* e = std::getenv("ATO_EVAL_TILE_LF")) h->tile_lf = std::atoi(e) != 0;
    if (const char* e = std::getenv("ATO_HESS_MASK")) h->hess_mask = std::atoi(e) != 0;
    *out = h;
    return ATO_OK;
}

int ato_destroy(ato_handle* h) {
    if (!h) return ATO_OK;
    release(h);
    delete h;
    return ATO_OK;
}

int ato_sizes(const ato_handle* h, int32_t* nw, int32_t* ng, int32_t* nnz) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    if (nw) *nw = h->L.p.nw;
    if (ng) *ng = h->L.p.ng;
    if (nnz) *nnz = h->L.p.nnz;
    return ATO_OK;
}

int ato_sparsity(const ato_handle* h, const int32_t** row_ptr, const int32_t** col) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    if (row_ptr) *row_ptr = h->L.row_ptr.data();
    if (col) *col = h->L.col.data();
    return ATO_OK;
}

int ato_set_instance_spheres(ato_handle* h, const double* centres, int64_t stride) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    if (centres && !h->L.p.has_spheres) return fail(ATO_ERR_ARG, "per-instance spheres need a problem with sphere rows");
    if (centres && stride < 1) return fail(ATO_ERR_ARG, "bad sphere table stride");
    for (ato::ProbD* p : {&h->pd, &h->pd_lf}) {
        p->isph = centres;
        p->isph_stride = centres ? stride : 0;
    }
    return ATO_OK;
}

int ato_sphere_rows(const ato_handle* h, int32_t* rows) {
    if (!h || !rows) return fail(ATO_ERR_ARG, "null argument");
    for (int q = 0; q < h->L.p.P; ++q) rows[q] = h->L.seg[((size_t)q * ato::NSEG + ato::SEG_SPHERE) * 2];
    return ATO_OK;
}

int ato_gradf_mode(ato_handle* h, int32_t sparse) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    for (ato::ProbD* p : {&h->pd, &h->pd_lf}) p->gf_sparse = sparse ? 1 : 0;
    return ATO_OK;
}

int ato_gradf_sparsity(const ato_handle* h, int32_t* nnz, int32_t* idx) {
    if (!h || !nnz) return fail(ATO_ERR_ARG, "null argument");
    // the entries the gradient passes write with a value (Layout units: interval n writes h_n, node
    // (n, k) its inputs u and input rates du); everything else is a structural zero of grad f
    const ato::ProbD& p = h->L.p;
    const int N = p.N, NZ = p.NZ, NU = p.NU, NV = p.NV;
    const int per_interval = p.K1;          // (RK4: K = 0, one node per interval)
    int32_t c = 0;
    for (int n = 0; n < N; ++n) {
        if (idx) idx[c] = n;
        ++c;
    }
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < per_interval; ++k)
            for (int i = 0; i < 2 * NU; ++i) {
                if (idx) idx[c] = N + (n * per_interval + k) * NV + NZ + i;
                ++c;
            }
    *nnz = c;
    return ATO_OK;
}

int ato_bounds(const ato_handle* h, double* lbg, double* ubg) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    for (size_t i = 0; i < h->L.lbg.size(); ++i) {
        if (lbg) lbg[i] = h->L.lbg[i];
        if (ubg) ubg[i] = h->L.ubg[i];
    }
    return ATO_OK;
}

// colours whose seeded passes share one launch: their scratch is held at once, within a byte budget
// (ATO_HESS_GROUP_BYTES, default 2 GiB) -- at B = 512 on the racetrack nine colours, at restoration widths
// all of them
static size_t hess_group_bytes() {
    static const size_t v = [] {
        const char* e = std::getenv("ATO_HESS_GROUP_BYTES");
        const long long b = e ? std::atoll(e) : (2LL << 30);
        return (size_t)(b > 0 ? b : 0);
    }();
    return v;
}

static int hess_reserve(ato_handle* h, int32_t max_batch) {
    if (max_batch <= h->hess_reserved) return ATO_OK;
    // the old scratch may still be read by kernels queued on any stream: drain before freeing
    if (h->d_dJ || h->d_dgf) ATO_HIP(hipDeviceSynchronize());
    (void)hipFree(h->d_dJ);
    (void)hipFree(h->d_dgf);
    h->d_dJ = h->d_dgf = nullptr;
    h->hess_reserved = 0;
    h->hess_colors = 0;
    const size_t per = ((size_t)std::max(h->L.p.nnz, 1) + (size_t)h->L.p.nw) * (size_t)max_batch * sizeof(double);
    const int nc = std::max(h->HL.n_colors, 1);
    const int g = (int)std::max<size_t>(1, std::min<size_t>((size_t)nc, hess_group_bytes() / std::max<size_t>(per, 1)));
    ATO_HIP(hipMalloc(&h->d_dJ, (size_t)g * std::max(h->L.p.nnz, 1) * max_batch * sizeof(double)));
    if (hipMalloc(&h->d_dgf, (size_t)g * h->L.p.nw * max_batch * sizeof(double)) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(h->d_dJ);
        h->d_dJ = nullptr;
        return fail(ATO_ERR_HIP, "hessian scratch: out of device memory");
    }
    h->hess_reserved = max_batch;
    h->hess_colors = g;
    return ATO_OK;
}

int ato_reserve(ato_handle* h, int32_t max_batch) {
    if (!h || max_batch < 1) return fail(ATO_ERR_ARG, "bad reserve arguments");
    if (h->hess_ready) {
        int rc = hess_reserve(h, max_batch);
        if (rc) return rc;
    }
    if (max_batch <= h->reserved) return ATO_OK;
    if (h->d_fpart) {
        ATO_HIP(hipDeviceSynchronize());        // queued evaluations may still write the old partials
        ATO_HIP(hipFree(h->d_fpart));
    }
    h->d_fpart = nullptr;
    h->reserved = 0;
    ATO_HIP(hipMalloc(&h->d_fpart, (size_t)h->L.p.N * max_batch * sizeof(double)));
    h->reserved = max_batch;
    return ATO_OK;
}

}  // extern "C"

template <class T>
static int eval_impl(ato_handle* h, int32_t batch, int32_t layout, const T* w, T* g, T* jac, T* f,
                     T* grad_f, void* stream) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    if (batch < 1) return fail(ATO_ERR_ARG, "batch must be >= 1");
    if (layout != ATO_LAYOUT_INTERLEAVED && layout != ATO_LAYOUT_INSTANCE_MAJOR)
        return fail(ATO_ERR_ARG, "unknown layout");
    if (!w) return fail(ATO_ERR_ARG, "w is null");
    const bool wf = f || grad_f;
    if (wf && !(f && grad_f)) return fail(ATO_ERR_ARG, "f and grad_f must be requested together");
    if (wf && batch > h->reserved) {
        int rc = ato_reserve(h, batch);
        if (rc) return rc;
    }
    // small batches run the long-first unit order (see Layout::build_units); larger ones run in
    // instance tiles of eval_tile chunks (long-first inside a tile when tile_lf)
    const bool tiled = batch > h->lf_max_batch && h->eval_tile > 0;
    const ato::ProbD& p = batch <= h->lf_max_batch || (tiled && h->tile_lf) ? h->pd_lf : h->pd;
    hipError_t e = hipSuccess;
    ato::with_model(p, [&]<class M>() {
        hipEvent_t* ev = nullptr;
        const bool sample = h->timing_stride <= 1 || h->timing_seen % h->timing_stride == 0;
        if (!h->events.empty()) ++h->timing_seen;
        if (sample && (size_t)(h->timed_calls + 1) * 3 <= h->events.size())
            ev = &h->events[(size_t)h->timed_calls++ * 3];
        e = ato::launch_eval<M, T>(p, batch, layout, w, g, jac, grad_f, f, (T*)h->d_fpart, (hipStream_t)stream,
                                   ev, tiled ? h->eval_tile : 0);
    });
    if (e != hipSuccess) return fail(ATO_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return ATO_OK;
}

extern "C" int ato_timing(ato_handle* h, int32_t max_calls) {
    if (!h || max_calls < 0) return fail(ATO_ERR_ARG, "bad timing arguments");
    for (hipEvent_t e : h->events) ATO_HIP(hipEventDestroy(e));
    h->events.clear();
    h->timed_calls = 0;
    h->timing_seen = 0;
    for (int i = 0; i < 3 * max_calls; ++i) {
        hipEvent_t e;
        // timing only: without the system-scope release the stop stamp is not delayed by the
        // write-back of the L2s the kernel's ~250 MB of stores stream through (hipExtLaunchKernel
        // stamps with default events read 52.4 us where rocprof's trace of the same launches
        // averaged 46.7 us, gpurun_out/r03i)
        ATO_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        h->events.push_back(e);
    }
    return ATO_OK;
}

extern "C" int ato_timing_stride(ato_handle* h, int32_t stride) {
    if (!h || stride < 1) return fail(ATO_ERR_ARG, "bad timing stride");
    h->timing_stride = stride;
    return ATO_OK;
}

extern "C" int ato_timing_read(ato_handle* h, double* eval_ms, double* reduce_ms, int32_t* calls) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    double se = 0.0, sr = 0.0;
    for (int32_t c = 0; c < h->timed_calls; ++c) {
        hipEvent_t* ev = &h->events[(size_t)c * 3];
        ATO_HIP(hipEventSynchronize(ev[2]));
        float a = 0.f, b = 0.f;
        ATO_HIP(hipEventElapsedTime(&a, ev[0], ev[1]));
        ATO_HIP(hipEventElapsedTime(&b, ev[1], ev[2]));
        se += a;
        sr += b;
    }
    if (eval_ms) *eval_ms = se;
    if (reduce_ms) *reduce_ms = sr;
    if (calls) *calls = h->timed_calls;
    return ATO_OK;
}

// Hessian structure, colouring and recovery tables (host analysis + upload), once per handle
static int ensure_hess_impl(ato_handle* h);
static int ensure_hess(ato_handle* h) { ATO_NOEXCEPT_BODY(ensure_hess_impl(h)) }
static int ensure_hess_impl(ato_handle* h) {
    if (h->hess_ready) return ATO_OK;
    std::string err = h->HL.build(h->L);
    if (!err.empty()) return fail(ATO_ERR_UNSUPPORTED, err);
    int rc;
    if ((rc = upload(h->HL.color, &h->d_color)) || (rc = upload(h->HL.take_e, &h->d_take_e)) ||
        (rc = upload(h->HL.take_r, &h->d_take_r)) || (rc = upload(h->HL.tk_ptr, &h->d_tk_ptr)) ||
        (rc = upload(h->HL.tk_ent, &h->d_tk_ent)) || (rc = upload(h->HL.tk_row, &h->d_tk_row)) ||
        (rc = upload(h->HL.tkf_ptr, &h->d_tkf_ptr)) || (rc = upload(h->HL.tkf_ent, &h->d_tkf_ent)) ||
        (rc = upload(h->HL.tkf_row, &h->d_tkf_row)) || (rc = upload(h->HL.amask, &h->d_amask)) ||
        (rc = upload(h->HL.take_off, &h->d_take_off)))
        return rc;
    h->hess_ready = true;
    return ATO_OK;
}

extern "C" int ato_hess_sparsity(ato_handle* h, int32_t* nnz, const int32_t** row_ptr, const int32_t** col,
                                 int32_t* n_colors) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    int rc = ensure_hess(h);
    if (rc) return rc;
    if (nnz) *nnz = h->HL.nnz();
    if (row_ptr) *row_ptr = h->HL.row_ptr.data();
    if (col) *col = h->HL.col.data();
    if (n_colors) *n_colors = h->HL.n_colors;
    return ATO_OK;
}

extern "C" int ato_hess_eval(ato_handle* h, int32_t batch, int32_t layout, const double* w, const double* lam,
                             const double* sigma, double* hess, void* stream) {
    if (!h) return fail(ATO_ERR_ARG, "null handle");
    if (batch < 1) return fail(ATO_ERR_ARG, "batch must be >= 1");
    if (layout != ATO_LAYOUT_INTERLEAVED && layout != ATO_LAYOUT_INSTANCE_MAJOR)
        return fail(ATO_ERR_ARG, "unknown layout");
    if (!w || !lam || !sigma || !hess) return fail(ATO_ERR_ARG, "null buffer");
    int rc = ensure_hess(h);
    if (rc) return rc;
    if ((rc = hess_reserve(h, batch))) return rc;
    const bool mk = h->hess_mask;
    const ato::HessDev hd{h->d_color, h->d_take_e, h->d_take_r, mk ? h->d_tk_ptr : h->d_tkf_ptr,
                          mk ? h->d_tk_ent : h->d_tkf_ent, mk ? h->d_tk_row : h->d_tkf_row,
                          mk ? h->d_amask : nullptr, h->HL.mask_words,
                          h->HL.take_off.data(), h->HL.n_colors, h->HL.nnz(), h->d_take_off,
                          // colours per launch at this batch: as many as the scratch holds
                          (int)std::max<long long>(1, std::min<long long>(h->HL.n_colors,
                              (long long)h->hess_colors * h->hess_reserved / batch))};
    hipError_t e = hipSuccess;
    ato::ProbD p = batch <= h->lf_max_batch ? h->pd_lf : h->pd;   // unit order as in ato_eval
    p.gf_sparse = 0;    // the seeded passes' grad f tangents fill a scratch buffer: every entry is written
    ato::with_model(p, [&]<class M>() {
        e = ato::launch_hess<M>(p, hd, batch, layout, w, lam, sigma, hess, h->d_dJ, h->d_dgf,
                                (hipStream_t)stream);
    });
    if (e != hipSuccess) return fail(ATO_ERR_HIP, std::string("hessian launch: ") + hipGetErrorString(e));
    return ATO_OK;
}

extern "C" int ato_eval(ato_handle* h, int32_t batch, int32_t layout, const double* w, double* g,
                        double* jac, double* f, double* grad_f, void* stream) {
    return eval_impl<double>(h, batch, layout, w, g, jac, f, grad_f, stream);
}

extern "C" int ato_eval_f32(ato_handle* h, int32_t batch, int32_t layout, const float* w, float* g,
                            float* jac, float* f, float* grad_f, void* stream) {
    return eval_impl<float>(h, batch, layout, w, g, jac, f, grad_f, stream);
}
