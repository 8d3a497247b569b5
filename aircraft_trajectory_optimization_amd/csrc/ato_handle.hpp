// ato_handle.hpp -- the opaque ato_handle of include/ato.h (library-internal).
#pragma once
#include <vector>
#include <hip/hip_runtime.h>
#include "ato_kernels.hpp"

struct ato_handle {
    ato::Layout L;
    int device = 0;
    ato::ProbD pd{};            // device-pointer copy of L.p (interval-major unit table)
    ato::ProbD pd_lf{};         // the same with the long-first unit table (batches <= lf_max_batch)
    int32_t lf_max_batch = 2048;
    // batches above lf_max_batch: the workgroup order runs eval_tile 64-instance chunks through every
    // unit before the next chunks start (0 = one pass per unit over the whole batch); tile_lf picks
    // the long-first unit table inside the tiles
    int32_t eval_tile = 8;
    bool tile_lf = true;
    double* d_geom = nullptr;
    double* d_node_s = nullptr;
    double* d_interval_s = nullptr;
    double* d_spheres = nullptr;
    double* d_cpc_wp = nullptr;
    ato_gate* d_gates = nullptr;
    int32_t* d_seg = nullptr;
    int32_t* d_tail = nullptr;
    int32_t* d_units = nullptr;
    int32_t* d_units_lf = nullptr;
    void* d_fpart = nullptr;    // [N][reserved] cost partials (double; reused for float)
    int32_t reserved = 0;
    std::vector<hipEvent_t> events;   // 3 per timed call
    int32_t timed_calls = 0;
    int32_t timing_stride = 1;        // events on every timing_stride-th evaluation
    int64_t timing_seen = 0;          // evaluations since ato_timing
    // Hessian of the Lagrangian (built on first use)
    bool hess_ready = false;
    ato::HessLayout HL;
    int32_t *d_color = nullptr, *d_take_e = nullptr, *d_take_r = nullptr;
    int32_t *d_tk_ptr = nullptr, *d_tk_ent = nullptr, *d_tk_row = nullptr;
    int32_t *d_tkf_ptr = nullptr, *d_tkf_ent = nullptr, *d_tkf_row = nullptr;
    uint32_t* d_amask = nullptr;
    bool hess_mask = false;           // ATO_HESS_MASK=1: the masked colour passes (HessLayout::amask)
    int32_t* d_take_off = nullptr;    // device copy of HL.take_off (the colour of a take, grouped passes)
    // seeded-pass scratch for hess_colors colours at hess_reserved instances: [colour][nnz][B] / [colour][nw][B]
    // (a launch runs as many colours as fit at its batch: fewer, larger launches)
    double* d_dJ = nullptr;
    double* d_dgf = nullptr;
    int32_t hess_reserved = 0;
    int32_t hess_colors = 0;
};
