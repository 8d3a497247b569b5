/*
 * ato_kkt.h -- batched factorisation and solve of the interior-point KKT system on the
 * device (part of libato.so).
 *
 * What it replaces. IPOPT, called by the reference through
 *     ca.nlpsol('solver', 'ipopt', ...)   drone3d/raceline/base_raceline.py:752-799
 * factorises its augmented system with MUMPS (or HSL MA97, :765-782) on every iteration
 * and reads the inertia from that factorisation; that is most of the reference's
 * `ipopt_time` (base_raceline.py:182-189). Here the same system
 *
 *     K = [ W + diag_x   J^T    ]      W: Lagrangian Hessian (lower CSR, ato_hess_sparsity)
 *         [ J            diag_r ]      J: constraint Jacobian  (CSR, ato_sparsity)
 *
 * is factorised for a BATCH of instances at once by a multifrontal symmetric-indefinite
 * LDL^T over an elimination tree of fronts (solver/kkt_plan.py: nested dissection of the
 * interval chain). A front's dense block -- its own positions and the trailing positions
 * its ancestors eliminate -- is assembled from the original entries assigned to it and the
 * contribution blocks of its children, held in registers, and its own positions are
 * eliminated with Bunch-Kaufman pivoting restricted to them; the trailing Schur complement
 * is its contribution to the parent. The fronts of one level are independent: one launch
 * per level over (front, instance) workgroups. The inertia (n+, n-, n0) of K is returned
 * per instance -- what IPOPT's inertia correction needs.
 *
 * All value pointers are DEVICE pointers; element e of instance b of every value array
 * (H, J, diag_x, diag_r, x) is at [e * stride_elem + b * stride_inst], so both the
 * interleaved ([e][B]: stride_elem = B, stride_inst = 1) and the instance-major layout work.
 */
#ifndef ATO_KKT_H
#define ATO_KKT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ato_kkt_plan_desc {
    int32_t n, m;               /* variables, constraint rows (KKT dim = n + m)                 */
    int32_t n_fronts;           /* F                                                            */
    int32_t n_levels;           /* L                                                            */
    const int32_t* level_ptr;   /* [L + 1] fronts of level l: level_ptr[l] .. level_ptr[l+1]-1   */
    const int32_t* level_tiles; /* [L] 32-wide register tiles of the level's largest front (<=8) */
    const int32_t* pos_ptr;     /* [F + 1] offsets into pos_index / parent_pos                   */
    const int32_t* n_own;       /* [F] eliminated (own) positions of every front, listed first  */
    const int32_t* pos_index;   /* [P] KKT index of every front position                        */
    const int32_t* parent_pos;  /* [P] trailing position -> position in the parent, -1 for own   */
    const int32_t* child_ptr;   /* [F + 1] offsets into child_list                               */
    const int32_t* child_list;  /* [C] children of every front (all in lower levels)             */
    const int32_t* ent_ptr;     /* [F * 9 + 1] entries of (front, 32-row strip), fronts <= 288      */
    const int32_t* ent_pos;     /* [E] (pa << 16) | pb, pa >= pb                                  */
    const int32_t* ent_src;     /* [E][2] (kind << 29) | index; kind 0 H, 1 J, 2 diag_x,          *
                                 * 3 diag_r; -1 = none. The value is the sum of both sources.    */
    const int64_t* l_off;       /* [F] factor-column offset of every front (doubles)             */
    int64_t l_size;             /* factor-column doubles per instance                           */
    const int32_t* piv_off;     /* [F] pivot-record offset of every front                        */
    const int64_t* cb_off;      /* [F] contribution-block offset (tq * tq doubles per front)     */
    int64_t cb_size;            /* contribution-block doubles per instance                      */
    const int32_t* sc_off;      /* [F] solve-contribution offset (tq doubles per front)          */
    int32_t sc_size;            /* solve-contribution doubles per instance                      */
    const int32_t* kres_ptr;    /* [n + m + 1] CSR of the whole K (both triangles): residuals    */
    const int32_t* kres_col;    /* [nnz_K] column (KKT index) of every entry                     */
    const int32_t* kres_src;    /* [nnz_K] source code of every entry (as ent_src, one source)   */
    const int32_t* n_sad;       /* [F] or NULL: nS of a SADDLE front (own = nS states, then their *
                                 * nS ODE defect rows; no children), 0 for the others. Its block  *
                                 * [[H, J^T], [J, 0]] is eliminated by an LU of the square J and *
                                 * dense products (inertia (nS, nS, 0)); Bunch-Kaufman when J is  *
                                 * singular or the rows carry a diagonal (delta_c).              */
} ato_kkt_plan_desc;

typedef struct ato_kkt ato_kkt;

int ato_kkt_create(const ato_kkt_plan_desc* desc, ato_kkt** out);
int ato_kkt_destroy(ato_kkt* kkt);

/* Device storage of the factors of instances 0 .. max_batch-1 (about l_size + cb_size doubles
 * each). */
int ato_kkt_reserve(ato_kkt* kkt, int32_t max_batch);

/* Factorise K for `batch` instances: instance list[i] (device int32 array; NULL = 0..batch-1)
 * is factorised into its own storage slot. H may be NULL (W = 0). inertia: device int32
 * [max_batch][3] = (positive, negative, zero) pivots, written for the listed instances.
 * Asynchronous on stream: levels whose fronts fall into several kernel classes also use a
 * second stream owned by the handle, forked from and joined into `stream` by events, so the
 * result is ordered on `stream`. One host thread per handle. */
int ato_kkt_factor(ato_kkt* kkt, int32_t batch, const int32_t* list, int64_t stride_elem,
                   int64_t stride_inst, const double* H, const double* J, const double* diag_x,
                   const double* diag_r, int32_t* inertia, void* stream);

/* Solve K x = rhs in place (x holds rhs on entry, KKT order: variables then rows) with the
 * factors of the listed instances. Asynchronous on stream. */
int ato_kkt_solve(ato_kkt* kkt, int32_t batch, const int32_t* list, int64_t stride_elem,
                  int64_t stride_inst, double* x, void* stream);

/* out = rhs - K x for all `batch` instances (x, rhs, out: [n + m] KKT order; H may be NULL),
 * the residual of IPOPT's iterative refinement of a KKT solve. Every instance sums its row
 * entries in a fixed order (deterministic). Asynchronous on stream. */
int ato_kkt_residual(ato_kkt* kkt, int32_t batch, int64_t stride_elem, int64_t stride_inst,
                     const double* H, const double* J, const double* diag_x, const double* diag_r,
                     const double* x, const double* rhs, double* out, void* stream);

/* The same for the listed instances only (device int32 list of `count` instance indices; NULL =
 * 0..count-1): iterative refinement of the instances whose residual is still above the ratio.
 * Columns of unlisted instances in `out` are left untouched. */
int ato_kkt_residual_list(ato_kkt* kkt, int32_t count, const int32_t* list, int64_t stride_elem,
                          int64_t stride_inst, const double* H, const double* J, const double* diag_x,
                          const double* diag_r, const double* x, const double* rhs, double* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ATO_KKT_H */
