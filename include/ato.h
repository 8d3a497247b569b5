/*
 * ato.h -- C ABI of the MI355X raceline NLP evaluation library (libato.so).
 *
 * What it replaces. The reference builds its collocation NLP as CasADi SX
 * expressions and hands them to IPOPT:
 *     ca.nlpsol('solver', 'ipopt', {'x': w, 'f': J, 'g': g}, opts)
 *         drone3d/raceline/base_raceline.py:752-799
 *     solver(x0=..., lbx=..., ubx=..., lbg=..., ubg=...)
 *         drone3d/raceline/base_raceline.py:157-191
 * Inside that call IPOPT evaluates CasADi's generated functions nlp_g, nlp_jac_g
 * (fixed sparsity), nlp_f and nlp_grad_f on every iterate. This library is the
 * drop-in for those evaluations, for a BATCH of independent problem instances
 * that share one structure (same track, N, K, model), on one HIP device.
 *
 *   ato_create        <- building w, g, J and the nlpsol structure
 *                        (base_raceline.py:218-239, 625-717)
 *   ato_sizes         <- w.numel(), g.numel(), jac_g sparsity nnz
 *   ato_sparsity      <- nlp_jac_g sparsity_out (CSR here; CasADi keeps CCS)
 *   ato_bounds        <- lbg / ubg lists built next to g (base_raceline.py:245-247)
 *   ato_eval          <- nlp_g + nlp_jac_g + nlp_f + nlp_grad_f for B instances
 *   ato_destroy, ato_last_error
 *
 * Conventions: all pointers to ato_eval are DEVICE pointers; tables in
 * ato_problem_desc are HOST pointers copied at ato_create. Every function
 * returns ATO_OK (0) or a negative error code, and ato_last_error() holds the
 * message for the calling thread. A handle belongs to the device that was
 * current when it was created; it is not shared between threads concurrently.
 */
#ifndef ATO_H
#define ATO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ATO_ABI_VERSION 3
#define ATO_KMAX 9            /* highest collocation degree supported */
#define ATO_GEOM_WIDTH 16     /* doubles per node in the geometry table */

enum { ATO_OK = 0, ATO_ERR_ARG = -1, ATO_ERR_UNSUPPORTED = -2, ATO_ERR_HIP = -3,
       ATO_ERR_STATE = -4 };

enum { ATO_MODEL_DRONE = 0, ATO_MODEL_POINT = 1 };
enum { ATO_ATT_ESP = 0, ATO_ATT_YPR = 1, ATO_ATT_DCM = 2 };  /* quaternion / yaw-pitch-roll / direction-cosine
                                                              matrix (build-side, config 5) */
enum { ATO_FRAME_GLOBAL = 0, ATO_FRAME_PARAMETRIC = 1 };
enum { ATO_TRANS_COLLOCATION = 0, ATO_TRANS_RK4 = 1 };
enum { ATO_GATE_CIRCLE = 0, ATO_GATE_SQUARE = 1 };
#define ATO_CPC_MAX 16
/* Batch layout of w, g, jac, grad_f on the device.
 * INTERLEAVED:      element e of instance b at [e * B + b]  (coalesced; default)
 * INSTANCE_MAJOR:   element e of instance b at [b * n + e]  (n = nw, ng or nnz) */
enum { ATO_LAYOUT_INTERLEAVED = 0, ATO_LAYOUT_INSTANCE_MAJOR = 1 };

/* One gate constraint (base_raceline.py:545-595, parametric placement
 * :986-1032, global placement :907-918). */
typedef struct ato_gate {
    int32_t interval;     /* interval n whose nodes interpolate the gate state   */
    int32_t shape;        /* ATO_GATE_CIRCLE / ATO_GATE_SQUARE                    */
    int32_t fix_center;   /* 1: x - gate_x == 0 (3 rows)                         */
    int32_t axial;        /* 1: axial equality row (global frame)                */
    int32_t at_end;       /* 1: state is z_F of the last interval                */
    int32_t n_coef;       /* weights in coef, on the consecutive nodes starting at   *
                           * node (interval, 0): K+1 (collocation), 1 (global frame:  *
                           * Z[interval, 0] itself), 2 (RK4: Z[n], Z[n+1] interpolated)*/
    double coef[ATO_KMAX + 1];  /* Lagrange weights l_k(d) on Z[interval, k]     */
    double gate_x[3];     /* gate centre                                          */
    double R[9];          /* gate orientation (row-major, columns e1 e2 e3)       */
    double xc[3], ey[3], en[3];  /* centreline point and frame at gate s (param.) */
    double d_max;         /* gate_ri - collision_radius                           */
} ato_gate;

typedef struct ato_problem_desc {
    int32_t abi_version;       /* ATO_ABI_VERSION */
    int32_t model;             /* ATO_MODEL_*  */
    int32_t attitude;          /* ATO_ATT_*    (drone only) */
    int32_t frame;             /* ATO_FRAME_*  */
    int32_t global_r;          /* 1: attitude relative to the global frame */
    int32_t transcription;     /* ATO_TRANS_*  */
    int32_t N, K;              /* intervals, collocation degree (0 for RK4) */
    int32_t closed;            /* periodic raceline */
    int32_t cleanly_closed;    /* centreline frame continuous at s_max -> s_min */
    int32_t quat_flip;         /* closure uses qF + q0 instead of qF - q0 */
    int32_t force_regularity;  /* curvature regularity rows */
    int32_t n_gates;
    int32_t phase_len;         /* global frame: intervals per gate phase (0: none) */
    int32_t has_spheres;       /* obstacle tube rows, one per node */
    int32_t pad0;
    double euler_wraps;        /* YPR closure offset count (2 pi * wraps) */
    double gamma;              /* regularity bound */
    /* vehicle (pytypes.py:357-402) */
    double m, g, b[3], I[3], bw[3], l, kt, T_max;
    double Rcost[16], dRcost[16];   /* input / input-rate cost matrices, nu x nu row-major */
    /* collocation coefficients (discretization_utils.py:8-34) */
    double tau[ATO_KMAX + 1], Bq[ATO_KMAX + 1];
    double C[(ATO_KMAX + 1) * (ATO_KMAX + 1)];   /* C[j * (K+1) + r] */
    double D[ATO_KMAX + 1];
    /* closure for parametric point mass on skew-closed lines (base_raceline.py:1209-1222) */
    double A_skew[4];
    /* host tables, copied at ato_create */
    const double* node_geom;   /* [P][ATO_GEOM_WIDTH]: Rp(9) ks ky kn |xc'| reg_active . . . */
    const double* node_s;      /* [P] fixed s of every node (parametric) */
    const double* interval_s;  /* [N+1] s at interval starts (parametric) */
    const ato_gate* gates;     /* [n_gates] */
    const double* spheres;     /* [P][3]: dy, dn, available radius (obstacle tube) */
    /* CPC gate progress (config 5; Foehn et al. 2021 time-optimal planning; build-side, the reference
     * only displays a CPC trajectory, cpc_utils.py:14-101). cpc_m > 0 (global frame, no gate rows):
     * per node q three blocks of cpc_m variables after the node variables -- progress lambda, its
     * decrease mu, tolerance nu -- and the rows, node by node after the obstacle rows:
     *   mu_j (|p_q - w_j|^2 - nu_j) = 0      (cpc_m complementarity rows)
     *   lambda_j - lambda_{j+1} <= 0        (cpc_m - 1 order rows)
     *   lambda_{q+1,j} - lambda_{q,j} + mu_{q,j} = 0   (cpc_m progress rows, not at the last node) */
    int32_t cpc_m;             /* waypoints (<= ATO_CPC_MAX); 0: no CPC */
    int32_t pad1;
    double cpc_wp[ATO_CPC_MAX * 3];   /* waypoint positions w_j */
} ato_problem_desc;

typedef struct ato_handle ato_handle;

int ato_create(const ato_problem_desc* desc, ato_handle** out);
int ato_destroy(ato_handle* h);

/* nw decision variables, ng constraint rows, nnz structural Jacobian entries. */
int ato_sizes(const ato_handle* h, int32_t* nw, int32_t* ng, int32_t* nnz);

/* CSR pattern of dg/dw in reference row order: row_ptr[ng+1], col[nnz] (host arrays
 * owned by the handle; valid until ato_destroy). Columns are ascending per row. */
int ato_sparsity(const ato_handle* h, const int32_t** row_ptr, const int32_t** col);

/* lbg / ubg (host arrays of ng doubles, caller owned). */
int ato_bounds(const ato_handle* h, double* lbg, double* ubg);

/* Structural nonzeros of grad f: idx (host, caller owned, may be NULL to query nnz) gets the
 * ascending indices of h_n and of every node's inputs u and input rates du -- the only variables
 * in the cost J = sum h_n B_k (u'Ru + du'dR du + 1) (base_raceline.py:601-623); the states'
 * entries are structural zeros. */
int ato_gradf_sparsity(const ato_handle* h, int32_t* nnz, int32_t* idx);

/* sparse != 0: ato_eval / ato_eval_f32 write only the ato_gradf_sparsity entries of grad_f and
 * leave the others untouched (the caller zero-fills its buffer once); 0 (default): every entry. */
int ato_gradf_mode(ato_handle* h, int32_t sparse);

/* Reserve device scratch for batches up to max_batch (call before graph capture). */
int ato_reserve(ato_handle* h, int32_t max_batch);

/* Evaluate g, J (values in ato_sparsity order), f and grad_f for `batch` instances.
 * w: [nw x batch] in `layout`; any of g / jac / f / grad_f may be NULL to skip it.
 * f is [batch]. stream is a hipStream_t (NULL = default stream). Asynchronous. */
int ato_eval(ato_handle* h, int32_t batch, int32_t layout, const double* w,
             double* g, double* jac, double* f, double* grad_f, void* stream);

/* Same evaluation in fp32 (w, outputs float). */
int ato_eval_f32(ato_handle* h, int32_t batch, int32_t layout, const float* w,
                 float* g, float* jac, float* f, float* grad_f, void* stream);

/* Hessian of the Lagrangian  sigma * grad^2 f + sum_i lam_i * grad^2 g_i  (IPOPT's nlp_hess_l,
 * base_raceline.py:752-799). Structure: lower triangle (col <= row) CSR with ascending columns
 * (host arrays owned by the handle). The first call analyses the structure and colours the
 * columns; n_colors seeded passes make up one evaluation. */
int ato_hess_sparsity(ato_handle* h, int32_t* nnz, const int32_t** row_ptr, const int32_t** col,
                      int32_t* n_colors);

/* hess [nnz_h x batch] (layout) for w [nw x batch], lam [ng x batch], sigma [batch] (fp64).
 * Asynchronous on stream; allocates its scratch on the first call for a larger batch
 * (ato_reserve after ato_hess_sparsity pre-allocates it). */
int ato_hess_eval(ato_handle* h, int32_t batch, int32_t layout, const double* w, const double* lam,
                  const double* sigma, double* hess, void* stream);

/* Per-instance obstacle-tube sphere centres (config 4's perturbed tubes; the reference builds one
 * ObstacleFreeTube per solve, mesh_obstacle.py:219-237, so a batch of perturbed tubes is a batch of
 * problems that differ only in these constants). centres: DEVICE array [P][2][stride] of doubles,
 * (dy, dn) of node p for instance b at index (2 p + c) * stride + b; it must stay valid while
 * evaluations use it. Applies to ato_eval / ato_eval_f32 / ato_hess_eval until replaced; NULL
 * returns to the descriptor's shared table. The rows' upper bounds (available radius^2) then
 * differ per instance and are the caller's (ato_sphere_rows gives their row indices). Requires a
 * problem with sphere rows (has_spheres). */
int ato_set_instance_spheres(ato_handle* h, const double* centres, int64_t stride);

/* Row index of each node's sphere row, rows[P] (-1: no sphere row at that node). */
int ato_sphere_rows(const ato_handle* h, int32_t* rows);

/* Triangle mesh of an obstacle environment (MeshObstacle, drone3d/obstacles/mesh_obstacle.py:18-161;
 * replaces trimesh.proximity.signed_distance / closest_point). vertices [nv][3], faces [nf][3]
 * (0-based triangles), host arrays copied at creation. */
typedef struct ato_mesh ato_mesh;
int ato_mesh_create(const double* vertices, int32_t n_vertices, const int32_t* faces, int32_t n_faces,
                    ato_mesh** out);
int ato_mesh_destroy(ato_mesh* mesh);

/* Signed distance of n points (device [n][3]) to the mesh into dist (device [n]): positive
 * outside, negative inside (ray-crossing parity). closest (device [n][3], may be NULL) gets the
 * closest surface point. Asynchronous on stream. */
int ato_mesh_signed_distance(ato_mesh* mesh, int32_t n, const double* points, double* dist, double* closest,
                             void* stream);

/* Per-kernel timing with HIP events recorded on the evaluation stream. ato_timing(h, n)
 * allocates n event slots and starts recording (n = 0 stops); while on, each ato_eval
 * records events around its Jacobian kernel and its cost-reduction kernel. ato_timing_read
 * waits for the recorded events and returns the summed durations (ms) and the call count. */
int ato_timing(ato_handle* h, int32_t max_calls);
int ato_timing_read(ato_handle* h, double* eval_ms, double* reduce_ms, int32_t* calls);
/* Sample the timing: while on, only every stride-th ato_eval (counted from the last ato_timing
 * call) records its events (stride 1, the default: every call). Each recorded call puts three
 * event packets into the stream, about 10 us of gaps at the benchmark size; sampling keeps the
 * kernel durations measured inside a timed loop without slowing the loop itself. */
int ato_timing_stride(ato_handle* h, int32_t stride);

const char* ato_last_error(void);

/* Library version string, e.g. "ato 1 gfx950". */
const char* ato_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ATO_H */
