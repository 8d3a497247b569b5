/*
 * ato_ipm.h -- fused column kernels of the batched interior-point iteration (part of libato.so).
 *
 * What it replaces. IPOPT (ca.nlpsol('solver', 'ipopt', ...), ref: drone3d/raceline/
 * base_raceline.py:752-799) runs its iteration's vector algebra -- optimality errors, barrier
 * gradient and right-hand side, fraction-to-the-boundary step sizes, filter measures, bound
 * multiplier updates -- on host vectors of one instance. The batched solver
 * (solver/batched_ipm.py) runs the same algebra for W instances ("columns") at once; each entry
 * point below does one of those steps in one or two launches instead of tens of elementwise
 * tensor operations, with per-column reductions in a fixed order (deterministic).
 *
 * Every vector is a DEVICE array in the interleaved layout [element][W]: element e of column b
 * is at e * W + b. Per-column scalars (mu, tau, f, ...) are device arrays [W]. Bounds are
 * +-infinity where absent; a bound is present where it is finite. The slack of inequality
 * row iin[i] is s[i]. IEEE operations are evaluated in the order of the host formulas (no
 * contraction), so elementwise outputs equal solver/batched_ipm.py's bit for bit; sums are
 * taken chunk by chunk in a fixed order.
 */
#ifndef ATO_IPM_H
#define ATO_IPM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ato_ipm_dims {
    int32_t n;                 /* variables                                          */
    int32_t m;                 /* constraint rows                                    */
    int32_t mi;                /* inequality rows (slacks)                           */
    int32_t meq;               /* equality rows                                      */
    const int32_t* iin;        /* [mi] device: row of every slack                   */
    const int32_t* ieq;        /* [meq] device: equality rows                       */
    int32_t W;                 /* columns (instances)                                */
} ato_ipm_dims;

typedef struct ato_ipm_bounds {
    const double* xL;          /* [n][W] variable bounds (relaxed)                  */
    const double* xU;
    const double* dL;          /* [mi][W] slack bounds (relaxed)                    */
    const double* dU;
} ato_ipm_bounds;

/* KKT diagonals of one inertia-correction pass (batched_ipm.py _kkt_step, IPOPT's perturbed
 * augmented system): dx = Sx + dw [n][W], Ds = Ss + dw [mi][W], dr [m][W] = -dc on equality rows and
 * -dc - 1 / Ds on slack rows; dw, dc [W] the per-column delta_w / delta_c. */
int ato_ipm_kkt_diag(const ato_ipm_dims* d, const double* Sx, const double* Ss, const double* dw, const double* dc,
                     double* dx, double* dr, double* Ds, void* stream);

/* doubles of workspace the reductions below need for these dimensions */
size_t ato_ipm_work_size(const ato_ipm_dims* d);

/* Optimality errors (IPOPT E_mu; batched_ipm.py _errors + the unscaled primal infeasibility).
 * dual_x = grad f + J^T y - zl + zu. out [5][W] = (E_mu, dual inf, primal inf, complementarity
 * inf, max |r / sg|) with r the constraint residual (g - c_rhs on equality rows, g - s on
 * slack rows) and s_max, n_bounds [W] the scaling of E_mu. */
int ato_ipm_errors(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                   const double* g, const double* c_rhs, const double* sg, const double* y, const double* zl,
                   const double* zu, const double* vl, const double* vu, const double* dual_x, const double* mu,
                   const double* n_bounds, double s_max, double* work, double* out, void* stream);

/* Barrier Newton system pieces (batched_ipm.py solve: Sx, Ss, _grad_phi, right-hand side):
 * Sx [n][W], Ss [mi][W], gx [n][W], gs [mi][W], rhs_x = -(gx + jty) [n][W],
 * rhs_s = -(gs - y[iin]) [mi][W], rhs_y = -r [m][W]. jty = J^T y. */
int ato_ipm_rhs(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                const double* g, const double* c_rhs, const double* gf, const double* jty, const double* y,
                const double* zl, const double* zu, const double* vl, const double* vu, const double* mu,
                double kappa_d, double* Sx, double* Ss, double* gx, double* gs, double* rhs_x, double* rhs_s,
                double* rhs_y, void* stream);

/* Bound multiplier steps and step sizes (IPOPT fraction to the boundary): dzl, dzu [n][W],
 * dvl, dvu [mi][W]; out [3][W] = (alpha_max of (x, s), alpha_z of the multipliers, the
 * directional derivative gx^T dx + gs^T ds). */
int ato_ipm_direction(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                      const double* dx, const double* ds, const double* zl, const double* zu, const double* vl,
                      const double* vu, const double* gx, const double* gs, const double* mu, const double* tau,
                      double* dzl, double* dzu, double* dvl, double* dvu, double* work, double* out, void* stream);

/* Filter measures of a point: out [2][W] = (theta = sum |r|, barrier objective phi). */
int ato_ipm_measures(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                     const double* g, const double* c_rhs, const double* f, const double* mu, double kappa_d,
                     double* work, double* out, void* stream);

/* Accepted step of the bound multipliers (in place): z += az dz, then IPOPT's kappa_sigma
 * safeguard against the slacks of the accepted (x, s). */
int ato_ipm_multipliers(const ato_ipm_dims* d, const ato_ipm_bounds* bd, const double* x, const double* s,
                        const double* mu, const double* az, double kappa_sigma, double* zl, double* zu, double* vl,
                        double* vu, const double* dzl, const double* dzu, const double* dvl, const double* dvu,
                        void* stream);

/* Filter line-search acceptance test of a trial point (batched_ipm.py _accept and the trial
 * bookkeeping around it; IPOPT A-5.4 - A-5.5, Waechter & Biegler 2006 eqs. (18)-(20)), one
 * thread per column. theta, phi: measures of the current iterate; gphi_d: barrier directional
 * derivative; alpha: trial step; tht, pht: measures of the trial point; F [W][fmax][2] the
 * filter entries (theta, phi) of every column, nf [W] (int64) how many are valid; theta_max,
 * theta_min [W]; pend, first [W] (bytes 0/1): columns still searching, first trial of the
 * search. prm = HOST array {s_phi, s_theta, delta, eta_phi, gamma_theta, gamma_phi, obj_max_inc, compare_tol,
 * max_filter_resets, filter_reset_trigger} (read on the host and passed to the kernel by value; every other
 * pointer is a device array). The sufficient-decrease and Armijo tests hold up to compare_tol |reference|
 * (IpUtils Compare_le). Outputs (bytes 0/1, [W]): ok = pend and accepted, arm = ok and the Armijo (f-type)
 * case, soc = pend, not accepted, first trial and tht >= theta (a second-order correction is tried).
 * fr_n, fr_cnt [W] int64, fr_last [W] bytes (in/out; all NULL: no heuristic): FilterLSAcceptor's filter reset
 * heuristic state of the pend columns (resets so far, successive iterations whose last rejection was the
 * filter's, last rejection was the filter's); a column whose filter is reset gets nf = 0. */
int ato_ipm_filter_accept(int32_t W, int32_t fmax, const double* theta, const double* phi, const double* gphi_d,
                          const double* alpha, const double* tht, const double* pht, const double* F,
                          int64_t* nf, const double* theta_max, const double* theta_min,
                          const uint8_t* pend, const uint8_t* first, const double* prm, int64_t* fr_n,
                          int64_t* fr_cnt, uint8_t* fr_last, uint8_t* ok, uint8_t* arm, uint8_t* soc, void* stream);

/* K successive backtracking trials of P columns tested in order (the lockstep line search's next K rounds at
 * once): trial k of column p has step alpha0[p] / 2^k and measures tht, pht [K][P]; theta, phi, gphi_d,
 * alpha_min, theta_max, theta_min [P]; F [P][fmax][2], nf [P] (in/out), the filter reset heuristic's state
 * fr_n, fr_cnt (int64), fr_last (bytes) [P] in/out, prm as ato_ipm_filter_accept's. A column stops at its first
 * trial with alpha <= alpha_min (failed = 1) or at its first accepted trial (kacc = k, arm = its Armijo case);
 * kacc = -1, failed = 0: none of the K trials decided. The heuristic runs on every tested trial, as K calls of
 * ato_ipm_filter_accept would. */
int ato_ipm_filter_multi(int32_t P, int32_t K, int32_t fmax, const double* theta, const double* phi,
                         const double* gphi_d, const double* alpha0, const double* alpha_min, const double* tht,
                         const double* pht, const double* F, int64_t* nf, const double* theta_max,
                         const double* theta_min, const double* prm, int64_t* fr_n, int64_t* fr_cnt, uint8_t* fr_last,
                         int32_t* kacc, uint8_t* failed, uint8_t* arm, void* stream);

/* IPOPT's PDPerturbationHandler per column (IpPDPerturbationHandler: ConsiderNewSystem,
 * PerturbForSingularity, PerturbForWrongInertia with the structural-degeneracy test; batched_ipm.py
 * BatchedPerturbation) and the bookkeeping of an inertia-correction pass (batched_ipm.py _kkt_step),
 * one thread per column. Handler state, device arrays [W]: hdeg, jdeg (0 unknown / 1 no / 2 yes),
 * diters, test (0 none, 1 C0X0, 2 CPX0, 3 C0XP, 4 CPXP), dx, dc (delta_w, delta_c), dx_last, dc_last.
 * pend [W] bytes 0/1, in/out. op 0 (new system): pend = columns to factorise, out: those that got a
 * perturbation. op 1 (after a factorisation of the pend columns; inertia [W][3] int32 = (positive,
 * negative, zero) eigenvalues, m constraint rows): a right inertia sets dw_out, dc_out = the column's
 * deltas and tosolve = 1; a singular matrix (zero eigenvalues or fewer than m negative ones) or a
 * wrong inertia (more than m negative) gets the next perturbation; out pend = columns to factorise
 * again. op 2 (after the solves): columns with tosolve = 1 and fin = 0 (unrefinable solve) count as
 * singular; tosolve is cleared, out pend as op 1. A column that runs out of perturbations (delta_w
 * above max) leaves pend = 0 without tosolve. prm = HOST array {delta_w_0, delta_w_min, delta_w_max,
 * kappa_w_minus, kappa_w_plus, kappa_w_plus_bar, delta_c_base, kappa_c, degen_iters_max}. */
int ato_ipm_perturb(int32_t op, int32_t W, int32_t m, const double* prm, int64_t* hdeg, int64_t* jdeg,
                    int64_t* diters, int64_t* test, double* dx, double* dc, double* dx_last, double* dc_last,
                    const double* mu, uint8_t* pend, const int32_t* inertia, double* dw_out, double* dc_out,
                    uint8_t* tosolve, const uint8_t* fin, void* stream);
/* Termination tests of a lockstep iteration (batched_ipm.py solve; IPOPT's ConvergenceCheck with the
 * acceptable-level counter), one thread per column, in place: act [W] bytes; n_acc, status [W] int64
 * (1 optimal, 2 acceptable, 3 max_iter; others unchanged). A column still active is optimal when
 * E0 <= tol, du / sf <= dual_inf_tol, pr_uns <= constr_viol_tol and co / sf <= compl_inf_tol; otherwise
 * its n_acc counts consecutive acceptable iterates (CurrentIsAcceptable: E0 <= acceptable_tol, du / sf <=
 * acceptable_dual_inf_tol, pr_uns <= acceptable_constr_viol_tol, co / sf <= acceptable_compl_inf_tol) and
 * acceptable_iter of them make it acceptable; then own >= lim ends it at max_iter. prm = HOST {tol,
 * dual_inf_tol, constr_viol_tol, compl_inf_tol, acceptable_tol, acceptable_iter, acceptable_dual_inf_tol,
 * acceptable_constr_viol_tol, acceptable_compl_inf_tol}. E0, du, pr_uns, co, sf fp64 [W]; own, lim int64 [W]. */
int ato_ipm_status(int32_t W, const double* prm, const double* E0, const double* du, const double* pr_uns,
                   const double* co, const double* sf, const int64_t* own, const int64_t* lim, uint8_t* act,
                   int64_t* n_acc, int64_t* status, void* stream);

/* One pass of the monotone barrier update (IPOPT MonotoneMuUpdate; batched_ipm.py solve), in place:
 * a column of mu_act wants a decrease when Emu <= kappa_eps mu or force; mu_new = max(min(kappa_mu mu,
 * mu^theta_mu), mu_min). A forced column whose mu cannot fall ends (status 8 tiny step, act = mu_act = 0);
 * otherwise a wanted change sets mu, tau = max(1 - mu, tau_min), nf = 0 and upd = 1 (else upd = 0);
 * force is cleared. prm = HOST {kappa_eps, kappa_mu, theta_mu, mu_min, tau_min}. */
int ato_ipm_barrier(int32_t W, const double* prm, const double* Emu, uint8_t* mu_act, uint8_t* force, uint8_t* act,
                    int64_t* status, double* mu, double* tau, int64_t* nf, uint8_t* upd, void* stream);

/* Iterative refinement of a batch of KKT solves (IPOPT's PDFullSpaceSolver; solver/batched_ipm.py
 * _refine): [N][W] vectors, per-column state [W].
 * ato_ipm_refine_work: the number of row chunks nch of the partial buffers ([nch][W] doubles each).
 * ato_ipm_refine_pass: where sel (NULL: every column) -- a += b on the columns with upd (b NULL: no
 *   update), then per row chunk the column maxima of |a| into part_a and of |c| into part_c (c NULL:
 *   none). NaN propagates.
 * ato_ipm_refine_decide (one workgroup): mode 0 -- rr = the column maxima of part_a (e.g. |rhs|);
 *   mode 1 -- the first residual of the solve (sel = the solved columns; part_a = |x|, part_c = |r|):
 *   rr = old = ratio |r| / (min(|x|, 1e6 nr) + nr) on sel (0 elsewhere), bad = 0, refine = sel;
 *   mode 2 -- after refinement step k >= 1 of the columns sel: rr = old = the new ratio, a column
 *   quits when (rr > ratio_max and k > max_steps) or (rr > old and k > min_steps), bad |= quit and
 *   rr > ratio_singular, refine = sel and not quit. Modes 1 and 2 then set need = refine, rr finite
 *   and (k >= min_steps ? rr > ratio_max : true), ok = rr finite and not bad, and write the columns
 *   with need in ascending order to list[1..], their count to list[0] (list: W + 1 int32).
 *   prm (host): ratio_max, ratio_singular, min_steps, max_steps. */
int ato_ipm_refine_work(int32_t N, int32_t W);
int ato_ipm_refine_pass(int32_t N, int32_t W, double* a, const double* b, const uint8_t* upd, const double* c,
                        const uint8_t* sel, double* part_a, double* part_c, void* stream);
int ato_ipm_refine_decide(int32_t N, int32_t W, int32_t mode, int32_t k, const double* prm, const double* part_a,
                          const double* part_c, const uint8_t* sel, const double* nr, double* rr, double* old,
                          uint8_t* bad, uint8_t* refine, uint8_t* need, int32_t* list, uint8_t* ok, void* stream);


/* Rows of the restoration phase's reduced KKT system (solver/batched_ipm.py _RestorationKKT): drow =
 * dr - 1/dp - 1/dn elementwise on [m][W], and cnt[b] (int32 [W][2], ADDED to: zero it first) +=
 * (number of dp, dn > 0, number of dp, dn < 0) over the m rows of column b. */
int ato_ipm_resto_rows(int32_t m, int32_t W, const double* dr, const double* dp, const double* dn, double* drow,
                       int32_t* cnt, void* stream);

/* The scaled Jacobian and its transpose product (solver/batched_ipm.py, the optimality check and the soft
 * restoration's primal-dual error; replaces `Js = jv * sg[jr]` and `_JTy(Js, y)`, the sparse products IPOPT's
 * dual infeasibility grad f + J^T y needs, ref: drone3d/raceline/base_raceline.py:752-799 via ca.nlpsol):
 * jv [nnz][W] Jacobian values in CSR entry order, sg [m][W] row scaling (NULL: Js = jv, js must be NULL),
 * y [m][W]; the entries of column i are src[col_ptr[i] .. col_ptr[i+1]) (entry indices, ascending within a
 * column) with rows row[.]. Writes js [nnz][W] = jv * sg[row] (when js is not NULL) and
 * jty [n][W] = sum over column i's entries, in that order from 0, of js * y[row] (no fused multiply-add). */
int ato_ipm_js_jty(int32_t n, int32_t nnz, int32_t W, const int32_t* col_ptr, const int32_t* src, const int32_t* row,
                   const double* jv, const double* sg, const double* y, double* js, double* jty, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ATO_IPM_H */
