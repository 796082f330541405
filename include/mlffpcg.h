/*
 * mlffpcg.h — C ABI of the MI355X (gfx950) preconditioned-CG solver for the
 * sGDML kernel linear system  (sigma_K * K + lam * I) x = b.
 *
 * This is the drop-in boundary for the hot path of bluecher31/mlff-preconditioner
 * (reference mounted at /root/reference; citations are relative to it).  The
 * reference wires its solve through scipy LinearOperators and
 * scipy.sparse.linalg.cg; every entry point below replaces one of those plug
 * points:
 *
 *   reference interface (file:line)                                   -> entry point here
 *   ---------------------------------------------------------------------------------------
 *   Iterative._init_kernel_operator / _K_vec
 *       src/sGDML/sgdml/solvers/iterative_solver.py:383-445          -> mlff_set_operator + mlff_matvec
 *   GDMLTrain._assemble_kernel_mat (+ worker)
 *       src/sGDML/sgdml/train.py:81-236, 1121-1308                   -> mlff_assemble_sgdml
 *   K_op as the reference evaluates it (GDMLPredict, alphas = v)
 *       src/sGDML/sgdml/predict.py:72-234, 400-449                   -> mlff_sgdml_operator
 *   Desc.from_R (descriptors + compact Jacobians)
 *       src/sGDML/sgdml/utils/desc.py:292-358                        -> mlff_sgdml_descriptors
 *   GDMLPredict energies on the training set (for _recov_int_const)
 *       src/sGDML/sgdml/predict.py:172-220; train.py:972-1119        -> mlff_sgdml_energies
 *   tools.utils.create_kernel_mat (synthetic RBF)
 *       src/tools/utils.py:173-187                                   -> mlff_gen_rbf
 *   set dense K from the caller (K_hat in custom_cg_solver)
 *       src/tools/custom_cg_solver.py:126-158                        -> mlff_set_matrix_host
 *   pivoted_cholesky + IterativeCholesky._init_precon_operator
 *       src/sGDML/sgdml/solvers/incomplete_cholesky.py:24-93
 *       src/sGDML/sgdml/solvers/iterative_cholesky.py:115-150        -> mlff_precon_pivchol
 *   Iterative._init_precon_operator (Nystrom, "_P_vec")
 *       src/sGDML/sgdml/solvers/iterative_solver.py:95-322           -> mlff_precon_nystrom(variant 0)
 *   Iterative._init_precon_operator_sb ("*_custom")
 *       src/sGDML/sgdml/solvers/iterative_solver.py:326-381          -> mlff_precon_nystrom(variant 1)
 *   svd_preconditioner (Woodbury on a supplied low-rank factor)
 *       src/sGDML/sgdml/solvers/iterative_solver.py:1313-1329        -> mlff_precon_lowrank
 *   P_op.matvec                                                       -> mlff_precon_apply
 *   scipy.sparse.linalg.cg(-K_op, y, x0, M=P_op, tol, atol=None, maxiter, callback)
 *       src/sGDML/sgdml/solvers/iterative_solver.py:995-1005         -> mlff_pcg_start / mlff_pcg_run /
 *                                                                       mlff_pcg_result
 *   _lev_scores (numeric part)
 *       src/sGDML/sgdml/solvers/iterative_solver.py:447-552          -> mlff_lev_scores
 *   _init_precon_operator_eigvals / _rank_k_leverage_scores (svd of K)
 *       src/sGDML/sgdml/solvers/iterative_solver.py:1110-1329        -> mlff_precon_eig
 *
 * Conventions
 *  - All matrices are fp64.  Host buffers are C-contiguous, owned by the
 *    caller, and never retained after a call returns.
 *  - One context = one GPU = one rank.  With world > 1 the N rows of K (and
 *    every N-vector) are split into contiguous row blocks, rank r owning rows
 *    [row0, row0 + nrows) (see mlff_shard_range).  "local" buffers have nrows
 *    entries, "global" buffers have N entries.
 *  - Every function returns MLFF_OK (0) or a negative MLFF_ERR_* code;
 *    mlff_last_error() gives the message.  Non-convergence is not an error:
 *    it is reported through `info` exactly as scipy does (0 converged,
 *    maxiter otherwise).
 */
#ifndef MLFFPCG_H
#define MLFFPCG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MLFF_OK 0
#define MLFF_ERR_ARG (-1)     /* bad argument (reference: ValueError / AssertionError on shapes) */
#define MLFF_ERR_HIP (-2)     /* HIP runtime failure */
#define MLFF_ERR_NOT_PSD (-3) /* pivot <= 0 in pivoted Cholesky (incomplete_cholesky.py:62 assert) */
#define MLFF_ERR_LINALG (-4)  /* Cholesky of a k x k block failed (scipy LinAlgError) */
#define MLFF_ERR_STATE (-5)   /* call order: e.g. mlff_pcg_start before a matrix is set */
#define MLFF_ERR_COMM (-6)    /* RCCL failure */
#define MLFF_ERR_NOMEM (-7)   /* device allocation failed */

/* preconditioner kinds reported by mlff_precon_info */
#define MLFF_PRECON_NONE 0
#define MLFF_PRECON_PIVCHOL 1  /* incomplete (pivoted) Cholesky + Woodbury (iterative_cholesky.py:115-150) */
#define MLFF_PRECON_NYSTROM 2  /* Nystrom, _init_precon_operator (iterative_solver.py:95-322) */
#define MLFF_PRECON_NYSTROM_SB 3 /* _init_precon_operator_sb (iterative_solver.py:326-381) */
#define MLFF_PRECON_LOWRANK 4  /* Woodbury on a caller-supplied factor (iterative_solver.py:1313-1329) */
#define MLFF_PRECON_EIG 5      /* truncated eigen-decomposition + Woodbury (iterative_solver.py:1177-1329) */

/* operator storage (mlff_set_storage / mlff_storage_info) */
#define MLFF_STORAGE_DENSE 0   /* dense row block, row GEMV: 8 N^2 bytes per mat-vec */
#define MLFF_STORAGE_SYMTILE 1 /* lower block triangle in 512 x 512 tiles: ~4 N^2 bytes */
#define MLFF_STORAGE_AUTO 2    /* cheapest available: MATFREE, SYMTILE or DENSE (default) */
#define MLFF_STORAGE_MATFREE 3 /* matrix-free sGDML operator (the reference's K_op), no N^2 bytes */

/* pcg status (mlff_pcg_result) */
#define MLFF_PCG_RUNNING 0
#define MLFF_PCG_CONVERGED 2
#define MLFF_PCG_MAXITER 3

typedef struct mlff_ctx mlff_ctx;

/* ---- library / devices ---------------------------------------------------- */
int mlff_version(void);                       /* 100 * major + minor */
/* Content hash (16 hex digits) of the csrc/ + include/ sources this binary was built from
 * (build_native.py src_hash, compiled in at link time): ties a shipped .so to its sources. */
const char *mlff_build_hash(void);
int mlff_device_count(int *n_out);
/* RCCL unique id (128 bytes) for a world > 1 context; rank 0 creates it and the
 * caller broadcasts it (torch.distributed / any channel) to the other ranks. */
int mlff_comm_unique_id(unsigned char id_out[128]);
/* Test hook: runs the library's RCCL allreduce / allgather (out of place and in place) /
 * reduce-scatter code on a ONE-rank RCCL communicator over `count` doubles, each between a
 * producing kernel and a consuming copy on the same stream, and returns the largest
 * deviation from the expected values (0 when correct, +inf for a poisoned entry).  The
 * multi-rank data path (sharded_pcg.py / api.hip comm_*) uses exactly these functions; a
 * one-GPU box can run no larger communicator.  No reference counterpart (torch.distributed
 * collectives in the reference's sharded callers are what comm_* replaces). */
int mlff_comm_selftest(int device, int64_t count, double *max_err_out);

/* ---- context --------------------------------------------------------------- */
/* n_global: kernel size N.  comm_id may be NULL when world == 1.  comm_id is a 128-byte
 * RCCL unique id, "LOCAL:<key>" (world contexts of one process joined in-process, the
 * multi-rank path on one GPU), or "SOLO:" (profiling only: this one rank of a world-way
 * split runs alone, every collective keeps only its own contribution, results are
 * meaningless). */
int mlff_ctx_create(int device, int rank, int world, const unsigned char *comm_id,
                    int64_t n_global, mlff_ctx **ctx_out);
int mlff_ctx_destroy(mlff_ctx *ctx);
const char *mlff_last_error(mlff_ctx *ctx); /* ctx may be NULL (thread-local last error) */
int mlff_shard_range(mlff_ctx *ctx, int64_t *row0_out, int64_t *nrows_out);
/* Abort this rank's communicator (ncclCommAbort; for an in-process "LOCAL:" group, the
 * whole group): peers blocked in, or later entering, a collective return MLFF_ERR_COMM,
 * and every later call on this context fails with MLFF_ERR_COMM (destroy still works).
 * The bindings call it when an entry point fails on a sharded context with anything
 * but MLFF_ERR_NOT_PSD / MLFF_ERR_LINALG, which every rank reaches together. */
int mlff_comm_abort(mlff_ctx *ctx);
/* leading dimension (doubles) of the device copy of K; rows are padded to 64 */
int mlff_matrix_ld(mlff_ctx *ctx, int64_t *ld_out);
int mlff_synchronize(mlff_ctx *ctx);
/* HIP stream the context launches on (hipStream_t as void*) */
int mlff_stream(mlff_ctx *ctx, void **stream_out);

/* ---- kernel matrix K (device resident, this rank's row block) --------------- */
/* K_local: nrows x N row-major with leading dimension ld_host (>= N).          */
int mlff_set_matrix_host(mlff_ctx *ctx, const double *K_local, int64_t ld_host);
/* copy rows [r0, r0+nr) (local indices) x all N columns back to the host */
int mlff_get_matrix_rows(mlff_ctx *ctx, int64_t r0, int64_t nr, double *out, int64_t ld_out);
/* synthetic SPD RBF kernel: K_ij = exp(-0.5 * |x_i/ell - x_j/ell|^2) + jitter*delta_ij
 * (sklearn RBF(length_scale=ell) as used by tools/utils.py:173-187).  X: N x d (all points). */
int mlff_gen_rbf(mlff_ctx *ctx, const double *X, int d, double length_scale, double jitter);
/* sGDML Matern-5/2 Hessian kernel assembly, GDMLTrain._assemble_kernel_mat with
 * col_idxs = all (train.py:81-236,1121-1308).  R_desc: M x D, R_d_desc: M x D x 3
 * (Desc.from_R layout, desc.py:292-358), perms: n_perms x n_atoms atom permutations
 * (task['perms']), sig: length scale.  N must equal 3 * n_atoms * M.           */
int mlff_assemble_sgdml(mlff_ctx *ctx, const double *R_desc, const double *R_d_desc,
                        int64_t M, int n_atoms, const int32_t *perms, int n_perms, double sig);
/* sGDML descriptors on the GPU (desc.py:203-358, no cutoff / no PBC):
 * R: M x n_atoms x 3  ->  R_desc: M x D (1/r_ij), R_d_desc: M x D x 3          */
/* Matrix-free sGDML operator (K_op / _K_vec, iterative_solver.py:383-445, i.e.
 * GDMLPredict force prediction with alphas = x, predict.py:72-234) from the same
 * inputs as mlff_assemble_sgdml, without forming K: O(M n_perms D) memory.
 * Mat-vecs, PCG iterations and the column-based builds run on it: pivoted
 * Cholesky, Nystrom and leverage scores fetch columns as K_op e_i (the
 * reference's get_col, iterative_cholesky.py:152-156) and the diagonal from the
 * diagonal blocks (_assemble_kernel_mat_diag, :241-380); only the eigen
 * preconditioner (all of K) needs mlff_assemble_sgdml, which also sets this
 * operator up.  For a permutation group it equals the assembled K; for other
 * permutation sets it is the reference's K_op. */
int mlff_sgdml_operator(mlff_ctx *ctx, const double *R_desc, const double *R_d_desc, int64_t M,
                        int n_atoms, const int32_t *perms, int n_perms, double sig);

/* Energy constraints (use_E_cstr), set BEFORE mlff_assemble_sgdml / mlff_sgdml_operator:
 * the system gets M energy rows / columns after the 3 n_atoms M force rows (the context's
 * N must be 3 n_atoms M + M).  The assembly appends the reference's K_fe / K_ee border
 * (train.py:212-236, _assemble_kernel_mat(use_E_cstr=True)); the matrix-free operator is
 * the reference's _K_vec with energy coefficients (iterative_solver.py:416-443: x = [x_F;
 * x_E], forces from GDMLPredict with alphas_E, predict.py:206-218, and the predicted
 * energies with a flipped sign); the diagonal includes K[E_i, E_i].  One rank only
 * (MLFF_ERR_ARG otherwise).  Replaces: the use_E_cstr argument of the reference's
 * assembly and operator (its Iterative.solve itself cannot run with it). */
int mlff_set_energy_constraints(mlff_ctx *ctx, int use_E_cstr);

/* Spectrum diagnostics of Iterative.solve(flag_eigvals=True) (iterative_solver.py:978-989,
 * 1100-1102; dev_utils.get_eigvals, dev_utils.py:8-25): eig_out (N) = the eigenvalues,
 * descending, of P_op A with the current low-rank preconditioner (preconditioned != 0 and
 * one is set) or of A = sigma_K K + lam I itself (the reference's eigvals_K).  P_op A is
 * similar to the symmetric R^T W R (A = R R^T), so its eigenvalues are real; the
 * reference's scipy.linalg.eigvals returns them as complex in LAPACK order.  Dense O(N^3)
 * on the device (Cholesky, GEMM, Jacobi); one rank. */
int mlff_spectrum(mlff_ctx *ctx, int preconditioned, double *eig_out);

/* Test hook (no reference counterpart): C = alpha op(A) op(B) + beta C through the library's
 * fp64 GEMM (matrix-core path for M >= 64, N >= 128, K >= 32; VALU otherwise), host arrays,
 * row-major; splits > 1 runs the split-K slab path and returns C - alpha op(A) op(B)
 * (beta must be 1).  Lets the tests check every operand layout with asymmetric data. */
int mlff_test_gemm(mlff_ctx *ctx, int ta, int tb, int64_t M, int64_t N, int64_t K, double alpha,
                   const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                   double *C, int64_t ldc, int splits);
/* Gram matrix G = W W^T (k x k, row-major) of a host k x ncols panel W (row-major) as the
 * Woodbury build forms L^T L (iterative_cholesky.py:141-142, `kernel = lam I + L^T L`):
 * mode 0 the fp64 matrix-core SYRK, 1 fp64 64-column chunks summed in double-double (the
 * default, MLFF_WB_GRAM=1), 2 every product exact and summed in double-double.  Test hook. */
int mlff_test_gram(mlff_ctx *ctx, const double *W, int64_t k, int64_t ncols, int mode,
                   double *G_out);
/* Iterative._cho_factor_stable (src/sGDML/sgdml/solvers/iterative_solver.py:555-583): the
 * smallest eigenvalue of the lower triangle of the host m x m matrix M (row-major) --
 * eigh(M, eigvals_only=True, eigvals=(0, 0)) at :577, computed on the device by Householder
 * tridiagonalisation and Sturm bisection as LAPACK's dsyevr/dstebz do --, the shift
 * M +- 1e-15 I (+ when lo_eig <= 0, :578-579) and the Cholesky factor (:580-582).  L_out
 * (m x m): the lower factor L = U^T of the reference's upper cho_factor (upper triangle
 * zero); lo_eig_out: the eigenvalue the sign was taken from.  MLFF_ERR_LINALG (-> LinAlgError)
 * when the shifted matrix is not positive definite.  The Nystrom builds (mlff_precon_nystrom
 * variant 0, mlff_lev_scores) call the same routine on their device matrices. */
int mlff_cho_factor_stable(mlff_ctx *ctx, const double *M, int64_t m, double *L_out,
                           double *lo_eig_out);
/* The eigenvalue test of mlff_cho_factor_stable alone: lo_eig_out = the smallest eigenvalue of
 * the lower triangle of M; d_out (m) / e_out (m - 1), optional: the tridiagonal matrix the
 * device reduction produced (its eigenvalues are M's). */
int mlff_sym_min_eig(mlff_ctx *ctx, const double *M, int64_t m, double *lo_eig_out,
                     double *d_out, double *e_out);
int mlff_sgdml_descriptors(const double *R, int64_t M, int n_atoms, double *R_desc_out,
                           double *R_d_desc_out);

/* operator A = sigma_K * K + lam * I.  sGDML: sigma_K = -1 (K is negative
 * semidefinite, the solved system is (-K + lam I) x = y, iterative_solver.py:995);
 * RBF: sigma_K = +1. */
/* Training-set energies of an sGDML model with coefficients `alphas` (N, global,
 * contiguous): E_out[i - i0] for the training points [i0, i0 + ni) this rank's rows
 * touch (E_out holds M entries).  This is GDMLPredict's E before the std scale and the
 * integration constant (predict.py:172-220, 1100-1108), the quantity
 * GDMLTrain._recov_int_const regresses on (train.py:972-1119).  Needs the
 * matrix-free operator data (mlff_sgdml_operator or mlff_assemble_sgdml). */
int mlff_sgdml_energies(mlff_ctx *ctx, const double *alphas, double *E_out, int64_t *i0_out,
                        int64_t *ni_out);

int mlff_set_operator(mlff_ctx *ctx, double sigma_K, double lam);
/* y_local = A v_global (v_global has N entries).  Collective over the ranks
 * when the symmetric tiled storage is in use (a reduce-scatter of the partial
 * products), so every rank calls it. */
int mlff_matvec(mlff_ctx *ctx, const double *v_global, double *y_local);
/* Storage of K used by the operator (K_op, iterative_solver.py:383-445; same
 * operator, different bytes).  AUTO (default): the matrix-free sGDML operator
 * when it exists and moves fewer bytes than the tiles; else symmetric tiles when K
 * was generated/assembled by this library (symmetric by construction) or, on one
 * rank, a host matrix passes an exact symmetry check; dense otherwise or when
 * the tile copy does not fit.  SYMTILE on a non-symmetric host matrix fails
 * with MLFF_ERR_ARG.  The tiles are a second copy next to the dense rows (the
 * preconditioner builds read the dense rows). */
int mlff_set_storage(mlff_ctx *ctx, int mode);
/* resolves the storage (building the tiles if needed) and reports the mode in
 * use and the algorithmic HBM bytes of one operator application on this rank */
int mlff_storage_info(mlff_ctx *ctx, int *mode_out, double *bytes_per_matvec_out);
/* form of the matrix-free sGDML operator (MLFF_STORAGE_MATFREE; the reference's K_op,
 * iterative_solver.py:383-445 / predict.py:172-220, evaluated three ways):
 * MLFF_MF_FORM_PAIR (pair sums, then F, then J^T), MLFF_MF_FORM_REC (record-factored: x-independent
 * per-pair records, many-atom / few-point systems such as the nanotube), MLFF_MF_FORM_PTILE
 * (pair-tile: query points in registers, training points streamed through LDS, fp64-vector
 * bound; few-atom / many-point systems such as ethanol).  -1 when no sGDML operator is set.
 * Environment MLFF_MF_FORM=pair|rec|pt (read by mlff_sgdml_operator) overrides the default. */
#define MLFF_MF_FORM_PAIR 0
#define MLFF_MF_FORM_REC 1
#define MLFF_MF_FORM_PTILE 2
int mlff_operator_form(mlff_ctx *ctx, int *form_out);
/* diag(sigma_K * K) (local) */
int mlff_get_diag(mlff_ctx *ctx, double *diag_local);

/* ---- preconditioners ------------------------------------------------------- */
int mlff_precon_none(mlff_ctx *ctx);
/* pivoted Cholesky of S = sigma_K*K to rank k (tie rule: first maximum in the
 * current permuted order, incomplete_cholesky.py:53) then Woodbury with lam:
 * T = chol(lam I + L^T L)^-1 L^T, apply z = (r - T^T T r) / lam.
 * index_columns_out (N, int64, optional): the permutation (first k = pivots).
 * build_woodbury = 0 only computes the pivots (truncated_cholesky selector); the
 * panel then holds L^T (k x N, rows in the original index order, as the
 * reference's L), readable with mlff_precon_get_panel, and PCG runs unpreconditioned. */
int mlff_precon_pivchol(mlff_ctx *ctx, int64_t k, int build_woodbury, int64_t *index_columns_out,
                        double *seconds_out);
/* per-column device seconds of the last pivoted-Cholesky build (time_cholesky of
 * incomplete_cholesky.py:48-80: event stamps every 4 columns, split evenly) and the
 * seconds of its Woodbury build */
int mlff_pivchol_times(mlff_ctx *ctx, double *col_seconds_out, int64_t k,
                       double *woodbury_seconds_out);
/* Nystrom from sorted column indices idx (k).  variant 0 = _init_precon_operator
 * (eig-sign diagonal shift, apply (B^T B r - r)/lam), variant 1 = _sb (1e-16
 * shift, apply -(r - P^T P r)/lam). */
int mlff_precon_nystrom(mlff_ctx *ctx, const int64_t *idx, int64_t k, int variant, double *seconds_out);
/* Woodbury on a caller-supplied factor L (N x k, given as Lt_local: k x nrows):
 * T = chol(lam I + L^T L)^-1 L^T, apply z = (r - T^T T r)/lam. */
int mlff_precon_lowrank(mlff_ctx *ctx, const double *Lt_local, int64_t k);
/* Truncated eigen-decomposition of S = sigma_K * K: the k largest |eigenvalues| s and
 * eigenvectors U (= scipy svd(K) of the reference), by block subspace iteration on the
 * operator in any storage (matrix-free included) with Rayleigh-Ritz and a device Jacobi
 * eigensolver (kernels_eig.hip; no LAPACK).  Collective over the ranks except mask 2.
 * mask_mode 0: K as is ('eigvec_precon'); 1: all entries zeroed
 * ('eigvec_precon_block_diagonal', iterative_solver.py:1255-1261); 2: only same-atom
 * 3x3 blocks and the max-|K| entries kept ('eigvec_precon_atomic_interactions',
 * :1238-1254; dim_i = 3 * n_atoms; needs the dense K and one rank).
 * build_woodbury = 1 installs the preconditioner
 * L = U sqrt(s)[:, :k] + Woodbury (svd_preconditioner :1313-1329).
 * evals_out (k) and rowlev_out (N, ||U[i, :k]||, :1172-1173) are optional. */
int mlff_precon_eig(mlff_ctx *ctx, int64_t k, int mask_mode, int64_t dim_i, int build_woodbury,
                    double *evals_out, double *rowlev_out);
int mlff_precon_info(mlff_ctx *ctx, int *kind_out, int64_t *k_out);
/* Convergence of the last truncated eigensolve (mlff_precon_eig): converged_out = 1 when every
 * one of the k leading Ritz pairs met ||S u - theta u|| <= 1e-11 |theta_0|; otherwise the
 * pairs after the iteration cap were accepted because they met 1e-6 (a slowly decaying
 * spectrum around k), rel_resid_out = the worst residual / |theta_0|.  The reference's full SVD
 * (iterative_solver.py:1297-1329) has no such state; the drop-in turns it into a warning. */
int mlff_eig_info(mlff_ctx *ctx, int *converged_out, double *rel_resid_out);
/* z_local = M r_local (collective over ranks for the low-rank part) */
int mlff_precon_apply(mlff_ctx *ctx, const double *r_local, double *z_local);
/* How this rank's low-rank apply (iterative_cholesky.py:145-148 z = (r - T^T T r) / lam)
 * runs: one_pass_out = 1 when each panel row is read once per apply by one workgroup (one
 * rank, rows that fit a workgroup's registers: k_lr_rows + k_lr_fin), 2 when a row is
 * shared by a cluster of workgroups (longer rows: k_lr_cluster + k_lr_fin), 0 for the
 * two-pass T r / T^T t apply; bytes_out = its algorithmic HBM bytes per apply (one pass:
 * 8 k N + 16 G N + 24 N, G = row groups or clusters; two passes: 16 k N + 24 N).  A cluster
 * whose hand-offs time out (its workgroups not all resident, ~1 s) is abandoned: that apply
 * (or PCG iteration) is redone with two passes and the context keeps the two-pass form (this
 * call then reports 0).  No reference counterpart. */
int mlff_precon_apply_traffic(mlff_ctx *ctx, int *one_pass_out, double *bytes_out);
/* the k x nrows Woodbury panel T (or B / P for Nystrom) of this rank */
int mlff_precon_get_panel(mlff_ctx *ctx, double *T_local, int64_t ld_out);

/* ridge leverage scores of the approximating columns idx (k): numeric part of
 * _lev_scores (iterative_solver.py:489-552); scores_out: N (global, every rank). */
int mlff_lev_scores(mlff_ctx *ctx, const int64_t *idx, int64_t k, double lam, double *scores_out);

/* ---- preconditioned CG (scipy 1.7.3 legacy semantics) ---------------------- */
/* Starts a solve of A x = b with x0 (local parts; x0 may be NULL = zeros).
 * tol: relative tolerance, atol = tol * ||b|| (scipy `atol=None` legacy mode);
 * maxiter: iteration cap (reference: 5N).  Returns *early_exit = 1 when scipy's
 * legacy pre-check ||A x0 - b|| <= tol ends the solve before any iteration. */
int mlff_pcg_start(mlff_ctx *ctx, const double *b_local, const double *x0_local, double tol,
                   int64_t maxiter, int *early_exit_out);
/* run up to n_iter more iterations (stops early on convergence / maxiter).
 * chunk: iterations launched between host status polls (0 = default 32).   */
int mlff_pcg_run(mlff_ctx *ctx, int64_t n_iter, int64_t chunk, int *status_out);
/* iterations done, status, last stop-test residual ||r||, scipy info code */
int mlff_pcg_result(mlff_ctx *ctx, int64_t *iters_out, int *status_out, double *resid_out,
                    int *info_out);
/* x_local of the current iterate */
int mlff_pcg_get_x(mlff_ctx *ctx, double *x_local);
/* residual trace: trace_out[0] = ||r_0||, trace_out[j] = stop-test ||r_j||, j = 1..iters */
int mlff_pcg_get_trace(mlff_ctx *ctx, double *trace_out, int64_t n);

/* ---- timing (device time of the hot kernels, hipEvents on the ctx stream) --- */
/* on = 0: off; 1: every PCG iteration bracketed; n > 1: every n-th iteration only (each
 * event costs GPU time between the kernels it brackets; the per-kernel averages are over
 * the bracketed iterations, whose count is the operator count of mlff_timing_read) */
int mlff_timing_enable(mlff_ctx *ctx, int on);
/* accumulated milliseconds and launch counts of the K mat-vec (GEMV) and of the
 * whole PCG iteration since the last reset */
int mlff_timing_read(mlff_ctx *ctx, double *gemv_ms, int64_t *gemv_count, double *iter_ms,
                     int64_t *iter_count);
/* summed HIP-event time of the low-rank preconditioner apply (T r, T^T t, z) inside
 * mlff_pcg_run while timing is on (one rank) */
int mlff_timing_read_precon(mlff_ctx *ctx, double *ms, int64_t *count);
/* summed HIP-event time of the collectives of the sharded iteration (allgather of z,
 * reduce-scatter / allreduce of p.q, allreduce of ||r||^2 | T r) and their count */
int mlff_timing_read_comm(mlff_ctx *ctx, double *ms, int64_t *count);
int mlff_timing_reset(mlff_ctx *ctx);
/* free / total bytes of the context's device (hipMemGetInfo) */
int mlff_device_memory(mlff_ctx *ctx, int64_t *free_out, int64_t *total_out);

#ifdef __cplusplus
}
#endif
#endif /* MLFFPCG_H */
