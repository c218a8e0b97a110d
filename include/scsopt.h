/*
 * scsopt.h -- C ABI of libscsopt, the MI355X (gfx950) implementation of the
 * SCORE inner iteration of SelfConcordantSmoothOptimization.jl.
 *
 * The reference has no FFI: its plugin boundary is Julia multiple dispatch on
 * `step!(method, model, reg_name, hμ, As, x, x_prev, ys, Cmat, iter)`
 * (src/algorithms/iterate.jl:52-54) plus the objective closures evaluated by
 * `optim_loop!` (iterate.jl:168, :189-190).  Each entry point below replaces
 * one of those Julia-side pieces; the Julia `ccall` binding a maintainer adds
 * is in INTEGRATION.md, the Python ctypes binding is
 * selfconcordantsmoothoptimization.jl_amd/scsopt/_lib.py.
 *
 * Conventions
 *   - All functions return SCS_OK (0) or an error code; the message is
 *     available from scs_last_error(ctx) (errors the reference raises with
 *     Base.error carry the reference's message text).
 *   - Host pointers are borrowed for the duration of the call.  Vectors of
 *     length m (x, x_prev, x_new, dx) are host fp64 arrays.
 *   - A is column-major (Julia Matrix{Float64} layout) with leading dimension
 *     lda >= N.  In a multi-rank context each rank holds rows
 *     [row0, row0 + N) of the global N_global x m matrix (row-sharded).
 *   - A context is not thread-safe; all device work is ordered on its stream.
 */
#ifndef SCSOPT_H
#define SCSOPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCS_OK 0
#define SCS_ERR_ARG 1      /* invalid argument / unsupported combination     */
#define SCS_ERR_HIP 2      /* HIP runtime / device failure                   */
#define SCS_ERR_SOLVE 3    /* factorization failed (singular system)         */
#define SCS_ERR_STATE 4    /* call order (e.g. step before data)             */
#define SCS_ERR_REF 5      /* an error the reference itself raises           */
#define SCS_ERR_COMM 6     /* all-reduce callback failed                     */
#define SCS_ERR_CALLBACK 7 /* a user loss callback returned non-zero         */

/* f(A, y, x) kinds -- closed forms of the reference's user callbacks.       */
enum scs_loss_kind {
  SCS_LOSS_LOGISTIC_MARGIN = 1, /* c*sum(log(1+exp(-y.*(A*x))))  test/test_algs.jl:9  */
  SCS_LOSS_LOGISTIC_CE = 2,     /* f(y, sigmoid(A*x)), cross-entropy  SURVEY §8a C3 */
  SCS_LOSS_LEAST_SQUARES = 3,   /* 0.5*sum((A*x-y).^2)*c           README.md:212-214 */
  SCS_LOSS_QUADRATIC = 4,       /* 1/2*(x'*(A*x)) + y'*x             test/test_algs.jl:90 */
  SCS_LOSS_ROSENBROCK = 5,      /* chained Rosenbrock, no data        README.md:49 */
  SCS_LOSS_CALLBACK = 6         /* the caller's f / grad_fx / hess_fx (scs_set_loss_callback) */
};

/* (out_fn, f(y, ŷ)) pairs used by ProxGGNSCORE (prox-GGN-SCORE.jl:44-56).    */
enum scs_ggn_kind {
  SCS_GGN_NONE = 0,
  SCS_GGN_SIGMOID_CE = 1,       /* Mfunc = sigmoid(A*x), CE on ŷ   test/test_algs.jl:10-11 */
  SCS_GGN_LINEAR_LS = 2         /* out_fn = A*x, 0.5*c*sum((ŷ-y).^2) README.md:233-239 */
};

/* reg_name strings of get_reg / invoke_prox (regularizers.jl:4-31,
 * prox-operators.jl:68-79).                                                 */
enum scs_reg_kind { SCS_REG_L1 = 1, SCS_REG_L2 = 2, SCS_REG_INDBOX = 3, SCS_REG_GL = 4 };

/* Smoother types (src/regularizers/: the *-smooth.jl files).                 */
enum scs_smoother_kind {
  SCS_SMOOTH_PHUBER_L1L2 = 1,   /* PHuberSmootherL1L2(μ)          phuber-smooth.jl:27   */
  SCS_SMOOTH_PHUBER_INDBOX = 2, /* PHuberSmootherIndBox(lb,ub,μ)  phuber-smooth.jl:59   */
  SCS_SMOOTH_PHUBER_GL = 3,     /* PHuberSmootherGL(μ, problem)   phuber-smooth.jl:137  */
  SCS_SMOOTH_EXP_INDBOX = 4,    /* ExponentialSmootherIndBox      exponential-smooth.jl:28 */
  SCS_SMOOTH_LOGEXP_INDBOX = 5, /* LogExpSmootherIndBox(lb,ub,μ)  log-exp-smooth.jl:28 */
  SCS_SMOOTH_OSBA_L1L2 = 6,     /* OsBaSmootherL1L2(μ)            ostrovskii-bach-smooth.jl:27 */
  SCS_SMOOTH_OSBA_GL = 7        /* OsBaSmootherGL(μ, problem)     ostrovskii-bach-smooth.jl:59 */
};

/* ProximalMethod subtypes (src/algorithms/prox-*-SCORE.jl).                 */
enum scs_method_kind { SCS_PROX_NSCORE = 1, SCS_PROX_GGNSCORE = 2, SCS_PROX_LQNSCORE = 3 };

typedef struct scs_ctx scs_ctx;

/* All-reduce hook for row-sharded contexts: sum `count` fp64 values in place
 * across ranks.  `dev_buf` is the device buffer registered with
 * scs_set_reduce_buffer (offset 0); `stream` is the context stream.  Return 0
 * on success.  Called between the local partial Gram/gradient and the m x m
 * solve (the only exchange point of the path).              */
typedef int (*scs_allreduce_fn)(void* dev_buf, int64_t count, void* stream, void* user);

/* Synthetic on-device data (counter-based RNG; every row is reproducible from
 * its global index, so any row shard is generated in place).               */
typedef struct scs_synth {
  int64_t N_global;  /* total rows                                        */
  int64_t row0;      /* first global row held by this context             */
  int64_t N;         /* rows held by this context                         */
  int64_t m;         /* columns                                           */
  uint64_t seed;
  int kind;          /* 1: A ~ N(0,1)/sqrt(m); y ~ Bernoulli(sigmoid(A x_true)) in {0,1}
                        2: A ~ N(0,1)/sqrt(m); y ~ ±1 with P(+1) = sigmoid(A x_true)
                        3: A ~ N(0,1);         y = A x_true + 0.1 eps
                        4: sparse A (scs_gen_sparse); x_true ~ U(-1.5,1.5), y = A x_true + 0.1 eps */
  double density;    /* fraction of nonzero entries of x_true             */
} scs_synth;

/* Per-kernel device-time accumulators (hipEvent elapsed, ms), read by bench. */
typedef struct scs_timing {
  double gram_ms;    int64_t gram_calls;   /* MFMA Aᵀ diag(w) A                */
  double gemv_ms;    int64_t gemv_calls;   /* A*x and Aᵀ*v streaming passes    */
  double solve_ms;   int64_t solve_calls;  /* m x m factor + solve             */
  double step_ms;    int64_t step_calls;   /* whole scs_step                   */
  double reduce_ms;  int64_t reduce_calls; /* all-reduce callback              */
} scs_timing;

/* ---- lifecycle ---------------------------------------------------------- */
const char* scs_version(void);
/* Create a context on HIP device `device`; `stream` = existing hipStream_t or
 * NULL to create one.                                                       */
int scs_create(int device, void* stream, scs_ctx** out);
int scs_destroy(scs_ctx* ctx);
/* One process, several GPUs (the reference's iterate! is one process, iterate.jl:56-76): a context
 * over devs[0..ndev) that splits the problem's rows across them (contiguous balanced blocks, the
 * first N % ndev devices one more row -- the blocks of one process per GPU), with an RCCL
 * communicator over the devices (ncclCommInitAll; one GPU each).  scs_set_data / scs_gen_data
 * take the WHOLE problem (N_global = N, row0 = 0); the problem / method / step / loop entry
 * points (scs_set_loss ... scs_iterate, scs_eval_*, scs_step*, scs_set_batches, timing) run on
 * every device at once, one host thread each, and return device 0's results (every device
 * holds the same replicated x and m-vectors).  scs_get_data gathers rows across devices;
 * kernel-level entry points and sparse data take a single-device context (SCS_ERR_ARG).
 * ndev = 1 is a plain one-device run.  A device that fails inside a collective aborts the
 * communicators (then every call returns SCS_ERR_COMM: destroy the context).                 */
int scs_create_multi(const int* devs, int ndev, scs_ctx** out);
/* The same with flags.  SCS_MULTI_HOST_EXCHANGE: the group's exchange through host memory instead of
 * RCCL (every device's payload to a host slot, a barrier, the slots summed in device order on every
 * device, written back) -- no RCCL, and devs may repeat a GPU (several sub-contexts on one device:
 * the group's fan-out, row split and exchange on a one-GPU machine).  Two host copies per exchange.  */
#define SCS_MULTI_HOST_EXCHANGE 1
int scs_create_multi_ex(const int* devs, int ndev, int flags, scs_ctx** out);
/* Devices of a context (1 for scs_create).                                                   */
int scs_group_size(scs_ctx* ctx, int* ndev);
const char* scs_last_error(const scs_ctx* ctx);
int scs_get_stream(scs_ctx* ctx, void** stream);

/* ---- row sharding ------------------------------------------------------- */
/* Two ways to run the exchange step (one in-place fp64 sum per step):
 *  (a) libscsopt's own RCCL communicator (the default of the Python and Julia hosts on GPUs):
 *      rank 0 calls scs_rccl_unique_id, the caller hands the 128 opaque bytes to every rank
 *      (MPI, torch.distributed, a file ...), and every rank calls scs_set_comm_rccl -- a
 *      collective call.  The context then calls ncclAllReduce itself, on its stream, in place
 *      in its reduce buffer (allocated by the library unless one is registered);
 *  (b) an all-reduce callback (scs_set_comm), e.g. torch.distributed with gloo for CPU tests. */
int scs_set_comm(scs_ctx* ctx, int rank, int nranks, scs_allreduce_fn fn, void* user);
int scs_rccl_unique_id(void* id /* 128 bytes */);
int scs_set_comm_rccl(scs_ctx* ctx, int rank, int nranks, const void* id /* 128 bytes */);
/* Run the exchange path (packed Gram tiles -> all-reduce -> unpack) even at one rank, so the
 * communicator is exercised on a one-GPU host (results are unchanged).                        */
int scs_set_comm_force(scs_ctx* ctx, int on);
/* Device buffer (>= scs_reduce_buffer_size() doubles) owned by the caller,
 * used as the in-place all-reduce payload.  The size depends on the data and
 * on the registered batch list (the sample-space all-gather of batches with
 * N_global + 1 <= m): query it again after scs_set_batches.                 */
int scs_reduce_buffer_size(scs_ctx* ctx, int64_t* ndoubles);
/* What the exchange actually runs on, read back from the library (for run records / scaling
 * checks): *kind = SCS_COMM_NONE / _RCCL (scs_set_comm_rccl) / _CALLBACK (scs_set_comm) /
 * _GROUP_RCCL (scs_create_multi) / _GROUP_HOST (SCS_MULTI_HOST_EXCHANGE); *nranks / *rank from the
 * communicator itself (ncclCommCount / ncclCommUserRank for RCCL; the group's device count and 0
 * for a group; the caller's values for a callback); *rccl_version = ncclGetVersion; lib (cap
 * bytes, may be NULL) = the path of the RCCL shared object this process resolved ncclAllReduce
 * from (dladdr).  Any output pointer may be NULL.                                              */
#define SCS_COMM_NONE 0
#define SCS_COMM_RCCL 1
#define SCS_COMM_CALLBACK 2
#define SCS_COMM_GROUP_RCCL 3
#define SCS_COMM_GROUP_HOST 4
int scs_comm_info(scs_ctx* ctx, int* kind, int* nranks, int* rank, int* rccl_version, char* lib, int64_t cap);
int scs_set_reduce_buffer(scs_ctx* ctx, void* dev_ptr, int64_t ndoubles);

/* ---- user callbacks (Problem(x0, f, λ; grad_fx, hess_fx), problems.jl:44-59; call sites
 * prox-N-SCORE.jl:49-56, prox-L-BFGS-SCORE.jl:85-91, iterate.jl:168) -------------------
 * SCS_LOSS_CALLBACK evaluates the loss on the caller's side (a data problem's closure captures
 * its own A, y: the device holds no data, as for a ProblemGeneric -- scs_set_data(N = 0,
 * A = NULL, m)); the smoother, the m x m solve, damping, prox and the loop stay on the device.
 * `what`: SCS_CB_F    out[0] = f(x)
 *         SCS_CB_GRAD out[0..m) = grad_fx(x)
 *         SCS_CB_HESS out = hess_fx(x), m x m column-major (ProxNSCORE)
 *         SCS_CB_FTEST out[0] = f(Atest, ytest, x), the held-out loss (iterate.jl:173), asked
 *                     only after scs_set_test_callback(ctx, 1)
 *         SCS_CB_GGN  out = [J (n x m, column-major) | r (n) | q (n)] with n = ggn_rows:
 *                     J = jac_yx, r = grad_fy, Q = diag(q) = hess_fy (prox-GGN-SCORE.jl:44-49);
 *                     a general symmetric Q is passed eigen-rotated (J̃ = VᵀJ, r̃ = Vᵀr,
 *                     q = its eigenvalues), which leaves JᵀQJ, Jᵀr and the sample-space
 *                     system of ggn_score_step unchanged (ProxGGNSCORE; multi-output targets
 *                     ny > 1 are n = N·ny rows)
 *         SCS_CB_GRAD_X out[0..m) = grad_fx(x) called with x ALONE: ProxGGNSCORE builds
 *                     grad_f = x -> model.grad_fx(x) (prox-GGN-SCORE.jl:58-59) and its ss_type 3
 *                     line search calls it (:83-84, utils.jl:31).  A data problem's
 *                     grad_fx(A, y, x) has no one-argument method: return SCS_CB_NO_METHOD and
 *                     the calling function fails with SCS_ERR_REF "MethodError: no method
 *                     matching grad_fx(::Vector{Float64})", the reference's error
 * x (m) and out are host arrays owned by the library, valid for the call; return 0 on
 * success, SCS_CB_NO_METHOD as above, anything else fails the calling ABI function with
 * SCS_ERR_CALLBACK.  There is no automatic differentiation on this path: ProxNSCORE needs
 * SCS_CB_HESS, ProxGGNSCORE ggn_rows > 0.                                                  */
#define SCS_CB_F 0
#define SCS_CB_GRAD 1
#define SCS_CB_HESS 2
#define SCS_CB_GGN 3
#define SCS_CB_FTEST 4
#define SCS_CB_GRAD_X 5
#define SCS_CB_NO_METHOD 2
typedef int (*scs_loss_fn)(void* user, int what, const double* x, int64_t m, double* out);
int scs_set_loss_callback(scs_ctx* ctx, scs_loss_fn fn, void* user, int64_t ggn_rows);

/* ---- data  (Problem(A, y, ...) -- problems.jl:61-81) --------------------- */
/* Upload host A (column-major, N x m, leading dim lda) and y (N).  N is the
 * local row count; N_global/row0 describe the shard.  A may be NULL with
 * m > 0 for a ProblemGeneric (problems.jl:44-59): SCS_LOSS_ROSENBROCK or SCS_LOSS_CALLBACK. */
int scs_set_data(scs_ctx* ctx, int64_t N, int64_t m, const double* A, int64_t lda,
                 const double* y, int64_t N_global, int64_t row0);
int scs_gen_data(scs_ctx* ctx, const scs_synth* spec);
/* ---- held-out data  (Problem(A, y, x0, f, λ; Atest, ytest), problems.jl:27-28,67-68) -------
 * optim_loop! evaluates ftest(x) = f(Atest, ytest, x) with the problem's own f (same loss kind,
 * same scale literal) at every stats push when BOTH Atest and ytest are given (iterate.jl:169-175,
 * utils.jl:55-57); the values become Solution.fvaltest (scs_history.fvaltest).  Call after the
 * data (a new scs_set_data / scs_gen_data / scs_set_sparse drops the test set).  Row-sharded
 * contexts pass their shard of the held-out rows (N local rows of N_global, every rank calls,
 * a rank may hold none); a multi-device context takes the whole set (N_global = N, row0 = 0)
 * and splits it like the data.  A = y = NULL clears the test set; exactly one of A, y NULL is the
 * reference's xor case (only one of Atest / ytest given, iterate.jl:170-171): recorded, and
 * scs_iterate_ex then raises the reference's UndefVarError at its first stats push.             */
int scs_set_test_data(scs_ctx* ctx, int64_t N, const double* A, int64_t lda, const double* y,
                      int64_t N_global, int64_t row0);
/* CSR held-out rows (0-based, m columns; values stored fp64, or fp32 with val_f32 = 1).       */
int scs_set_test_sparse(scs_ctx* ctx, int64_t N, int64_t nnz, const int64_t* rowptr, const int32_t* colidx,
                        const double* val, int val_f32, const double* y, int64_t N_global, int64_t row0);
/* Rows [row0, row0 + N) of the scs_gen_data generator (dense kinds 1-3, spec->m = the data's m):
 * with row0 >= the data's N_global they are held-out samples of the same distribution.  A
 * multi-device context splits spec->N rows across its devices.                                */
int scs_gen_test_data(scs_ctx* ctx, const scs_synth* spec);
/* A callback loss (SCS_LOSS_CALLBACK) keeps its held-out data on the caller's side: on = 1 makes
 * the loop ask SCS_CB_FTEST at every push.                                                     */
int scs_set_test_callback(scs_ctx* ctx, int on);
/* ftest(x) now; *on = 1 when the context holds test data.                                      */
int scs_eval_ftest(scs_ctx* ctx, const double* x, double* fval);
int scs_has_test(scs_ctx* ctx, int* on);

/* Copy device A rows [r0, r0+nr) (column-major, lda_out) and y back.       */
int scs_get_data(scs_ctx* ctx, int64_t r0, int64_t nr, double* A, int64_t lda_out, double* y);
int scs_get_dims(scs_ctx* ctx, int64_t* N, int64_t* m, int64_t* N_global, int64_t* row0);

/* ---- sparse A  (Problem(A::SparseMatrixCSC, y, ...); README.md:105 builds it
 * with sprandn(N, m, 0.01) -- BASELINE configs[4]).  Held twice on the device:
 * CSR for A*x and a CSC copy for Aᵀ*v, so both products are gathers with a
 * fixed summation order (no atomics).  Indices are 0-based; the CSC copy
 * describes the same local rows (rowidx in [0, N)).  val_f32 = 1 stores the
 * values as fp32 (the fp32-value arm of the study; accumulation stays fp64).
 * All methods run on sparse A: the products stay sparse; ProxNSCORE /
 * ProxGGNSCORE form their Gram on a dense device mirror of A, built once and
 * refused (SCS_ERR_ARG) when it does not fit in device memory.               */
int scs_set_sparse(scs_ctx* ctx, int64_t N, int64_t m, int64_t nnz,
                   const int64_t* rowptr, const int32_t* colidx, const double* val,
                   const int64_t* colptr, const int32_t* rowidx, const double* valT,
                   int val_f32, const double* y, int64_t N_global, int64_t row0);
/* Synthetic sparse A (single context): k = round(density*m) nonzeros per row
 * in a layered-bijection pattern (N a power of two, m | N; every column then
 * holds k*N/m), values N(0,1)/sqrt(k); x_true ~ U(-1.5, 1.5) and
 * y = A x_true + 0.1 eps (spec->kind must be 4; spec->density is ρ).        */
int scs_gen_sparse(scs_ctx* ctx, const scs_synth* spec, int val_f32);
int scs_get_nnz(scs_ctx* ctx, int64_t* nnz);
/* CSR copy back to the host (values widened to fp64).                       */
int scs_get_sparse(scs_ctx* ctx, int64_t* rowptr, int32_t* colidx, double* val);

/* ---- problem / regularizer / smoother ----------------------------------- */
int scs_set_loss(scs_ctx* ctx, int loss_kind, int ggn_kind, double scale);
/* λ: nlam = 1 (scalar) or 2 ([λ1, λ2] for "gl").  Box (indbox): lb/ub are
 * nbound = 1 scalars or nbound = m vectors (C_set).  Groups (gl): ind is the
 * 3 x ngroups Int matrix of get_P (column-major, 1-based start, end, weight;
 * prox-reg-utils.jl:27-62); the ranges must partition 1..m (any order) --
 * what get_Cmat (prox-reg-utils.jl:121-142) and the GL smoothers accept.    */
int scs_set_reg(scs_ctx* ctx, int reg_kind, const double* lam, int nlam,
                const double* lb, const double* ub, int64_t nbound,
                const int64_t* ind, int64_t ngroups);
/* Opt-in: reuse AᵀQA across steps when it does not depend on x -- least
 * squares under ProxNSCORE (hess_fx = c·AᵀA) or under ProxGGNSCORE with the
 * linear out_fn (J = A, Q = c·I).  The reference recomputes it every step
 * (prox-GGN-SCORE.jl:129, prox-N-SCORE.jl:55) and that stays the default;
 * with the cache on, later steps copy the (all-reduced) Gram of the first and
 * only the gradient is all-reduced.  Bit-identical results.  Costs one more
 * m_pad² fp64 buffer.                                                        */
int scs_set_gram_cache(scs_ctx* ctx, int on);
/* The compute arm of the fp32-vs-fp64 tolerance study (BASELINE configs[4]): on = 1 runs the
 * sparse products of fp32-stored values (scs_set_sparse val_f32 = 1) and the L-BFGS two-loop
 * recursion in fp32 ARITHMETIC (fp32 products, fp32 accumulation and dots, results widened to fp64);
 * everything else (f / η / step / prox / the m x m solves) stays fp64.  0 (default): fp64.      */
int scs_set_compute_f32(scs_ctx* ctx, int on);
/* The m x m (and the GGN sample-space (N+1)²) systems' solver.  SCS_SOLVER_DEFAULT: blocked
 * Cholesky on MFMA with the LU fallback (sample space: LU) -- equal to the reference's solves to
 * O(cond·eps).  SCS_SOLVER_REFERENCE: the reference's own factorizations -- Householder QR
 * (LAPACK dgeqrf / dlarfg / dlarft conventions, 128-column compact-WY panels) for ProxGGNSCORE's
 * `qr(JQJ) \ Je` and `qr(I + A) \ residual` (prox-GGN-SCORE.jl:126,131) and the LU for
 * ProxNSCORE's `(H + λ·Diagonal(Hr)) \ ∇q` (prox-N-SCORE.jl:70) -- for parity work on
 * ill-conditioned systems; slower (the QR panel is a column-by-column chain).                  */
#define SCS_SOLVER_DEFAULT 0
#define SCS_SOLVER_REFERENCE 1
int scs_set_solver(scs_ctx* ctx, int kind);
/* G of get_P(n, G, ind) (1-based, a permutation of 1..m): get_reg's group
 * term reads P.matrix*x = x[G] (prox-reg-utils.jl:31, regularizers.jl:24-27);
 * the prox (ProxL2) and the GL smoothers (Cmat) index x directly, as in the
 * reference.  Call after scs_set_reg(gl); the default is G = 1:m.           */
int scs_set_group_map(scs_ctx* ctx, const int64_t* G, int64_t ntotal);
/* Mh/nu as in the smoother struct (e.g. 2.0/2.6 for pseudo-Huber).  lb/ub
 * (indbox smoothers) follow bounds_sanity_check (prox-reg-utils.jl:144-158). */
int scs_set_smoother(scs_ctx* ctx, int kind, double mu, double Mh, double nu,
                     const double* lb, const double* ub, int64_t nbound);
/* model.L (nothing <=> has_L = 0); iterate!(…; α) sets L = 1/α.            */
int scs_set_L(scs_ctx* ctx, int has_L, double L);

/* ---- method  (init! / step!) -------------------------------------------- */
/* init!(method, x): select the method and reset its state (L-BFGS memory,
 * prox-L-BFGS-SCORE.jl:31-36).  mem = ProxLQNSCORE.m.                       */
int scs_method_init(scs_ctx* ctx, int method, int ss_type, int use_prox, int mem);
/* f(A, y, x) (iterate.jl:168).                                             */
int scs_eval_f(scs_ctx* ctx, const double* x, double* fval);
/* ∇f(A, y, x) (grad_fx; the ForwardDiff gradient of f when the user gives none,
 * prox-L-BFGS-SCORE.jl:84-97).                                              */
int scs_eval_grad(scs_ctx* ctx, const double* x, double* g);
/* get_reg(model, x, reg_name) (regularizers.jl:4-31).                      */
int scs_eval_reg(scs_ctx* ctx, const double* x, double* gval);
/* Minibatches: the collected DataLoader batch list of optim_loop!
 * (iterate.jl:124-146; utils.jl:18-25 get_data_loader / get_loader_subset).
 * Batch b is the local rows rows[offsets[b] .. offsets[b+1]) (0-based, any
 * order -- a shuffled loader's permutation is the caller's), gathered on the
 * device as the As, ys its step! sees (iterate.jl:205-207).  scs_iterate runs
 * the inner `for (i, sample) in enumerate(data)` loop over the registered
 * list; scs_select_batch(b) makes batch b the As, ys of the following scs_step
 * calls (b = -1: the full data).  f / get_reg / the histories always use the
 * full data (iterate.jl:168).  nbatch = 0 clears the list.  One rank; a
 * sparse A's batches are gathered dense (the reference's Matrix(As')).                                                                          */
int scs_set_batches(scs_ctx* ctx, const int64_t* rows, const int64_t* offsets, int64_t nbatch);
int scs_select_batch(scs_ctx* ctx, int64_t b);
/* step!(method, model, reg_name, hμ, As, x, x_prev, ys, Cmat, iter;
 *       return_dx) (prox-N-SCORE.jl:34, prox-GGN-SCORE.jl:34,
 * prox-L-BFGS-SCORE.jl:69).  dx may be NULL.                               */
int scs_step(scs_ctx* ctx, const double* x, const double* x_prev, int64_t iter,
             double* x_new, double* dx, double* pri_res_norm);
/* step!(...; ∇fx) (iterate.jl:52-54): the caller's gradient replaces grad_f at every point the
 * step evaluates it (`grad_f = x -> ∇fx`, prox-N-SCORE.jl:66-68 and prox-L-BFGS-SCORE.jl:98-100:
 * ∇q, the BB step's ∇q_prev, the line search and the L-BFGS pair's γh); ProxGGNSCORE takes no ∇fx
 * (prox-GGN-SCORE.jl:34-135 never reads it).  grad_fx (m, host) NULL = scs_step.              */
int scs_step_grad(scs_ctx* ctx, const double* x, const double* x_prev, int64_t iter, const double* grad_fx,
                  double* x_new, double* dx, double* pri_res_norm);

/* ---- loop level  (iterate!(method, model, reg_name, hμ; max_epoch, x_tol,
 * f_tol) -> Solution, iterate.jl:56-76 / optim_loop! :100-267) ------------ */
/* History arrays of a Solution (iterate.jl:3-32), caller-owned, capacity
 * 2 * max_epoch + 1 each (times may be NULL): an epoch pushes its start entry
 * (:214) and, when a step stops on f_rel_error <= f_tol but the refreshed
 * f_rel_error no longer passes the test at :257, a terminate entry (:246)
 * too.  pri_res_norm[0] is the reference's `nothing` (NaN).                  */
typedef struct scs_history {
  double* obj;
  double* fval;
  double* pri_res_norm;
  double* rel;      /* rel_error: max(‖x − x*‖ / max(‖x*‖, 1), x_tol), or the
                       mean_square_error for reg "gl" (rel_kind = 1)       */
  double* objrel;   /* f_rel_error: max(|obj − obj*| / |obj*|, f_tol)       */
  double* times;    /* seconds since the start, millisecond resolution       */
  double* fvaltest; /* (r04) ftest(x) = f(Atest, ytest, x) of every pushed point when the
                       context holds test data (scs_set_test_*; iterate.jl:169-175,
                       utils.jl:55-57: one entry per obj entry); may be NULL.  Written only
                       through scs_iterate_ex, and only when test data is held  */
} scs_history;
/* optim_loop! on the device: init! + per epoch f(x) + get_reg(x) + one step!
 * per batch (the full batch, or the scs_set_batches list in order), the
 * reference's termination tests and history pushes.  x_star is
 * model.x (the comparison solution).  Outputs: final x, *n_hist entries,
 * *epochs (Solution.epochs).  Metrics / verbose printing stay in the host loop
 * (scsopt.iterate).  Requires scs_method_init.
 * ABI note (r05 -> r06): scs_iterate reads the six-field (r03) history and never writes
 * fvaltest; a context holding test data (scs_set_test_*) is refused with SCS_ERR_STATE --
 * callers built against the r04 seven-field struct call scs_iterate_ex instead.          */
int scs_iterate(scs_ctx* ctx, const double* x0, const double* x_star, int64_t max_epoch, double x_tol,
                double f_tol, int rel_kind, double* x_out, const scs_history* hist, int64_t* n_hist,
                int64_t* epochs);
/* The same loop with a sized history: hist_size = sizeof(scs_history) as the caller compiled it.
 * Fields beyond hist_size are taken as NULL, so a caller built against the six-field (r03) layout
 * is never written past its struct; scs_iterate itself is scs_iterate_ex with the six-field size
 * (it never touches fvaltest).  A context given exactly one of Atest / ytest (scs_set_test_data
 * with A or y NULL: the reference's xor case, iterate.jl:170-171) fails with SCS_ERR_REF
 * "UndefVarError: `ftest` not defined ..." at the loop's first stats push, as the reference's
 * first show_stat! (:201) does.                                                                 */
int scs_iterate_ex(scs_ctx* ctx, const double* x0, const double* x_star, int64_t max_epoch, double x_tol,
                   double f_tol, int rel_kind, double* x_out, const scs_history* hist, size_t hist_size,
                   int64_t* n_hist, int64_t* epochs);

/* ---- kernel-level entry points (parity tests) --------------------------- */
/* hμ.grad(Cmat, x), hμ.hess(Cmat, x)                                       */
int scs_smoother_eval(scs_ctx* ctx, const double* x, double* gr, double* Hr);
/* prox_step(invoke_prox(model, reg_name, z, 1 ./ Hr, λ, α))                */
int scs_prox_eval(scs_ctx* ctx, const double* z, const double* Hr, double lam,
                  double alpha, double* out);
/* G = Aᵀ diag(w) A (local rows; lower triangle + diagonal tiles), ldg >= m. */
int scs_gram_eval(scs_ctx* ctx, const double* w, double* G, int64_t ldg);
/* out = Aᵀ v (local rows)                                                  */
int scs_gemv_t_eval(scs_ctx* ctx, const double* v, double* out);
/* out = A x (local rows)                                                   */
int scs_gemv_n_eval(scs_ctx* ctx, const double* x, double* out);

/* The m x m system of ProxNSCORE / ProxGGNSCORE, (Aᵀ diag(w) A + diag(dvec)) x = rhs
 * ((H + λ·Diagonal(Hr)) \ ∇q, prox-N-SCORE.jl:69-70; qr(JQJ) \ Je, prox-GGN-SCORE.jl:129-131),
 * through the step's own path: MFMA Gram, then the solver scs_set_solver selects (mode 0: by
 * default the hand-written Cholesky with the LU fallback), the hand-written LU alone (mode 1) or
 * the Householder QR (mode 2).  *used_lu = 1 when the LU ran.                                */
int scs_solve_eval(scs_ctx* ctx, const double* w, const double* dvec, const double* rhs, int mode,
                   double* x, int* used_lu);
/* Julia's `A \ b` for a dense square Matrix (LAPACK getrf + getrs) by the hand-written
 * blocked LU: A is row-major n x n; ipiv receives getrf's pivot rows (0-based), info its
 * first zero pivot (1-based; x is then not written, ipiv is dgetrf's).  A cooperative panel whose
 * candidate exchange timed out (a workgroup never became resident) is redone with the
 * column-step panels, the same factor bit for bit (scs_fallback_counts).
 * Needs a context only.                                                                    */
int scs_lu_eval(scs_ctx* ctx, int64_t n, const double* A, const double* b, double* x, int32_t* ipiv,
                int* info);
/* Columns cols[0..ncols) of the local (dense) A, column-major N x ncols.                 */
int scs_get_columns(scs_ctx* ctx, const int64_t* cols, int64_t ncols, double* out);
/* The production Gram launch for weights w, with Aᵀv formed in the same pass where a step
 * fuses it (*fused = 1): entries G(ij[2k], ij[2k+1]) for k < n, and Aᵀv (m).              */
int scs_gram_atv_eval(scs_ctx* ctx, const double* w, const double* v, const int64_t* ij, int64_t n,
                      double* gvals, double* atv, int* fused);

/* ---- timing ------------------------------------------------------------- */
/* on = 0: off; 1: HIP events around every Gram / product / solve / step; n > 1: in
 * scs_iterate's pipelined ProxLQNSCORE loop only every n-th epoch's launches are bracketed
 * (each event record costs a dispatch gap), everything else as for 1.                      */
int scs_timing_enable(scs_ctx* ctx, int on);
int scs_timing_get(scs_ctx* ctx, scs_timing* out);
int scs_timing_reset(scs_ctx* ctx);
/* The kernels of the latest main Gram launch and sparse product launch, as rocprofv3 names them
 * ("" when none ran), NUL-terminated, truncated to the capacities.                          */
int scs_kernel_names(scs_ctx* ctx, char* gram, int64_t gram_cap, char* product, int64_t product_cap);
/* Fallbacks taken instead of failing (r06), counted since the context was created (a
 * multi-device context: summed over its devices).  counts[i] for i < n:
 *   SCS_FB_LU_COOP_REFUSED  LU panels whose cooperative launch the runtime refused (run as column steps)
 *   SCS_FB_LU_COOP_REDO     LU factorizations redone with column-step panels after the one-launch
 *                           panel's candidate exchange timed out (info = -1)
 *   SCS_FB_SOLVE_BLOCKS     Cholesky solves redone by per-block launches after a one-launch solve's
 *                           dependency wait gave up
 *   SCS_FB_QR_BLOCKS        QR backward solves redone by per-block launches (the same, for QR)
 *   SCS_FB_CHAIN_REDO       Cholesky factors redone with one launch per operation after a wait of
 *                           the dependency-driven chain (SCS_CHOL_DAG=1) gave up
 *   SCS_FB_PIPE_REDO        steps whose Gram + factor were redone unpipelined after a strip wait of
 *                           the pipelined factor (SCS_CHOL_PIPE) gave up
 *   SCS_FB_QR_COOP_REFUSED  QR panels whose cooperative launch the runtime refused (run as column steps)
 *   SCS_FB_QR_COOP_REDO     QR solves redone from the saved system with the per-column launches after
 *                           a one-launch panel's record exchange timed out
 * Each redo gives the bits of the mode it falls back to.                                   */
#define SCS_FB_LU_COOP_REFUSED 0
#define SCS_FB_LU_COOP_REDO 1
#define SCS_FB_SOLVE_BLOCKS 2
#define SCS_FB_QR_BLOCKS 3
#define SCS_FB_CHAIN_REDO 4
#define SCS_FB_PIPE_REDO 5
#define SCS_FB_QR_COOP_REFUSED 6
#define SCS_FB_QR_COOP_REDO 7
#define SCS_FB_N 8
int scs_fallback_counts(scs_ctx* ctx, int64_t* counts, int n);
/* Wait for all work on the context stream.                                 */
int scs_sync(scs_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* SCSOPT_H */
