// Launcher declarations shared by the kernel files and the orchestration.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>
#include "../../include/scsopt.h"

namespace scs {

// host-side mirror of the prox/regularizer parameters (device pointers inside)
struct ProxArgsH {
  int reg = 0;
  int use_prox = 1;
  double lam = 0.0, lam2 = 0.0;
  const double* lb = nullptr;
  const double* ub = nullptr;
  const int* gstart = nullptr;
  const int* gend = nullptr;
  const double* gw = nullptr;
  int ngroups = 0;
  const int* gmap = nullptr;
};

// ---- gram.hip
void gram_tile_list(int nb, int2* out, int* ntiles);
void gram_tile_list_tall(int nb, int2* out, int* ntiles);
// Main Gram on the panel-blocked A (lda = S = Npad / 16); `packed` bit 0 = packed slots (else the
// upper triangle), bit 1 = accumulate into G.  tall = 1: 256 x 128 tiles from
// gram_tile_list_tall (nb even); packed slots are then the 128 x 128 halves (2t, 2t+1) of
// launch tile t.  gram_launch_gen operates on column-major operands (the Cholesky updates).
// v != nullptr: the same launch also forms Aᵀv (fused, gram_fuse_ok kernels only) into VP: one row
// (stride vps >= mpad) per K piece (nsplit rows for the scheduled launch, zeroed beforehand when
// nsplit > 1), reduced by gram_vfinal_launch.
// rocprofv3's name of the kernel the latest gram_launch / gram_launch_sched ran
const char* gram_main_kernel_name();
hipError_t gram_launch(const double* A, int64_t lda, const double* w, int64_t Nk, const int2* tiles, int ntiles,
                       double* G, int64_t ldg, int packed, int tall, hipStream_t st, const double* v = nullptr,
                       double* VP = nullptr, int64_t vps = 0);
int gram_fuse_ok(int tall);
hipError_t gram_vfinal_launch(const double* VP, int npiece, int64_t vps, int64_t m, double* out, hipStream_t st);
void gram_tile_list_rowmajor(int nb, int2* out);
hipError_t gram_launch_gen(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                           int64_t k0, int64_t k1, const int2* tiles, int ntiles, double* G, int64_t ldg, int flags,
                           hipStream_t st);
// the same as CU-bounded persistent launches leaving the CUs of `skip` (ids within a shader engine)
// free; ctr: 9 device counters, zeroed in stream order by the call (zeroed: already zero)
// K-split work list over two column-major operands: partial tiles to P (gram.hip; the QR's Vᵀ products)
hipError_t gram_launch_work_cm(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                               int64_t K, const int4* work, int seglen, int nsplit, double* P, hipStream_t st);
hipError_t gram_launch_bounded(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                               int64_t k0, int64_t k1, const int2* tiles, int ntiles, double* G, int64_t ldg, int flags,
                               unsigned* ctr, unsigned skip, int slots, hipStream_t st, bool zeroed = false);
// the latency form of gram_launch_gen (128 x 16/32 strips per workgroup, loads 8 stages ahead);
// the same bits per tile as gram_launch_gen's other kernels
hipError_t gram_launch_small(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                             int64_t k0, int64_t k1, const int2* tiles, int ntiles, double* G, int64_t ldg, int flags,
                             hipStream_t st);
// Tail-balanced schedule of the main Gram (see gram.hip): work items (bi, bj, ks, idx),
// combine items (bi, bj, tix, first partial slot)
int gram_schedule(const int2* tiles, int ntiles, int slots_per_xcd, std::vector<int4>& work, std::vector<int4>& comb,
                  int* nsplit, int* npart, int diag_first_gti = 0);
hipError_t gram_launch_sched(const double* A, int64_t lda, const double* w, int64_t Nk, const int4* work, int seglen,
                             int nsplit, const int4* comb, int ncomb, double* P, double* G, int64_t ldg, int packed,
                             int tall, hipStream_t st, const double* v = nullptr, double* VP = nullptr,
                             int64_t vps = 0, unsigned* scnt = nullptr, int sob = 0);
// scnt: per-strip completion counts (each finished whole tile adds 1 to scnt[bj / sob]); the
// factor stream waits for a strip with strip_wait_launch (flag: set on a timed-out wait)
hipError_t strip_wait_launch(const unsigned* cnt, unsigned target, int* flag, hipStream_t st);
hipError_t gram_pack_launch(const double* G, int64_t ldg, const int2* tiles, int ntiles, double* P, hipStream_t st);
hipError_t gram_unpack_launch(const double* P, const int2* tiles, int ntiles, double* G, int64_t ldg,
                              hipStream_t st);

// ---- chol.hip (upper Cholesky on MFMA; W holds the inverted diagonal blocks)
// One strip task of the Cholesky's dependency-driven chain launches (chol_dag_kernel): a latency
// Gram strip (gram_small_strip<16>) with its operands as offsets, the counters it waits for and
// the ones it advances when done.
struct DagTask {
  int64_t a1, a2, out;   // element offsets: A1 in W (a1w) or G; A2 and the output strip origin in G
  int32_t lda1, a1w;     // A1 leading dimension (128 for W, ld for G), A1 in W?
  int32_t k0, nk;        // contraction [k0, k0 + nk), whole 8-stage rings
  int32_t wneg, flags;   // weights +1 (0) or -1 (1); GRAM_ACCUMULATE | GRAM_UPPER
  int32_t dep0, ndep;    // its dependencies: deps[dep0 .. dep0 + ndep)
  int32_t sig0, sig1;    // counters advanced on completion (-1: none)
};
struct DagDep {
  int32_t c, target;     // counter c has reached target (in this run)
};
struct DagList {
  int t0 = 0, nt = 0;    // task range
  unsigned gen = 0;      // runs so far (the counters only grow: run g waits for (g-1)·period + target)
};

struct CholAux {             // device constants of the two-level factorization (chol_aux_init)
  double* w = nullptr;       // [128 x +1.0 | mpad x -1.0] Gram weights (panel solve | block updates)
  int2* rect = nullptr;      // R x nblk rectangle tile lists, R = 1..4 (bj-major)
  hipStream_t st2 = nullptr; // lookahead: the bulk stream (strip solve beyond the next block, C12)
  hipStream_t stc = nullptr; // lookahead: the chain's own high-priority stream (SCS_CHOL_CHAIN=1)
  hipStream_t st2h = nullptr;   // lookahead: the bulk stream at high priority (default: its own HW queue)
  hipEvent_t ev1 = nullptr, ev2 = nullptr, ev3 = nullptr, ev4 = nullptr, ev0 = nullptr, ev5 = nullptr;
  int nblk = 0;
  // the bulk stream's launches as CU-bounded persistent launches (gram_launch_bounded): claim /
  // arrival counters, the skipped CU ids (SCS_CHOL_BULK_SKIP), workgroup slots of the device
  // (BCTR_SLOTS sets of 16, zeroed together; each launch takes the next set -- no memset per launch)
  unsigned* bctr = nullptr;
  // the lower-triangle tile list in 8 x 8 super-blocks (super-rows ascending): rows < 8R are a
  // prefix, so the bulk update's tiles of rows [2OB, nc) are one slice when 8 divides 2OB and nc
  int2* sbl = nullptr;
  unsigned bskip = 0;
  int bslots = 0;
  mutable int bslot = 0;   // the next unused counter set
  // the streams' hardware-queue guard (SCS_CHOL_CHAIN, chol.hip): 2 where the process also holds RCCL's
  // streams (the caller sets it), else 0
  mutable int chain_mode = 0;
  // the chain's strip solve as right-looking step launches (strip_solve_steps): two rows of
  // 128 x (16 x 128) doubles for a step's leaf (its copy-back is the next step's)
  double* sscr = nullptr;
  // strip pipeline (chol_pipe_init): the left-looking update of each outer strip s as a
  // tail-balanced scheduled launch over the pairs (i >= j, j < OB) of its trailing columns
  struct StripSched {
    int4* work = nullptr;
    int seglen = 0, nsplit = 1;
    int4* comb = nullptr;
    int ncomb = 0;
  };
  std::vector<StripSched> ssched;
  double* spart = nullptr;   // K-split partial tiles of those launches
  // one-launch triangular solves (chol_solve): per-block flags (2 nblk), their error flag, and
  // the generation number the next solve stamps
  unsigned* sflags = nullptr;
  int* serr = nullptr;
  unsigned sgen = 0;
  // fallbacks (scsopt.cpp): the per-block solves instead of the one-launch ones after a solve's wait gave
  // up; the launch-per-operation chain instead of the dependency-driven one after a chain wait gave up
  mutable bool no_persist = false;
  mutable bool no_dag = false;
  // dependency-driven chain launches (chol_dag_build, built for one outer block size dag_ob): per
  // inner block k the A-phase step (row panel + trailing strips inside the outer block), per outer
  // block t the next block's strip solve + diagonal triangle (Ba + C1a)
  mutable int dag_ob = 0;
  mutable int64_t dag_ld = 0;
  mutable DagTask* dtasks = nullptr;
  mutable DagDep* ddeps = nullptr;
  mutable unsigned* dcnt = nullptr;
  mutable unsigned* dper = nullptr;
  mutable std::vector<DagList> dstep, dnext;
};
hipError_t chol_aux_init(CholAux* a, int64_t mpad, hipStream_t st);
void chol_aux_free(CholAux* a);
// the 128 x 128 diagonal block k: factor in place, W_k = U_kk⁻¹ (SCS_CHOL_DIAG=0: phase-serial kernel)
hipError_t launch_chol_diag(double* G, int64_t ld, int k, double* W, int* info, hipStream_t st);
// L11⁻¹ and U11⁻¹ (row-major 128 x 128) of the LU's factored diagonal block at (r0, r0) (chol.hip)
hipError_t launch_lu_tri_inv(const double* A, int64_t ld, int64_t r0, double* Linv, double* Uinv, hipStream_t st);
hipError_t chol_factor(double* G, int64_t ld, int64_t m, int64_t mpad, double* W, const CholAux* aux,
                       const int2* trilist, int* info, hipStream_t st);
hipError_t chol_solve(const double* G, int64_t ld, int64_t mpad, const double* W, double* b, double* y, CholAux* a,
                      hipStream_t st);
// whether chol_factor would run the dependency-driven chain (SCS_CHOL_DAG=1, not switched off)
bool chol_dag_active(const CholAux* a);
// U x = y by the per-block launches (y is consumed as scratch), the fallback of chol_back_solve
hipError_t chol_back_blocks(const double* U, int64_t ld, int64_t mpad, const double* W, double* y, double* x,
                            hipStream_t st);
// Strip pipeline (scsopt.cpp gram_factor_pipelined): the factor runs left-looking behind a Gram
// computed strip by strip.  Strip s = inner blocks [s·OB, min((s+1)·OB, nblk)).
int chol_outer_block();
hipError_t chol_pipe_init(CholAux* a, int64_t mpad, hipStream_t st);
// strip s -= U[0:i0, strip]ᵀ U[0:i0, strip..] (all earlier strips at once, K = i0·128)
hipError_t chol_strip_update(double* G, int64_t ld, int s, const CholAux* a, hipStream_t st);
// A and B of strip s: its diagonal block by the 128-blocked loop, then its row strip solved
hipError_t chol_strip_factor(double* G, int64_t ld, int s, double* W, const CholAux* a, const int2* trilist, int* info,
                             hipStream_t st);
// dst(r0:r1, c0:c1) = src(r0:r1, c0:c1), column-major with leading dimension ld (r0 even)
hipError_t chol_copy_rows(double* dst, const double* src, int64_t ld, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                          hipStream_t st);
// G[i, i] = 1 for i in [lo, hi) (the padding of block-diag(A, I))
hipError_t chol_diag_pad(double* G, int64_t ld, int64_t lo, int64_t hi, hipStream_t st);
// the Cholesky's column-major form of the scheduled Gram: A1 = A2 = X (lda = ld), K rows [k0, k1)
hipError_t gram_launch_sched_cm(const double* X, int64_t ld, const double* w, int64_t k0, int64_t k1, const int4* work,
                                int seglen, int nsplit, const int4* comb, int ncomb, double* P, double* G, int64_t ldg,
                                int flags, hipStream_t st);

// ---- lu.hip (blocked LU with partial pivoting, row-major, in place; lu_solve after lu_factor)
struct LUAux {
  int64_t npad = 0;          // capacity (lu_aux_init)
  double* cand = nullptr;    // [2][256] per-workgroup pivot candidates |a| of the next column
  int* candi = nullptr;      // [2][256] their rows
  double* candrow = nullptr; // [2][256][128] their panel rows
  double* rowj = nullptr;    // [2][128] copy of row j (the row the pivot row displaces)
  unsigned long long* gran = nullptr;   // cooperative panel: {tag, word} granules (candidates, rows), abort word
  int* ipiv = nullptr;       // [npad] pivot row of each column (0-based, absolute)
  int2* pairs = nullptr;     // [nblk][256] composed row moves of each block (dst, src)
  int* npairs = nullptr;     // [nblk]
  double* Linv = nullptr;    // [nblk][128 x 128] row-major L11⁻¹
  double* Uinv = nullptr;    // [nblk][128 x 128] row-major U11⁻¹
  double* T = nullptr;       // [npad][128] A12ᵀ staging
  double* UT = nullptr;      // [npad][128] U12 as K-contiguous columns
  double* UTo = nullptr;     // [npad][512] an outer block's U rows on the trailing columns, K-contiguous
  int2* rect = nullptr;      // row-major nblk x c tile rectangles, c = 1 .. 4 (updates inside an outer block;
                             // 4: the lookahead's next outer block)
  double* w = nullptr;       // [128 x +1 | 512 x -1]
  mutable int ob = 1;        // panels per outer block of the last lu_factor (lu_solve follows its row order)
  int2* sq = nullptr;        // square-shell tile list (trailing updates)
  int2* row1 = nullptr;      // (0, j) tile list (TRSM)
  // the cooperative one-launch panel: off for a redo after a timed-out candidate exchange (info = -1,
  // scsopt.cpp lu_factor_checked); launches the runtime refused (the panel ran as column steps)
  mutable bool no_coop = false;
  mutable int64_t coop_refused = 0;
  // the lookahead outer step (SCS_LU_LA, r06): the bulk stream that updates the trailing columns beyond
  // the next outer block while the next block's panels run, its two events (panels done / bulk done),
  // its own A12ᵀ staging, the (i < LU_OB, j) tile list of the bulk's top rows and the counter sets of
  // its CU-bounded launches (LU_LCTR sets of 16, zeroed once per factorization)
  mutable hipStream_t st2 = nullptr;
  mutable hipEvent_t evp = nullptr, evb = nullptr;
  double* T2 = nullptr;
  int2* col4 = nullptr;
  unsigned* lctr = nullptr;
  mutable int lslot = 0;
};
hipError_t lu_aux_init(LUAux* a, int64_t npad, hipStream_t st);
void lu_aux_free(LUAux* a);
// A: npad x npad row-major (row stride ld), rows/cols [n, npad) zero; *info must be 0 on
// entry and receives the first zero pivot (1-based) -- the factorization still completes.
hipError_t lu_factor(double* A, int64_t ld, int64_t n, int64_t npad, const LUAux* a, int* info, hipStream_t st);
// b (npad, zero-padded) <- A⁻¹ b
hipError_t lu_solve(const double* A, int64_t ld, int64_t npad, const LUAux* a, double* b, hipStream_t st);

// ---- qr.hip: Householder QR solve (LAPACK dgeqrf / dlarfg / dlarft conventions), the reference
// solver mode (scs_set_solver).  A: column-major npad x npad, rows/cols [n, npad) the identity;
// A is overwritten, b (npad) receives x.
struct QRAux {
  int64_t npad = 0;
  double *part = nullptr, *tw = nullptr, *tau = nullptr, *scal = nullptr, *V = nullptr, *Vt = nullptr,
         *Wm = nullptr, *Ym = nullptr, *Gv = nullptr, *T = nullptr, *ones = nullptr, *W = nullptr, *rowc = nullptr, *xs = nullptr;
  int2* tiles = nullptr;
  std::vector<int64_t> rect_off;   // per panel: offset of its update rectangle in tiles
  struct KList {                   // a K-split work list (qr_ksplit)
    int64_t off = 0;
    int seglen = 0, nsplit = 1, nj = 1;
  };
  std::vector<KList> klists;       // per panel: [Gv, Wm]
  int4* kwork = nullptr;
  double* kpart = nullptr;         // the pieces' partial tiles
  // the one-launch backward solve's block flags (generation-stamped, never reset) and its
  // dependency-wait error flag (set when a wait gives up after ~30 s: never expected)
  unsigned* flags = nullptr;
  int* err = nullptr;
  unsigned gen = 0;
  // the cooperative one-launch panel (r06): {tag, word} granules (records, row c, abort word), its info
  // (-1: a sweep gave up -- scsopt.cpp qr_run redoes the solve with no_coop); launches the runtime refused
  unsigned long long* gran = nullptr;
  int* cinfo = nullptr;
  mutable bool no_coop = false;
  mutable int64_t coop_refused = 0;
  // the lookahead trailing update (SCS_QR_LA, r06): the bulk stream that applies panel p's block
  // reflector to the columns beyond the next panel while panel p + 1 runs, its events, the second V / T
  // (panel parity) and the bulk's own Wm / Ym / Vᵀ / K-split partials; klists[2 nbk + p]: its Wm list
  hipStream_t st2 = nullptr;
  hipEvent_t evp = nullptr, evb = nullptr;
  double *V2 = nullptr, *T2 = nullptr, *Wm2 = nullptr, *Ym2 = nullptr, *Vt2 = nullptr, *kpart2 = nullptr;
};
// set the identity padding of a column-major system in place / build it from a row-major one
hipError_t qr_prepare(double* A, int64_t ld, int64_t n, int64_t npad, hipStream_t st);
hipError_t qr_from_rowmajor(const double* S, int64_t lds, double* D, int64_t ldd, int64_t n, int64_t npad,
                            hipStream_t st);
hipError_t qr_aux_init(QRAux* a, int64_t npad, hipStream_t st);
void qr_aux_free(QRAux* a);
hipError_t qr_solve(double* A, int64_t ld, int64_t npad, QRAux* a, double* b, hipStream_t st);
// whether qr_solve of order npad may run cooperative panels (SCS_QR_COOP, read per call): the caller then
// keeps a copy of A and b for a redo after a sweep that gave up (QRAux::cinfo = -1)
bool qr_coop_wanted(int64_t npad);
// chol.hip pieces the QR solve reuses: the inverses of the 128 x 128 upper diagonal blocks of R
// (W, as the Cholesky's), and the one-launch backward solve U x = y
// T (128 x 128, upper) of a compact WY block from Gv = VᵀV and tau (chol.hip; the QR's panels)
hipError_t wy_t_build(const double* Gv, const double* tau, double* T, hipStream_t st);
hipError_t chol_tri_inverse(const double* R, int64_t ld, int nblk, double* W, hipStream_t st);
hipError_t chol_back_solve(const double* U, int64_t ld, int64_t mpad, const double* W, double* y, double* x,
                           unsigned* flags, unsigned gen, int* err, hipStream_t st);

// ---- vec.hip
hipError_t launch_smoother(int kind, const double* x, int64_t m, double mu, const double* a, const double* b,
                           const double* wel, double* gr, double* Hr, hipStream_t st);
hipError_t launch_score_tail(const double* x, const double* d, const double* gr, const double* Hr, int64_t m,
                             double lam, double Mg, double step_host, const double* step_dev, const ProxArgsH& P,
                             double* hinv, double* zbuf, double* x_new, double* dx, double* scal, hipStream_t st);
hipError_t launch_prox_only(const ProxArgsH& P, const double* z, const double* Hr, double step, int64_t m,
                            double* hinv, double* out, hipStream_t st);
hipError_t launch_reg_value(const ProxArgsH& P, const double* x, int64_t m, double* out, double* part,
                            hipStream_t st);
hipError_t launch_dot(const double* a, const double* b, int64_t m, double* out, hipStream_t st);
// fused ProxLQNSCORE epoch passes (vec.hip): R = LQ_NPART x 256 partials
enum { LQ_DG = 0, LQ_GG, LQ_ETA, LQ_REG, LQ_NA, LQ_NB, LQ_NC, LQ_PRI, LQ_NPART };
constexpr int LQ_G = 256;
hipError_t launch_lqn_eta(const double* gr, const double* Hr, int64_t m, double lam, double* hinv, double* R,
                          hipStream_t st);
hipError_t launch_lqn_tail(const double* x, const double* d, int neg, int64_t m, double Mg, double step,
                           const ProxArgsH& P, const double* hinv, double* x_new, double* dx, double* dh, double* R,
                           double* scal, hipStream_t st);
// ring (device [order[0..mem] | k | spare]) non-null: the pair goes to slot ring[mem+2] and the
// memory decision is taken on the device (H0 -> scal[h0_slot]); null: slot `slot`, the host decides.
// A second kernel forms the sums (and, with valpart, the loss sum as sum_partials does -> scal[zf_slot]),
// then copies scal[0..nmap) to hmap (device-mapped pinned host memory; nmap <= 64, 0: none).  (A last-
// workgroup reduction inside lqn_post measured slower: each workgroup's device-scope release writes
// back the XCD's L2.)
hipError_t launch_lqn_post(const double* tpart, int nchunk, int64_t ldp, int64_t m, double lam, int skind, double mu,
                           const double* sa, const double* sb, const ProxArgsH& P, const double* xs, const double* x,
                           const double* xn, const double* gq, const double* dh, double* gqn, double* S, double* Y,
                           int64_t lds, int* ring, int mem, int slot, double* gr, double* Hr, double* hinv, double* R,
                           const double* valpart, int nval, double* scal, int zf_slot, int rx_slot, int nrm_slot,
                           int h0_slot, double* hmap, int nmap, hipStream_t st);
// out[0..3) = Σ(x − xs)², Σx², Σ(xn − x)² (xs / xn may be null); part: 3 x 256 doubles
hipError_t launch_norms3(const double* x, const double* xs, const double* xn, int64_t m, double* out, double* part,
                         hipStream_t st);
hipError_t launch_axpby(const double* a, double lam, const double* b, int64_t m, double* out, hipStream_t st);
hipError_t launch_sub(const double* a, const double* b, int64_t m, double* out, hipStream_t st);
hipError_t launch_neg(const double* a, int64_t m, double* out, hipStream_t st);
hipError_t launch_trial_point(const double* x, const double* d, double alpha, int64_t m, double* out,
                              hipStream_t st);
hipError_t launch_bb_step(const double* x, const double* xp, const double* g, const double* gp, int64_t m,
                          double* out, hipStream_t st);
// m <= TWO_LOOP_SINGLE_MAX: one workgroup; above: TWO_LOOP_MAX_WG workgroups at most, one launch per
// recursion step; work holds (kcap + 4) * TWO_LOOP_MAX_WG doubles (kcap >= k).  kp / H0p non-null: the
// ring size and H0 are read on the device (scs_iterate's pipelined loop) and k is only their upper bound.
constexpr int64_t TWO_LOOP_SINGLE_MAX = 16384;
constexpr int TWO_LOOP_MAX_WG = 256;
// f32 = 1: fp32 arithmetic (the compute arm of the C5 tolerance study, scs_set_compute_f32)
hipError_t launch_two_loop(const double* S, const double* Y, int64_t ld, const int* order, int k, double H0,
                           const double* g, int64_t m, double* q, double* d, double* ab, double* work, int kcap,
                           const int* kp, const double* H0p, hipStream_t st, int f32 = 0);
hipError_t launch_lbfgs_update(const double* dh, const double* gq_new, const double* gq, int64_t m, double* Sslot,
                               double* Yslot, double* scal, double* part, hipStream_t st);
hipError_t launch_diag_add(double* G, int64_t ldg, int64_t m, double lam, const double* Hr, hipStream_t st);
hipError_t launch_nonfinite(const double* G, int64_t ldg, int64_t m, const double* rhs, int* flag, hipStream_t st);
hipError_t launch_fill(double* a, int64_t n, double v, hipStream_t st);
hipError_t launch_symmetrize(double* G, int64_t ldg, int64_t m, hipStream_t st);
hipError_t launch_half_sym(const double* A, int64_t S, int64_t m, double* G, int64_t ldg, hipStream_t st);
hipError_t launch_rosen(const double* x, int64_t m, int what, double* out, double* G, int64_t ldg, hipStream_t st);

// ---- data.hip
// z-partials: out[split][ldo] ; returns the number of splits used
int gemv_n_splits(int64_t Npad, int64_t m);
// A is panel-blocked (common.h tiled_off), S = Npad / 16; x has m_pad entries (zero beyond m)
hipError_t launch_gemv_n(const double* A, int64_t S, int64_t Npad, int64_t mpad, const double* x, int nsplit,
                         double* part, int64_t ldo, hipStream_t st);
// loss epilogue over samples: sums the z-partials, writes z / coefficient vectors and
// per-block loss partials.  Returns the number of value partials written.
// EPI_SQR (with EPI_GGN): write s -> g, q -> h, r -> w instead of s²q / s·r (GGN sample-space branch)
enum { EPI_Z = 1, EPI_VAL = 2, EPI_GRAD = 4, EPI_HESS = 8, EPI_GGN = 16, EPI_SQR = 32 };
int epilogue_blocks(int64_t Npad);
hipError_t launch_epilogue(int loss, int ggn, int flags, const double* zpart, int nsplit, int64_t ldz,
                           const double* y, int64_t N, int64_t Npad, double c, double* z, double* g, double* h,
                           double* w, double* v, double* valpart, hipStream_t st);
// out[0] = Σ part[0..n)  (fixed order)
hipError_t launch_sum_partials(const double* part, int n, double* out, hipStream_t st);
hipError_t launch_marker(hipStream_t st);
// the line search's trial products (incremental form): out[0..Npad) = z0, out[Npad..2 Npad) = α·zd, so
// the epilogue over these two "partials" forms z0 + α·zd = A x + α·A d
hipError_t launch_ls_pair(const double* z0, const double* zd, double alpha, int64_t Npad, double* out,
                          hipStream_t st);
// Aᵀ v (column partial sums over row chunks, then a fixed-order finalize)
int gemv_t_chunks(int64_t Npad);
hipError_t launch_gemv_t(const double* A, int64_t S, int64_t Npad, int64_t m, int64_t mpad, const double* v,
                         double* part, hipStream_t st);
// panel p: column-major Npad x 128 buffer C <-> tiled A (to_tiled = 1: C -> A)
hipError_t launch_retile(double* C, double* A, int64_t Npad, int64_t p, int to_tiled, hipStream_t st);
// out[j] = Σ_chunk part[chunk][j] (+ lam*add[j] if add)
hipError_t launch_gemv_t_finalize(const double* part, int nchunk, int64_t mpad, int64_t m, double* out,
                                  hipStream_t st);
hipError_t launch_densify(const int64_t* rowptr, const int* col, const void* val, int f32, int64_t N, int64_t Npad,
                          double* Ad, hipStream_t st);
// CSR rows [r0, r0 + n) into a zeroed panel-blocked slot of Npad_b rows (zero = 1: clear them again)
hipError_t launch_densify_range(const int64_t* rowptr, const int* col, const void* val, int f32, int64_t r0,
                                int64_t n, int64_t Npad_b, int zero, double* Ab, hipStream_t st);
hipError_t launch_densify_rows(const int64_t* rowptr, const int* col, const void* val, int f32, const int64_t* rows,
                               int64_t n, int64_t Npad_b, const double* y, double* Ab, double* yb, hipStream_t st);
hipError_t launch_gather_rows(const double* A, int64_t Npad, const double* y, const int64_t* rows, int64_t n,
                              int64_t Npad_b, int64_t mpad, double* Ab, double* yb, hipStream_t st);
hipError_t launch_transpose(const double* A, int64_t Npad, int64_t N, int64_t m, double* At, int64_t ldt,
                            int64_t nt, hipStream_t st);
// selected columns of the panel-blocked A -> column-major N x ncols (cols on the device)
hipError_t launch_get_columns(const double* A, int64_t S, const int64_t* cols, int64_t ncols, int64_t N, double* out,
                              hipStream_t st);
// out[k] = G(ij[k].x, ij[k].y) of a column-major matrix
hipError_t launch_gather_entries(const double* G, int64_t ld, const int2* ij, int n, double* out, hipStream_t st);
// GGN sample-space branch (vec.hip)
hipError_t launch_ggn_sample_prep(const double* Hr, const double* gr, double lam, int64_t m, int64_t mpad,
                                  double* hvec, double* hg, hipStream_t st);
hipError_t launch_ggn_sample_assemble(const double* P, int64_t ldp, const double* s, const double* q,
                                      const double* r, const double* u, const double* kNN, int64_t N, double* M,
                                      int64_t ldm, double* b, hipStream_t st);
hipError_t launch_ggn_sample_scale(const double* s, const double* B, int64_t N, int64_t Npad, double* v,
                                   hipStream_t st);
hipError_t launch_ggn_sample_direction(const double* hvec, const double* t, const double* hg, const double* B,
                                       int64_t N, int64_t m, double* d, hipStream_t st);
// synthetic data
hipError_t launch_gen_A(double* A, int64_t Npad, int64_t N, int64_t m, int64_t mpad, int64_t row0, uint64_t seed,
                        double scale, hipStream_t st);
hipError_t launch_gen_xtrue(double* x, int64_t m, uint64_t seed, double density, hipStream_t st);
hipError_t launch_gen_y(int kind, const double* z, double* y, int64_t N, int64_t row0, uint64_t seed,
                        hipStream_t st);

// ---- sparse.hip (LDS-blocked gathers; out[b*ldo + r] = Σ_{p in row r, block b} val[p] x[(b<<shift) + lidx[p]])
int spmv_blk_shift(int64_t ncols);
int spmv_pad_index();   // padding index of the blocked layouts (the SpMV's zero slot)
int spmv_slot_width(int f32);   // segments padded to whole slots of 4 (fp64) / 8 (fp32) entries
// segments padded to whole slots (blk_pad), padding index spmv_pad_index(), value 0
// f32: 0 fp64 values, 1 fp32-stored values (fp64 arithmetic), 2 fp32-stored values with fp32 arithmetic
const char* spmv_kernel_name(int f32);
hipError_t launch_spmv_blk(const int64_t* ptr, const uint16_t* lidx, const void* val, int f32, const double* x,
                           int64_t nrows, int64_t ncols, int shift, int64_t nnz, double* out, int64_t ldo,
                           hipStream_t st);
hipError_t blk_count(const int64_t* ptr, const int* idx, int64_t nrows, int shift, int64_t* cnt, int64_t* first,
                     hipStream_t st);
hipError_t blk_pad(int64_t* cnt, int64_t n, int f32, hipStream_t st);
hipError_t blk_scan(void* temp, size_t* temp_bytes, const int64_t* cnt, int64_t* bptr, int64_t n, hipStream_t st);
hipError_t blk_scatter(const int64_t* ptr, const int* idx, const void* val, int f32, int64_t nrows, int shift,
                       const int64_t* bptr, const int64_t* first, uint16_t* lidx, void* bval, hipStream_t st);
// sparse Gram G = Aᵀ diag(w) A (upper part, column j up to the end of its diagonal tile) from the
// CSC copy and a Gram-blocked CSR copy (block width 2^shift, unpadded segments): Σ_r nnz_r² work
int sparse_gram_shift();
int64_t sparse_gram_items(int64_t j0, int64_t j1, int shift);   // work items of columns [j0, j1)
// variant 8 (sparse.hip): the segment copy (value + index records, 8-B units), the per-triple table
// T[tptr[j] + b·n_j + k] = n << 40 | unit, and sw[p] = w[rowidx[p]]·valT[p] formed per Gram
int64_t seg_units_host(int64_t n, int f32);
int sparse_gram_requested();   // SCS_SPARSE_GRAM_KERNEL (default 8)
hipError_t seg_units(const int64_t* cnt, int64_t n, int f32, int64_t* ucnt, hipStream_t st);
hipError_t seg_scatter(const int64_t* ptr, const int* idx, const void* val, int f32, int64_t nrows, int shift,
                       const int64_t* cnt, const int64_t* first, const int64_t* uptr, uint64_t* seg, hipStream_t st);
hipError_t seg_table(const int64_t* colptr, const int* rowidx, const int64_t* cnt, const int64_t* uptr, int64_t nrows,
                     int64_t m, int shift, const int64_t* tptr, uint64_t* T, hipStream_t st);
hipError_t csc_weight(const int* rowidx, const void* valT, int f32, const double* w, int64_t nnz, double* sw,
                      hipStream_t st);
hipError_t launch_sparse_gram_seg(const int64_t* colptr, const double* sw, const int64_t* tptr, const uint64_t* T,
                                  const uint64_t* seg, int f32, int64_t m, int shift, double* G, int64_t ldg,
                                  hipStream_t st);
// the variant launch_sparse_gram runs (SCS_SPARSE_GRAM_KERNEL) for a copy of `entries` entries
const char* sparse_gram_kernel_name(int f32, int64_t entries);
hipError_t launch_sparse_gram(const int64_t* colptr, const int* rowidx, const void* valT, const int64_t* bptr,
                              const uint16_t* lidx, const void* bval, int64_t entries, int f32, const double* w,
                              int64_t nrows, int64_t m, int shift, double* G, int64_t ldg, hipStream_t st);
size_t sparse_layer_map_bytes(int k);
void sparse_layer_maps(uint64_t seed, int k, int64_t N, void* out_host);
hipError_t launch_gen_sparse(int64_t N, int64_t m, int k, uint64_t seed, const void* Ldev, int f32, double scale,
                             int64_t* rowptr, int* col, void* val, int64_t* colptr, int* row, void* valT,
                             hipStream_t st);
hipError_t sort_segments(void* temp, size_t* temp_bytes, const int* kin, int* kout, const void* vin, void* vout,
                         int f32, int64_t nnz, int64_t nseg, const int64_t* off, int end_bit, hipStream_t st);
hipError_t launch_gen_uniform(double* x, int64_t m, uint64_t seed, double lo, double hi, hipStream_t st);

}  // namespace scs
