// libscsopt: C ABI + per-method step orchestration of the SCORE inner
// iteration on MI355X.  Device work is issued on the context stream; the host
// reads back only the scalars the reference's control flow needs.
//
// Method map (reference -> here):
//   step!(::ProxNSCORE)   prox-N-SCORE.jl:34-119     -> step_newton(NSCORE)
//   step!(::ProxGGNSCORE) prox-GGN-SCORE.jl:34-135   -> step_newton(GGN)
//   step!(::ProxLQNSCORE) prox-L-BFGS-SCORE.jl:69-169 -> step_lqn
//   linesearch / inv_BB_step  utils.jl:27-48           -> line_search / bb kernel
//   get_Mg                    smoothing.jl:12-25        -> get_Mg
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/scsopt.h"
#include "common.h"
#include "kernels.h"
#include "shard_plan.h"

using namespace scs;

namespace {

struct Pending {
  int cat;
  hipEvent_t e0, e1;
};
enum { T_GRAM = 0, T_GEMV, T_SOLVE, T_STEP, T_REDUCE, T_N };
constexpr int ZF_SLOT = 24;   // scal / hscal slot of the deferred f(x) (forward with need_val = false)
// scs_iterate's device-resident loop: f(x) and get_reg(x) of the epoch's x, the norms (3 slots)
constexpr int FX_SLOT = 25, RX_SLOT = 26, NRM_SLOT = 28, LOOP_SLOTS = 32;
constexpr int TF_SLOT = 31;   // ftest(x) of the held-out data (inside LOOP_SLOTS: it rides the loop's hand-off)
constexpr int H0_SLOT = 19;   // the device ring's H0 (scs_iterate's pipelined ProxLQNSCORE loop)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// The N-dependent state of a context: the data rows with their sample-space workspace and the
// GGN sample-space caches.  A minibatch (scs_set_batch) is a second view swapped in for the
// duration of scs_step (the As, ys handed to step!, iterate.jl:205-207).
struct NView {
  double* A = nullptr;
  double* y = nullptr;
  int64_t N = 0, Npad = 0, nstage = 0, Nglob = 0;
  int nsplit = 1, nval = 1, nchunk = 1;
  double *zpart = nullptr, *z = nullptr, *gN = nullptr, *hN = nullptr, *wN = nullptr, *vN = nullptr,
         *valpart = nullptr, *tpart = nullptr;
  double *At = nullptr, *Ps = nullptr, *Ms = nullptr, *bS = nullptr, *uN = nullptr, *hvec = nullptr, *hg = nullptr;
  int64_t NpS = 0;
  int2* stiles = nullptr;
  int nstiles = 0;
  int64_t n1pad = 0;     // row stride of Ms: round_up(N + 1, 128) (lu.hip)
  bool sparse = false;   // a batch view is always dense (Matrix(As'), iterate.jl:207)
};

}  // namespace

struct scs_ctx {
  int dev = 0;
  hipStream_t st = nullptr;
  bool own_stream = false;
  std::string err;

  // row sharding: the exchange runs through libscsopt's own RCCL communicator (rccl) or the
  // caller's all-reduce callback (ar); comm_force runs the exchange path at one rank too
  int rank = 0, nranks = 1;
  scs_allreduce_fn ar = nullptr;
  void* ar_user = nullptr;
  ncclComm_t rccl = nullptr;
  bool comm_force = false;
  double* red = nullptr;
  int64_t red_cap = 0;
  bool own_red = false;   // red allocated by the library (no scs_set_reduce_buffer)

  // data
  int64_t N = 0, Npad = 0, m = 0, mpad = 0, Nglob = 0, row0 = 0;
  int64_t Nglob_data = 0;   // N_global of the full data (Nglob follows the swapped-in view)
  int64_t nstage = 0;  // Npad / 16: stages of the panel-blocked A (common.h tiled_off)
  bool has_data = false;
  bool generic = false;  // ProblemGeneric (no A)
  double* A = nullptr;
  double* y = nullptr;
  // sparse A: CSR (rows) + CSC copy (columns), values fp64 or fp32
  bool sparse = false;
  int sp_f32 = 0;
  // scs_set_compute_f32: fp32 ARITHMETIC in the sparse products (fp32-stored values) and the L-BFGS
  // two-loop -- the compute arm of BASELINE configs[4]'s fp32-vs-fp64 study; 0 (fp64) by default
  int f32c = 0;
  int64_t nnz = 0;
  int64_t *rowptr = nullptr, *colptr = nullptr;
  int *colidx = nullptr, *rowidx = nullptr;
  void *val = nullptr, *valT = nullptr;
  struct SpBlk {
    int shift = 0, nblk = 0;
    int64_t nnz = 0;   // entries of the copy
    int64_t* ptr = nullptr;
    uint16_t* lidx = nullptr;
    void* val = nullptr;
  } bcsr, bcsc;  // LDS-blocked copies used by the products (sparse.hip)
  SpBlk bgram;    // the sparse Gram's row copy: 2^sparse_gram_shift()-wide blocks, unpadded (built on first use)
  struct SegGram {   // the sparse Gram's variant-8 structure (build_gram_seg, on first use)
    int state = 0;   // 0 not tried, 1 built, -1 not built (memory / size): the Gram-blocked walk instead
    int shift = 0;
    uint64_t* seg = nullptr;   // per (block, row) segment records, 8-B units
    uint64_t* T = nullptr;     // per (column, upper block, row of the column): n << 40 | unit
    int64_t* tptr = nullptr;   // T's column offsets
    double* sw = nullptr;      // w[rowidx[p]]·valT[p], per Gram
  } sgseg;
  int sp_gram = 0;   // the Gram of a sparse A: 0 undecided, 1 priced by nnz (sparse_gram_kernel), 2 dense tiles
  double* Ad = nullptr;  // dense panel-blocked mirror of a sparse A (Gram-based methods only)
  // ... or, when the mirror does not fit under the cap, a ring of two R-row dense slots the Gram
  // streams through chunk by chunk (gram_main_stream)
  int sp_mode = 0;              // 0: undecided, 1: mirror, 2: stream
  double* ringA = nullptr;
  int64_t ring_rows = 0;
  int64_t ring_r0[2] = {-1, -1}, ring_n[2] = {0, 0};
  // x-independent Gram reuse (scs_set_gram_cache): Gk holds AᵀQA of data generation gk_gen;
  // data_gen moves on every change of the rows or the loss (new data, batch view swaps)
  int gram_cache = 0;
  double* Gk = nullptr;
  uint64_t data_gen = 1, gk_gen = 0;
  bool g_from_cache = false;   // this step's G was copied from Gk (solve_system)

  // problem
  int loss = 0, ggn = 0;
  double scale = 1.0;
  bool loss_set = false;
  int reg = 0;
  double lam = 0.0, lam2 = 0.0;
  int nlam = 1;
  bool reg_set = false;
  double* clb = nullptr;  // C_set (raw) bounds, length mpad
  double* cub = nullptr;
  int ngroups = 0;
  int* gstart = nullptr;
  int* gend = nullptr;
  double* gw = nullptr;
  double* wel = nullptr;  // per-element group weight (Cmat diagonal)
  int* gmap = nullptr;    // get_P's G, 0-based (null: identity)
  int smooth = 0;
  double mu = 1.0, Mh = 2.0, nu = 2.6;
  bool smooth_set = false;
  double* slb = nullptr;  // sanitized smoother bounds
  double* sub = nullptr;
  bool has_L = false;
  double L = 0.0;

  // method
  int method = 0, ss_type = 1, use_prox = 1, mem = 10;
  bool method_set = false;
  double* S = nullptr;  // [mem+1][mpad]
  double* Yv = nullptr;
  std::vector<int> ring;  // physical slots, oldest -> newest
  int spare = 0;
  int* d_order = nullptr;
  int* hring = nullptr;       // pinned copy of the ring order (asynchronous upload)
  // SCS_LOSS_CALLBACK: the caller's f / grad_fx / hess_fx, with a pinned [x | out] exchange buffer
  scs_loss_fn cb = nullptr;
  void* cb_user = nullptr;
  double* cbh = nullptr;
  size_t cbh_cap = 0;
  int64_t cb_nout = 0;        // rows of the SCS_CB_GGN Jacobian (0: no GGN callback)
  NView cbv;                  // that Jacobian, panel-blocked, swapped in for the GGN step
  double* cbstage = nullptr;  // column-major staging panel for its upload
  const double* gfix = nullptr; // scs_step_grad: the caller's ∇fx (device copy) for the step's duration
  bool lbfgs_pending = false; // scs_iterate's device loop: the memory update's dg/gg are read at the epoch end
  int lbfgs_slot = 0;
  double H0 = 1.0;

  // m-space workspace
  double *x = nullptr, *xp = nullptr, *xn = nullptr, *dxv = nullptr, *gr = nullptr, *Hr = nullptr, *hinv = nullptr,
         *zb = nullptr, *d = nullptr, *gq = nullptr, *gqn = nullptr, *gtmp = nullptr, *gtmp2 = nullptr, *q = nullptr,
         *ab = nullptr, *tlwork = nullptr, *scal = nullptr, *gcache[2] = {nullptr, nullptr};
  double* hscal = nullptr;  // pinned host scalars
  int* hserr = nullptr;     // pinned: the one-launch triangular solves' timeout flag, copied after each solve
  double* xstar = nullptr;  // model.x on the device (scs_iterate's rel_error)
  double* lqR = nullptr;    // fused ProxLQNSCORE epoch: LQ_NPART x 256 partial sums
  double* hloop = nullptr;  // pinned: the pipelined loop's per-epoch scalars, two epochs (parity)
  double* hloop_dev = nullptr;   // its device-side address
  hipEvent_t loop_ev[2] = {nullptr, nullptr};
  bool dev_loop = false;    // scs_iterate's device-resident loop: steps leave x_new / pri on the device
  // N-space workspace
  int nsplit = 1;
  double *zpart = nullptr, *z = nullptr, *gN = nullptr, *hN = nullptr, *wN = nullptr, *vN = nullptr,
         *valpart = nullptr;
  int nval = 1;
  int nchunk = 1;
  double* tpart = nullptr;
  // Gram / solve
  double *G = nullptr, *Gc = nullptr;
  int2* tiles = nullptr;    // Gram launch list
  int ntiles = 0;
  int tall = 0;             // 1: 256 x 128 launch tiles (nb even), packed slots = their 128 x 128 halves
  int2* utiles = nullptr;   // 128 x 128 slot list (unpack)
  int nslots = 0;
  int4* gwork = nullptr;    // tail-balanced schedule (gram_schedule): work items, combine items, partials
  int4* gcomb = nullptr;
  int gseglen = 0, gncomb = 0, gnsplit = 1;
  double* gpart = nullptr;
  double* vpart = nullptr;   // fused Aᵀv partials: max(gnsplit, strip nsplits, 1) rows of mpad
  // strip pipeline (gram_factor_pipelined): the Gram's tile list cut into the factor's outer
  // strips (tiles with bj in strip s), one tail-balanced schedule each; the factor stream and
  // one event per strip
  struct GStrip {
    int4* work = nullptr;
    int4* comb = nullptr;
    int seglen = 0, nsplit = 1, ncomb = 0;
  };
  std::vector<GStrip> gstrip;
  // the one-launch form (SCS_CHOL_PIPE=2): every strip's tiles in one scheduled launch, each XCD's
  // segment strip-major (its share of strip 0, then of strip 1, ...), K-split pieces in the last
  // strip only; whole tiles count into gp_cnt[strip], gp_target[s] = whole tiles of strip s
  GStrip gpipe;
  std::vector<unsigned> gp_target;
  unsigned* gp_cnt = nullptr;
  int* gp_flag = nullptr;
  int vpieces = 1;           // rows of vpart
  hipStream_t sf = nullptr;
  std::vector<hipEvent_t> evstrip;
  hipEvent_t evfac = nullptr;
  double* W = nullptr;      // inverted diagonal blocks of the Cholesky factor [mpad/128][128*128]
  double* ysol = nullptr;   // triangular-solve scratch (mpad)
  int2* trilist = nullptr;  // row-major lower tiles
  int* cinfo = nullptr;
  CholAux caux;             // two-level factorization constants (chol.hip)
  LUAux lu;                 // blocked LU (lu.hip): the non-SPD fallback and the GGN sample-space system
  // scs_set_solver: SCS_SOLVER_REFERENCE solves the way the reference does -- Householder QR for
  // ProxGGNSCORE's systems (prox-GGN-SCORE.jl:126,131), LU (Julia's `\`) for ProxNSCORE's
  int solver = 0;
  QRAux qr;                 // qr.hip workspace
  double* qrM = nullptr;    // the sample-space system transposed to column-major for the QR
  int64_t qrM_n = 0;
  double* luM = nullptr;    // scs_lu_eval's system / rhs / info, kept so the LU graphs replay
  double* lub = nullptr;
  int* luinfo = nullptr;
  int64_t lu_np = 0;
  // GGN sample-space branch (N + 1 <= m): Aᵀ copy, sample Gram, (N+1)² system
  double *At = nullptr, *Ps = nullptr, *Ms = nullptr, *bS = nullptr, *uN = nullptr, *hvec = nullptr, *hg = nullptr;
  int64_t NpS = 0;
  int2* stiles = nullptr;
  int nstiles = 0;
  int64_t n1pad = 0;
  // minibatches (scs_set_batches / scs_select_batch): the collected DataLoader batch list of
  // iterate.jl:141-146 as one device row list; each distinct batch size owns a gathered view
  // (NView) that is swapped in for the steps on that batch
  // On several ranks the list holds GLOBAL row indices: each rank keeps the batch's rows it
  // owns (possibly none) and their positions in the batch (bpos, for the sample-space gather);
  // the batch's global size (bglob) drives the branch choice and the exchange covers the rest.
  int64_t* brows = nullptr;
  std::vector<int64_t> boff;   // batch b = brows[boff[b] .. boff[b + 1]) (local rows)
  std::vector<int64_t> bglob;  // global size of batch b
  std::vector<int64_t> bpos;   // position in its batch of each local row of brows (host)
  std::vector<NView> bpool;    // gathered views, one per distinct (local, global) batch size
  std::vector<int64_t> bheld;  // the batch each pool view currently holds (-1: none)
  int bview = -1;              // the selected batch's pool view (-1: the full data)
  int64_t bsel = -1;           // the selected batch (-1: the full data)
  // all ranks' rows of the full data or of the selected batch (GGN sample-space branch with
  // N_global + 1 <= m on several ranks)
  NView gview;
  // held-out data (Problem(...; Atest, ytest), problems.jl:27-28,67-68): a view of its own (rows, y,
  // the f workspace; a sparse set also its CSR + LDS-blocked copy) swapped in only to evaluate
  // ftest(x) = f(Atest, ytest, x) at the loop's stats pushes (iterate.jl:169-175, utils.jl:55-57).
  // `host`: a callback loss evaluates it on the caller's side (SCS_CB_FTEST)
  struct TestSet {
    NView v;
    bool on = false, host = false;
    // exactly one of Atest / ytest given: optim_loop! logs "Will skip testing..." and leaves
    // `ftest` unassigned (iterate.jl:170-171), so its first show_stat! call (:201) raises
    // UndefVarError -- scs_iterate fails the same way at its first stats push
    bool xor_case = false;
    int sp_f32 = 0;
    int64_t nnz = 0;
    SpBlk bcsr;
    int64_t* rowptr = nullptr;
    int* colidx = nullptr;
    void* val = nullptr;
  } tset;
  bool gview_ok = false;
  int64_t gview_batch = -1;    // the batch gview holds (-1: the full data) ...
  uint64_t gview_gen = 0;      // ... of batch list generation gview_gen
  uint64_t batch_gen = 1;      // bumped whenever the batch list changes (scs_set_batches)
  bool lu_fallback_used = false;
  // the incremental line search's N-space scratch: [z0 | α·A d] trial pair (2 Npad) + A d (Npad)
  double* lsbuf = nullptr;
  int64_t lscap = 0;
  int64_t ls_direct = 0;   // incremental trials re-decided on the direct form (near the Armijo threshold)
  // fallbacks taken instead of failing (scs_fallback_counts): SCS_FB_* in include/scsopt.h
  int64_t fb[SCS_FB_N] = {};
  double* rbk = nullptr;   // (m_pad) the right-hand side before a one-launch solve, for its per-block redo
  double* Gbk = nullptr;   // (m_pad²) the system before a cooperative-panel LU, for its column-step redo
  int64_t Gbk_n = 0;
  double* qbk = nullptr;   // (npad² + npad) A and b before a cooperative-panel QR solve, for its redo
  int64_t qbk_n = 0;

  // caches (CSE of identical evaluations; keyed by the host x content)
  std::vector<double> zkey;
  bool zvalid = false;
  double zfval = 0.0;  // f(x) for zkey (global, scaled)
  bool zf_pending = false;   // zfval still in flight to hscal[8] (forward with need_val = false)
  std::vector<double> gkey[2];
  bool gvalid[2] = {false, false};
  // scs_iterate's host vectors carry version tags (bumped on every write), so the f / ∇q caches
  // compare a tag instead of m doubles and keep no copy; untagged pointers (the per-call ABI)
  // use the content keys above.  A key's tag is 0 for a content key.
  struct XTag {
    const double* p = nullptr;
    uint64_t v = 0;
  } xtags[3];
  uint64_t xtag_next = 1;
  uint64_t ztag = 0, gtag[2] = {0, 0};
  int gnext = 0;

  // the kernels the dominant launches used (scs_kernel_names; rocprofv3's names)
  std::string gram_kname, prod_kname;
  // timing
  bool timing = false;
  int timing_every = 1;     // scs_iterate's pipelined loop: kernel-timing events on every n-th epoch only
  std::vector<Pending> pending;
  double tms[T_N] = {0, 0, 0, 0, 0};
  int64_t tcalls[T_N] = {0, 0, 0, 0, 0};

  std::vector<DevBuf> allocs;

  // a multi-device context (scs_create_multi): one sub-context per device holding its row block
  // (row_plan), one RCCL communicator over the devices (ncclCommInitAll); the entry points a group
  // supports run on every sub-context at once, one host thread each (group_run)
  std::vector<scs_ctx*> subs;
  std::vector<RowBlock> plan;
  int64_t grpN = 0, grpm = 0;   // the whole problem's rows and columns
  bool group_broken = false;
  // one persistent host thread per device (group_run hands each call's per-device work to them:
  // no thread spawn per ABI call); `aborting` is shared with the sub-contexts (comm_abort), which
  // check it before every RCCL call once a failing device has aborted the communicators
  struct Workers;
  std::unique_ptr<Workers> workers;
  std::shared_ptr<std::atomic<bool>> comm_abort;
  // SCS_MULTI_HOST_EXCHANGE groups: the exchange through host memory instead of RCCL
  struct HostExchange;
  std::unique_ptr<HostExchange> hx;
  ~scs_ctx();
};

// ---------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------
namespace {

struct Fail {
  int code;
};

void set_err(scs_ctx* c, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
}

#define HCK(expr)                                                                                      \
  do {                                                                                                 \
    hipError_t e__ = (expr);                                                                           \
    if (e__ != hipSuccess) {                                                                           \
      set_err(c, "HIP error '%s' at %s:%d (%s)", hipGetErrorString(e__), __FILE__, __LINE__, #expr); \
      throw Fail{SCS_ERR_HIP};                                                                         \
    }                                                                                                  \
  } while (0)

[[noreturn]] void fail(scs_ctx* c, int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  c->err = buf;
  throw Fail{code};
}

template <class F>
int guarded(scs_ctx* c, F&& f) {
  if (!c) return SCS_ERR_ARG;
  if (!c->subs.empty()) {   // the group-aware entry points branch to group_* before this
    c->err = "this entry point takes a single-device context (scs_create), not a multi-device one";
    return SCS_ERR_ARG;
  }
  try {
    c->err.clear();
    f();
    return SCS_OK;
  } catch (const Fail& e) {
    return e.code;
  } catch (const std::exception& e) {
    c->err = e.what();
    return SCS_ERR_HIP;
  }
}

template <class T>
T* dalloc(scs_ctx* c, size_t n) {
  void* p = nullptr;
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) fail(c, SCS_ERR_HIP, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
  HCK(hipMemsetAsync(p, 0, bytes, c->st));
  c->allocs.push_back({p, bytes});
  return (T*)p;
}

void dfree(scs_ctx* c, void*& p) {
  if (!p) return;
  for (size_t i = 0; i < c->allocs.size(); ++i)
    if (c->allocs[i].p == p) {
      c->allocs.erase(c->allocs.begin() + i);
      break;
    }
  (void)hipFree(p);
  p = nullptr;
}
template <class T>
void dfree_t(scs_ctx* c, T*& p) {
  void* v = (void*)p;
  dfree(c, v);
  p = nullptr;
}

void h2d(scs_ctx* c, double* dst, const double* src, int64_t n) {
  HCK(hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
}
void d2h(scs_ctx* c, double* dst, const double* src, int64_t n) {
  HCK(hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToHost, c->st));
}
// Drain the stream.  A triangular solve whose block wait gave up (~30 s, never expected) flagged
// caux.serr; its copy lands in hserr behind the solve, so the first drain after that solve reports
// it (the step's direction is invalid) instead of the next factor's chain check.
void sync(scs_ctx* c) {
  HCK(hipStreamSynchronize(c->st));
  if (c->hserr && *c->hserr) {
    *c->hserr = 0;
    if (c->caux.serr) HCK(hipMemsetAsync(c->caux.serr, 0, sizeof(int), c->st));
    HCK(hipStreamSynchronize(c->st));
    fail(c, SCS_ERR_HIP, "Cholesky triangular solve: a block wait timed out; this step's direction is invalid");
  }
}

// after a chol_solve on the context stream: its timeout flag -> hserr (checked by sync)
void solve_flag_copy(scs_ctx* c) {
  if (c->hserr && c->caux.serr) HCK(hipMemcpyAsync(c->hserr, c->caux.serr, sizeof(int), hipMemcpyDeviceToHost, c->st));
}

void tbegin(scs_ctx* c, int cat, hipEvent_t* e0) {
  if (!c->timing) return;
  HCK(hipEventCreate(e0));
  HCK(hipEventRecord(*e0, c->st));
  (void)cat;
}
void tend(scs_ctx* c, int cat, hipEvent_t e0) {
  if (!c->timing) return;
  hipEvent_t e1;
  HCK(hipEventCreate(&e1));
  HCK(hipEventRecord(e1, c->st));
  c->pending.push_back({cat, e0, e1});
}
void tresolve(scs_ctx* c) {
  if (c->pending.empty()) return;
  for (auto& p : c->pending) {
    HCK(hipEventSynchronize(p.e1));
    float ms = 0.f;
    HCK(hipEventElapsedTime(&ms, p.e0, p.e1));
    c->tms[p.cat] += ms;
    c->tcalls[p.cat] += 1;
    (void)hipEventDestroy(p.e0);
    (void)hipEventDestroy(p.e1);
  }
  c->pending.clear();
}

// get_Mg (smoothing.jl:12-25)
double get_Mg(scs_ctx* c, double Mh, double nu, double mu, int64_t n) {
  if (Mh < 0) fail(c, SCS_ERR_REF, "Mh must be nonnegative.");
  if (mu <= 0) fail(c, SCS_ERR_REF, "μ must be positive.");
  if (0 < nu && nu <= 3) return std::pow((double)n, (3 - nu) / 2) * std::pow(mu, nu / 2 - 2) * Mh;
  if (nu > 3) return std::pow(mu, 4 - 3 * nu / 2) * Mh;
  fail(c, SCS_ERR_REF, "ν must be positive.");
}

double jl_min_h(double x, double y) {
  auto isless = [](double a, double b) { return (a < b) || (std::signbit(a) && !std::signbit(b)); };
  return (std::isnan(x) || (!std::isnan(y) && isless(x, y))) ? x : y;
}

bool same_x(const std::vector<double>& key, const double* x, int64_t m) {
  return (int64_t)key.size() == m && std::memcmp(key.data(), x, sizeof(double) * m) == 0;
}

uint64_t xtag_of(const scs_ctx* c, const double* x) {
  for (const auto& t : c->xtags)
    if (t.p && t.p == x) return t.v;
  return 0;
}
// cache key (content `key` or tag `ktag`) matches the host vector x; x = nullptr: a device-only
// vector (a line-search trial point) that never hits and is keyed by a fresh tag
bool key_hit(const scs_ctx* c, const std::vector<double>& key, uint64_t ktag, const double* x) {
  if (!x) return false;
  const uint64_t t = xtag_of(c, x);
  if (t) return ktag == t;
  return ktag == 0 && same_x(key, x, c->m);
}
void key_set(scs_ctx* c, std::vector<double>& key, uint64_t& ktag, const double* x) {
  if (!x) {
    key.clear();
    ktag = c->xtag_next++;
    return;
  }
  ktag = xtag_of(c, x);
  if (ktag)
    key.clear();
  else
    key.assign(x, x + c->m);
}

ProxArgsH prox_args(scs_ctx* c) {
  ProxArgsH P;
  P.reg = c->reg;
  P.use_prox = c->use_prox;
  P.lam = c->lam;
  P.lam2 = c->lam2;
  P.lb = c->clb;
  P.ub = c->cub;
  P.gstart = c->gstart;
  P.gend = c->gend;
  P.gw = c->gw;
  P.ngroups = c->ngroups;
  P.gmap = c->gmap;
  return P;
}

void require_ready(scs_ctx* c, bool need_method) {
  if (!c->has_data) fail(c, SCS_ERR_STATE, "no data: call scs_set_data / scs_gen_data first");
  if (!c->loss_set) fail(c, SCS_ERR_STATE, "no loss: call scs_set_loss first");
  if (!c->reg_set) fail(c, SCS_ERR_STATE, "no regularizer: call scs_set_reg first");
  if (need_method && !c->smooth_set) fail(c, SCS_ERR_STATE, "no smoother: call scs_set_smoother first");
  if (need_method && !c->method_set) fail(c, SCS_ERR_STATE, "no method: call scs_method_init first");
}

// the exchange step is active: several ranks, or one rank with the exchange forced
bool sharded(const scs_ctx* c) { return c->nranks > 1 || c->comm_force; }

// doubles of the in-place all-reduce payload: packed Gram tiles ‖ Aᵀv (GGN / NSCORE), the
// m-vector (LQN), or the all-gather of the rows for the sharded GGN sample-space branch
int64_t reduce_buffer_doubles(const scs_ctx* c) {
  const int64_t nb = c->mpad / 128;
  const int64_t tsz = (nb * (nb + 1) / 2 + nb) * 128 * 128;   // 128 x 128 slots (tall lists add <= nb)
  int64_t need = std::max<int64_t>(tsz + c->mpad, c->mpad);
  // GGN sample-space branch across ranks: the all-gather of the rows (Ng x m_pad) and y of the
  // full data when N_global + 1 <= m, and of every registered batch whose global size b has
  // b + 1 <= m -- sized from those sizes, not from m (the buffer outlives view swaps; a new batch
  // list that needs more reallocates a library-owned buffer, scs_set_batches)
  int64_t ng = 0;
  if (c->Nglob_data + 1 <= c->m) ng = c->Nglob_data;
  for (int64_t b : c->bglob)
    if (b + 1 <= c->m) ng = std::max(ng, b);
  if (c->bsel < 0 && c->Nglob + 1 <= c->m) ng = std::max(ng, c->Nglob);
  if (ng > 0) {
    const int64_t Ng = round_up(ng, 16);
    need = std::max<int64_t>(need, Ng * c->mpad + Ng);
  }
  return need + 64;
}

// the payload buffer: the caller's (scs_set_reduce_buffer) or one the library owns
void ensure_red(scs_ctx* c) {
  if (c->red || !sharded(c)) return;
  if (!c->has_data) fail(c, SCS_ERR_STATE, "the reduce buffer needs the data dimensions");
  const int64_t need = reduce_buffer_doubles(c);
  c->red = dalloc<double>(c, need);
  c->red_cap = need;
  c->own_red = true;
}

void allreduce(scs_ctx* c, double* buf, int64_t count) {
  if (!sharded(c)) return;
  if (buf != c->red) fail(c, SCS_ERR_COMM, "internal: all-reduce payload must live in the reduce buffer");
  if (count > c->red_cap) fail(c, SCS_ERR_COMM, "reduce buffer too small (%lld < %lld doubles)",
                               (long long)c->red_cap, (long long)count);
  hipEvent_t e0;
  tbegin(c, T_REDUCE, &e0);
  if (c->comm_abort && c->comm_abort->load(std::memory_order_acquire))
    fail(c, SCS_ERR_COMM, "the multi-device context's communicators were aborted by a failing device");
  // fault injection for the abort path's tests: this rank's exchanges fail (read per call)
  if (const char* fe = std::getenv("SCS_FAULT_EXCHANGE_RANK"))
    if (c->nranks > 1 && std::atoi(fe) == c->rank) fail(c, SCS_ERR_COMM, "injected exchange failure at rank %d", c->rank);
  if (c->rccl) {   // in place, on the context stream (one fp64 sum per exchange)
    const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, c->rccl, c->st);
    if (r != ncclSuccess) fail(c, SCS_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
    // RCCL launches its kernel on c->st, so the events around it time it.  At world 1 the in-place
    // all-reduce launches nothing (0.02 ms, profiles/r05/rccltrace/: no RCCL kernel on any queue);
    // the +7 ms the r04 verdict saw in `solve` with RCCL forced was the factor's two streams sharing
    // one hardware queue once torch and RCCL had created theirs (chol.hip, create_chain_stream).
    // The empty dispatch keeps the end event behind the collective should RCCL ever join c->st by a
    // stream wait instead (an event recorded right after a wait takes the last dispatch's time).
    if (c->timing) HCK(launch_marker(c->st));
  } else {
    if (!c->ar) fail(c, SCS_ERR_COMM, "multi-rank context without a communicator");
    int rc = c->ar(buf, count, (void*)c->st, c->ar_user);
    if (rc != 0) fail(c, SCS_ERR_COMM, "all-reduce callback returned %d", rc);
  }
  tend(c, T_REDUCE, e0);
}

// ---------------------------------------------------------------------------
// workspace
// ---------------------------------------------------------------------------
void alloc_mspace(scs_ctx* c) {
  const int64_t mp = c->mpad;
  double** vs[] = {&c->x, &c->xp, &c->xn, &c->dxv, &c->gr, &c->Hr, &c->hinv, &c->zb, &c->d,
                   &c->gq, &c->gqn, &c->gtmp, &c->gtmp2, &c->q, &c->gcache[0], &c->gcache[1], &c->rbk};
  for (double** v : vs) {
    dfree_t(c, *v);
    *v = dalloc<double>(c, mp);
  }
  dfree_t(c, c->cinfo);
  c->cinfo = dalloc<int>(c, 1);   // factorization info (Cholesky pivot check, LU zero pivot, NaN scan)
  dfree_t(c, c->scal);
  // scalars + the partials of the multi-workgroup tail / L-BFGS update (64..), get_reg (64 + 2·256)
  // and the loop norms (64 + 3·256)
  c->scal = dalloc<double>(c, 64 + 6 * 256);
  dfree_t(c, c->xstar);
  c->xstar = dalloc<double>(c, mp);
  dfree_t(c, c->lqR);
  c->lqR = dalloc<double>(c, (size_t)LQ_NPART * LQ_G);
  if (!c->hscal) HCK(hipHostMalloc((void**)&c->hscal, 64 * sizeof(double), hipHostMallocDefault));
  if (!c->hserr) {
    HCK(hipHostMalloc((void**)&c->hserr, sizeof(int), hipHostMallocDefault));
    *c->hserr = 0;
  }
  if (!c->hloop) {   // written by kernels (lqn_post): fine-grained, device-mapped
    HCK(hipHostMalloc((void**)&c->hloop, 2 * LOOP_SLOTS * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped));
    HCK(hipHostGetDevicePointer((void**)&c->hloop_dev, c->hloop, 0));
  }
}

void alloc_nspace(scs_ctx* c) {
  if (c->generic) return;
  c->nsplit = c->sparse ? c->bcsr.nblk : gemv_n_splits(c->Npad, c->m);
  c->nval = epilogue_blocks(c->Npad);
  c->nchunk = c->sparse ? c->bcsc.nblk : gemv_t_chunks(c->Npad);
  dfree_t(c, c->zpart);
  dfree_t(c, c->z);
  dfree_t(c, c->gN);
  dfree_t(c, c->hN);
  dfree_t(c, c->wN);
  dfree_t(c, c->vN);
  dfree_t(c, c->valpart);
  dfree_t(c, c->tpart);
  c->zpart = dalloc<double>(c, (size_t)c->nsplit * c->Npad);
  c->z = dalloc<double>(c, c->Npad);
  c->gN = dalloc<double>(c, c->Npad);
  c->hN = dalloc<double>(c, c->Npad);
  c->wN = dalloc<double>(c, c->Npad);
  c->vN = dalloc<double>(c, c->Npad);
  c->valpart = dalloc<double>(c, c->nval);
  c->tpart = dalloc<double>(c, (size_t)c->nchunk * c->mpad);
}

void ensure_gram(scs_ctx* c) {
  if (c->G) return;
  const int64_t mp = c->mpad;
  c->G = dalloc<double>(c, (size_t)mp * mp);
  c->Gc = dalloc<double>(c, (size_t)mp * mp);
  const int nb = (int)(mp / 128);
  std::vector<int2> tl((size_t)nb * (nb + 1) / 2 + nb), ul;
  int nt = 0;
  const char* sq = std::getenv("SCS_GRAM_TALL");
  // 256 x 128 tiles from m = 12288 on (interleaved kernels: C3 73-74 TF/s; at m = 8192 the 128 x 128
  // tiles with 2 workgroups / CU are ~1 % faster, 72.5 vs 71.6 TF/s at C2)
  c->tall = (nb % 2 == 0) && nb >= 96 && !(sq && sq[0] == '0');
  if (sq && sq[0] == '1') c->tall = (nb % 2 == 0);
  if (c->tall) {
    gram_tile_list_tall(nb, tl.data(), &nt);
    ul.resize(2 * (size_t)nt);
    for (int t = 0; t < nt; ++t) {
      ul[2 * t] = make_int2(2 * tl[t].x, tl[t].y);
      ul[2 * t + 1] = make_int2(2 * tl[t].x + 1, tl[t].y);
    }
  } else {
    gram_tile_list(nb, tl.data(), &nt);
    ul.assign(tl.begin(), tl.begin() + nt);
  }
  c->tiles = dalloc<int2>(c, nt);
  HCK(hipMemcpyAsync(c->tiles, tl.data(), sizeof(int2) * nt, hipMemcpyHostToDevice, c->st));
  c->ntiles = nt;
  c->nslots = (int)ul.size();
  {
    const char* ev = std::getenv("SCS_GRAM_SCHED");
    if (!(ev && ev[0] == '0')) {
      std::vector<int4> wk, cb;
      int npart = 0;
      // the AV launches' designated tiles first in each XCD's order on 256 x 128 tiles (C3 Gram
      // 3863.7 -> 3846.6 ms); on 128 x 128 tiles it measured slower (C2 Gram +0.3 ms unfused, +0.9 fused;
      // profiles/r05/diagfirst/).  SCS_GRAM_DIAGFIRST=0 / 1: off / also on 128 x 128 tiles (A/B)
      const char* df = std::getenv("SCS_GRAM_DIAGFIRST");
      const int dfg = (df && df[0] == '0') ? 0 : c->tall ? 256 : (df && df[0] == '1') ? 128 : 0;
      c->gseglen = gram_schedule(tl.data(), nt, 32 * (c->tall ? 1 : 2), wk, cb, &c->gnsplit, &npart, dfg);
      c->gncomb = (int)cb.size();
      c->gwork = dalloc<int4>(c, wk.size());
      HCK(hipMemcpyAsync(c->gwork, wk.data(), sizeof(int4) * wk.size(), hipMemcpyHostToDevice, c->st));
      if (c->gncomb > 0) {
        c->gcomb = dalloc<int4>(c, cb.size());
        HCK(hipMemcpyAsync(c->gcomb, cb.data(), sizeof(int4) * cb.size(), hipMemcpyHostToDevice, c->st));
        c->gpart = dalloc<double>(c, (size_t)npart * (c->tall ? 256 : 128) * 128);
      }
    }
  }
  {
    // the strips of the pipeline: tiles whose column block (bj, 128-wide) lies in outer strip s
    const int OB = chol_outer_block(), ns = (nb + OB - 1) / OB;
    c->gstrip.assign(ns, scs_ctx::GStrip());
    c->vpieces = std::max(c->gnsplit, 1);
    int npart_max = 0;
    for (int s2 = 0; s2 < ns; ++s2) {
      std::vector<int2> st;
      for (int t = 0; t < nt; ++t)
        if (tl[t].y / OB == s2) st.push_back(tl[t]);
      std::vector<int4> wk, cb;
      int nsplit = 1, npart = 0;
      scs_ctx::GStrip& g = c->gstrip[s2];
      g.seglen = gram_schedule(st.data(), (int)st.size(), 32 * (c->tall ? 1 : 2), wk, cb, &nsplit, &npart);
      g.nsplit = nsplit;
      g.ncomb = (int)cb.size();
      g.work = dalloc<int4>(c, wk.size());
      HCK(hipMemcpyAsync(g.work, wk.data(), sizeof(int4) * wk.size(), hipMemcpyHostToDevice, c->st));
      if (!cb.empty()) {
        g.comb = dalloc<int4>(c, cb.size());
        HCK(hipMemcpyAsync(g.comb, cb.data(), sizeof(int4) * cb.size(), hipMemcpyHostToDevice, c->st));
      }
      npart_max = std::max(npart_max, npart);
      c->vpieces = std::max(c->vpieces, nsplit);
    }
    // the one-launch schedule: strips 0 .. ns-2 cut into 8 contiguous per-XCD chunks (no split),
    // the last strip as gram_schedule lays it out (tail pieces + combine items)
    {
      const int slots = 32 * (c->tall ? 1 : 2);
      std::vector<std::vector<int4>> seg(8);
      c->gp_target.assign(ns, 0u);
      std::vector<int4> cbl;
      int nsplit = 1, npart = 0;
      for (int s2 = 0; s2 < ns; ++s2) {
        std::vector<int2> st;
        std::vector<int> ix;
        for (int t = 0; t < nt; ++t)
          if (tl[t].y / OB == s2) {
            st.push_back(tl[t]);
            ix.push_back(t);
          }
        const int n = (int)st.size();
        if (s2 + 1 < ns) {
          c->gp_target[s2] = (unsigned)n;
          const int q = n / 8, r = n % 8;
          int t0 = 0;
          for (int x = 0; x < 8; ++x) {
            const int nx = q + (x < r ? 1 : 0);
            for (int i = 0; i < nx; ++i) seg[x].push_back(make_int4(st[t0 + i].x, st[t0 + i].y, -1, ix[t0 + i]));
            t0 += nx;
          }
        } else {
          std::vector<int4> wk;
          const int sl = gram_schedule(st.data(), n, slots, wk, cbl, &nsplit, &npart);
          for (int x = 0; x < 8; ++x)
            for (int i = 0; i < sl; ++i) {
              int4 it = wk[(size_t)x * sl + i];
              if (it.x < 0) continue;
              if (it.z < 0) it.w = ix[it.w];   // whole tile: its canonical index
              seg[x].push_back(it);
            }
          for (auto& cb : cbl) cb.z = ix[cb.z];
        }
      }
      size_t seglen = 0;
      for (auto& v : seg) seglen = std::max(seglen, v.size());
      std::vector<int4> wk(8 * seglen, make_int4(-1, -1, -1, -1));
      for (int x = 0; x < 8; ++x)
        for (size_t i = 0; i < seg[x].size(); ++i) wk[x * seglen + i] = seg[x][i];
      scs_ctx::GStrip& g = c->gpipe;
      g.seglen = (int)seglen;
      g.nsplit = nsplit;
      g.ncomb = (int)cbl.size();
      g.work = dalloc<int4>(c, wk.size());
      HCK(hipMemcpyAsync(g.work, wk.data(), sizeof(int4) * wk.size(), hipMemcpyHostToDevice, c->st));
      if (!cbl.empty()) {
        g.comb = dalloc<int4>(c, cbl.size());
        HCK(hipMemcpyAsync(g.comb, cbl.data(), sizeof(int4) * cbl.size(), hipMemcpyHostToDevice, c->st));
      }
      npart_max = std::max(npart_max, npart);
      c->vpieces = std::max(c->vpieces, nsplit);
      c->gp_cnt = dalloc<unsigned>(c, ns);
      c->gp_flag = dalloc<int>(c, 1);
      HCK(hipMemsetAsync(c->gp_flag, 0, sizeof(int), c->st));
    }
    if (npart_max > 0) {
      const size_t need = (size_t)npart_max * (c->tall ? 256 : 128) * 128;
      // gpart is shared with the one-launch schedule: size it for the larger user
      size_t have = 0;
      for (auto& a : c->allocs)
        if (a.p == c->gpart) have = a.bytes / sizeof(double);
      if (need > have) {
        if (c->gpart) dfree_t(c, c->gpart);
        c->gpart = dalloc<double>(c, need);
      }
    }
  }
  c->vpart = dalloc<double>(c, (size_t)c->vpieces * mp);
  c->utiles = dalloc<int2>(c, ul.size());
  HCK(hipMemcpyAsync(c->utiles, ul.data(), sizeof(int2) * ul.size(), hipMemcpyHostToDevice, c->st));
  {
    const int nb2 = (int)(mp / 128);
    c->W = dalloc<double>(c, (size_t)mp * 128);
    c->ysol = dalloc<double>(c, mp);
    std::vector<int2> tr((size_t)nb2 * (nb2 + 1) / 2);
    gram_tile_list_rowmajor(nb2, tr.data());
    c->trilist = dalloc<int2>(c, tr.size());
    HCK(hipMemcpyAsync(c->trilist, tr.data(), sizeof(int2) * tr.size(), hipMemcpyHostToDevice, c->st));
    HCK(chol_aux_init(&c->caux, mp, c->st));
  }
  sync(c);
}

void invalidate_caches(scs_ctx* c) {
  c->zvalid = false;
  c->zf_pending = false;
  c->gvalid[0] = c->gvalid[1] = false;
}

// ---------------------------------------------------------------------------
// f / ∇f building blocks
// ---------------------------------------------------------------------------
// finalize a loss sum: the per-kind constant of f (see epilogue_kernel)
// exchange the context's N-dependent fields with v (the full data <-> a minibatch)
void swap_view(scs_ctx* c, NView& v) {
  ++c->data_gen;
  std::swap(c->sparse, v.sparse);
  std::swap(c->A, v.A);
  std::swap(c->y, v.y);
  std::swap(c->N, v.N);
  std::swap(c->Npad, v.Npad);
  std::swap(c->nstage, v.nstage);
  std::swap(c->Nglob, v.Nglob);
  std::swap(c->nsplit, v.nsplit);
  std::swap(c->nval, v.nval);
  std::swap(c->nchunk, v.nchunk);
  for (auto pr : {std::make_pair(&c->zpart, &v.zpart), std::make_pair(&c->z, &v.z), std::make_pair(&c->gN, &v.gN),
                  std::make_pair(&c->hN, &v.hN), std::make_pair(&c->wN, &v.wN), std::make_pair(&c->vN, &v.vN),
                  std::make_pair(&c->valpart, &v.valpart), std::make_pair(&c->tpart, &v.tpart),
                  std::make_pair(&c->At, &v.At), std::make_pair(&c->Ps, &v.Ps), std::make_pair(&c->Ms, &v.Ms),
                  std::make_pair(&c->bS, &v.bS), std::make_pair(&c->uN, &v.uN), std::make_pair(&c->hvec, &v.hvec),
                  std::make_pair(&c->hg, &v.hg)})
    std::swap(*pr.first, *pr.second);
  std::swap(c->NpS, v.NpS);
  std::swap(c->stiles, v.stiles);
  std::swap(c->nstiles, v.nstiles);
  std::swap(c->n1pad, v.n1pad);
}

void free_view(scs_ctx* c, NView& v) {
  for (double** p : {&v.A, &v.y, &v.zpart, &v.z, &v.gN, &v.hN, &v.wN, &v.vN, &v.valpart, &v.tpart, &v.At, &v.Ps,
                     &v.Ms, &v.bS, &v.uN, &v.hvec, &v.hg})
    dfree_t(c, *p);
  dfree_t(c, v.stiles);
  v = NView();
}

// the held-out view <-> the context's data fields (f's fields only: rows, y, the products'
// workspace and, for a sparse set, the CSR arrays and the SpMV's blocked copy).  Not a data
// change: the data generation (the Gram cache's key) and the product kernel name are kept.
void swap_test(scs_ctx* c) {
  auto& t = c->tset;
  const uint64_t gen = c->data_gen;
  swap_view(c, t.v);
  c->data_gen = gen;
  std::swap(c->sp_f32, t.sp_f32);
  std::swap(c->nnz, t.nnz);
  std::swap(c->bcsr, t.bcsr);
  std::swap(c->rowptr, t.rowptr);
  std::swap(c->colidx, t.colidx);
  std::swap(c->val, t.val);
}

struct TestScope {
  scs_ctx* c;
  std::string pk;
  explicit TestScope(scs_ctx* cc) : c(cc), pk(cc->prod_kname) { swap_test(c); }
  ~TestScope() {
    swap_test(c);
    c->prod_kname = pk;
  }
};

void free_test(scs_ctx* c) {
  auto& t = c->tset;
  free_view(c, t.v);
  dfree_t(c, t.bcsr.ptr);
  dfree_t(c, t.bcsr.lidx);
  dfree(c, t.bcsr.val);
  t.bcsr = scs_ctx::SpBlk();
  dfree_t(c, t.rowptr);
  dfree_t(c, t.colidx);
  dfree(c, t.val);
  t.nnz = 0;
  t.sp_f32 = 0;
  t.on = t.host = t.xor_case = false;
}

// scs_step on the selected minibatch view: swapped in (and the data-keyed caches dropped) for
// the call, swapped back even when the step fails
struct BatchScope {
  scs_ctx* c;
  int k;
  explicit BatchScope(scs_ctx* cc) : c(cc), k(cc->bview) {
    if (k >= 0) {
      swap_view(c, c->bpool[k]);
      invalidate_caches(c);
    }
  }
  ~BatchScope() {
    if (k >= 0) {
      swap_view(c, c->bpool[k]);
      invalidate_caches(c);
    }
  }
};

void clear_batches(scs_ctx* c) {
  // the gathered rows of a batch index belong to the list they came from: a new list (a
  // reshuffle, another slice) must not reuse them
  ++c->batch_gen;
  if (c->gview_ok && c->gview_batch >= 0) {
    free_view(c, c->gview);
    c->gview = NView();
    c->gview_ok = false;
  }
  for (NView& v : c->bpool) free_view(c, v);
  c->bpool.clear();
  c->bheld.clear();
  c->boff.clear();
  c->bglob.clear();
  c->bpos.clear();
  dfree_t(c, c->brows);
  c->bview = -1;
  c->bsel = -1;
}

// select batch b (-1: the full data) for the following steps: its size's pool view is
// allocated on first use (A / y rows + the sample-space workspace sized by its own Npad)
// and re-gathered only when it holds another batch
void select_batch(scs_ctx* c, int64_t b) {
  c->bview = -1;
  c->bsel = b < 0 ? -1 : b;
  if (b < 0) return;
  // f(A, y, x) = 1/2 x'(A x) + y'x reads A as an m x m operator, not as samples
  if (c->loss == SCS_LOSS_QUADRATIC) fail(c, SCS_ERR_ARG, "the quadratic loss has no samples to batch");
  const int64_t n = c->boff[b + 1] - c->boff[b], ng = c->bglob[b];
  int k = -1;
  for (int i = 0; i < (int)c->bpool.size(); ++i)
    if (c->bpool[i].N == n && c->bpool[i].Nglob == ng) k = i;
  if (k < 0) {
    NView v;
    v.N = n;
    v.Nglob = ng;
    // a rank that owns none of the batch's rows keeps one zero 16-row stage (the kernels mask
    // rows >= N, so it contributes nothing to the exchanged sums)
    v.Npad = round_up(std::max<int64_t>(n, 1), 16);
    v.nstage = v.Npad / 16;
    v.A = dalloc<double>(c, (size_t)v.Npad * c->mpad);
    v.y = dalloc<double>(c, v.Npad);
    swap_view(c, v);
    alloc_nspace(c);
    swap_view(c, v);
    c->bpool.push_back(v);
    c->bheld.push_back(-1);
    k = (int)c->bpool.size() - 1;
  }
  if (c->bheld[k] != b) {
    NView& v = c->bpool[k];
    if (n == 0) {
      HCK(hipMemsetAsync(v.A, 0, sizeof(double) * (size_t)v.Npad * c->mpad, c->st));
      HCK(hipMemsetAsync(v.y, 0, sizeof(double) * v.Npad, c->st));
    } else if (c->sparse) {   // CSR rows -> the dense batch (the reference's Matrix(As') of a sparse A)
      HCK(hipMemsetAsync(v.A, 0, sizeof(double) * (size_t)v.Npad * c->mpad, c->st));
      HCK(launch_densify_rows(c->rowptr, c->colidx, c->val, c->sp_f32, c->brows + c->boff[b], n, v.Npad, c->y,
                              v.A, v.y, c->st));
    } else {
      HCK(launch_gather_rows(c->A, c->Npad, c->y, c->brows + c->boff[b], n, v.Npad, c->mpad, v.A, v.y, c->st));
    }
    // the view's GGN sample-space Aᵀ copy (built once per A, ggn_sample_step) follows its rows
    if (v.At) HCK(launch_transpose(v.A, v.Npad, n, c->m, v.At, c->mpad, v.NpS, c->st));
    c->bheld[k] = b;
  }
  c->bview = k;
}

double loss_scale_value(scs_ctx* c, double s) {
  switch (c->loss) {
    case SCS_LOSS_LOGISTIC_MARGIN: return c->scale * s;
    case SCS_LOSS_LOGISTIC_CE: return -c->scale * s;
    case SCS_LOSS_LEAST_SQUARES: return 0.5 * s * c->scale;
    default: return s;
  }
}

// z-partials of A x into c->zpart (dense: `nsplit` column splits; sparse: one
// CSR gather pass).  Returns the number of partials written.
int matvec_n(scs_ctx* c, const double* xd, int nsplit) {
  if (c->sparse) {
    const auto& B = c->bcsr;
    const int vk = c->sp_f32 ? (c->f32c ? 2 : 1) : 0;
    HCK(launch_spmv_blk(B.ptr, B.lidx, B.val, vk, xd, c->N, c->m, B.shift, c->nnz, c->zpart, c->Npad, c->st));
    c->prod_kname = spmv_kernel_name(vk);
    return B.nblk;
  }
  HCK(launch_gemv_n(c->A, c->nstage, c->Npad, c->mpad, xd, nsplit, c->zpart, c->Npad, c->st));
  return nsplit;
}

// the partial rows of Aᵀ v over the local rows into c->tpart (stride mpad); returns their count
int matvec_t_part(scs_ctx* c, const double* v) {
  if (c->sparse) {
    const auto& B = c->bcsc;
    const int vk = c->sp_f32 ? (c->f32c ? 2 : 1) : 0;
    HCK(launch_spmv_blk(B.ptr, B.lidx, B.val, vk, v, c->m, c->N, B.shift, c->nnz, c->tpart, c->mpad, c->st));
    return B.nblk;
  }
  HCK(launch_gemv_t(c->A, c->nstage, c->Npad, c->m, c->mpad, v, c->tpart, c->st));
  return c->nchunk;
}

// out (device, m) = Aᵀ v over the local rows (dense: chunked column sums +
// fixed-order finalize; sparse: one CSC gather pass)
void matvec_t(scs_ctx* c, const double* v, double* out) {
  const int np = matvec_t_part(c, v);
  HCK(launch_gemv_t_finalize(c->tpart, np, c->mpad, c->m, out, c->st));
}

void require_dense(scs_ctx* c, const char* what) {
  if (c->sparse)
    fail(c, SCS_ERR_ARG, "%s needs a dense A (sparse A supports f, ∇f and ProxLQNSCORE)", what);
}

// Forward pass at the device vector xd whose host copy is xh: z = A x (or the
// cached z), then the epilogue with `flags`.  Always refreshes the f-value
// cache; returns f(x) (global).
double forward(scs_ctx* c, const double* xh, const double* xd, int flags, bool need_val = true) {
  const bool cached = c->zvalid && key_hit(c, c->zkey, c->ztag, xh);
  hipEvent_t e0;
  if (!cached) {
    tbegin(c, T_GEMV, &e0);
    const int ns = matvec_n(c, xd, c->nsplit);
    tend(c, T_GEMV, e0);
    flags |= EPI_Z | EPI_VAL;
    HCK(launch_epilogue(c->loss, c->ggn, flags, c->zpart, ns, c->Npad, c->y, c->N, c->Npad, c->scale, c->z,
                        c->gN, c->hN, c->wN, c->vN, c->valpart, c->st));
    // loss sum -> scal[ZF_SLOT] (reduce buffer slot 0 in multi-rank); a slot of its own: the value
    // stays in flight until the next use (no host round trip when the caller only needs z)
    ensure_red(c);
    double* dst = sharded(c) ? c->red : c->scal + ZF_SLOT;
    HCK(launch_sum_partials(c->valpart, c->nval, dst, c->st));
    allreduce(c, c->red, 1);
    if (sharded(c)) HCK(hipMemcpyAsync(c->scal + ZF_SLOT, c->red, sizeof(double), hipMemcpyDeviceToDevice, c->st));
    d2h(c, c->hscal + ZF_SLOT, c->scal + ZF_SLOT, 1);
    c->zf_pending = true;
    key_set(c, c->zkey, c->ztag, xh);
    c->zvalid = true;
  } else if (flags & ~(EPI_VAL | EPI_Z)) {
    flags &= ~(EPI_Z | EPI_VAL);
    HCK(launch_epilogue(c->loss, c->ggn, flags, c->z, 1, c->Npad, c->y, c->N, c->Npad, c->scale, c->z, c->gN, c->hN,
                        c->wN, c->vN, c->valpart, c->st));
  }
  if (need_val && c->zf_pending) {
    sync(c);
    c->zfval = loss_scale_value(c, c->hscal[ZF_SLOT]);
    c->zf_pending = false;
  }
  return c->zfval;
}

// out (device, m) = Aᵀ v over the local rows (no reduction)
void gemv_t_local(scs_ctx* c, const double* v, double* out) {
  hipEvent_t e0;
  tbegin(c, T_GEMV, &e0);
  matvec_t(c, v, out);
  tend(c, T_GEMV, e0);
}

// out (device, m) = Aᵀ v (local, then all-reduced across ranks)
void gemv_t_global(scs_ctx* c, const double* v, double* out) {
  hipEvent_t e0;
  tbegin(c, T_GEMV, &e0);
  ensure_red(c);
  matvec_t(c, v, sharded(c) ? c->red : out);
  tend(c, T_GEMV, e0);
  if (sharded(c)) {
    allreduce(c, c->red, c->m);
    HCK(hipMemcpyAsync(out, c->red, sizeof(double) * c->m, hipMemcpyDeviceToDevice, c->st));
  }
}

// SCS_LOSS_CALLBACK: call the caller's loss with x (the host copy xh, or xd downloaded) and
// return the host output area (nout doubles) of the pinned exchange buffer.  The stream is
// drained first: the previous upload from the buffer must have landed before it is reused.
double* cb_eval(scs_ctx* c, int what, const double* xh, const double* xd, size_t nout) {
  if (!c->cb) fail(c, SCS_ERR_STATE, "no loss callback: call scs_set_loss_callback");
  const int64_t m = c->m;
  const size_t need = (size_t)m + nout;
  sync(c);
  if (need > c->cbh_cap) {
    if (c->cbh) HCK(hipHostFree(c->cbh));
    c->cbh = nullptr;
    c->cbh_cap = 0;
    HCK(hipHostMalloc((void**)&c->cbh, need * sizeof(double), hipHostMallocDefault));
    c->cbh_cap = need;
  }
  double* xb = c->cbh;
  if (xh) {
    std::memcpy(xb, xh, sizeof(double) * m);
  } else {
    d2h(c, xb, xd, m);
    sync(c);
  }
  const int rc = c->cb(c->cb_user, what, xb, m, xb + m);
  if (rc == SCS_CB_NO_METHOD && what == SCS_CB_GRAD_X)   // prox-GGN-SCORE.jl:59 called grad_fx(x)
    fail(c, SCS_ERR_REF, "MethodError: no method matching grad_fx(::Vector{Float64}) (ProxGGNSCORE calls "
                         "model.grad_fx(x) with one argument in its ss_type 3 line search, "
                         "prox-GGN-SCORE.jl:58-59,83-84)");
  if (rc != 0) fail(c, SCS_ERR_CALLBACK, "loss callback (what = %d) returned %d", what, rc);
  return xb + m;
}

// f(x) for a device vector with host copy xh
double eval_f_dev(scs_ctx* c, const double* xh, const double* xd) {
  if (c->loss == SCS_LOSS_CALLBACK) return cb_eval(c, SCS_CB_F, xh, xd, 1)[0];
  if (c->loss == SCS_LOSS_ROSENBROCK) {
    HCK(launch_rosen(xd, c->m, 0, c->scal + 8, nullptr, 0, c->st));
    d2h(c, c->hscal + 8, c->scal + 8, 1);
    sync(c);
    return c->hscal[8];
  }
  if (c->loss == SCS_LOSS_QUADRATIC) {
    // 1/2*(x'*(A*x)) + y'*x
    require_dense(c, "the quadratic loss");
    HCK(launch_gemv_n(c->A, c->nstage, c->Npad, c->mpad, xd, 1, c->zpart, c->Npad, c->st));
    HCK(launch_dot(xd, c->zpart, c->m, c->scal + 8, c->st));
    HCK(launch_dot(c->y, xd, c->m, c->scal + 9, c->st));
    d2h(c, c->hscal + 8, c->scal + 8, 2);
    sync(c);
    return 0.5 * c->hscal[8] + c->hscal[9];
  }
  return forward(c, xh, xd, 0);
}

// ftest(x) = f(Atest, ytest, x) (iterate.jl:173) at the device vector xd, enqueued: the loss sum of
// the held-out rows lands in scal[TF_SLOT] (all-reduced across ranks for a row-sharded test set);
// loss_scale_value(hscal / hloop[TF_SLOT]) is the value.  The same products and epilogue as f(x),
// on the held-out view; the z / f caches of the data are not touched.
void ftest_enqueue(scs_ctx* c, const double* xd) {
  ensure_red(c);   // sized by the data's view, before the held-out one is swapped in
  TestScope ts(c);
  const int ns = matvec_n(c, xd, c->nsplit);
  HCK(launch_epilogue(c->loss, c->ggn, EPI_VAL, c->zpart, ns, c->Npad, c->y, c->N, c->Npad, c->scale, c->z, c->gN,
                      c->hN, c->wN, c->vN, c->valpart, c->st));
  double* dst = sharded(c) ? c->red : c->scal + TF_SLOT;
  HCK(launch_sum_partials(c->valpart, c->nval, dst, c->st));
  allreduce(c, c->red, 1);
  if (sharded(c)) HCK(hipMemcpyAsync(c->scal + TF_SLOT, c->red, sizeof(double), hipMemcpyDeviceToDevice, c->st));
}

// ftest(x) now (host copy xh, may be null, and device copy xd)
double eval_ftest_dev(scs_ctx* c, const double* xh, const double* xd) {
  if (!c->tset.on) fail(c, SCS_ERR_STATE, "no test data: call scs_set_test_data first");
  if (c->tset.host) return cb_eval(c, SCS_CB_FTEST, xh, xd, 1)[0];
  if (c->loss == SCS_LOSS_QUADRATIC) {   // 1/2*(x'*(Atest*x)) + ytest'*x
    // Atest*x and x' need Atest to be m x m (and ytest length m); Julia raises DimensionMismatch.
    // The test view holds only its own rows, so a non-square Atest must not reach eval_f_dev
    if (c->tset.v.Nglob != c->m)
      fail(c, SCS_ERR_ARG, "DimensionMismatch: the quadratic loss 1/2*(x'*(Atest*x)) + ytest'*x needs an m x m "
                           "Atest (m = %lld), got %lld rows", (long long)c->m, (long long)c->tset.v.Nglob);
    TestScope ts(c);
    return eval_f_dev(c, xh, xd);
  }
  ftest_enqueue(c, xd);
  d2h(c, c->hscal + TF_SLOT, c->scal + TF_SLOT, 1);
  sync(c);
  return loss_scale_value(c, c->hscal[TF_SLOT]);
}

// ∇f(x) -> out (device)
// (cb_what: SCS_CB_GRAD = grad_fx(A, y, x); SCS_CB_GRAD_X = ProxGGNSCORE's one-argument call)
void grad_f_dev(scs_ctx* c, const double* xh, const double* xd, double* out, int cb_what = SCS_CB_GRAD) {
  if (c->gfix) {   // step!(...; ∇fx): grad_f = x -> ∇fx at every point (prox-L-BFGS-SCORE.jl:98-100)
    if (out != c->gfix) HCK(hipMemcpyAsync(out, c->gfix, sizeof(double) * c->m, hipMemcpyDeviceToDevice, c->st));
    return;
  }
  if (c->loss == SCS_LOSS_CALLBACK) {
    const double* g = cb_eval(c, cb_what, xh, xd, c->m);
    HCK(hipMemcpyAsync(out, g, sizeof(double) * c->m, hipMemcpyHostToDevice, c->st));
    return;
  }
  if (c->loss == SCS_LOSS_ROSENBROCK) {
    HCK(launch_rosen(xd, c->m, 1, out, nullptr, 0, c->st));
    return;
  }
  if (c->loss == SCS_LOSS_QUADRATIC) {
    // 0.5*(A*x + Aᵀ*x) + y
    require_dense(c, "the quadratic loss");
    HCK(launch_gemv_n(c->A, c->nstage, c->Npad, c->mpad, xd, 1, c->zpart, c->Npad, c->st));
    gemv_t_global(c, xd, c->gtmp2);
    HCK(launch_axpby(c->zpart, 1.0, c->gtmp2, c->m, c->gtmp2, c->st));
    HCK(launch_axpby(c->y, 0.5, c->gtmp2, c->m, out, c->st));  // y + 0.5*(Ax + Aᵀx)
    return;
  }
  forward(c, xh, xd, EPI_GRAD, false);
  gemv_t_global(c, c->gN, out);
}

// ∇q(x) = ∇f(x) + λ hμ.grad(x) -> out (device); uses the 2-slot cache.
void grad_q_dev(scs_ctx* c, const double* xh, const double* xd, double* out, int cb_what = SCS_CB_GRAD) {
  // (a one-argument grad_fx call is always made: a cached grad_fx(A, y, x) must not stand in for it)
  const bool cacheable = !(c->loss == SCS_LOSS_CALLBACK && cb_what == SCS_CB_GRAD_X);
  for (int s = 0; s < 2 && cacheable; ++s)
    if (c->gvalid[s] && key_hit(c, c->gkey[s], c->gtag[s], xh)) {
      HCK(hipMemcpyAsync(out, c->gcache[s], sizeof(double) * c->m, hipMemcpyDeviceToDevice, c->st));
      return;
    }
  grad_f_dev(c, xh, xd, c->gtmp, cb_what);
  HCK(launch_smoother(c->smooth, xd, c->m, c->mu, c->slb, c->sub, c->wel, c->zb, c->hinv, c->st));
  HCK(launch_axpby(c->gtmp, c->lam, c->zb, c->m, out, c->st));
  if (!cacheable) return;
  const int s = c->gnext;
  c->gnext ^= 1;
  HCK(hipMemcpyAsync(c->gcache[s], out, sizeof(double) * c->m, hipMemcpyDeviceToDevice, c->st));
  key_set(c, c->gkey[s], c->gtag[s], xh);
  c->gvalid[s] = true;
}

double eval_reg_dev(scs_ctx* c, const double* xd) {
  HCK(launch_reg_value(prox_args(c), xd, c->m, c->scal + 10, c->scal + 64 + 2 * 256, c->st));
  d2h(c, c->hscal + 10, c->scal + 10, 1);
  sync(c);
  return c->hscal[10];
}

// linesearch (utils.jl:27-35): Armijo with ρ = 0.5, c = 1e-4 and no cap.
// obj(x) and grad_q(x) are evaluated once (the reference re-evaluates the
// same deterministic values on every trial).  For the data losses the trial's
// f(x + αd) is formed incrementally: A(x + αd) = Ax + α·Ad with
// Ax from f(x)'s forward pass and ONE extra pass for Ad, then O(N) per trial (the
// epilogue over z0 + α·zd) instead of a full pass over A per trial.  The values
// equal the direct form to rounding (SCS_LS_INCR=0 keeps the direct form).
bool ls_incremental(const scs_ctx* c) {
  const char* e = std::getenv("SCS_LS_INCR");   // read per call (A/B within one process)
  const bool off = e && e[0] == '0';
  return !off && !c->generic && (c->loss == SCS_LOSS_LOGISTIC_MARGIN || c->loss == SCS_LOSS_LOGISTIC_CE ||
                                 c->loss == SCS_LOSS_LEAST_SQUARES);
}

double line_search(scs_ctx* c, const double* xh, const double* xd, const double* dd) {
  const double f0 = eval_f_dev(c, xh, xd) + eval_reg_dev(c, xd);
  // ProxGGNSCORE's grad_f is x -> model.grad_fx(x), one argument (prox-GGN-SCORE.jl:58-59,83-84):
  // a callback loss is asked for that call (a data problem's grad_fx(A, y, x) raises MethodError)
  grad_q_dev(c, xh, xd, c->gqn, c->method == SCS_PROX_GGNSCORE ? SCS_CB_GRAD_X : SCS_CB_GRAD);
  HCK(launch_dot(c->gqn, dd, c->m, c->scal + 11, c->st));
  d2h(c, c->hscal + 11, c->scal + 11, 1);
  sync(c);
  const double gd = c->hscal[11];
  const bool incr = ls_incremental(c);
  double* zd = nullptr;
  double* pair = nullptr;
  if (incr) {
    // z0 = A x: f(x) above left it in c->z (forward with EPI_Z); A d once into zd
    forward(c, xh, xd, 0);
    if (c->lscap < 3 * c->Npad) {
      dfree_t(c, c->lsbuf);
      c->lsbuf = dalloc<double>(c, 3 * c->Npad);
      c->lscap = 3 * c->Npad;
    }
    pair = c->lsbuf;
    zd = c->lsbuf + 2 * c->Npad;
    hipEvent_t e0;
    tbegin(c, T_GEMV, &e0);
    const int ns = matvec_n(c, dd, c->nsplit);
    tend(c, T_GEMV, e0);
    HCK(launch_epilogue(c->loss, c->ggn, EPI_Z, c->zpart, ns, c->Npad, c->y, c->N, c->Npad, c->scale, zd, nullptr,
                        nullptr, nullptr, nullptr, c->valpart, c->st));
    ensure_red(c);
  }
  // the band (relative) within which an incremental trial is re-decided on the direct form;
  // SCS_LS_NEAR overrides it (tests: a huge band re-decides every trial).  The incremental form's own
  // rounding is one extra addition per z_i (<= eps·(|Ax|_i + α|Ad|_i)): ~1e-16 relative in f; both
  // forms share the dot products' rounding.  1e-12 leaves four orders of margin (the first r05
  // value, 1e-9, re-decided trials whose margin was a million times the incremental form's rounding)
  const char* ne = std::getenv("SCS_LS_NEAR");
  const double near = ne ? std::atof(ne) : 1e-12;
  double alpha = 1.0;
  for (int trial = 0; trial < 100000; ++trial) {
    // the trial point lives on the device only (no host copy: it is keyed by a fresh tag)
    HCK(launch_trial_point(xd, dd, alpha, c->m, c->gtmp2, c->st));
    double ft;
    if (incr) {
      HCK(launch_ls_pair(c->z, zd, alpha, c->Npad, pair, c->st));
      HCK(launch_epilogue(c->loss, c->ggn, EPI_VAL, pair, 2, c->Npad, c->y, c->N, c->Npad, c->scale, nullptr, nullptr,
                          nullptr, nullptr, nullptr, c->valpart, c->st));
      double* dst = sharded(c) ? c->red : c->scal + 14;
      HCK(launch_sum_partials(c->valpart, c->nval, dst, c->st));
      allreduce(c, c->red, 1);
      if (sharded(c)) HCK(hipMemcpyAsync(c->scal + 14, c->red, sizeof(double), hipMemcpyDeviceToDevice, c->st));
      d2h(c, c->hscal + 14, c->scal + 14, 1);
      const double rg = eval_reg_dev(c, c->gtmp2);   // syncs: hscal[14] has landed too
      ft = loss_scale_value(c, c->hscal[14]) + rg;
      // Ax + fl(α·Ad) differs from the reference's A·fl(x + αd) (utils.jl:27-35) in the last bits
      // of each z_i: a trial whose Armijo test sits within `near` (relative) of its threshold is
      // decided on the direct form instead, so the accepted α is the reference's form's
      if (std::fabs(ft - (f0 + 1e-4 * alpha * gd)) <= near * std::max(std::fabs(f0), std::fabs(ft))) {
        ft = eval_f_dev(c, nullptr, c->gtmp2) + eval_reg_dev(c, c->gtmp2);
        ++c->ls_direct;
        // that pass left A·(x + αd) in c->z: restore z0 = A x for the later incremental trials
        if (ft > f0 + 1e-4 * alpha * gd) forward(c, xh, xd, 0, false);
      }
    } else {
      ft = eval_f_dev(c, nullptr, c->gtmp2) + eval_reg_dev(c, c->gtmp2);
    }
    if (!(ft > f0 + 1e-4 * alpha * gd)) return alpha;
    alpha = 0.5 * alpha;
  }
  fail(c, SCS_ERR_REF, "linesearch did not terminate");
}

// solve (G + λ diag Hr) sol = rhs in place (rhs -> sol, length m_pad, zero-padded).
// Hand-written blocked Cholesky on MFMA (chol.hip) first; the hand-written blocked LU with
// partial pivoting (lu.hip; the reference's `\`, prox-N-SCORE.jl:70) from the saved copy when
// a pivot is not positive (e.g. the indefinite Q of a CE loss on ±1 labels,
// test/test_algs.jl:10), or always with force_lu (scs_solve_eval).
// SCS_FAULT_LATE (tests; read per call): a bit mask of the dependency waits to report as timed out,
// as the device would after ~30 s (never expected), so that each fallback below can be driven:
// 1 the one-launch triangular solves, 2 the QR's one-launch backward solve, 4 the dependency-driven
// Cholesky chain (SCS_CHOL_DAG=1), 8 the pipelined factor's strip wait (SCS_CHOL_PIPE).  The
// cooperative LU panel's own give-up path is driven on the device instead (SCS_LU_COOP_SPIN=0).
static bool fault_late(int bit) {
  const char* e = std::getenv("SCS_FAULT_LATE");
  return e && (std::atoi(e) & bit);
}

// lu_factor(M) with the cooperative panel's fallback (r06).  A panel launch the runtime refuses runs as
// column steps inside lu_factor; a candidate exchange that timed out (info = -1: a workgroup of the
// one-launch panel never became resident -- the plain launch mode, SCS_LU_COOP_LAUNCH=0, or a device
// shared with other work) leaves M undefined, so `rebuild` restores the system and the factorization
// is redone with the column-step panels, which give the same factor and pivots bit for bit
// (test_lu_coop_panel_largest_grid).  Returns the factorization's info (0, or the first zero pivot).
template <class F>
int lu_factor_checked(scs_ctx* c, double* M, int64_t ld, int64_t n, int64_t npad, int* dinfo, F&& rebuild) {
  int info = 0;
  const int64_t refused0 = c->lu.coop_refused;
  HCK(hipMemsetAsync(dinfo, 0, sizeof(int), c->st));
  HCK(lu_factor(M, ld, n, npad, &c->lu, dinfo, c->st));
  HCK(hipMemcpyAsync(&info, dinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
  sync(c);
  c->fb[SCS_FB_LU_COOP_REFUSED] += c->lu.coop_refused - refused0;
  if (info != -1) return info;
  ++c->fb[SCS_FB_LU_COOP_REDO];
  rebuild();
  c->lu.no_coop = true;
  HCK(hipMemsetAsync(dinfo, 0, sizeof(int), c->st));
  const hipError_t e = lu_factor(M, ld, n, npad, &c->lu, dinfo, c->st);
  c->lu.no_coop = false;
  HCK(e);
  HCK(hipMemcpyAsync(&info, dinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
  sync(c);
  if (info < 0) fail(c, SCS_ERR_HIP, "LU: info %d from the column-step panels", info);
  return info;
}

// chol_solve with the one-launch solves' fallback (r06): a dependency wait of chol_fwd/bwd_persist_kernel
// that gave up (~30 s, never expected: a block waits only on blocks dispatched before it) sets caux.serr
// and leaves rhs undefined; the solve is redone from the saved right-hand side by the per-block launches
// (SCS_SOLVE_PERSIST=0's form)
void chol_solve_checked(scs_ctx* c, double* rhs) {
  const int64_t ld = c->mpad;
  HCK(hipMemcpyAsync(c->rbk, rhs, sizeof(double) * ld, hipMemcpyDeviceToDevice, c->st));
  HCK(chol_solve(c->G, ld, ld, c->W, rhs, c->ysol, &c->caux, c->st));
  int late = 0;
  if (c->caux.serr) HCK(hipMemcpyAsync(&late, c->caux.serr, sizeof(int), hipMemcpyDeviceToHost, c->st));
  sync(c);
  if (!late && !fault_late(1)) return;
  if (c->caux.serr) HCK(hipMemsetAsync(c->caux.serr, 0, sizeof(int), c->st));
  ++c->fb[SCS_FB_SOLVE_BLOCKS];
  HCK(hipMemcpyAsync(rhs, c->rbk, sizeof(double) * ld, hipMemcpyDeviceToDevice, c->st));
  c->caux.no_persist = true;
  const hipError_t e = chol_solve(c->G, ld, ld, c->W, rhs, c->ysol, &c->caux, c->st);
  c->caux.no_persist = false;
  HCK(e);
}

// the LU fallback: the full symmetric system from the copy Gc (rebuilt from the cached Gram when
// this step's Gram came from the cache), the reference's `\` (prox-N-SCORE.jl:70)
void solve_lu_fallback(scs_ctx* c, double* rhs, hipEvent_t e0) {
  const int64_t m = c->m, ld = c->mpad;
  int info = 0;
  if (c->g_from_cache) {
    HCK(hipMemcpyAsync(c->Gc, c->Gk, sizeof(double) * ld * ld, hipMemcpyDeviceToDevice, c->st));
    HCK(launch_diag_add(c->Gc, c->mpad, m, c->lam, c->Hr, c->st));
  }
  // the full symmetric matrix: its column-major storage is also the row-major one lu.hip factors
  HCK(launch_symmetrize(c->Gc, ld, m, c->st));
  // a NaN / Inf in the system (a smoother's NaN, Appendix A) is no SingularException in the
  // reference: LAPACK getrf only flags exact zero pivots, and the solve comes out NaN
  HCK(hipMemsetAsync(c->cinfo, 0, sizeof(int), c->st));
  HCK(launch_nonfinite(c->Gc, ld, m, rhs, c->cinfo, c->st));
  HCK(hipMemcpyAsync(&info, c->cinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
  sync(c);
  c->lu_fallback_used = true;
  if (info != 0) {
    HCK(launch_fill(rhs, m, std::numeric_limits<double>::quiet_NaN(), c->st));
    tend(c, T_SOLVE, e0);
    return;
  }
  HCK(lu_aux_init(&c->lu, ld, c->st));
  // the system the factor overwrites, kept for a column-step redo (lu_factor_checked)
  if (c->Gbk_n != ld) {
    dfree_t(c, c->Gbk);
    c->Gbk = dalloc<double>(c, (size_t)ld * ld);
    c->Gbk_n = ld;
  }
  HCK(hipMemcpyAsync(c->Gbk, c->Gc, sizeof(double) * ld * ld, hipMemcpyDeviceToDevice, c->st));
  info = lu_factor_checked(c, c->Gc, ld, m, ld, c->cinfo, [&] {
    HCK(hipMemcpyAsync(c->Gc, c->Gbk, sizeof(double) * ld * ld, hipMemcpyDeviceToDevice, c->st));
  });
  if (info != 0) fail(c, SCS_ERR_SOLVE, "SingularException(%d)", info);
  HCK(lu_solve(c->Gc, ld, ld, &c->lu, rhs, c->st));
  tend(c, T_SOLVE, e0);
}

// solve (G + λ diag Hr) sol = rhs in place (rhs -> sol, length m_pad, zero-padded).
// Hand-written blocked Cholesky on MFMA (chol.hip) first; the hand-written blocked LU with
// partial pivoting (lu.hip; the reference's `\`, prox-N-SCORE.jl:70) from the saved copy when
// a pivot is not positive (e.g. the indefinite Q of a CE loss on ±1 labels,
// test/test_algs.jl:10), or always with force_lu (scs_solve_eval).
// the reference's own solver (scs_set_solver(SCS_SOLVER_REFERENCE)): qr(JQJ) \ Je by Householder QR
// (prox-GGN-SCORE.jl:131) on the symmetrized copy Gc; a NaN / Inf system gives a NaN direction
// Householder QR solve of the column-major npad x npad system A (identity-padded) with b := A \ b;
// a backward-solve dependency wait that gave up (~30 s, never expected) fails the call
// r06: the panels as cooperative launches (qr.hip qr_panel_coop_kernel) -- a refused launch runs that panel
// by column steps inside qr_solve; a sweep that gave up (cinfo = -1: a workgroup never became resident)
// leaves A and b undefined, so the solve is redone from the saved copy with the per-column launches
static void qr_run(scs_ctx* c, double* A, int64_t npad, double* b) {
  const bool coop = qr_coop_wanted(npad);
  const size_t nA = (size_t)npad * npad;
  if (coop) {
    if (c->qbk_n != npad) {
      dfree_t(c, c->qbk);
      c->qbk = dalloc<double>(c, nA + (size_t)npad);
      c->qbk_n = npad;
    }
    HCK(hipMemcpyAsync(c->qbk, A, sizeof(double) * nA, hipMemcpyDeviceToDevice, c->st));
    HCK(hipMemcpyAsync(c->qbk + nA, b, sizeof(double) * npad, hipMemcpyDeviceToDevice, c->st));
  }
  const int64_t refused0 = c->qr.coop_refused;
  HCK(qr_solve(A, npad, npad, &c->qr, b, c->st));
  int late = 0, cinfo = 0;
  HCK(hipMemcpyAsync(&late, c->qr.err, sizeof(int), hipMemcpyDeviceToHost, c->st));
  if (coop) HCK(hipMemcpyAsync(&cinfo, c->qr.cinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
  sync(c);
  c->fb[SCS_FB_QR_COOP_REFUSED] += c->qr.coop_refused - refused0;
  if (cinfo == -1) {
    ++c->fb[SCS_FB_QR_COOP_REDO];
    HCK(hipMemcpyAsync(A, c->qbk, sizeof(double) * nA, hipMemcpyDeviceToDevice, c->st));
    HCK(hipMemcpyAsync(b, c->qbk + nA, sizeof(double) * npad, hipMemcpyDeviceToDevice, c->st));
    c->qr.no_coop = true;
    const hipError_t e = qr_solve(A, npad, npad, &c->qr, b, c->st);
    c->qr.no_coop = false;
    HCK(e);
    HCK(hipMemcpyAsync(&late, c->qr.err, sizeof(int), hipMemcpyDeviceToHost, c->st));
    sync(c);
  }
  if (late || fault_late(2)) {
    // R is complete and qr.Ym still holds Qᵀb (the one-launch kernel only reads it): the backward
    // solve again by the per-block launches
    HCK(hipMemsetAsync(c->qr.err, 0, sizeof(int), c->st));
    ++c->fb[SCS_FB_QR_BLOCKS];
    HCK(chol_back_blocks(A, npad, npad, c->qr.W, c->qr.Ym, b, c->st));
  }
}

void solve_qr(scs_ctx* c, double* rhs, hipEvent_t e0) {
  const int64_t m = c->m, ld = c->mpad;
  if (c->g_from_cache) {
    HCK(hipMemcpyAsync(c->Gc, c->Gk, sizeof(double) * ld * ld, hipMemcpyDeviceToDevice, c->st));
    HCK(launch_diag_add(c->Gc, c->mpad, m, c->lam, c->Hr, c->st));
  }
  HCK(launch_symmetrize(c->Gc, ld, m, c->st));
  int info = 0;
  HCK(hipMemsetAsync(c->cinfo, 0, sizeof(int), c->st));
  HCK(launch_nonfinite(c->Gc, ld, m, rhs, c->cinfo, c->st));
  HCK(hipMemcpyAsync(&info, c->cinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
  sync(c);
  c->lu_fallback_used = false;
  if (info != 0) {
    HCK(launch_fill(rhs, m, std::numeric_limits<double>::quiet_NaN(), c->st));
    tend(c, T_SOLVE, e0);
    return;
  }
  HCK(qr_prepare(c->Gc, ld, m, ld, c->st));
  qr_run(c, c->Gc, ld, rhs);
  tend(c, T_SOLVE, e0);
}

void solve_system(scs_ctx* c, double* rhs, bool force_lu = false, bool force_qr = false) {
  const int64_t m = c->m, ld = c->mpad;
  hipEvent_t e0;
  tbegin(c, T_SOLVE, &e0);
  // the LU fallback needs the system the in-place factor destroys: copied up front, or -- when
  // this step's Gram came from the cache -- rebuilt from it only if the factor fails
  if (!c->g_from_cache) HCK(hipMemcpyAsync(c->Gc, c->G, sizeof(double) * ld * ld, hipMemcpyDeviceToDevice, c->st));
  if (c->solver == SCS_SOLVER_REFERENCE && !force_lu && !force_qr) {
    if (c->method == SCS_PROX_GGNSCORE) force_qr = true;   // qr(JQJ) \ Je
    else force_lu = true;                                  // (H + λHr) \ ∇q: Julia's `\` = LU
  }
  if (force_qr) {
    solve_qr(c, rhs, e0);
    return;
  }
  int info = 0;
  if (!force_lu) {
    HCK(hipMemsetAsync(c->cinfo, 0, sizeof(int), c->st));
    c->caux.chain_mode = c->rccl ? 2 : 0;   // RCCL's streams in the process: keep the factor's two apart
    HCK(chol_factor(c->G, ld, m, ld, c->W, &c->caux, c->trilist, c->cinfo, c->st));
    HCK(hipMemcpyAsync(&info, c->cinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
    int late = 0;   // a dependency wait of the chain launches gave up (~30 s): never expected
    HCK(hipMemcpyAsync(&late, c->caux.serr, sizeof(int), hipMemcpyDeviceToHost, c->st));
    sync(c);
    if (late || (fault_late(4) && chol_dag_active(&c->caux))) {
      // the factor is incomplete: the system again (Gc, or the cached Gram + λ diag Hr), and the
      // factor redone with one launch per operation (r06; was SCS_ERR_HIP)
      HCK(hipMemsetAsync(c->caux.serr, 0, sizeof(int), c->st));
      ++c->fb[SCS_FB_CHAIN_REDO];
      if (c->g_from_cache) {
        HCK(hipMemcpyAsync(c->G, c->Gk, sizeof(double) * ld * ld, hipMemcpyDeviceToDevice, c->st));
        HCK(launch_diag_add(c->G, c->mpad, m, c->lam, c->Hr, c->st));
      } else {
        HCK(hipMemcpyAsync(c->G, c->Gc, sizeof(double) * ld * ld, hipMemcpyDeviceToDevice, c->st));
      }
      HCK(hipMemsetAsync(c->cinfo, 0, sizeof(int), c->st));
      c->caux.no_dag = true;
      const hipError_t e = chol_factor(c->G, ld, m, ld, c->W, &c->caux, c->trilist, c->cinfo, c->st);
      c->caux.no_dag = false;
      HCK(e);
      HCK(hipMemcpyAsync(&info, c->cinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
      sync(c);
    }
    if (info == 0) {
      chol_solve_checked(c, rhs);
      solve_flag_copy(c);
      c->lu_fallback_used = false;
      tend(c, T_SOLVE, e0);
      return;
    }
  }
  solve_lu_fallback(c, rhs, e0);
}

// the pipelined path's solve: the factor (and Gc) are already enqueued (gram_factor_pipelined,
// which opened the T_SOLVE interval at the end of the Gram).  false: a strip wait gave up (~30 s,
// never expected) and the strip was factored incomplete -- the caller redoes the Gram, the factor
// and the solve without the pipeline (r06; was SCS_ERR_STATE)
bool solve_factored(scs_ctx* c, double* rhs, hipEvent_t e0) {
  int info = 0, late = 0;
  HCK(hipMemcpyAsync(&info, c->cinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
  if (c->gp_flag) HCK(hipMemcpyAsync(&late, c->gp_flag, sizeof(int), hipMemcpyDeviceToHost, c->st));
  sync(c);
  if (late || fault_late(8)) {
    if (c->gp_flag) HCK(hipMemsetAsync(c->gp_flag, 0, sizeof(int), c->st));
    ++c->fb[SCS_FB_PIPE_REDO];
    tend(c, T_SOLVE, e0);
    return false;
  }
  if (info == 0) {
    chol_solve_checked(c, rhs);
    solve_flag_copy(c);
    c->lu_fallback_used = false;
    tend(c, T_SOLVE, e0);
    return true;
  }
  solve_lu_fallback(c, rhs, e0);
  return true;
}

// the main Gram launch (scheduled when gram_schedule built a work list)
// the panel-blocked A the Gram kernels read: A itself, or for a sparse A its dense mirror, built
// once (Jt*Q*Jt' of a SparseMatrixCSC, prox-GGN-SCORE.jl:129 / hess_fx, prox-N-SCORE.jl:55; the
// products Ax, Aᵀv keep running on the sparse copies)
const double* dense_A(scs_ctx* c) {
  if (!c->sparse) return c->A;
  if (c->Ad) return c->Ad;
  const size_t bytes = (size_t)c->Npad * c->mpad * sizeof(double);
  size_t fr = 0, tot = 0;
  HCK(hipMemGetInfo(&fr, &tot));
  if (bytes + (size_t)c->mpad * c->mpad * 16 > fr)
    fail(c, SCS_ERR_ARG,
         "the GGN sample-space branch on a sparse A forms Aᵀ from a dense mirror of A (%.1f GiB) plus the "
         "m x m system; the device has %.1f GiB free",
         bytes / 1073741824.0, fr / 1073741824.0);
  c->Ad = dalloc<double>(c, bytes / sizeof(double));
  HCK(hipMemsetAsync(c->Ad, 0, bytes, c->st));
  HCK(launch_densify(c->rowptr, c->colidx, c->val, c->sp_f32, c->N, c->Npad, c->Ad, c->st));
  return c->Ad;
}

// The Gram of a sparse A priced by nnz (sparse_gram_kernel: Σ_r nnz_r² multiply-adds) instead of
// dense MFMA tiles over a densified A (N·m² whatever the density): chosen when Σ_r nnz_r² is below
// N·m²/64 (the dense tiles run ~50x more flops per second), or forced by SCS_SPARSE_GRAM=1 / 0.
// The sparse Gram's row copy: the (sorted) CSR cut into 2^sparse_gram_shift()-wide column blocks,
// unpadded (blk_count / blk_scan / blk_scatter with no slot rounding).
void build_gram_blocked(scs_ctx* c) {
  scs_ctx::SpBlk& B = c->bgram;
  const int64_t nrows = c->N;
  B.shift = sparse_gram_shift();
  B.nblk = (int)ceil_div(c->m, int64_t(1) << B.shift);
  const int64_t nk = (int64_t)B.nblk * nrows;
  int64_t* cnt = dalloc<int64_t>(c, nk + 1);
  int64_t* first = dalloc<int64_t>(c, nk + 1);
  B.ptr = dalloc<int64_t>(c, nk + 1);
  int64_t nnz = 0;
  if (nrows > 0) {
    HCK(blk_count(c->rowptr, c->colidx, nrows, B.shift, cnt, first, c->st));
    size_t tb = 0;
    HCK(blk_scan(nullptr, &tb, cnt, B.ptr, nk + 1, c->st));
    void* tmp = dalloc<char>(c, tb);
    HCK(blk_scan(tmp, &tb, cnt, B.ptr, nk + 1, c->st));
    HCK(hipMemcpyAsync(&nnz, B.ptr + nk, sizeof(int64_t), hipMemcpyDeviceToHost, c->st));
    sync(c);
    dfree(c, tmp);
  }
  B.nnz = nnz;
  B.lidx = dalloc<uint16_t>(c, nnz + 8);
  B.val = c->sp_f32 ? (void*)dalloc<float>(c, (size_t)nnz + 8) : (void*)dalloc<double>(c, (size_t)nnz + 8);
  if (nrows > 0)
    HCK(blk_scatter(c->rowptr, c->colidx, c->val, c->sp_f32, nrows, B.shift, B.ptr, first, B.lidx, B.val, c->st));
  sync(c);
  dfree_t(c, cnt);
  dfree_t(c, first);
}

// The variant-8 structure (sparse.hip, r04): the segment records, the per-triple table and the sw
// buffer.  Built only when it fits (free memory less 4 GiB) and its units fit 32 bits; else state -1
// and gram_sparse takes the Gram-blocked walk (variant 6).  C5 shape: T 47 GB, seg 6.9 GB, sw 5.5 GB.
bool build_gram_seg(scs_ctx* c) {
  scs_ctx::SegGram& S = c->sgseg;
  if (S.state) return S.state > 0;
  S.state = -1;
  const int64_t nrows = c->N, m = c->m;
  const int shift = sparse_gram_shift();
  const int64_t nblk = ceil_div(m, int64_t(1) << shift);
  const int64_t nk = nblk * nrows;
  std::vector<int64_t> cp((size_t)m + 1), tp((size_t)m + 1, 0);
  HCK(hipMemcpyAsync(cp.data(), c->colptr, sizeof(int64_t) * (m + 1), hipMemcpyDeviceToHost, c->st));
  sync(c);
  for (int64_t j = 0; j < m; ++j) tp[(size_t)j + 1] = tp[(size_t)j] + ((j >> shift) + 1) * (cp[(size_t)j + 1] - cp[(size_t)j]);
  const int64_t nT = tp[(size_t)m], nnz = cp[(size_t)m];
  const double units_max = (double)seg_units_host(1, c->sp_f32) * (double)nnz + 2.0 * (double)nk;
  const double need = 8.0 * ((double)nT + (double)nnz + units_max + 4.0 * (double)(nk + 1)) + 4.0 * 1073741824.0;
  size_t fr = 0, tot = 0;
  HCK(hipMemGetInfo(&fr, &tot));
  if (nrows <= 0 || need > (double)fr) return false;
  int64_t* cnt = dalloc<int64_t>(c, nk + 1);
  int64_t* first = dalloc<int64_t>(c, nk + 1);
  int64_t* ucnt = dalloc<int64_t>(c, nk + 1);
  int64_t* uptr = dalloc<int64_t>(c, nk + 1);
  HCK(blk_count(c->rowptr, c->colidx, nrows, shift, cnt, first, c->st));
  HCK(seg_units(cnt, nk, c->sp_f32, ucnt, c->st));
  size_t tb = 0;
  HCK(blk_scan(nullptr, &tb, ucnt, uptr, nk + 1, c->st));
  void* tmp = dalloc<char>(c, tb);
  HCK(blk_scan(tmp, &tb, ucnt, uptr, nk + 1, c->st));
  int64_t units = 0;
  HCK(hipMemcpyAsync(&units, uptr + nk, sizeof(int64_t), hipMemcpyDeviceToHost, c->st));
  sync(c);
  dfree(c, tmp);
  dfree_t(c, ucnt);
  if (units < ((int64_t)1 << 31)) {   // the kernel keeps record positions in 32 bits
    S.seg = dalloc<uint64_t>(c, units + 1);
    HCK(seg_scatter(c->rowptr, c->colidx, c->val, c->sp_f32, nrows, shift, cnt, first, uptr, S.seg, c->st));
    S.tptr = dalloc<int64_t>(c, m + 1);
    HCK(hipMemcpyAsync(S.tptr, tp.data(), sizeof(int64_t) * (m + 1), hipMemcpyHostToDevice, c->st));
    S.T = dalloc<uint64_t>(c, nT);
    HCK(seg_table(c->colptr, c->rowidx, cnt, uptr, nrows, m, shift, S.tptr, S.T, c->st));
    S.sw = dalloc<double>(c, nnz);
    S.shift = shift;
    S.state = 1;
  }
  sync(c);   // the temporaries' last readers
  dfree_t(c, cnt);
  dfree_t(c, first);
  dfree_t(c, uptr);
  return S.state > 0;
}

bool sparse_gram(scs_ctx* c) {
  if (!c->sparse) return false;
  if (const char* e = std::getenv("SCS_SPARSE_GRAM")) return e[0] == '1';   // read per call (A/B tests)
  if (c->sp_gram == 0) {
    std::vector<int64_t> rp((size_t)c->N + 1);
    HCK(hipMemcpyAsync(rp.data(), c->rowptr, sizeof(int64_t) * (c->N + 1), hipMemcpyDeviceToHost, c->st));
    sync(c);
    double s2 = 0.0;
    for (int64_t r = 0; r < c->N; ++r) s2 += (double)(rp[r + 1] - rp[r]) * (double)(rp[r + 1] - rp[r]);
    c->sp_gram = (64.0 * s2 <= (double)c->N * (double)c->m * (double)c->m) ? 1 : 2;
  }
  return c->sp_gram == 1;
}

// the sparse Gram -> out (upper part, ldg = m_pad), or packed 128 x 128 slots (multi-rank) through G
void gram_sparse(scs_ctx* c, const double* w, double* out, int packed) {
  double* dst = (packed & 1) ? c->G : out;
  if (packed & 2) fail(c, SCS_ERR_ARG, "internal: the sparse Gram does not accumulate");
  if (sparse_gram_requested() == 8 && build_gram_seg(c)) {   // variant 8 (default)
    const scs_ctx::SegGram& S = c->sgseg;
    HCK(csc_weight(c->rowidx, c->valT, c->sp_f32, w, c->nnz, S.sw, c->st));
    HCK(launch_sparse_gram_seg(c->colptr, S.sw, S.tptr, S.T, S.seg, c->sp_f32, c->m, S.shift, dst, c->mpad, c->st));
    c->gram_kname = c->sp_f32 ? "sparse_gram_seg_kernel<float, 0>" : "sparse_gram_seg_kernel<double, 0>";   // rocprofv3's names
    if (packed & 1) HCK(gram_pack_launch(c->G, c->mpad, c->utiles, c->nslots, out, c->st));
    return;
  }
  if (!c->bgram.ptr) build_gram_blocked(c);
  HCK(launch_sparse_gram(c->colptr, c->rowidx, c->valT, c->bgram.ptr, c->bgram.lidx, c->bgram.val, c->bgram.nnz,
                         c->sp_f32, w, c->N, c->m, c->bgram.shift, dst, c->mpad, c->st));
  c->gram_kname = sparse_gram_kernel_name(c->sp_f32, c->bgram.nnz);
  if (packed & 1) HCK(gram_pack_launch(c->G, c->mpad, c->utiles, c->nslots, out, c->st));
}

// How the Gram of a sparse A gets its dense operand tiles: a mirror of all of A when it fits
// under the cap (SCS_SPARSE_MIRROR_MAX_GB, default: the free device memory less the m x m
// system and 4 GiB), else the streaming ring (memory O(nnz + R·m + m²) for any N).
bool sparse_streams(scs_ctx* c) {
  if (!c->sparse) return false;
  if (c->sp_mode == 0) {
    const double bytes = (double)c->Npad * c->mpad * sizeof(double);
    size_t fr = 0, tot = 0;
    HCK(hipMemGetInfo(&fr, &tot));
    double cap = (double)fr - (double)c->mpad * c->mpad * 24 - 4.0 * 1073741824.0;
    if (const char* e = std::getenv("SCS_SPARSE_MIRROR_MAX_GB")) cap = std::atof(e) * 1073741824.0;
    c->sp_mode = (bytes <= cap) ? 1 : 2;
  }
  return c->sp_mode == 2;
}

// Streaming sparse Gram (Jt*Q*Jt' of a SparseMatrixCSC, prox-GGN-SCORE.jl:114,129 / a hess_fx Gram):
// rows are densified R at a time into one of two panel-blocked ring slots (the CSR scatter is
// O(nnz), the slot's previous chunk is cleared by scattering zeros at its own positions) and the
// production Gram launch accumulates each chunk's Aᵀ diag(w) A into G -- the MFMA tiles are the
// dense kernel's, K split into N/R chunks.
void gram_main_stream(scs_ctx* c, const double* w, double* out, int packed) {
  if (!c->ringA) {
    int64_t R = 0;
    if (const char* e = std::getenv("SCS_SPARSE_CHUNK_ROWS")) R = round_up(std::max<int64_t>(16, std::atoll(e)), 16);
    if (R == 0) {   // two slots within min(16 GiB, a quarter of the free memory)
      size_t fr = 0, tot = 0;
      HCK(hipMemGetInfo(&fr, &tot));
      const double budget = std::min(16.0 * 1073741824.0, 0.25 * (double)fr);
      R = std::max<int64_t>(2048, (int64_t)(budget / (2.0 * c->mpad * sizeof(double))) / 2048 * 2048);
    }
    c->ring_rows = std::min(R, c->Npad);
    c->ringA = dalloc<double>(c, (size_t)2 * c->ring_rows * c->mpad);
    c->ring_r0[0] = c->ring_r0[1] = -1;
  }
  const int64_t R = c->ring_rows;
  const int64_t nchunk = ceil_div(std::max<int64_t>(c->N, 1), R);
  for (int64_t k = 0; k < nchunk; ++k) {
    const int s = (int)(k & 1);
    double* slot = c->ringA + (size_t)s * R * c->mpad;
    const int64_t r0 = k * R, n = std::min(R, c->N - r0);
    if (c->ring_r0[s] >= 0)
      HCK(launch_densify_range(c->rowptr, c->colidx, c->val, c->sp_f32, c->ring_r0[s], c->ring_n[s], R, 1, slot, c->st));
    HCK(launch_densify_range(c->rowptr, c->colidx, c->val, c->sp_f32, r0, n, R, 0, slot, c->st));
    c->ring_r0[s] = r0;
    c->ring_n[s] = n;
    const int mode = packed | (k > 0 ? 2 : 0);
    const int64_t nk = round_up(std::max<int64_t>(n, 1), 16);   // w + r0 + nk <= w + Npad
    if (c->gwork)
      HCK(gram_launch_sched(slot, R / 16, w + r0, nk, c->gwork, c->gseglen, c->gnsplit, c->gcomb, c->gncomb, c->gpart,
                            out, c->mpad, mode, c->tall, c->st));
    else
      HCK(gram_launch(slot, R / 16, w + r0, nk, c->tiles, c->ntiles, out, c->mpad, mode, c->tall, c->st));
    c->gram_kname = gram_main_kernel_name();
  }
}

// v != nullptr: the same launch forms Aᵀv of the local rows into vout (fused, gram_fuse_ok)
void gram_main(scs_ctx* c, const double* w, double* out, int packed, const double* v = nullptr,
               double* vout = nullptr) {
  if (sparse_gram(c)) {
    if (v) fail(c, SCS_ERR_ARG, "internal: the sparse Gram forms no Aᵀv");
    gram_sparse(c, w, out, packed);
    return;
  }
  if (sparse_streams(c)) {
    if (v) fail(c, SCS_ERR_ARG, "internal: the streaming sparse Gram forms no Aᵀv");
    gram_main_stream(c, w, out, packed);
    return;
  }
  const double* A = dense_A(c);
  const int npiece = (v && c->gwork) ? std::max(c->gnsplit, 1) : 1;
  if (v && npiece > 1) HCK(hipMemsetAsync(c->vpart, 0, sizeof(double) * npiece * c->mpad, c->st));
  if (c->gwork)
    HCK(gram_launch_sched(A, c->nstage, w, c->Npad, c->gwork, c->gseglen, c->gnsplit, c->gcomb, c->gncomb, c->gpart,
                          out, c->mpad, packed, c->tall, c->st, v, c->vpart, c->mpad));
  else
    HCK(gram_launch(A, c->nstage, w, c->Npad, c->tiles, c->ntiles, out, c->mpad, packed, c->tall, c->st, v, c->vpart,
                    c->mpad));
  c->gram_kname = gram_main_kernel_name();
  if (v) HCK(gram_vfinal_launch(c->vpart, npiece, c->mpad, c->m, vout, c->st));
}

// Gram of the local rows with weights w -> c->G (single rank) or the packed
// reduce buffer (multi-rank; then all-reduced together with `vec`).
// AᵀQA does not depend on x: least squares under ProxNSCORE (hess_fx = c·AᵀA) or under
// ProxGGNSCORE with the linear out_fn (J = A, Q = c·I); the reference still recomputes it every
// step (prox-GGN-SCORE.jl:129), which stays the default
bool gram_x_independent(const scs_ctx* c) {
  if (c->loss != SCS_LOSS_LEAST_SQUARES) return false;
  return c->method == SCS_PROX_NSCORE || (c->method == SCS_PROX_GGNSCORE && c->ggn == SCS_GGN_LINEAR_LS);
}

// vec_dev = Aᵀv of the local rows (then reduced with the Gram): formed inside the Gram launch
// (gram_sia_kernel AV) unless the Gram is served from the cache (a cached run never fuses, so
// its steps all take the same separate Aᵀv pass) or SCS_GRAM_FUSE=0
void gram_and_reduce(scs_ctx* c, const double* w, const double* v, double* vec_dev) {
  ensure_gram(c);
  ensure_red(c);
  hipEvent_t e0;
  const bool cacheable = c->gram_cache && gram_x_independent(c);
  const size_t gbytes = sizeof(double) * (size_t)c->mpad * c->mpad;
  // sparse A: Aᵀv from the CSC copy (a streaming Gram has no whole-A pass to ride on)
  const bool fuse = !cacheable && !c->sparse && gram_fuse_ok(c->tall);
  if (!fuse) gemv_t_local(c, v, vec_dev);
  if (cacheable && c->Gk && c->gk_gen == c->data_gen) {   // the reduced Gram of an earlier step
    c->g_from_cache = true;
    HCK(hipMemcpyAsync(c->G, c->Gk, gbytes, hipMemcpyDeviceToDevice, c->st));
    if (sharded(c)) {
      HCK(hipMemcpyAsync(c->red, vec_dev, sizeof(double) * c->m, hipMemcpyDeviceToDevice, c->st));
      allreduce(c, c->red, c->m);
      HCK(hipMemcpyAsync(vec_dev, c->red, sizeof(double) * c->m, hipMemcpyDeviceToDevice, c->st));
    }
    return;
  }
  if (sharded(c)) {
    const int64_t tsz = (int64_t)c->nslots * 128 * 128;
    tbegin(c, T_GRAM, &e0);
    gram_main(c, w, c->red, 1, fuse ? v : nullptr, vec_dev);
    tend(c, T_GRAM, e0);
    HCK(hipMemcpyAsync(c->red + tsz, vec_dev, sizeof(double) * c->m, hipMemcpyDeviceToDevice, c->st));
    allreduce(c, c->red, tsz + c->m);
    HCK(gram_unpack_launch(c->red, c->utiles, c->nslots, c->G, c->mpad, c->st));
    HCK(hipMemcpyAsync(vec_dev, c->red + tsz, sizeof(double) * c->m, hipMemcpyDeviceToDevice, c->st));
  } else {
    tbegin(c, T_GRAM, &e0);
    gram_main(c, w, c->G, 0, fuse ? v : nullptr, vec_dev);
    tend(c, T_GRAM, e0);
  }
  if (cacheable) {
    if (!c->Gk) c->Gk = dalloc<double>(c, (size_t)c->mpad * c->mpad);
    HCK(hipMemcpyAsync(c->Gk, c->G, gbytes, hipMemcpyDeviceToDevice, c->st));
    c->gk_gen = c->data_gen;
  }
}

// The factor hidden under the Gram (SCS_CHOL_PIPE=1; off by default, see below): one scheduled Gram launch per
// outer strip of the system on the context stream; on a second stream, as each strip lands:
// λ·Hr on its diagonal (and the padding's 1s), its copy into Gc (the LU fallback's system), the
// left-looking update from every earlier strip, its diagonal block and row strip
// (chol_strip_update / chol_strip_factor).  Only the last strip's factor and the two triangular
// solves remain after the Gram.  Single rank, dense A, Gram not served from the cache; m/128 >= 3
// outer blocks.  The result is the same factor up to the summation order of the updates
// (left- instead of right-looking).
// Measured at C2 (m = 8192, one box, same build): step 118.5 ms piped vs 107.7 ms classic.  The
// exposed solve drops 13.1 -> 6.2 ms, but the Gram grows 93.3 -> 110.9 ms: a strip launch is less
// than one round of the chip (strip 0: 484 tiles on 512 slots took 24.3 ms alone against its 21.5 ms
// share -- the interleaved kernel does not run a lone workgroup per CU twice as fast), and the
// factor's workgroups share CUs with MFMA-bound Gram waves (the left-looking updates ran at ~11 %
// of their alone rate).  At C3 (16 strips of 256 x 128 tiles) the partial rounds alone would cost
// seconds.  Hiding the factor needs the one-launch Gram with per-strip completion counters.
// SCS_CHOL_PIPE=2: ONE scheduled Gram launch whose per-XCD segments run the strips in order and
// count each finished tile into its strip; the factor stream waits for a strip's count
// (strip_wait_kernel) instead of an event after a per-strip launch, so the Gram keeps whole
// rounds.  (gram_factor_pipelined)
int pipe_mode(const scs_ctx* c, bool cacheable) {
  const char* e = std::getenv("SCS_CHOL_PIPE");   // read per step (tests toggle it in-process)
  const int mode = e ? std::atoi(e) : 0;
  const int64_t nblk = c->mpad / 128;
  const bool ok = !cacheable && !sharded(c) && !c->sparse && c->gwork && c->solver == 0 &&
                  nblk >= 3 * chol_outer_block();
  return ok && (mode == 1 || mode == 2) ? mode : 0;
}
bool pipe_ok(const scs_ctx* c, bool cacheable) { return pipe_mode(c, cacheable) != 0; }

// Gram (+ fused Aᵀv into vec_dev) and the factor of G + λ diag(Hr); Gc receives the system.
// Returns with the factor enqueued on c->st (info in c->cinfo).
hipEvent_t gram_factor_pipelined(scs_ctx* c, const double* w, const double* v, double* vec_dev) {
  const int64_t m = c->m, ld = c->mpad;
  const int nb = (int)(ld / 128), OB = chol_outer_block(), ns = (int)c->gstrip.size();
  HCK(chol_pipe_init(&c->caux, ld, c->st));
  if (!c->sf) {
    HCK(hipStreamCreateWithFlags(&c->sf, hipStreamNonBlocking));
    HCK(hipEventCreateWithFlags(&c->evfac, hipEventDisableTiming));
  }
  while ((int)c->evstrip.size() < ns + 1) {
    hipEvent_t e;
    HCK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->evstrip.push_back(e);
  }
  const bool fuse = !c->sparse && gram_fuse_ok(c->tall);
  if (!fuse) gemv_t_local(c, v, vec_dev);
  const double* A = dense_A(c);
  if (fuse && c->vpieces > 1) HCK(hipMemsetAsync(c->vpart, 0, sizeof(double) * c->vpieces * ld, c->st));
  HCK(hipMemsetAsync(c->cinfo, 0, sizeof(int), c->st));
  const bool one = pipe_mode(c, false) == 2;
  if (one) HCK(hipMemsetAsync(c->gp_cnt, 0, sizeof(unsigned) * ns, c->st));
  hipEvent_t e0;
  tbegin(c, T_GRAM, &e0);
  // the factor stream starts after everything already on st (weights, smoother, info reset)
  HCK(hipEventRecord(c->evstrip[ns], c->st));
  HCK(hipStreamWaitEvent(c->sf, c->evstrip[ns], 0));
  if (one) {
    const scs_ctx::GStrip& g = c->gpipe;
    HCK(gram_launch_sched(A, c->nstage, w, c->Npad, g.work, g.seglen, g.nsplit, g.comb, g.ncomb, c->gpart, c->G, ld,
                          0, c->tall, c->st, fuse ? v : nullptr, c->vpart, ld, c->gp_cnt, OB));
    HCK(hipEventRecord(c->evstrip[ns - 1], c->st));   // the last strip (and its combined pieces)
  } else {
    for (int s2 = 0; s2 < ns; ++s2) {
      const scs_ctx::GStrip& g = c->gstrip[s2];
      HCK(gram_launch_sched(A, c->nstage, w, c->Npad, g.work, g.seglen, g.nsplit, g.comb, g.ncomb, c->gpart, c->G, ld,
                            0, c->tall, c->st, fuse ? v : nullptr, c->vpart, ld));
      HCK(hipEventRecord(c->evstrip[s2], c->st));
    }
  }
  tend(c, T_GRAM, e0);
  hipEvent_t es;
  tbegin(c, T_SOLVE, &es);   // the solve's share of the step: what runs after the Gram
  if (fuse) HCK(gram_vfinal_launch(c->vpart, c->vpieces, ld, m, vec_dev, c->st));
  for (int s2 = 0; s2 < ns; ++s2) {
    if (one && s2 + 1 < ns)
      HCK(strip_wait_launch(c->gp_cnt + s2, c->gp_target[s2], c->gp_flag, c->sf));
    else
      HCK(hipStreamWaitEvent(c->sf, c->evstrip[s2], 0));
    const int64_t r0 = (int64_t)s2 * OB * 128, r1 = std::min<int64_t>((int64_t)(s2 + 1) * OB * 128, ld);
    if (r0 < m) HCK(launch_diag_add(c->G + r0 * ld + r0, ld, std::min(r1, m) - r0, c->lam, c->Hr + r0, c->sf));
    HCK(chol_diag_pad(c->G, ld, std::max(r0, m), r1, c->sf));
    // strip rows [r0, r1), columns [r0, ld) -> Gc
    HCK(chol_copy_rows(c->Gc, c->G, ld, r0, r1, r0, ld, c->sf));
    HCK(chol_strip_update(c->G, ld, s2, &c->caux, c->sf));
    HCK(chol_strip_factor(c->G, ld, s2, c->W, &c->caux, c->trilist, c->cinfo, c->sf));
  }
  (void)nb;
  HCK(hipEventRecord(c->evfac, c->sf));
  HCK(hipStreamWaitEvent(c->st, c->evfac, 0));
  return es;
}

// fixed step-size rules shared by ProxNSCORE / ProxGGNSCORE
double step_size_newton(scs_ctx* c, int64_t iter, bool* needs_ls) {
  *needs_ls = false;
  if (c->ss_type == 1 && c->has_L) return jl_min_h(1 / c->L, 1.0);
  if (c->ss_type == 1 && !c->has_L) return 0.5;
  if (c->ss_type == 2) {
    if (iter == 1) return 1.0;
    // prox-N-SCORE.jl:81-83 / prox-GGN-SCORE.jl:78-80 call hμ.grad(x_prev) with one
    // argument and use an undefined ∇f: the reference raises a MethodError here.
    fail(c, SCS_ERR_REF, "MethodError: ss_type=2 calls hμ.grad(x_prev) with the wrong arity (reference bug, "
                         "prox-N-SCORE.jl:81 / prox-GGN-SCORE.jl:78)");
  }
  if (c->ss_type == 3) {
    *needs_ls = true;
    return 0.0;
  }
  fail(c, SCS_ERR_REF, "Please, choose ss_type in [1, 2, 3].");
}

// ggn_score_step's sample-space branch (prox-GGN-SCORE.jl:124-127, N + 1 <= m) -> c->d
void ggn_sample_direction(scs_ctx* c, const double* xh);

// The sample-space branch across ranks: its (N+1) x (N+1) system couples every pair of
// samples, so the ranks' rows are all-gathered once (each rank writes its rows into the
// zeroed reduce buffer at their global positions; the sum is the full A and y, at most
// N_global·m <= m² doubles -- the size of the feature branch's Gram exchange) and every
// rank runs the single-rank branch on that view, redundantly, as it does the m x m solve.
void ggn_sample_direction_sharded(scs_ctx* c, const double* xh) {
  if (c->sparse) fail(c, SCS_ERR_ARG, "the sharded GGN sample-space branch needs a dense A");
  ensure_red(c);
  const int64_t Ng = c->Nglob, Npg = round_up(std::max<int64_t>(Ng, 1), 16);
  const uint64_t gen = c->bsel < 0 ? 0 : c->batch_gen;
  const bool held = c->gview_ok && c->gview_batch == c->bsel && c->gview_gen == gen;
  if (c->gview_ok && !held && c->gview.N != Ng) {   // another size: new buffers
    free_view(c, c->gview);
    c->gview = NView();
    c->gview_ok = false;
  }
  if (!held) {
    if (Npg * c->mpad + Npg > c->red_cap) fail(c, SCS_ERR_COMM, "reduce buffer too small for the row all-gather");
    // each local row at its global position: in the data (row0 + r) or in the selected batch
    std::vector<int64_t> rows(Ng, -1);
    if (c->bsel < 0) {
      for (int64_t r = 0; r < c->N; ++r) rows[c->row0 + r] = r;
    } else {
      const int64_t o = c->boff[c->bsel];
      for (int64_t r = 0; r < c->N; ++r) rows[c->bpos[o + r]] = r;
    }
    int64_t* drows = dalloc<int64_t>(c, Ng);
    HCK(hipMemcpyAsync(drows, rows.data(), sizeof(int64_t) * Ng, hipMemcpyHostToDevice, c->st));
    HCK(launch_gather_rows(c->A, c->Npad, c->y, drows, Ng, Npg, c->mpad, c->red, c->red + Npg * c->mpad, c->st));
    allreduce(c, c->red, Npg * c->mpad + Npg);
    NView& v = c->gview;
    const bool fresh = !c->gview_ok;   // same size as the view held: refill its buffers in place
    if (fresh) {
      v.N = v.Nglob = Ng;
      v.Npad = Npg;
      v.nstage = Npg / 16;
      v.A = dalloc<double>(c, (size_t)Npg * c->mpad);
      v.y = dalloc<double>(c, Npg);
    }
    HCK(hipMemcpyAsync(v.A, c->red, sizeof(double) * Npg * c->mpad, hipMemcpyDeviceToDevice, c->st));
    HCK(hipMemcpyAsync(v.y, c->red + Npg * c->mpad, sizeof(double) * Npg, hipMemcpyDeviceToDevice, c->st));
    // a refilled view's Aᵀ copy (built once per A by ggn_sample_direction) follows its rows
    if (!fresh && v.At) HCK(launch_transpose(v.A, v.Npad, Ng, c->m, v.At, c->mpad, v.NpS, c->st));
    sync(c);
    dfree_t(c, drows);
    if (fresh) {
      swap_view(c, v);
      alloc_nspace(c);
      swap_view(c, v);
    }
    c->gview_ok = true;
    c->gview_batch = c->bsel;
    c->gview_gen = gen;
  }
  struct Scope {   // the gathered rows on one logical rank, restored even when the step fails
    scs_ctx* c;
    int nr;
    bool force;
    explicit Scope(scs_ctx* cc) : c(cc), nr(cc->nranks), force(cc->comm_force) {
      swap_view(c, c->gview);
      c->nranks = 1;
      c->comm_force = false;
      invalidate_caches(c);
    }
    ~Scope() {
      swap_view(c, c->gview);
      c->nranks = nr;
      c->comm_force = force;
      invalidate_caches(c);
    }
  } scope(c);
  ggn_sample_direction(c, xh);
}

void ggn_sample_direction(scs_ctx* c, const double* xh) {
  const int64_t N = c->N, m = c->m;
  if (sharded(c)) return ggn_sample_direction_sharded(c, xh);
  if (c->At && c->loss == SCS_LOSS_CALLBACK)   // the caller's J changes every step
    HCK(launch_transpose(c->A, c->Npad, N, m, c->At, c->mpad, c->NpS, c->st));
  if (!c->At) {
    const double* A = dense_A(c);
    c->NpS = round_up(N, 128);
    c->At = dalloc<double>(c, (size_t)c->NpS * c->mpad);
    HCK(launch_transpose(A, c->Npad, N, m, c->At, c->mpad, c->NpS, c->st));
    c->Ps = dalloc<double>(c, (size_t)c->NpS * c->NpS);
    c->n1pad = round_up(N + 1, 128);   // row-major, zero padding (lu.hip)
    c->Ms = dalloc<double>(c, (size_t)c->n1pad * c->n1pad);
    c->bS = dalloc<double>(c, c->n1pad);
    c->uN = dalloc<double>(c, c->Npad);
    c->hvec = dalloc<double>(c, c->mpad);
    c->hg = dalloc<double>(c, c->mpad);
    const int nb = (int)(c->NpS / 128);
    std::vector<int2> tl((size_t)nb * (nb + 1) / 2);
    int nt = 0;
    gram_tile_list(nb, tl.data(), &nt);
    c->stiles = dalloc<int2>(c, nt);
    HCK(hipMemcpyAsync(c->stiles, tl.data(), sizeof(int2) * nt, hipMemcpyHostToDevice, c->st));
    c->nstiles = nt;
  }
  // s, q, r (prox-GGN-SCORE.jl:44-56) -> gN, hN, wN (a callback loss filled them: ggn_cb_load)
  if (c->loss != SCS_LOSS_CALLBACK) forward(c, xh, c->x, EPI_GGN | EPI_SQR, false);
  HCK(launch_ggn_sample_prep(c->Hr, c->gr, c->lam, m, c->mpad, c->hvec, c->hg, c->st));
  hipEvent_t e0;
  tbegin(c, T_GRAM, &e0);
  HCK(gram_launch_gen(c->At, c->mpad, c->At, c->mpad, c->hvec, 0, c->mpad, c->stiles, c->nstiles, c->Ps, c->NpS,
                      /*GRAM_UPPER*/ 4, c->st));
  tend(c, T_GRAM, e0);
  HCK(launch_symmetrize(c->Ps, c->NpS, N, c->st));
  const int ns = matvec_n(c, c->hg, c->nsplit);   // u = A (h∘λgr)
  HCK(launch_epilogue(SCS_LOSS_LEAST_SQUARES, SCS_GGN_NONE, EPI_Z, c->zpart, ns, c->Npad, c->y, N, c->Npad, 1.0,
                      c->uN, nullptr, nullptr, nullptr, nullptr, c->valpart, c->st));
  HCK(launch_ggn_sample_assemble(c->Ps, c->NpS, c->gN, c->hN, c->wN, c->uN, nullptr, N, c->Ms, c->n1pad, c->bS,
                                      c->st));
  tbegin(c, T_SOLVE, &e0);
  const int64_t n1 = N + 1, np1 = c->n1pad;
  int info = 0;
  // NaN / Inf in the system: the reference's qr(...) \ b comes out NaN (no SingularException)
  HCK(hipMemsetAsync(c->cinfo, 0, sizeof(int), c->st));
  HCK(launch_nonfinite(c->Ms, np1, n1, c->bS, c->cinfo, c->st));
  HCK(hipMemcpyAsync(&info, c->cinfo, sizeof(int), hipMemcpyDeviceToHost, c->st));
  sync(c);
  if (info != 0) {
    HCK(launch_fill(c->bS, n1, std::numeric_limits<double>::quiet_NaN(), c->st));
  } else if (c->solver == SCS_SOLVER_REFERENCE) {
    // qr(I + A) \ residual (prox-GGN-SCORE.jl:126): the row-major system transposed into a
    // column-major copy with identity padding, Householder QR
    if (c->qrM_n != np1) {
      dfree_t(c, c->qrM);
      c->qrM = dalloc<double>(c, (size_t)np1 * np1);
      c->qrM_n = np1;
    }
    HCK(qr_from_rowmajor(c->Ms, np1, c->qrM, np1, n1, np1, c->st));
    qr_run(c, c->qrM, np1, c->bS);
  } else {
    HCK(lu_aux_init(&c->lu, np1, c->st));
    info = lu_factor_checked(c, c->Ms, np1, n1, np1, c->cinfo, [&] {   // the system assembled again
      HCK(launch_ggn_sample_assemble(c->Ps, c->NpS, c->gN, c->hN, c->wN, c->uN, nullptr, N, c->Ms, c->n1pad, c->bS,
                                     c->st));
    });
    if (info != 0) fail(c, SCS_ERR_SOLVE, "SingularException(%d)", info);
    HCK(lu_solve(c->Ms, np1, np1, &c->lu, c->bS, c->st));
  }
  tend(c, T_SOLVE, e0);
  HCK(launch_ggn_sample_scale(c->gN, c->bS, N, c->Npad, c->vN, c->st));
  gemv_t_local(c, c->vN, c->gtmp);   // Aᵀ(s∘B)
  HCK(launch_ggn_sample_direction(c->hvec, c->gtmp, c->hg, c->bS, N, m, c->d, c->st));
}

// host column-major rows (N x m, lda) -> panel-blocked dst (Npad x mpad), one 128-column panel
// at a time through the column-major staging buffer C (Npad x 128)
static void upload_panels(scs_ctx* c, const double* A, int64_t N, int64_t lda, int64_t Npad, double* dst, double* C) {
  const int64_t m = c->m;
  for (int64_t p = 0; p < c->mpad / 128; ++p) {
    const int64_t j0 = p * 128, nc = std::min<int64_t>(128, m - j0);
    HCK(hipMemsetAsync(C, 0, sizeof(double) * Npad * 128, c->st));
    if (nc > 0 && N > 0)
      HCK(hipMemcpy2DAsync(C, sizeof(double) * Npad, A + j0 * lda, sizeof(double) * lda, sizeof(double) * N, nc,
                           hipMemcpyHostToDevice, c->st));
    HCK(launch_retile(C, dst, Npad, p, 1, c->st));
  }
}

// ProxGGNSCORE on a callback loss (jac_yx / grad_fy / hess_fy, prox-GGN-SCORE.jl:44-49): the
// caller hands over J (n x m, column-major), r and the diagonal q of Q (a general symmetric Q
// arrives eigen-rotated: J̃ = VᵀJ, r̃ = Vᵀr, q = eigenvalues -- JᵀQJ, Jᵀr and the sample-space
// system are unchanged).  J is uploaded into the callback view, which then stands in for the
// data with s = 1: w = q, v = r in the feature branch; (s, q, r) = (1, q, r) in the sample one.
void ggn_cb_load(scs_ctx* c, const double* xh, bool sample) {
  const int64_t n = c->cb_nout, m = c->m;
  const double* out = cb_eval(c, SCS_CB_GGN, xh, c->x, (size_t)n * (m + 2));
  NView& v = c->cbv;
  if (!v.A) {
    v.N = v.Nglob = n;
    v.Npad = round_up(std::max<int64_t>(n, 1), 16);
    v.nstage = v.Npad / 16;
    v.A = dalloc<double>(c, (size_t)v.Npad * c->mpad);
    v.y = dalloc<double>(c, v.Npad);
    swap_view(c, v);
    c->generic = false;
    alloc_nspace(c);
    c->generic = true;
    swap_view(c, v);
    c->cbstage = dalloc<double>(c, (size_t)v.Npad * 128);
  }
  upload_panels(c, out, n, n, v.Npad, v.A, c->cbstage);
  const double* r = out + (size_t)n * m;
  const double* q = r + n;
  if (sample) {
    HCK(launch_fill(v.gN, n, 1.0, c->st));
    HCK(hipMemcpyAsync(v.hN, q, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
    HCK(hipMemcpyAsync(v.wN, r, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
  } else {
    HCK(hipMemcpyAsync(v.wN, q, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
    HCK(hipMemcpyAsync(v.vN, r, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
  }
}

// the callback view in place of the (absent) data for one GGN step, restored even on failure
struct CbScope {
  scs_ctx* c;
  explicit CbScope(scs_ctx* cc) : c(cc) {
    swap_view(c, c->cbv);
    c->generic = false;
    invalidate_caches(c);
  }
  ~CbScope() {
    swap_view(c, c->cbv);
    c->generic = true;
    invalidate_caches(c);
  }
};

// ProxNSCORE / ProxGGNSCORE step
void step_newton(scs_ctx* c, const double* xh, int64_t iter, double* x_new, double* dx, double* pri) {
  const int64_t m = c->m;
  c->g_from_cache = false;
  HCK(launch_smoother(c->smooth, c->x, m, c->mu, c->slb, c->sub, c->wel, c->gr, c->Hr, c->st));
  const bool cbggn = c->method == SCS_PROX_GGNSCORE && c->loss == SCS_LOSS_CALLBACK;
  const bool sample_space = (c->method == SCS_PROX_GGNSCORE) &&
                            (cbggn ? c->cb_nout + 1 <= m : (c->Nglob + 1 <= m && c->ggn != SCS_GGN_NONE));
  if (cbggn) ggn_cb_load(c, xh, sample_space);
  if (sample_space) {
    if (cbggn) {
      CbScope scope(c);
      ggn_sample_direction(c, xh);
    } else {
      ggn_sample_direction(c, xh);
    }
  } else {
  ensure_gram(c);
  if (c->method == SCS_PROX_NSCORE) {
    // H = hess_fx, ∇q = grad_fx + λ gr  (prox-N-SCORE.jl:183-204)
    if (c->loss == SCS_LOSS_ROSENBROCK) {
      HCK(launch_rosen(c->x, m, 2, nullptr, c->G, c->mpad, c->st));
      HCK(launch_rosen(c->x, m, 1, c->gtmp, nullptr, 0, c->st));
    } else if (c->loss == SCS_LOSS_CALLBACK) {
      // H = hess_fx(x) (m x m, column-major) into the leading block of G; the padded rows /
      // columns keep block-diag(H, I) (zero from the allocation, the padded diagonal set by
      // chol_factor)
      const double* H = cb_eval(c, SCS_CB_HESS, xh, c->x, (size_t)m * m);
      HCK(hipMemcpy2DAsync(c->G, sizeof(double) * c->mpad, H, sizeof(double) * m, sizeof(double) * m, m,
                           hipMemcpyHostToDevice, c->st));
      grad_f_dev(c, xh, c->x, c->gtmp);
    } else if (c->loss == SCS_LOSS_QUADRATIC) {
      require_dense(c, "the quadratic loss");
      HCK(launch_half_sym(c->A, c->nstage, m, c->G, c->mpad, c->st));
      grad_f_dev(c, xh, c->x, c->gtmp);
    } else {
      forward(c, xh, c->x, EPI_GRAD | EPI_HESS, false);
      // local Aᵀg (not yet reduced; fused into the Gram pass); reduced together with the Gram
      if (pipe_ok(c, c->gram_cache && gram_x_independent(c))) {
        ensure_gram(c);
        const hipEvent_t es = gram_factor_pipelined(c, c->hN, c->gN, c->gtmp);
        if (c->gfix) grad_f_dev(c, xh, c->x, c->gtmp);   // ∇fx replaces the fused Aᵀg
        HCK(launch_axpby(c->gtmp, c->lam, c->gr, m, c->gq, c->st));
        if (solve_factored(c, c->gq, es)) {
          HCK(launch_neg(c->gq, m, c->d, c->st));
          goto newton_tail;
        }
        // (a strip wait gave up: the unpipelined Gram, factor and solve below)
      }
      gram_and_reduce(c, c->hN, c->gN, c->gtmp);
    }
  } else if (cbggn) {
    CbScope scope(c);
    gram_and_reduce(c, c->wN, c->vN, c->gtmp);   // JᵀQJ + Jᵀr of the caller's J (w = q, v = r)
  } else {
    if (c->ggn == SCS_GGN_NONE) fail(c, SCS_ERR_ARG, "ProxGGNSCORE needs an out_fn / GGN loss kind");
    // J, residual, Q (prox-GGN-SCORE.jl:44-56) -> w = s²q, v = s·r
    forward(c, xh, c->x, EPI_GGN, false);
    if (pipe_ok(c, c->gram_cache && gram_x_independent(c))) {
      ensure_gram(c);
      const hipEvent_t es = gram_factor_pipelined(c, c->wN, c->vN, c->gtmp);
      HCK(launch_axpby(c->gtmp, c->lam, c->gr, m, c->gq, c->st));
      if (solve_factored(c, c->gq, es)) {
        HCK(launch_neg(c->gq, m, c->d, c->st));
        goto newton_tail;
      }
      // (a strip wait gave up: the unpipelined Gram, factor and solve below)
    }
    gram_and_reduce(c, c->wN, c->vN, c->gtmp);   // Gram + Jᵀr in one pass over A
  }
  // rhs = ∇f + λ gr (NSCORE) | Jᵀr + λ gr (GGN: Jt*[r;1], prox-GGN-SCORE.jl:121-130); a caller's
  // ∇fx replaces ∇f in ProxNSCORE (prox-N-SCORE.jl:66-69; ProxGGNSCORE takes no ∇fx)
  if (c->gfix && c->method == SCS_PROX_NSCORE) grad_f_dev(c, xh, c->x, c->gtmp);
  HCK(launch_axpby(c->gtmp, c->lam, c->gr, m, c->gq, c->st));
  HCK(launch_diag_add(c->G, c->mpad, m, c->lam, c->Hr, c->st));
  solve_system(c, c->gq);
  HCK(launch_neg(c->gq, m, c->d, c->st));  // d = -sol
  }
newton_tail:
  bool ls = false;
  double step = step_size_newton(c, iter, &ls);
  if (ls) step = line_search(c, xh, c->x, c->d);
  const double Mg = get_Mg(c, c->Mh, c->nu, c->mu, m);
  HCK(launch_score_tail(c->x, c->d, c->gr, c->Hr, m, c->lam, Mg, step, nullptr, prox_args(c), c->hinv, c->zb, c->xn,
                        c->dxv, c->scal, c->st));
  if (c->dev_loop) return;   // x_new stays in c->xn, pri_res_norm in scal[0]
  d2h(c, x_new, c->xn, m);
  if (dx) d2h(c, dx, c->dxv, m);
  d2h(c, c->hscal, c->scal, 4);
  sync(c);
  *pri = c->hscal[0];
}

// L-BFGS memory update decision (prox-L-BFGS-SCORE.jl:154-162) from the device's δhᵀγh, γhᵀγh:
// accept the pair written to `slot` when δhᵀγh > 1e-10 (absolute), FIFO capped at mem
void lbfgs_accept(scs_ctx* c, int slot, double dg, double gg) {
  if (!(dg > 1e-10)) return;
  if ((int)c->ring.size() == c->mem) {
    c->spare = c->ring.front();
    c->ring.erase(c->ring.begin());
  } else {
    // the next unused physical slot becomes the spare
    std::vector<bool> used(c->mem + 1, false);
    for (int r : c->ring) used[r] = true;
    used[slot] = true;
    for (int i = 0; i <= c->mem; ++i)
      if (!used[i]) {
        c->spare = i;
        break;
      }
  }
  c->ring.push_back(slot);
  c->H0 = dg / gg;
}

// a memory update left in flight by the device loop: its dg / gg are in hscal[16..17] once the
// epoch-end copy has landed (scs_iterate syncs before calling this)
void lbfgs_settle(scs_ctx* c, bool synced) {
  if (!c->lbfgs_pending) return;
  if (!synced) {
    d2h(c, c->hscal + 16, c->scal + 16, 2);
    sync(c);
  }
  c->lbfgs_pending = false;
  lbfgs_accept(c, c->lbfgs_slot, c->hscal[16], c->hscal[17]);
}

// ProxLQNSCORE step (prox-L-BFGS-SCORE.jl:69-169)
void step_lqn(scs_ctx* c, const double* xh, const double* xph, int64_t iter, double* x_new, double* dx,
              double* pri) {
  const int64_t m = c->m;
  lbfgs_settle(c, false);
  HCK(launch_smoother(c->smooth, c->x, m, c->mu, c->slb, c->sub, c->wel, c->gr, c->Hr, c->st));
  grad_q_dev(c, xh, c->x, c->gq);  // ∇q = grad_f(x) + λgr
  const int k = (int)c->ring.size();
  if (iter == 1 || k == 0) {
    HCK(launch_neg(c->gq, m, c->d, c->st));
  } else {
    std::memcpy(c->hring, c->ring.data(), sizeof(int) * k);   // pinned: a truly asynchronous upload
    HCK(hipMemcpyAsync(c->d_order, c->hring, sizeof(int) * k, hipMemcpyHostToDevice, c->st));
    HCK(launch_two_loop(c->S, c->Yv, c->mpad, c->d_order, k, c->H0, c->gq, m, c->q, c->d, c->ab, c->tlwork, c->mem,
                        nullptr, nullptr, c->st, c->f32c));
  }
  double step = 0.0;
  const double* step_dev = nullptr;
  if (c->ss_type == 1 && c->has_L) {
    step = jl_min_h(1 / c->L, 1.0);
  } else if (c->ss_type == 1 && !c->has_L) {
    step = 0.5;
  } else if (c->ss_type == 2 || !c->has_L) {
    if (iter == 1) {
      step = 1.0;
    } else {
      grad_q_dev(c, xph, c->xp, c->gqn);  // ∇q(x_prev)
      HCK(launch_bb_step(c->x, c->xp, c->gq, c->gqn, m, c->scal + 12, c->st));
      step_dev = c->scal + 12;
    }
  } else if (c->ss_type == 3) {
    step = line_search(c, xh, c->x, c->d);
  } else {
    fail(c, SCS_ERR_REF, "Please, choose ss_type in [1, 2, 3].");
  }
  const double Mg = get_Mg(c, c->Mh, c->nu, c->mu, m);
  HCK(launch_score_tail(c->x, c->d, c->gr, c->Hr, m, c->lam, Mg, step, step_dev, prox_args(c), c->hinv, c->zb, c->xn,
                        c->dxv, c->scal, c->st));
  if (!c->dev_loop) {
    d2h(c, x_new, c->xn, m);
    if (dx) d2h(c, dx, c->dxv, m);
    d2h(c, c->hscal, c->scal, 4);
    sync(c);
    *pri = c->hscal[0];
  }
  // δh = x_new − x (prox) | dx (into q / dxv: grad_q_dev's smoother scratch is zb, hinv);
  // ∇q_new = grad_f(x_new) + λ gr(x_new)
  const double* dh = c->dxv;
  if (c->use_prox) {
    HCK(launch_sub(c->xn, c->x, m, c->q, c->st));
    dh = c->q;
  }
  grad_q_dev(c, x_new, c->xn, c->gqn);
  const int slot = c->spare;
  HCK(launch_lbfgs_update(dh, c->gqn, c->gq, m, c->S + (int64_t)slot * c->mpad, c->Yv + (int64_t)slot * c->mpad,
                          c->scal + 16, c->scal + 64, c->st));
  c->lbfgs_pending = true;
  c->lbfgs_slot = slot;
  if (!c->dev_loop) lbfgs_settle(c, false);
}

}  // namespace

namespace {
bool is_group(const scs_ctx* c);
template <class F>
int group_run(scs_ctx* g, F&& f);
int group_destroy(scs_ctx* g);
int group_set_data(scs_ctx* g, int64_t N, int64_t m, const double* A, int64_t lda, const double* y, int64_t Nglob,
                   int64_t row0);
int group_gen_data(scs_ctx* g, const scs_synth* sp);
int group_get_data(scs_ctx* g, int64_t r0, int64_t nr, double* A, int64_t lda_out, double* y);
int group_set_test_data(scs_ctx* g, int64_t N, const double* A, int64_t lda, const double* y, int64_t Nglob,
                        int64_t row0);
int group_gen_test_data(scs_ctx* g, const scs_synth* sp);
int group_eval(scs_ctx* g, const double* x, double* out, int64_t nout, int (*fn)(scs_ctx*, const double*, double*));
int group_step(scs_ctx* g, const double* x, const double* x_prev, int64_t iter, const double* grad_fx, double* x_new,
               double* dx, double* pri);
int group_iterate(scs_ctx* g, const double* x0, const double* x_star, int64_t max_epoch, double x_tol, double f_tol,
                  int rel_kind, double* x_out, const scs_history* h, int64_t* n_hist, int64_t* epochs);
}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

// SCS_SEGV_TRACE=1: a fatal-signal handler that names the shared object and offset of every
// frame (dladdr), for faults outside this library's symbols (e.g. runtime teardown at exit).
// Diagnostics only; installed when the library is loaded.
static void scs_fatal_trace(int sig, siginfo_t* si, void*) {
  void* fr[48];
  const int n = backtrace(fr, 48);
  fprintf(stderr, "[scsopt] signal %d, fault address %p, %d frames:\n", sig, si ? si->si_addr : nullptr, n);
  for (int i = 0; i < n; ++i) {
    Dl_info d;
    if (dladdr(fr[i], &d) && d.dli_fname)
      fprintf(stderr, "  #%-2d %s +0x%lx %s\n", i, d.dli_fname, (unsigned long)((char*)fr[i] - (char*)d.dli_fbase),
              d.dli_sname ? d.dli_sname : "");
    else
      fprintf(stderr, "  #%-2d %p\n", i, fr[i]);
  }
  fflush(stderr);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void scs_install_trace() {
  const char* e = getenv("SCS_SEGV_TRACE");
  if (!e || e[0] != '1') return;
  void* warm[2];
  (void)backtrace(warm, 2);   // loads the unwinder now, not inside the handler
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = scs_fatal_trace;
  sa.sa_flags = SA_SIGINFO;
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGBUS, &sa, nullptr);
  sigaction(SIGABRT, &sa, nullptr);
}

const char* scs_version(void) { return "libscsopt 0.1.0 (gfx950)"; }

int scs_create(int device, void* stream, scs_ctx** out) {
  if (!out) return SCS_ERR_ARG;
  *out = nullptr;
  scs_ctx* c = new scs_ctx();
  int rc = guarded(c, [&] {
    HCK(hipSetDevice(device));
    c->dev = device;
    if (stream) {
      c->st = (hipStream_t)stream;
    } else {
      HCK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
      c->own_stream = true;
    }
  });
  if (rc != SCS_OK) {
    delete c;
    return rc;
  }
  *out = c;
  return SCS_OK;
}

int scs_destroy(scs_ctx* c) {
  if (is_group(c)) return group_destroy(c);
  if (!c) return SCS_OK;
  (void)hipSetDevice(c->dev);
  (void)hipStreamSynchronize(c->st);
  for (auto& p : c->pending) {
    (void)hipEventDestroy(p.e0);
    (void)hipEventDestroy(p.e1);
  }
  if (c->rccl) (void)ncclCommDestroy(c->rccl);
  for (auto& a : c->allocs) (void)hipFree(a.p);
  if (c->hscal) (void)hipHostFree(c->hscal);
  if (c->hserr) (void)hipHostFree(c->hserr);
  if (c->hring) (void)hipHostFree(c->hring);
  if (c->hloop) (void)hipHostFree(c->hloop);
  for (hipEvent_t e : c->loop_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->cbh) (void)hipHostFree(c->cbh);
  lu_aux_free(&c->lu);
  qr_aux_free(&c->qr);
  if (c->sf) {
    (void)hipStreamSynchronize(c->sf);
    (void)hipStreamDestroy(c->sf);
  }
  for (hipEvent_t e : c->evstrip) (void)hipEventDestroy(e);
  if (c->evfac) (void)hipEventDestroy(c->evfac);
  if (c->own_stream) (void)hipStreamDestroy(c->st);
  delete c;
  return SCS_OK;
}

const char* scs_last_error(const scs_ctx* c) { return c ? c->err.c_str() : "null context"; }

int scs_get_stream(scs_ctx* c, void** stream) {
  if (is_group(c)) return (*stream = (void*)c->st), SCS_OK;
  return guarded(c, [&] { *stream = (void*)c->st; });
}

int scs_set_comm(scs_ctx* c, int rank, int nranks, scs_allreduce_fn fn, void* user) {
  return guarded(c, [&] {
    if (nranks < 1 || rank < 0 || rank >= nranks) fail(c, SCS_ERR_ARG, "bad rank/nranks %d/%d", rank, nranks);
    if (nranks > 1 && !fn) fail(c, SCS_ERR_ARG, "nranks > 1 needs an all-reduce callback");
    if (c->rccl) {
      (void)ncclCommDestroy(c->rccl);
      c->rccl = nullptr;
    }
    c->rank = rank;
    c->nranks = nranks;
    c->ar = fn;
    c->ar_user = user;
  });
}

int scs_rccl_unique_id(void* id) {
  if (!id) return SCS_ERR_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return SCS_ERR_COMM;
  std::memcpy(id, &u, sizeof(u));
  return SCS_OK;
}

int scs_set_comm_rccl(scs_ctx* c, int rank, int nranks, const void* id) {
  return guarded(c, [&] {
    if (nranks < 1 || rank < 0 || rank >= nranks || !id)
      fail(c, SCS_ERR_ARG, "bad rank/nranks %d/%d or null id", rank, nranks);
    HCK(hipSetDevice(c->dev));
    sync(c);
    if (c->rccl) {
      (void)ncclCommDestroy(c->rccl);
      c->rccl = nullptr;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, nranks, u, rank);   // collective over the ranks
    if (r != ncclSuccess) fail(c, SCS_ERR_COMM, "ncclCommInitRank(%d of %d): %s", rank, nranks, ncclGetErrorString(r));
    c->rccl = comm;
    c->rank = rank;
    c->nranks = nranks;
    c->ar = nullptr;
    c->ar_user = nullptr;
  });
}

int scs_set_comm_force(scs_ctx* c, int on) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_comm_force(s_, on); });
  return guarded(c, [&] {
    if (on && !c->rccl && !c->ar) fail(c, SCS_ERR_STATE, "scs_set_comm_force needs a communicator");
    c->comm_force = on != 0;
  });
}

int scs_reduce_buffer_size(scs_ctx* c, int64_t* nd) {
  return guarded(c, [&] {
    if (!c->has_data) fail(c, SCS_ERR_STATE, "reduce buffer size needs the data dimensions");
    *nd = reduce_buffer_doubles(c);
  });
}

int scs_set_reduce_buffer(scs_ctx* c, void* p, int64_t nd) {
  return guarded(c, [&] {
    if (c->own_red) {
      dfree_t(c, c->red);
      c->own_red = false;
    }
    c->red = (double*)p;
    c->red_cap = nd;
  });
}

static void set_dims(scs_ctx* c, int64_t N, int64_t m, int64_t Nglob, int64_t row0) {
  if (m <= 0 || N < 0) fail(c, SCS_ERR_ARG, "bad dimensions N=%lld m=%lld", (long long)N, (long long)m);
  c->N = N;
  c->m = m;
  c->Npad = std::max<int64_t>(round_up(std::max<int64_t>(N, 1), 16), 16);
  c->mpad = round_up(m, 128);
  c->nstage = c->Npad / 16;
  c->Nglob = Nglob > 0 ? Nglob : N;
  c->Nglob_data = c->Nglob;
  c->row0 = row0;
}

static void reset_data(scs_ctx* c) {
  if (c->own_red) {   // sized by the old dimensions
    dfree_t(c, c->red);
    c->red_cap = 0;
    c->own_red = false;
  }
  dfree_t(c, c->A);
  dfree_t(c, c->rowptr);
  dfree_t(c, c->colptr);
  dfree_t(c, c->colidx);
  dfree_t(c, c->rowidx);
  dfree(c, c->val);
  dfree(c, c->valT);
  for (auto* B : {&c->bcsr, &c->bcsc, &c->bgram}) {
    dfree_t(c, B->ptr);
    dfree_t(c, B->lidx);
    dfree(c, B->val);
    B->nblk = B->shift = 0;
    B->nnz = 0;
  }
  dfree_t(c, c->sgseg.seg);
  dfree_t(c, c->sgseg.T);
  dfree_t(c, c->sgseg.tptr);
  dfree_t(c, c->sgseg.sw);
  c->sgseg.state = 0;
  c->sparse = false;
  dfree_t(c, c->Ad);
  dfree_t(c, c->ringA);
  c->sp_mode = 0;
  c->sp_gram = 0;
  c->ring_rows = 0;
  c->ring_r0[0] = c->ring_r0[1] = -1;
  dfree_t(c, c->Gk);
  free_view(c, c->cbv);
  dfree_t(c, c->cbstage);
  ++c->data_gen;
  c->nnz = 0;
  dfree_t(c, c->y);
  dfree_t(c, c->G);
  dfree_t(c, c->Gc);
  dfree_t(c, c->tiles);
  dfree_t(c, c->utiles);
  for (double** v : {&c->At, &c->Ps, &c->Ms, &c->bS, &c->uN, &c->hvec, &c->hg}) dfree_t(c, *v);
  dfree_t(c, c->stiles);
  c->n1pad = 0;
  c->NpS = 0;
  c->nstiles = 0;
  dfree_t(c, c->gwork);
  dfree_t(c, c->gcomb);
  dfree_t(c, c->gpart);
  dfree_t(c, c->vpart);
  for (auto& g : c->gstrip) {
    dfree_t(c, g.work);
    dfree_t(c, g.comb);
  }
  c->gstrip.clear();
  c->vpieces = 1;
  c->gseglen = c->gncomb = 0;
  c->gnsplit = 1;
  dfree_t(c, c->W);
  dfree_t(c, c->ysol);
  dfree_t(c, c->trilist);
  dfree_t(c, c->cinfo);
  dfree_t(c, c->lsbuf);
  c->lscap = 0;
  chol_aux_free(&c->caux);
  clear_batches(c);
  free_view(c, c->gview);
  free_test(c);
  c->gview_ok = false;
  c->ntiles = c->nslots = 0;
  invalidate_caches(c);
  c->has_data = false;
  c->reg_set = c->smooth_set = c->method_set = false;
}

int scs_set_data(scs_ctx* c, int64_t N, int64_t m, const double* A, int64_t lda, const double* y, int64_t Nglob,
                 int64_t row0) {
  if (is_group(c)) return group_set_data(c, N, m, A, lda, y, Nglob, row0);
  return guarded(c, [&] {
    HCK(hipSetDevice(c->dev));
    reset_data(c);
    set_dims(c, N, m, Nglob, row0);
    c->generic = (A == nullptr);
    if (!c->generic) {
      if (lda < N) fail(c, SCS_ERR_ARG, "lda (%lld) < N (%lld)", (long long)lda, (long long)N);
      c->A = dalloc<double>(c, (size_t)c->Npad * c->mpad);
      c->y = dalloc<double>(c, c->Npad);
      if (N > 0) {
        // panel by panel: host columns -> column-major staging buffer -> panel-blocked A
        double* C = dalloc<double>(c, (size_t)c->Npad * 128);
        upload_panels(c, A, N, lda, c->Npad, c->A, C);
        sync(c);
        dfree_t(c, C);
        if (y) h2d(c, c->y, y, N);
      }
    }
    alloc_mspace(c);
    alloc_nspace(c);
    sync(c);
    c->has_data = true;
  });
}

int scs_gen_data(scs_ctx* c, const scs_synth* s) {
  if (is_group(c)) return group_gen_data(c, s);
  return guarded(c, [&] {
    if (!s) fail(c, SCS_ERR_ARG, "null synth spec");
    HCK(hipSetDevice(c->dev));
    reset_data(c);
    set_dims(c, s->N, s->m, s->N_global, s->row0);
    c->generic = false;
    c->A = dalloc<double>(c, (size_t)c->Npad * c->mpad);
    c->y = dalloc<double>(c, c->Npad);
    alloc_mspace(c);
    alloc_nspace(c);
    const double scale = (s->kind == 3) ? 1.0 : 1.0 / std::sqrt((double)s->m);
    HCK(launch_gen_A(c->A, c->Npad, c->N, c->m, c->mpad, c->row0, s->seed, scale, c->st));
    HCK(launch_gen_xtrue(c->xn, c->m, s->seed, s->density, c->st));
    HCK(launch_gemv_n(c->A, c->nstage, c->Npad, c->mpad, c->xn, 1, c->zpart, c->Npad, c->st));
    HCK(launch_gen_y(s->kind, c->zpart, c->y, c->N, c->row0, s->seed, c->st));
    sync(c);
    c->has_data = true;
  });
}

int scs_get_data(scs_ctx* c, int64_t r0, int64_t nr, double* A, int64_t lda_out, double* y) {
  if (is_group(c)) return group_get_data(c, r0, nr, A, lda_out, y);
  return guarded(c, [&] {
    if (!c->has_data || c->generic) fail(c, SCS_ERR_STATE, "no data");
    if (c->sparse && A) fail(c, SCS_ERR_ARG, "sparse A: use scs_get_sparse");
    if (r0 < 0 || nr < 0 || r0 + nr > c->N) fail(c, SCS_ERR_ARG, "row range out of bounds");
    if (A && nr > 0) {
      double* C = dalloc<double>(c, (size_t)c->Npad * 128);
      for (int64_t p = 0; p < c->mpad / 128; ++p) {
        const int64_t j0 = p * 128, nc = std::min<int64_t>(128, c->m - j0);
        if (nc <= 0) break;
        HCK(launch_retile(C, c->A, c->Npad, p, 0, c->st));
        HCK(hipMemcpy2DAsync(A + j0 * lda_out, sizeof(double) * lda_out, C + r0, sizeof(double) * c->Npad,
                             sizeof(double) * nr, nc, hipMemcpyDeviceToHost, c->st));
      }
      sync(c);
      dfree_t(c, C);
    }
    if (y && nr > 0) d2h(c, y, c->y + r0, nr);
    sync(c);
  });
}

int scs_get_dims(scs_ctx* c, int64_t* N, int64_t* m, int64_t* Ng, int64_t* r0) {
  if (is_group(c)) {   // the group holds the whole problem
    if (N) *N = c->grpN;
    if (m) *m = c->grpm;
    if (Ng) *Ng = c->grpN;
    if (r0) *r0 = 0;
    return SCS_OK;
  }
  return guarded(c, [&] {
    if (N) *N = c->N;
    if (m) *m = c->m;
    if (Ng) *Ng = c->Nglob;
    if (r0) *r0 = c->row0;
  });
}

static void* dalloc_vals(scs_ctx* c, int64_t n, int f32) {
  return f32 ? (void*)dalloc<float>(c, (size_t)n) : (void*)dalloc<double>(c, (size_t)n);
}

static void upload_vals(scs_ctx* c, void* dst, const double* src, int64_t n, int f32) {
  if (!f32) {
    HCK(hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
    sync(c);
    return;
  }
  std::vector<float> h((size_t)n);
  for (int64_t i = 0; i < n; ++i) h[i] = (float)src[i];
  HCK(hipMemcpyAsync(dst, h.data(), sizeof(float) * n, hipMemcpyHostToDevice, c->st));
  sync(c);
}

// Sort each row's entries by index (in place: the arrays are replaced by sorted
// copies) and build the LDS-blocked copy B (sparse.hip).
static void build_blocked(scs_ctx* c, int64_t nrows, int64_t ncols, int64_t* ptr, int*& idx, void*& val,
                          scs_ctx::SpBlk& B) {
  const int64_t nnz = c->nnz;
  size_t tb = 0;
  if (nnz > 0 && nrows > 0) {
    int end_bit = 1;
    while ((int64_t(1) << end_bit) < ncols) ++end_bit;
    int* idx_s = dalloc<int>(c, nnz);
    void* val_s = dalloc_vals(c, nnz, c->sp_f32);
    HCK(sort_segments(nullptr, &tb, idx, idx_s, val, val_s, c->sp_f32, nnz, nrows, ptr, end_bit, c->st));
    void* tmp = dalloc<char>(c, tb);
    HCK(sort_segments(tmp, &tb, idx, idx_s, val, val_s, c->sp_f32, nnz, nrows, ptr, end_bit, c->st));
    sync(c);
    dfree(c, tmp);
    dfree_t(c, idx);
    dfree(c, val);
    idx = idx_s;
    val = val_s;
  }
  B.shift = spmv_blk_shift(ncols);
  B.nblk = (int)ceil_div(ncols, int64_t(1) << B.shift);
  const int64_t nk = (int64_t)B.nblk * nrows;
  int64_t* cnt = dalloc<int64_t>(c, nk + 1);
  int64_t* first = dalloc<int64_t>(c, nk + 1);
  B.ptr = dalloc<int64_t>(c, nk + 1);
  if (nrows > 0) {
    HCK(blk_count(ptr, idx, nrows, B.shift, cnt, first, c->st));
    // segments in whole slots of 4 (fp64) / 8 (fp32) entries (padding: index 16384 = the SpMV's
    // zero slot, value 0; launch_spmv_blk)
    HCK(blk_pad(cnt, nk, c->sp_f32, c->st));
    tb = 0;
    HCK(blk_scan(nullptr, &tb, cnt, B.ptr, nk + 1, c->st));
    void* tmp = dalloc<char>(c, tb);
    HCK(blk_scan(tmp, &tb, cnt, B.ptr, nk + 1, c->st));
    int64_t nnzp = 0;
    HCK(hipMemcpyAsync(&nnzp, B.ptr + nk, sizeof(int64_t), hipMemcpyDeviceToHost, c->st));
    sync(c);
    dfree(c, tmp);
    B.lidx = dalloc<uint16_t>(c, nnzp + 8);
    HCK(hipMemsetD16Async((hipDeviceptr_t)B.lidx, (unsigned short)spmv_pad_index(), (size_t)(nnzp + 8), c->st));
    B.val = dalloc_vals(c, nnzp + 8, c->sp_f32);
    HCK(blk_scatter(ptr, idx, val, c->sp_f32, nrows, B.shift, B.ptr, first, B.lidx, B.val, c->st));
    sync(c);
  } else {
    B.lidx = dalloc<uint16_t>(c, 4);
    B.val = dalloc_vals(c, 4, c->sp_f32);
  }
  sync(c);
  dfree_t(c, cnt);
  dfree_t(c, first);
}

int scs_set_sparse(scs_ctx* c, int64_t N, int64_t m, int64_t nnz, const int64_t* rowptr, const int32_t* colidx,
                   const double* val, const int64_t* colptr, const int32_t* rowidx, const double* valT, int f32,
                   const double* y, int64_t Nglob, int64_t row0) {
  return guarded(c, [&] {
    if (nnz < 0 || !rowptr || !colptr || (nnz > 0 && (!colidx || !val || !rowidx || !valT)))
      fail(c, SCS_ERR_ARG, "sparse A: null arrays");
    if (rowptr[0] != 0 || rowptr[N] != nnz || colptr[0] != 0 || colptr[m] != nnz)
      fail(c, SCS_ERR_ARG, "sparse A: rowptr/colptr must start at 0 and end at nnz");
    for (int64_t i = 0; i < N; ++i)
      if (rowptr[i + 1] < rowptr[i]) fail(c, SCS_ERR_ARG, "sparse A: rowptr not monotone at %lld", (long long)i);
    for (int64_t j = 0; j < m; ++j)
      if (colptr[j + 1] < colptr[j]) fail(c, SCS_ERR_ARG, "sparse A: colptr not monotone at %lld", (long long)j);
    for (int64_t p = 0; p < nnz; ++p)
      if (colidx[p] < 0 || colidx[p] >= m || rowidx[p] < 0 || rowidx[p] >= N)
        fail(c, SCS_ERR_ARG, "sparse A: index out of range at %lld", (long long)p);
    if (nnz > INT32_MAX * 64LL) fail(c, SCS_ERR_ARG, "sparse A: nnz too large");
    HCK(hipSetDevice(c->dev));
    reset_data(c);
    set_dims(c, N, m, Nglob, row0);
    c->generic = false;
    c->sparse = true;
    c->sp_f32 = f32 ? 1 : 0;
    c->nnz = nnz;
    c->rowptr = dalloc<int64_t>(c, N + 1);
    c->colptr = dalloc<int64_t>(c, m + 1);
    c->colidx = dalloc<int>(c, nnz);
    c->rowidx = dalloc<int>(c, nnz);
    c->val = dalloc_vals(c, nnz, c->sp_f32);
    c->valT = dalloc_vals(c, nnz, c->sp_f32);
    HCK(hipMemcpyAsync(c->rowptr, rowptr, sizeof(int64_t) * (N + 1), hipMemcpyHostToDevice, c->st));
    HCK(hipMemcpyAsync(c->colptr, colptr, sizeof(int64_t) * (m + 1), hipMemcpyHostToDevice, c->st));
    if (nnz > 0) {
      HCK(hipMemcpyAsync(c->colidx, colidx, sizeof(int) * nnz, hipMemcpyHostToDevice, c->st));
      HCK(hipMemcpyAsync(c->rowidx, rowidx, sizeof(int) * nnz, hipMemcpyHostToDevice, c->st));
      upload_vals(c, c->val, val, nnz, c->sp_f32);
      upload_vals(c, c->valT, valT, nnz, c->sp_f32);
    }
    c->y = dalloc<double>(c, c->Npad);
    if (y && N > 0) h2d(c, c->y, y, N);
    build_blocked(c, N, m, c->rowptr, c->colidx, c->val, c->bcsr);
    build_blocked(c, m, N, c->colptr, c->rowidx, c->valT, c->bcsc);
    alloc_mspace(c);
    alloc_nspace(c);
    sync(c);
    c->has_data = true;
  });
}

int scs_gen_sparse(scs_ctx* c, const scs_synth* s, int f32) {
  return guarded(c, [&] {
    if (!s) fail(c, SCS_ERR_ARG, "null synth spec");
    if (s->kind != 4) fail(c, SCS_ERR_ARG, "scs_gen_sparse: kind must be 4");
    const int64_t N = s->N, m = s->m;
    if (N <= 0 || (N & (N - 1)) != 0 || m <= 0 || N % m != 0)
      fail(c, SCS_ERR_ARG, "scs_gen_sparse: N must be a power of two and a multiple of m");
    if ((s->N_global > 0 && s->N_global != N) || s->row0 != 0)
      fail(c, SCS_ERR_ARG, "scs_gen_sparse: single-context generator (shard with scs_set_sparse)");
    const int k = (int)std::max<int64_t>(1, std::llround(s->density * (double)m));
    if (k > m) fail(c, SCS_ERR_ARG, "scs_gen_sparse: density > 1");
    const int64_t nnz = N * (int64_t)k;
    HCK(hipSetDevice(c->dev));
    reset_data(c);
    set_dims(c, N, m, N, 0);
    c->generic = false;
    c->sparse = true;
    c->sp_f32 = f32 ? 1 : 0;
    c->nnz = nnz;
    c->rowptr = dalloc<int64_t>(c, N + 1);
    c->colptr = dalloc<int64_t>(c, m + 1);
    c->colidx = dalloc<int>(c, nnz);
    c->rowidx = dalloc<int>(c, nnz);
    c->val = dalloc_vals(c, nnz, c->sp_f32);
    c->valT = dalloc_vals(c, nnz, c->sp_f32);
    c->y = dalloc<double>(c, c->Npad);
    alloc_mspace(c);
    std::vector<char> maps(sparse_layer_map_bytes(k));
    sparse_layer_maps(s->seed, k, N, maps.data());
    void* dmaps = dalloc<char>(c, maps.size());
    HCK(hipMemcpyAsync(dmaps, maps.data(), maps.size(), hipMemcpyHostToDevice, c->st));
    HCK(launch_gen_sparse(N, m, k, s->seed, dmaps, c->sp_f32, 1.0 / std::sqrt((double)k), c->rowptr, c->colidx,
                          c->val, c->colptr, c->rowidx, c->valT, c->st));
    build_blocked(c, N, m, c->rowptr, c->colidx, c->val, c->bcsr);
    build_blocked(c, m, N, c->colptr, c->rowidx, c->valT, c->bcsc);
    alloc_nspace(c);
    HCK(launch_gen_uniform(c->xn, m, s->seed, -1.5, 1.5, c->st));
    const int ns = matvec_n(c, c->xn, c->nsplit);
    HCK(launch_epilogue(SCS_LOSS_LEAST_SQUARES, SCS_GGN_NONE, EPI_Z, c->zpart, ns, c->Npad, c->y, c->N, c->Npad, 1.0,
                        c->z, nullptr, nullptr, nullptr, nullptr, c->valpart, c->st));
    HCK(launch_gen_y(3, c->z, c->y, c->N, 0, s->seed, c->st));
    sync(c);
    dfree(c, dmaps);
    c->has_data = true;
  });
}

int scs_get_nnz(scs_ctx* c, int64_t* nnz) {
  return guarded(c, [&] {
    if (!c->has_data || !c->sparse) fail(c, SCS_ERR_STATE, "no sparse data");
    *nnz = c->nnz;
  });
}

int scs_get_sparse(scs_ctx* c, int64_t* rowptr, int32_t* colidx, double* val) {
  return guarded(c, [&] {
    if (!c->has_data || !c->sparse) fail(c, SCS_ERR_STATE, "no sparse data");
    if (rowptr) HCK(hipMemcpyAsync(rowptr, c->rowptr, sizeof(int64_t) * (c->N + 1), hipMemcpyDeviceToHost, c->st));
    if (colidx && c->nnz)
      HCK(hipMemcpyAsync(colidx, c->colidx, sizeof(int) * c->nnz, hipMemcpyDeviceToHost, c->st));
    if (val && c->nnz) {
      if (c->sp_f32) {
        std::vector<float> h((size_t)c->nnz);
        HCK(hipMemcpyAsync(h.data(), c->val, sizeof(float) * c->nnz, hipMemcpyDeviceToHost, c->st));
        sync(c);
        for (int64_t p = 0; p < c->nnz; ++p) val[p] = h[p];
      } else {
        HCK(hipMemcpyAsync(val, c->val, sizeof(double) * c->nnz, hipMemcpyDeviceToHost, c->st));
      }
    }
    sync(c);
  });
}

// ---- held-out data (Problem(...; Atest, ytest), problems.jl:27-28,67-68) -----------------------
// the rows of a new held-out view (after free_test): Npad, nstage and the buffers of its dense form
static void test_view_dims(scs_ctx* c, int64_t N, int64_t Nglob, bool sparse) {
  if (!c->has_data || c->generic)
    fail(c, SCS_ERR_STATE, "test data needs a data problem: call scs_set_data / scs_gen_data / scs_set_sparse first");
  if (N < 0) fail(c, SCS_ERR_ARG, "test data: N = %lld", (long long)N);
  NView& v = c->tset.v;
  v.N = N;
  v.Nglob = Nglob > 0 ? Nglob : N;
  v.Npad = std::max<int64_t>(round_up(std::max<int64_t>(N, 1), 16), 16);
  v.nstage = v.Npad / 16;
  v.sparse = sparse;
  v.y = dalloc<double>(c, v.Npad);
  if (!sparse) v.A = dalloc<double>(c, (size_t)v.Npad * c->mpad);
}

int scs_set_test_data(scs_ctx* c, int64_t N, const double* A, int64_t lda, const double* y, int64_t Nglob,
                      int64_t row0) {
  if (is_group(c)) return group_set_test_data(c, N, A, lda, y, Nglob, row0);
  return guarded(c, [&] {
    HCK(hipSetDevice(c->dev));
    free_test(c);
    if (!A && !y) return;   // clears the held-out set
    if (!A || !y) {         // the reference's xor case (iterate.jl:170-171): recorded, not an error here
      c->tset.xor_case = true;
      return;
    }
    if (lda < N) fail(c, SCS_ERR_ARG, "test data: lda (%lld) < N (%lld)", (long long)lda, (long long)N);
    (void)row0;
    test_view_dims(c, N, Nglob, false);
    TestScope ts(c);
    if (N > 0) {
      double* C = dalloc<double>(c, (size_t)c->Npad * 128);
      upload_panels(c, A, N, lda, c->Npad, c->A, C);
      h2d(c, c->y, y, N);
      sync(c);
      dfree_t(c, C);
    }
    alloc_nspace(c);
    sync(c);
    c->tset.on = true;
  });
}

int scs_set_test_sparse(scs_ctx* c, int64_t N, int64_t nnz, const int64_t* rowptr, const int32_t* colidx,
                        const double* val, int f32, const double* y, int64_t Nglob, int64_t row0) {
  if (is_group(c)) {
    c->err = "sparse test data takes a single-device context";
    return SCS_ERR_ARG;
  }
  return guarded(c, [&] {
    HCK(hipSetDevice(c->dev));
    free_test(c);
    if (!rowptr || !y || nnz < 0 || (nnz > 0 && (!colidx || !val)))
      fail(c, SCS_ERR_ARG, "sparse test data: null arrays (Atest and ytest are both required)");
    if (N < 0 || rowptr[0] != 0 || rowptr[N] != nnz)
      fail(c, SCS_ERR_ARG, "sparse test data: rowptr must start at 0 and end at nnz");
    for (int64_t i = 0; i < N; ++i)
      if (rowptr[i + 1] < rowptr[i]) fail(c, SCS_ERR_ARG, "sparse test data: rowptr not monotone at %lld", (long long)i);
    for (int64_t p = 0; p < nnz; ++p)
      if (colidx[p] < 0 || colidx[p] >= c->m)
        fail(c, SCS_ERR_ARG, "sparse test data: column index out of range at %lld", (long long)p);
    if (nnz > INT32_MAX * 64LL) fail(c, SCS_ERR_ARG, "sparse test data: nnz too large");
    (void)row0;
    test_view_dims(c, N, Nglob, true);
    TestScope ts(c);
    c->sp_f32 = f32 ? 1 : 0;
    c->nnz = nnz;
    c->rowptr = dalloc<int64_t>(c, N + 1);
    c->colidx = dalloc<int>(c, nnz);
    c->val = dalloc_vals(c, nnz, c->sp_f32);
    HCK(hipMemcpyAsync(c->rowptr, rowptr, sizeof(int64_t) * (N + 1), hipMemcpyHostToDevice, c->st));
    if (nnz > 0) {
      HCK(hipMemcpyAsync(c->colidx, colidx, sizeof(int) * nnz, hipMemcpyHostToDevice, c->st));
      upload_vals(c, c->val, val, nnz, c->sp_f32);
    }
    if (N > 0) h2d(c, c->y, y, N);
    build_blocked(c, N, c->m, c->rowptr, c->colidx, c->val, c->bcsr);
    alloc_nspace(c);
    sync(c);
    c->tset.on = true;
  });
}

int scs_gen_test_data(scs_ctx* c, const scs_synth* s) {
  if (is_group(c)) return group_gen_test_data(c, s);
  return guarded(c, [&] {
    if (!s) fail(c, SCS_ERR_ARG, "null synth spec");
    if (s->kind < 1 || s->kind > 3) fail(c, SCS_ERR_ARG, "scs_gen_test_data: dense kinds 1-3");
    if (s->m != c->m) fail(c, SCS_ERR_ARG, "scs_gen_test_data: m = %lld, the data has %lld", (long long)s->m,
                           (long long)c->m);
    HCK(hipSetDevice(c->dev));
    free_test(c);
    test_view_dims(c, s->N, s->N_global, false);
    TestScope ts(c);
    alloc_nspace(c);
    const double scale = (s->kind == 3) ? 1.0 : 1.0 / std::sqrt((double)s->m);
    // rows [row0, row0 + N) of the same generator as scs_gen_data: with row0 >= the data's N_global
    // they are held-out samples of the same distribution (the same x_true)
    HCK(launch_gen_A(c->A, c->Npad, c->N, c->m, c->mpad, s->row0, s->seed, scale, c->st));
    HCK(launch_gen_xtrue(c->xn, c->m, s->seed, s->density, c->st));
    HCK(launch_gemv_n(c->A, c->nstage, c->Npad, c->mpad, c->xn, 1, c->zpart, c->Npad, c->st));
    HCK(launch_gen_y(s->kind, c->zpart, c->y, c->N, s->row0, s->seed, c->st));
    sync(c);
    c->tset.on = true;
  });
}

int scs_set_test_callback(scs_ctx* c, int on) {
  if (is_group(c)) {
    c->err = "a callback loss takes a single-device context";
    return SCS_ERR_ARG;
  }
  return guarded(c, [&] {
    free_test(c);
    if (!on) return;
    if (c->loss != SCS_LOSS_CALLBACK || !c->cb)
      fail(c, SCS_ERR_STATE, "scs_set_test_callback: the loss is not a callback (scs_set_loss_callback first)");
    c->tset.on = c->tset.host = true;
  });
}

int scs_eval_ftest(scs_ctx* c, const double* x, double* fval) {
  if (is_group(c)) return group_eval(c, x, fval, 1, scs_eval_ftest);
  return guarded(c, [&] {
    if (!x || !fval) fail(c, SCS_ERR_ARG, "scs_eval_ftest: null argument");
    if (!c->has_data || !c->loss_set) fail(c, SCS_ERR_STATE, "scs_eval_ftest: needs the data and the loss");
    HCK(hipSetDevice(c->dev));
    h2d(c, c->xn, x, c->m);
    *fval = eval_ftest_dev(c, x, c->xn);
  });
}

int scs_has_test(scs_ctx* c, int* on) {
  if (!on) return SCS_ERR_ARG;
  if (is_group(c)) return scs_has_test(c->subs[0], on);
  *on = c->tset.on ? 1 : 0;
  return SCS_OK;
}

int scs_set_loss(scs_ctx* c, int loss, int ggn, double scale) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_loss(s_, loss, ggn, scale); });
  return guarded(c, [&] {
    if (loss < SCS_LOSS_LOGISTIC_MARGIN || loss > SCS_LOSS_CALLBACK) fail(c, SCS_ERR_ARG, "unknown loss %d", loss);
    if (ggn < SCS_GGN_NONE || ggn > SCS_GGN_LINEAR_LS) fail(c, SCS_ERR_ARG, "unknown ggn kind %d", ggn);
    if ((loss == SCS_LOSS_QUADRATIC || loss == SCS_LOSS_ROSENBROCK || loss == SCS_LOSS_CALLBACK) && sharded(c))
      fail(c, SCS_ERR_ARG, "quadratic / Rosenbrock / callback problems are not row-sharded");
    if (loss == SCS_LOSS_CALLBACK && (!c->has_data || !c->generic))
      fail(c, SCS_ERR_ARG, "a callback loss holds no device data: scs_set_data(N = 0, A = NULL, m) first");
    if (loss == SCS_LOSS_CALLBACK && ggn != SCS_GGN_NONE)
      fail(c, SCS_ERR_ARG, "a callback loss has no out_fn kind (its GGN pieces come from the callback)");
    c->loss = loss;
    c->ggn = ggn;
    c->scale = scale;
    c->loss_set = true;
    ++c->data_gen;
    invalidate_caches(c);
  });
}

int scs_set_loss_callback(scs_ctx* c, scs_loss_fn fn, void* user, int64_t ggn_rows) {
  return guarded(c, [&] {
    if (ggn_rows < 0) fail(c, SCS_ERR_ARG, "ggn_rows must be >= 0");
    c->cb = fn;
    c->cb_user = user;
    if (ggn_rows != c->cb_nout) {
      free_view(c, c->cbv);
      dfree_t(c, c->cbstage);
      c->cb_nout = ggn_rows;
    }
    invalidate_caches(c);
  });
}

static double* upload_bounds(scs_ctx* c, double* old, const double* v, int64_t nb, bool sanitize, bool lower) {
  dfree_t(c, old);
  std::vector<double> h(c->mpad, 0.0);
  for (int64_t i = 0; i < c->m; ++i) {
    double b = (nb == 1) ? v[0] : v[i];
    if (sanitize) {
      if (lower && b == -INFINITY) b = -1e32;  // L_INF_CACHE, prox-reg-utils.jl:6
      if (!lower && b == INFINITY) b = 1e32;   // U_INF_CACHE
    }
    h[i] = b;
  }
  double* d = dalloc<double>(c, c->mpad);
  h2d(c, d, h.data(), c->mpad);
  sync(c);
  return d;
}

int scs_set_reg(scs_ctx* c, int reg, const double* lam, int nlam, const double* lb, const double* ub, int64_t nbound,
                const int64_t* ind, int64_t ngroups) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_reg(s_, reg, lam, nlam, lb, ub, nbound, ind, ngroups); });
  return guarded(c, [&] {
    if (!c->has_data) fail(c, SCS_ERR_STATE, "set the data before the regularizer");
    if (reg < SCS_REG_L1 || reg > SCS_REG_GL) fail(c, SCS_ERR_REF, "reg_name not valid.");
    if (nlam < 1 || nlam > 2 || !lam) fail(c, SCS_ERR_ARG, "λ must have 1 or 2 entries");
    if (reg == SCS_REG_GL && nlam != 2)
      fail(c, SCS_ERR_REF, "Please provide a Tuple or Vector with exactly two entries for λ, e.g. [λ1, λ2]");
    c->reg = reg;
    c->nlam = nlam;
    c->lam = lam[0];  // step! uses λ = model.λ[1] when length(λ) > 1
    c->lam2 = nlam > 1 ? lam[1] : 0.0;
    if (reg == SCS_REG_INDBOX) {
      if (!lb || !ub || (nbound != 1 && nbound != c->m)) fail(c, SCS_ERR_ARG, "indbox needs C_set bounds (1 or m)");
      c->clb = upload_bounds(c, c->clb, lb, nbound, false, true);
      c->cub = upload_bounds(c, c->cub, ub, nbound, false, false);
    }
    if (reg == SCS_REG_GL) {
      if (!ind || ngroups < 1) fail(c, SCS_ERR_ARG, "gl needs the group index matrix");
      std::vector<int> hs(ngroups), he(ngroups);
      std::vector<double> hw(ngroups), wel(c->mpad, 0.0);
      // get_Cmat (prox-reg-utils.jl:121-142) needs the ranges to cover 1..n exactly once, in any
      // order (a gap leaves a zero column index, an overlap makes Cmat longer than x)
      std::vector<char> seen(c->m, 0);
      for (int64_t g = 0; g < ngroups; ++g) {
        const int64_t s = ind[3 * g], e = ind[3 * g + 1], w = ind[3 * g + 2];
        if (s < 1 || e < s || e > c->m)
          fail(c, SCS_ERR_ARG, "group %lld = %lld:%lld is outside 1..%lld", (long long)g + 1, (long long)s,
               (long long)e, (long long)c->m);
        for (int64_t k = s - 1; k < e; ++k) {
          if (seen[k]) fail(c, SCS_ERR_ARG, "groups overlap at %lld: they must partition 1..m", (long long)k + 1);
          seen[k] = 1;
          wel[k] = (double)w;
        }
        hs[g] = (int)(s - 1);
        he[g] = (int)(e - 1);
        hw[g] = (double)w;
      }
      for (int64_t k = 0; k < c->m; ++k)
        if (!seen[k]) fail(c, SCS_ERR_ARG, "groups must partition 1..m (%lld is in no group)", (long long)k + 1);
      dfree_t(c, c->gmap);
      dfree_t(c, c->gstart);
      dfree_t(c, c->gend);
      dfree_t(c, c->gw);
      dfree_t(c, c->wel);
      c->gstart = dalloc<int>(c, ngroups);
      c->gend = dalloc<int>(c, ngroups);
      c->gw = dalloc<double>(c, ngroups);
      c->wel = dalloc<double>(c, c->mpad);
      HCK(hipMemcpyAsync(c->gstart, hs.data(), sizeof(int) * ngroups, hipMemcpyHostToDevice, c->st));
      HCK(hipMemcpyAsync(c->gend, he.data(), sizeof(int) * ngroups, hipMemcpyHostToDevice, c->st));
      h2d(c, c->gw, hw.data(), ngroups);
      h2d(c, c->wel, wel.data(), c->mpad);
      c->ngroups = (int)ngroups;
      sync(c);
    }
    c->reg_set = true;
  });
}

int scs_set_compute_f32(scs_ctx* c, int on) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_compute_f32(s_, on); });
  return guarded(c, [&] {
    sync(c);
    c->f32c = on ? 1 : 0;
    invalidate_caches(c);
  });
}

int scs_set_solver(scs_ctx* c, int kind) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_solver(s_, kind); });
  return guarded(c, [&] {
    if (kind != SCS_SOLVER_DEFAULT && kind != SCS_SOLVER_REFERENCE) fail(c, SCS_ERR_ARG, "scs_set_solver: kind %d", kind);
    c->solver = kind;
  });
}

int scs_set_gram_cache(scs_ctx* c, int on) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_gram_cache(s_, on); });
  return guarded(c, [&] {
    c->gram_cache = on ? 1 : 0;
    ++c->data_gen;
    if (!on) dfree_t(c, c->Gk);
  });
}

int scs_set_group_map(scs_ctx* c, const int64_t* G, int64_t ntotal) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_group_map(s_, G, ntotal); });
  return guarded(c, [&] {
    if (!c->reg_set || c->reg != SCS_REG_GL) fail(c, SCS_ERR_STATE, "scs_set_group_map needs reg gl set first");
    if (!G || ntotal != c->m)
      fail(c, SCS_ERR_ARG, "G must select every variable once (length %lld, m = %lld)", (long long)ntotal,
           (long long)c->m);
    std::vector<int> h(ntotal);
    std::vector<char> seen(c->m, 0);
    bool ident = true;
    for (int64_t k = 0; k < ntotal; ++k) {
      if (G[k] < 1 || G[k] > c->m || seen[G[k] - 1]) fail(c, SCS_ERR_ARG, "G must be a permutation of 1..m");
      seen[G[k] - 1] = 1;
      h[k] = (int)(G[k] - 1);
      ident = ident && (G[k] == k + 1);
    }
    dfree_t(c, c->gmap);
    if (ident) return;
    c->gmap = dalloc<int>(c, ntotal);
    HCK(hipMemcpyAsync(c->gmap, h.data(), sizeof(int) * ntotal, hipMemcpyHostToDevice, c->st));
    sync(c);
  });
}

int scs_set_smoother(scs_ctx* c, int kind, double mu, double Mh, double nu, const double* lb, const double* ub,
                     int64_t nbound) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_smoother(s_, kind, mu, Mh, nu, lb, ub, nbound); });
  return guarded(c, [&] {
    if (!c->has_data) fail(c, SCS_ERR_STATE, "set the data before the smoother");
    if (kind < SCS_SMOOTH_PHUBER_L1L2 || kind > SCS_SMOOTH_OSBA_GL) fail(c, SCS_ERR_ARG, "unknown smoother %d", kind);
    if (kind == SCS_SMOOTH_PHUBER_INDBOX || kind == SCS_SMOOTH_EXP_INDBOX || kind == SCS_SMOOTH_LOGEXP_INDBOX) {
      if (!lb || !ub || (nbound != 1 && nbound != c->m))
        fail(c, SCS_ERR_REF, "Lengths of the bounds do not match that of the variable.");
      c->slb = upload_bounds(c, c->slb, lb, nbound, true, true);
      c->sub = upload_bounds(c, c->sub, ub, nbound, true, false);
    }
    if ((kind == SCS_SMOOTH_PHUBER_GL || kind == SCS_SMOOTH_OSBA_GL) && !c->wel)
      fail(c, SCS_ERR_STATE, "%s needs the gl groups (scs_set_reg)",
           kind == SCS_SMOOTH_PHUBER_GL ? "PHuberSmootherGL" : "OsBaSmootherGL");
    c->smooth = kind;
    c->mu = mu;
    c->Mh = Mh;
    c->nu = nu;
    c->smooth_set = true;
    invalidate_caches(c);
  });
}

int scs_set_L(scs_ctx* c, int has_L, double L) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_L(s_, has_L, L); });
  return guarded(c, [&] {
    c->has_L = has_L != 0;
    c->L = L;
  });
}

int scs_method_init(scs_ctx* c, int method, int ss_type, int use_prox, int mem) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_method_init(s_, method, ss_type, use_prox, mem); });
  return guarded(c, [&] {
    if (!c->has_data) fail(c, SCS_ERR_STATE, "set the data before the method");
    if (method < SCS_PROX_NSCORE || method > SCS_PROX_LQNSCORE) fail(c, SCS_ERR_ARG, "unknown method %d", method);
    if (method == SCS_PROX_GGNSCORE && c->loss == SCS_LOSS_CALLBACK && c->cb_nout <= 0)
      fail(c, SCS_ERR_ARG, "ProxGGNSCORE on a callback loss needs jac_yx / grad_fy / hess_fy (ggn_rows > 0)");
    if (method == SCS_PROX_GGNSCORE && c->loss != SCS_LOSS_CALLBACK && (c->generic || c->loss == SCS_LOSS_QUADRATIC))
      fail(c, SCS_ERR_ARG, "ProxGGNSCORE needs a data problem with an out_fn (GGN kind)");
    c->method = method;
    c->ss_type = ss_type;
    c->use_prox = use_prox;
    c->mem = mem;
    if (method == SCS_PROX_LQNSCORE) {
      if (mem < 1) fail(c, SCS_ERR_ARG, "L-BFGS memory must be >= 1");
      dfree_t(c, c->S);
      dfree_t(c, c->Yv);
      dfree_t(c, c->d_order);
      dfree_t(c, c->ab);
      dfree_t(c, c->tlwork);
      c->tlwork = dalloc<double>(c, (size_t)(mem + 5) * TWO_LOOP_MAX_WG);
      c->S = dalloc<double>(c, (size_t)(mem + 1) * c->mpad);
      c->Yv = dalloc<double>(c, (size_t)(mem + 1) * c->mpad);
      c->d_order = dalloc<int>(c, mem + 3);   // order[0..mem] | k | spare (the device ring)
      if (c->hring) (void)hipHostFree(c->hring);
      c->hring = nullptr;
      HCK(hipHostMalloc((void**)&c->hring, sizeof(int) * (mem + 3), hipHostMallocDefault));
      c->ab = dalloc<double>(c, 2 * (mem + 1));
      sync(c);
    }
    // init! (prox-L-BFGS-SCORE.jl:31-36)
    c->ring.clear();
    c->spare = 0;
    c->H0 = 1.0;
    c->lbfgs_pending = false;
    c->method_set = true;
    invalidate_caches(c);
  });
}

int scs_eval_f(scs_ctx* c, const double* x, double* fval) {
  if (is_group(c)) return group_eval(c, x, fval, 1, scs_eval_f);
  return guarded(c, [&] {
    if (!c->has_data) fail(c, SCS_ERR_STATE, "no data: call scs_set_data / scs_gen_data first");
    if (!c->loss_set) fail(c, SCS_ERR_STATE, "no loss: call scs_set_loss first");
    HCK(hipSetDevice(c->dev));
    h2d(c, c->xn, x, c->m);
    *fval = eval_f_dev(c, x, c->xn);
  });
}

int scs_eval_grad(scs_ctx* c, const double* x, double* g) {
  if (is_group(c)) return group_eval(c, x, g, c->grpm, scs_eval_grad);
  return guarded(c, [&] {
    if (!c->has_data) fail(c, SCS_ERR_STATE, "no data: call scs_set_data / scs_gen_data first");
    if (!c->loss_set) fail(c, SCS_ERR_STATE, "no loss: call scs_set_loss first");
    HCK(hipSetDevice(c->dev));
    h2d(c, c->xn, x, c->m);
    grad_f_dev(c, x, c->xn, c->gqn);
    d2h(c, g, c->gqn, c->m);
    sync(c);
  });
}

int scs_eval_reg(scs_ctx* c, const double* x, double* gval) {
  if (is_group(c)) return group_eval(c, x, gval, 1, scs_eval_reg);
  return guarded(c, [&] {
    require_ready(c, false);
    HCK(hipSetDevice(c->dev));
    h2d(c, c->xn, x, c->m);
    *gval = eval_reg_dev(c, c->xn);
  });
}

int scs_set_batches(scs_ctx* c, const int64_t* rows, const int64_t* offsets, int64_t nbatch) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_set_batches(s_, rows, offsets, nbatch); });
  return guarded(c, [&] {
    HCK(hipSetDevice(c->dev));
    sync(c);
    clear_batches(c);
    invalidate_caches(c);
    if (nbatch == 0) return;
    if (!c->has_data) fail(c, SCS_ERR_STATE, "no data: call scs_set_data / scs_gen_data first");
    if (c->generic) fail(c, SCS_ERR_ARG, "a ProblemGeneric has no samples to batch");
    if (nbatch < 0 || !rows || !offsets || offsets[0] != 0) fail(c, SCS_ERR_ARG, "scs_set_batches: bad batch list");
    for (int64_t b = 0; b < nbatch; ++b)
      if (offsets[b + 1] <= offsets[b]) fail(c, SCS_ERR_ARG, "scs_set_batches: batch %lld is empty", (long long)b);
    const int64_t tot = offsets[nbatch];
    // rows are global indices (row0 = 0, Nglob = N on one rank): keep this rank's rows of each batch
    for (int64_t i = 0; i < tot; ++i)
      if (rows[i] < 0 || rows[i] >= c->Nglob)
        fail(c, SCS_ERR_ARG, "scs_set_batches: row %lld out of range", (long long)rows[i]);
    std::vector<int64_t> loc;
    c->boff.assign(1, 0);
    for (int64_t b = 0; b < nbatch; ++b) {
      for (int64_t i = offsets[b]; i < offsets[b + 1]; ++i)
        if (rows[i] >= c->row0 && rows[i] < c->row0 + c->N) {
          loc.push_back(rows[i] - c->row0);
          c->bpos.push_back(i - offsets[b]);
        }
      c->boff.push_back((int64_t)loc.size());
      c->bglob.push_back(offsets[b + 1] - offsets[b]);
    }
    c->brows = dalloc<int64_t>(c, std::max<size_t>(loc.size(), 1));
    if (!loc.empty())
      HCK(hipMemcpyAsync(c->brows, loc.data(), sizeof(int64_t) * loc.size(), hipMemcpyHostToDevice, c->st));
    sync(c);
    // the exchange payload of the new list's sample-space batches (reduce_buffer_doubles)
    if (c->own_red && c->red && reduce_buffer_doubles(c) > c->red_cap) {
      dfree_t(c, c->red);
      c->red_cap = 0;
      c->own_red = false;
      ensure_red(c);
    }
  });
}

int scs_select_batch(scs_ctx* c, int64_t b) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_select_batch(s_, b); });
  return guarded(c, [&] {
    const int64_t nb = c->boff.empty() ? 0 : (int64_t)c->boff.size() - 1;
    if (b < -1 || b >= nb) fail(c, SCS_ERR_ARG, "scs_select_batch: batch %lld of %lld", (long long)b, (long long)nb);
    HCK(hipSetDevice(c->dev));
    select_batch(c, b);
    sync(c);
  });
}

static void step_call(scs_ctx* c, const double* x, const double* x_prev, int64_t iter, const double* grad_fx,
                      double* x_new, double* dx, double* pri) {
  require_ready(c, true);
  HCK(hipSetDevice(c->dev));
  hipEvent_t e0;
  tbegin(c, T_STEP, &e0);
  BatchScope bs(c);
  h2d(c, c->x, x, c->m);
  h2d(c, c->xp, x_prev ? x_prev : x, c->m);
  std::vector<double> xnew_h(c->m);
  {
    // ∇fx lives in its own buffer for the call (gtmp2 is line-search scratch)
    double* gbuf = nullptr;
    // ProxGGNSCORE takes ∇fx and never reads it (prox-GGN-SCORE.jl:34-135: its grad_f -- the line
    // search's ∇q, :58-63,83-84 -- is the model's gradient): only NSCORE / LQN install it
    if (grad_fx && c->method != SCS_PROX_GGNSCORE) {
      gbuf = dalloc<double>(c, c->mpad);
      h2d(c, gbuf, grad_fx, c->m);
      invalidate_caches(c);
      c->gfix = gbuf;
    }
    struct Release {
      scs_ctx* c;
      double* g;
      ~Release() {
        if (!g) return;
        c->gfix = nullptr;
        invalidate_caches(c);
        (void)hipStreamSynchronize(c->st);
        dfree_t(c, g);
      }
    } rel{c, gbuf};
    if (c->method == SCS_PROX_LQNSCORE)
      step_lqn(c, x, x_prev ? x_prev : x, iter, xnew_h.data(), dx, pri);
    else
      step_newton(c, x, iter, xnew_h.data(), dx, pri);
  }
  std::memcpy(x_new, xnew_h.data(), sizeof(double) * c->m);
  tend(c, T_STEP, e0);
  if (c->timing) tresolve(c);
}

int scs_step(scs_ctx* c, const double* x, const double* x_prev, int64_t iter, double* x_new, double* dx,
             double* pri) {
  if (is_group(c)) return group_step(c, x, x_prev, iter, nullptr, x_new, dx, pri);
  return guarded(c, [&] { step_call(c, x, x_prev, iter, nullptr, x_new, dx, pri); });
}

int scs_step_grad(scs_ctx* c, const double* x, const double* x_prev, int64_t iter, const double* grad_fx,
                  double* x_new, double* dx, double* pri) {
  if (is_group(c)) return group_step(c, x, x_prev, iter, grad_fx, x_new, dx, pri);
  return guarded(c, [&] { step_call(c, x, x_prev, iter, grad_fx, x_new, dx, pri); });
}

// optim_loop! (iterate.jl:100-267), full-batch, in C++ around the same device calls the
// per-call entry points make (f(x) + get_reg(x) + step! per epoch), so a caller pays one
// ABI crossing per solve instead of three per epoch.  Histories follow iterate.jl exactly:
// one push per epoch (the pre-step values), the duplicated entry at max_epoch
// (:219-231) or the post-step entry on termination (:235-247); pri_res_norm[0] is
// `nothing` (NaN here).  Termination uses the pre-step f_rel_error (:234, :257).
// scs_iterate: the r03 six-field history (obj .. times) -- fvaltest is never read or written
int scs_iterate(scs_ctx* c, const double* x0, const double* x_star, int64_t max_epoch, double x_tol, double f_tol,
                int rel_kind, double* x_out, const scs_history* h, int64_t* n_hist, int64_t* epochs_out) {
  // r05 made this entry the six-field (r03) layout: it never writes fvaltest.  A context that holds test
  // data expects Solution.fvaltest, which only scs_iterate_ex returns -- refused rather than dropped
  // silently (r04 C callers: call scs_iterate_ex with sizeof(scs_history))
  int on = 0;
  if (c && scs_has_test(c, &on) == SCS_OK && on) {
    c->err = "scs_iterate has no fvaltest (six-field history) and this context holds test data: call scs_iterate_ex "
             "with sizeof(scs_history)";
    return SCS_ERR_STATE;
  }
  return scs_iterate_ex(c, x0, x_star, max_epoch, x_tol, f_tol, rel_kind, x_out, h, offsetof(scs_history, fvaltest),
                        n_hist, epochs_out);
}

int scs_iterate_ex(scs_ctx* c, const double* x0, const double* x_star, int64_t max_epoch, double x_tol, double f_tol,
                   int rel_kind, double* x_out, const scs_history* hist, size_t hist_size, int64_t* n_hist,
                   int64_t* epochs_out) {
  // the caller's struct as far as it reaches (a shorter, older layout leaves the later fields NULL)
  scs_history hcopy{};
  if (hist) std::memcpy(&hcopy, hist, std::min(hist_size, sizeof(scs_history)));
  const scs_history* h = hist ? &hcopy : nullptr;
  if (is_group(c)) return group_iterate(c, x0, x_star, max_epoch, x_tol, f_tol, rel_kind, x_out, h, n_hist, epochs_out);
  return guarded(c, [&] {
    require_ready(c, true);
    if (!x0 || !x_star || !x_out || !h || !n_hist || !epochs_out) fail(c, SCS_ERR_ARG, "scs_iterate: null argument");
    if (hist_size < offsetof(scs_history, fvaltest))
      fail(c, SCS_ERR_ARG, "scs_iterate_ex: hist_size %zu < the six history arrays", hist_size);
    if (max_epoch < 1) fail(c, SCS_ERR_ARG, "scs_iterate: max_epoch must be >= 1");
    HCK(hipSetDevice(c->dev));
    const int64_t m = c->m;
    // Σ (a − b)² (b may be null) in a fixed order: eight interleaved partial sums (vectorized;
    // the one-accumulator loop was ~90 us per call at m = 65536, three calls per epoch, on the
    // C5 step's critical path), then a fixed tree and the tail.  Julia's norm is BLAS nrm2, a
    // different order again; termination compares at x_tol, not ulps.
    auto sumsq = [&](const double* a, const double* b) {
      double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      int64_t i = 0;
      if (b) {
        for (; i + 8 <= m; i += 8)
          for (int l = 0; l < 8; ++l) {
            const double d = a[i + l] - b[i + l];
            acc[l] += d * d;
          }
      } else {
        for (; i + 8 <= m; i += 8)
          for (int l = 0; l < 8; ++l) acc[l] += a[i + l] * a[i + l];
      }
      double t = 0.0;
      for (; i < m; ++i) {
        const double d = b ? a[i] - b[i] : a[i];
        t += d * d;
      }
      return (((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]))) + t;
    };
    auto nrm = [&](const double* a, const double* b) { return std::sqrt(sumsq(a, b)); };   // ‖a − b‖
    auto jmax = [](double a, double b) {   // Julia max: NaN propagates, -0.0 < +0.0
      if (std::isnan(a)) return a;
      if (std::isnan(b)) return b;
      return (b < a || (std::signbit(b) && !std::signbit(a))) ? a : b;
    };
    // f(x) + get_reg(x) with one upload of x (c->xn holds it for both)
    // the tagged host vector the device buffers c->x / c->xn hold (0: unknown), so a vector
    // already on the device is not uploaded again (x = the last step's x_new = c->xn)
    uint64_t dev_x = 0, dev_xn = 0;
    auto fobj_of = [&](const double* xx, double* fv) {
      const uint64_t t = xtag_of(c, xx);
      if (!(t && t == dev_xn)) {
        h2d(c, c->xn, xx, m);
        dev_xn = t;
      }
      *fv = eval_f_dev(c, xx, c->xn);
      return *fv + eval_reg_dev(c, c->xn);
    };
    // ftest(x) of a host vector (uploaded to c->xn unless it is already there, as fobj_of)
    auto ftest_of = [&](const double* xx) -> double {
      if (!c->tset.on) return std::numeric_limits<double>::quiet_NaN();
      const uint64_t t = xtag_of(c, xx);
      if (!(t && t == dev_xn)) {
        h2d(c, c->xn, xx, m);
        dev_xn = t;
      }
      return eval_ftest_dev(c, xx, c->xn);
    };
    const double nstar = nrm(x_star, nullptr);
    auto rel_of = [&](const double* xx) {
      if (rel_kind == 1) return sumsq(x_star, xx) / (double)m;   // mean_square_error (utils.jl:3-5), the "gl" rel_error
      return jmax(nrm(xx, x_star) / jmax(nstar, 1.0), x_tol);
    };
    const auto t0 = std::chrono::steady_clock::now();
    auto now = [&] {   // Dates.now() differences: millisecond resolution
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      return std::floor(sec * 1000.0) / 1000.0;
    };
    double fstar = 0.0;
    const double obj_star = fobj_of(x_star, &fstar);
    auto frel_of = [&](double ob) { return jmax(std::fabs(ob - obj_star) / std::fabs(obj_star), f_tol); };
    int64_t nh = 0;
    // show_stat! + update_stat! (utils.jl:50-57,106-113): with held-out data every push carries
    // ftest of the pushed point too (the `fvaltests` vector, iterate.jl:169-175), so the test
    // history has one entry per obj entry
    const bool tst = c->tset.on;
    const double nan = std::numeric_limits<double>::quiet_NaN();
    auto push = [&](double ob, double fv, double pr, double rl, double fr, double dt, double ft) {
      if (c->tset.xor_case)   // iterate.jl:170-171 then :201: ftest is unassigned at the first show_stat!
        fail(c, SCS_ERR_REF, "UndefVarError: `ftest` not defined (only one of Atest / ytest was given: "
                             "iterate.jl:170-171 leave ftest unassigned, show_stat! at :201 reads it)");
      h->obj[nh] = ob;
      h->fval[nh] = fv;
      h->pri_res_norm[nh] = pr;
      h->rel[nh] = rl;
      h->objrel[nh] = fr;
      if (h->times) h->times[nh] = dt;
      if (tst && h->fvaltest) h->fvaltest[nh] = ft;
      ++nh;
    };
    // init!(method, x): reset the method state (prox-L-BFGS-SCORE.jl:31-36)
    c->ring.clear();
    c->spare = 0;
    c->H0 = 1.0;
    c->lbfgs_pending = false;
    invalidate_caches(c);
    // x, x_prev, x_new in pinned host memory: their per-epoch uploads / the x_new download are
    // DMA transfers instead of staged pageable copies (the arrays are only touched after syncs)
    struct Pinned {
      double* p = nullptr;
      ~Pinned() {
        if (p) (void)hipHostFree(p);
      }
    } pin;
    HCK(hipHostMalloc((void**)&pin.p, sizeof(double) * 3 * std::max<int64_t>(m, 1), hipHostMallocDefault));
    double* x = pin.p;
    double* x_prev = pin.p + m;
    double* x_new = pin.p + 2 * m;
    std::memcpy(x, x0, sizeof(double) * m);
    std::memcpy(x_prev, x0, sizeof(double) * m);
    // version tags of the three buffers for the f / ∇q caches (unregistered on exit)
    struct Untag {
      scs_ctx* c;
      ~Untag() {
        for (auto& t : c->xtags) t = scs_ctx::XTag{};
      }
    } untag{c};
    auto tag_slot = [&](const double* p) -> scs_ctx::XTag& {
      for (auto& t : c->xtags)
        if (t.p == p) return t;
      fail(c, SCS_ERR_STATE, "scs_iterate: untracked buffer");
      return c->xtags[0];
    };
    c->xtags[0] = {x, c->xtag_next};
    c->xtags[1] = {x_prev, c->xtag_next++};   // same content as x
    c->xtags[2] = {x_new, c->xtag_next++};
    double pri = std::numeric_limits<double>::quiet_NaN();
    int64_t epochs = 0;
    // the collected batches (iterate.jl:146): the registered list, else the one full batch
    const int64_t nb = c->boff.empty() ? 0 : (int64_t)c->boff.size() - 1;
    const int64_t iend = std::max<int64_t>(nb, 1);
    struct Unselect {
      scs_ctx* c;
      ~Unselect() { c->bview = -1; }
    } unselect{c};
    double last_nx = 0.0, last_ndx = 0.0;
    // Device-resident loop (the full batch of a data loss): x, x_prev, x_new never leave the
    // device; get_reg(x), f(x), rel_error and the two norms of the termination test are reduced
    // on the device and read back with pri_res_norm (and L-BFGS's δhᵀγh) in ONE copy + sync at the
    // end of each epoch -- the GPU only idles for that hand-off.  Same kernels, same order as the
    // per-call path, so the histories equal the host loop's (the norms differ in summation order
    // only; test_device_loop_matches_host_loop).
    // (a Rosenbrock ProblemGeneric runs here too: its f / ∇f / ∇²f are device kernels; the
    // quadratic loss and the host callbacks keep the per-call path)
    const bool dev_ok = nb == 0 && c->loss != SCS_LOSS_QUADRATIC && c->loss != SCS_LOSS_CALLBACK &&
                        (!c->generic || c->loss == SCS_LOSS_ROSENBROCK);
    if (dev_ok) {
      struct DevLoop {
        scs_ctx* c;
        explicit DevLoop(scs_ctx* cc) : c(cc) { c->dev_loop = true; }
        ~DevLoop() { c->dev_loop = false; }
      } devloop(c);
      h2d(c, c->xstar, x_star, m);
      h2d(c, c->x, x0, m);
      HCK(hipMemcpyAsync(c->xp, c->x, sizeof(double) * m, hipMemcpyDeviceToDevice, c->st));
      double* hs = c->hscal;
      auto rel_from = [&](double ss) {
        if (rel_kind == 1) return ss / (double)m;
        return jmax(std::sqrt(ss) / jmax(nstar, 1.0), x_tol);
      };
      // ProxLQNSCORE, fused epoch (lqn_tail / lqn_post, vec.hip): 7 launches per epoch around the two
      // products instead of ~22; every quantity the history and the termination test read for the
      // NEXT x is produced by this epoch's post pass, so the hand-off at the epoch end is the only
      // one.  Same per-element arithmetic and partial-sum order as the unfused step (bit-identical
      // x, obj, fval, pri_res_norm; SCS_LQN_FUSED=0 selects the unfused epoch).
      const char* fz = std::getenv("SCS_LQN_FUSED");
      const bool fused = c->method == SCS_PROX_LQNSCORE && c->ss_type == 1 && m >= 16384 && !sharded(c) &&
                         c->smooth != SCS_SMOOTH_PHUBER_GL && c->smooth != SCS_SMOOTH_OSBA_GL &&
                         !(c->use_prox && c->reg == SCS_REG_GL) && c->reg != SCS_REG_GL && !(fz && fz[0] == '0');
      if (fused) {
        const double Mg = get_Mg(c, c->Mh, c->nu, c->mu, m);
        const double step = c->has_L ? jl_min_h(1 / c->L, 1.0) : 0.5;
        // state at x0: ∇q(x0) -> gq, then smoother(x0) -> gr, Hr, hinv and η's partials, f / get_reg / norms
        grad_q_dev(c, x, c->x, c->gq);
        HCK(launch_smoother(c->smooth, c->x, m, c->mu, c->slb, c->sub, c->wel, c->gr, c->Hr, c->st));
        HCK(launch_lqn_eta(c->gr, c->Hr, m, c->lam, c->hinv, c->lqR, c->st));
        HCK(launch_reg_value(prox_args(c), c->x, m, c->scal + RX_SLOT, c->scal + 64 + 2 * 256, c->st));
        HCK(launch_norms3(c->x, c->xstar, nullptr, m, c->scal + NRM_SLOT, c->scal + 64 + 3 * 256, c->st));
        forward(c, x, c->x, 0, false);   // cached: the z of x0 from ∇q(x0)
        if (tst) ftest_enqueue(c, c->x);
        d2h(c, hs, c->scal, LOOP_SLOTS);
        sync(c);
        double fcur = loss_scale_value(c, hs[ZF_SLOT]), regcur = hs[RX_SLOT];
        double ftcur = tst ? loss_scale_value(c, hs[TF_SLOT]) : nan;
        double relcur = rel_from(hs[NRM_SLOT]), nxcur = std::sqrt(hs[NRM_SLOT + 1]);
        // Pipelined by one epoch: epoch e+1 is enqueued before the host reads epoch e's scalars, so
        // the GPU never idles for the hand-off.  What the next epoch needs from this one stays on
        // the device: the L-BFGS ring ([order | k | spare] in d_order, H0 in scal[H0_SLOT]) is
        // advanced by lqn_post's last workgroup, and the two-loop launches for an upper bound of k
        // (the ring grows by at most one per epoch in flight; surplus launches return at once).
        // The host keeps the mirror (lbfgs_accept on the same δhᵀγh, γhᵀγh) for the history and
        // the state after the call.  An epoch enqueued past the stopping one writes only x_prev's
        // buffer, the spare pair slot and scratch; its buffer rotation is undone.
        const int mem = c->mem;
        for (int i = 0; i < mem + 3; ++i) c->hring[i] = 0;   // init!: empty ring, spare slot 0
        HCK(hipMemcpyAsync(c->d_order, c->hring, sizeof(int) * (mem + 3), hipMemcpyHostToDevice, c->st));
        HCK(launch_fill(c->scal + H0_SLOT, 1, 1.0, c->st));
        for (auto& ev : c->loop_ev)
          if (!ev) HCK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        struct Rot {
          double *x, *xp, *xn, *gq, *gqn;
        };
        auto rot_get = [&] { return Rot{c->x, c->xp, c->xn, c->gq, c->gqn}; };
        // the epoch's scalars: written by lqn_post's final kernel straight into the pinned buffer
        // (SCS_LOOP_HOSTMAP=0: a device-to-host copy after it)
        const char* hm_env = std::getenv("SCS_LOOP_HOSTMAP");
        const bool hostmap = !(hm_env && hm_env[0] == '0');
        int64_t enq = 0, done = 0;
        Rot before_last{};   // the rotation state before the latest enqueue
        // k = 0 is speculated while the host's ring is empty (no two-loop launches: the tail takes
        // d = -∇q); when the epoch in flight turns out to have accepted the first pair, the epoch
        // enqueued behind it is discarded and re-run (once per call: the ring never empties).
        bool spec_k0 = false;   // the latest enqueue assumed k = 0
        auto enqueue = [&](int64_t e) {
          before_last = rot_get();
          const bool timed = c->timing && (e % c->timing_every == 0);
          const bool tsave = c->timing;
          c->timing = timed;   // timing events cost a dispatch gap each: sample the epochs
          const int kmax = c->ring.empty() ? 0 : std::min<int>(mem, (int)c->ring.size() + (int)(enq - done));
          spec_k0 = kmax == 0;
          hipEvent_t e0;
          tbegin(c, T_STEP, &e0);
          if (kmax > 0)
            HCK(launch_two_loop(c->S, c->Yv, c->mpad, c->d_order, kmax, 1.0, c->gq, m, c->q, c->d, c->ab, c->tlwork,
                                mem, c->d_order + mem + 1, c->scal + H0_SLOT, c->st, c->f32c));
          HCK(launch_lqn_tail(c->x, kmax > 0 ? c->d : c->gq, kmax > 0 ? 0 : 1, m, Mg, step, prox_args(c), c->hinv,
                              c->xn, c->dxv, c->q, c->lqR, c->scal, c->st));
          if (tst) ftest_enqueue(c, c->xn);   // -> scal[TF_SLOT], carried to the host by lqn_post_final
          // z = A x_new, r = ∂f/∂z, f(x_new) -> scal[ZF_SLOT] (forward()'s passes, no host copies)
          hipEvent_t e1;
          tbegin(c, T_GEMV, &e1);
          const int ns = matvec_n(c, c->xn, c->nsplit);
          tend(c, T_GEMV, e1);
          HCK(launch_epilogue(c->loss, c->ggn, EPI_GRAD | EPI_Z | EPI_VAL, c->zpart, ns, c->Npad, c->y, c->N, c->Npad,
                              c->scale, c->z, c->gN, c->hN, c->wN, c->vN, c->valpart, c->st));   // Σ: lqn_post
          hipEvent_t e2;
          tbegin(c, T_GEMV, &e2);
          const int np = matvec_t_part(c, c->gN);       // Aᵀ r partials
          tend(c, T_GEMV, e2);
          HCK(launch_lqn_post(c->tpart, np, c->mpad, m, c->lam, c->smooth, c->mu, c->slb, c->sub, prox_args(c),
                              c->xstar, c->x, c->xn, c->gq, c->q, c->gqn, c->S, c->Yv, c->mpad, c->d_order, mem, 0,
                              c->gr, c->Hr, c->hinv, c->lqR, c->valpart, c->nval, c->scal, ZF_SLOT, RX_SLOT, NRM_SLOT,
                              H0_SLOT, c->hloop_dev + (e & 1) * LOOP_SLOTS, hostmap ? LOOP_SLOTS : 0, c->st));
          tend(c, T_STEP, e0);
          if (!hostmap) d2h(c, c->hloop + (e & 1) * LOOP_SLOTS, c->scal, LOOP_SLOTS);
          HCK(hipEventRecord(c->loop_ev[e & 1], c->st));
          double* t = c->xp;   // x_prev <- x, x <- x_new
          c->xp = c->x;
          c->x = c->xn;
          c->xn = t;
          std::swap(c->gq, c->gqn);   // ∇q(x) of the next epoch
          ++enq;
          c->timing = tsave;
        };
        auto restore_last = [&] {   // undo the rotation of the latest enqueue
          c->x = before_last.x;
          c->xp = before_last.xp;
          c->xn = before_last.xn;
          c->gq = before_last.gq;
          c->gqn = before_last.gqn;
        };
        enqueue(1);
        for (int64_t epoch = 1; epoch <= max_epoch; ++epoch) {
          const double dt = now();
          const double obj = fcur + regcur;
          const double frel = frel_of(obj);
          push(obj, fcur, pri, relcur, frel, dt, ftcur);
          if (epoch == max_epoch) push(obj, fcur, pri, relcur, frel, now(), ftcur);   // iterate.jl:219-231
          if (epoch < max_epoch) enqueue(epoch + 1);
          HCK(hipEventSynchronize(c->loop_ev[epoch & 1]));
          const double* he = c->hloop + (epoch & 1) * LOOP_SLOTS;
          ++done;
          const bool was_empty = c->ring.empty();
          lbfgs_accept(c, c->spare, he[16], he[17]);   // the device took the same decision
          if (was_empty && !c->ring.empty() && enq > done && spec_k0) {
            // epoch + 1 ran with d = -∇q but the memory now holds a pair: discard it.  Restore the
            // rotation, the ring (host mirror) and H0, and the smoother / η state at x_{epoch+1}
            // that its post pass overwrote (the same kernels as the setup), then enqueue it again.
            sync(c);
            restore_last();
            enq = done;
            const int k = (int)c->ring.size();
            for (int i = 0; i < mem + 3; ++i) c->hring[i] = 0;
            for (int i = 0; i < k; ++i) c->hring[i] = c->ring[i];
            c->hring[mem + 1] = k;
            c->hring[mem + 2] = c->spare;
            HCK(hipMemcpyAsync(c->d_order, c->hring, sizeof(int) * (mem + 3), hipMemcpyHostToDevice, c->st));
            HCK(launch_fill(c->scal + H0_SLOT, 1, c->H0, c->st));
            HCK(launch_smoother(c->smooth, c->x, m, c->mu, c->slb, c->sub, c->wel, c->gr, c->Hr, c->st));
            HCK(launch_lqn_eta(c->gr, c->Hr, m, c->lam, c->hinv, c->lqR, c->st));
            enqueue(epoch + 1);
          }
          pri = he[0];
          const double ndx = std::sqrt(he[NRM_SLOT + 2]);
          const double fnext = loss_scale_value(c, he[ZF_SLOT]), regnext = he[RX_SLOT];
          const double relnext = rel_from(he[NRM_SLOT]), nxnext = std::sqrt(he[NRM_SLOT + 1]);
          const double ftnext = tst ? loss_scale_value(c, he[TF_SLOT]) : nan;
          const bool stop = ndx < x_tol * std::max(nxcur, 1.0) || frel <= f_tol || pri < x_tol;
          if (stop && epoch != max_epoch)   // iterate.jl:235-247: stats of x_new
            push(fnext + regnext, fnext, pri, relnext, frel_of(fnext + regnext), now(), ftnext);
          fcur = fnext;
          ftcur = ftnext;
          regcur = regnext;
          relcur = relnext;
          nxcur = nxnext;
          ++epochs;
          if (stop) {
            if (enq > done) restore_last();   // the epoch enqueued past this one
            break;
          }
        }
        sync(c);
        c->lbfgs_pending = false;
        invalidate_caches(c);   // z, f and ∇q of the last enqueued point, which may be past the stop
        d2h(c, x_out, c->x, m);
        sync(c);
        *n_hist = nh;
        *epochs_out = epochs;
        if (c->timing) tresolve(c);
        return;
      }
      for (int64_t epoch = 1; epoch <= max_epoch; ++epoch) {
        double dt = now();
        // f(x): the z of x is cached (the previous step's ∇q(x_new) / the Newton step's forward)
        // except at epoch 1; its value is copied out of the deferred slot before the step's
        // forward at x_new reuses it
        if (c->loss == SCS_LOSS_ROSENBROCK) {
          HCK(launch_rosen(c->x, m, 0, c->scal + FX_SLOT, nullptr, 0, c->st));
        } else {
          forward(c, x, c->x, 0, false);
          HCK(hipMemcpyAsync(c->scal + FX_SLOT, c->scal + ZF_SLOT, sizeof(double), hipMemcpyDeviceToDevice, c->st));
        }
        HCK(launch_reg_value(prox_args(c), c->x, m, c->scal + RX_SLOT, c->scal + 64 + 2 * 256, c->st));
        if (tst) ftest_enqueue(c, c->x);   // -> scal[TF_SLOT], read back with the epoch's scalars
        hipEvent_t e0;
        tbegin(c, T_STEP, &e0);
        tag_slot(x_new).v = c->xtag_next++;   // the step writes x_new (c->xn)
        if (c->method == SCS_PROX_LQNSCORE)
          step_lqn(c, x, x_prev, epoch, x_new, nullptr, &pri);
        else
          step_newton(c, x, epoch, x_new, nullptr, &pri);
        tend(c, T_STEP, e0);
        HCK(launch_norms3(c->x, c->xstar, c->xn, m, c->scal + NRM_SLOT, c->scal + 64 + 3 * 256, c->st));
        d2h(c, hs, c->scal, LOOP_SLOTS);
        sync(c);
        lbfgs_settle(c, true);
        const double fval = loss_scale_value(c, hs[FX_SLOT]);
        const double obj = fval + hs[RX_SLOT];
        const double rel = rel_from(hs[NRM_SLOT]);
        const double frel = frel_of(obj);
        const double ft = tst ? loss_scale_value(c, hs[TF_SLOT]) : nan;
        push(obj, fval, pri, rel, frel, dt, ft);
        if (epoch == max_epoch) push(obj, fval, pri, rel, frel, now(), ft);   // iterate.jl:219-231
        pri = hs[0];
        const double nx = std::sqrt(hs[NRM_SLOT + 1]), ndx = std::sqrt(hs[NRM_SLOT + 2]);
        const bool stop = ndx < x_tol * std::max(nx, 1.0) || frel <= f_tol || pri < x_tol;
        if (stop && epoch != max_epoch) {   // iterate.jl:235-247: stats of x_new
          dt = now();
          double fv = eval_f_dev(c, x_new, c->xn);
          const double ob = fv + eval_reg_dev(c, c->xn);
          const double ft = tst ? eval_ftest_dev(c, x_new, c->xn) : nan;
          HCK(launch_norms3(c->xn, c->xstar, nullptr, m, c->scal + NRM_SLOT, c->scal + 64 + 3 * 256, c->st));
          d2h(c, hs + NRM_SLOT, c->scal + NRM_SLOT, 1);
          sync(c);
          push(ob, fv, pri, rel_from(hs[NRM_SLOT]), frel_of(ob), dt, ft);
        }
        // x_prev <- x, x <- x_new: rotate the device buffers and the host identities' tags
        std::swap(x_prev, x);
        tag_slot(x).v = tag_slot(x_new).v;
        double* t = c->xp;
        c->xp = c->x;
        c->x = c->xn;
        c->xn = t;
        ++epochs;
        if (stop) break;
      }
      d2h(c, x_out, c->x, m);
      sync(c);
      *n_hist = nh;
      *epochs_out = epochs;
      if (c->timing) tresolve(c);
      return;
    }
    for (int64_t epoch = 1; epoch <= max_epoch; ++epoch) {
      double dt = now();
      double fval = 0.0;
      double obj = fobj_of(x, &fval);
      double ft = ftest_of(x);
      double rel = rel_of(x);
      double frel = frel_of(obj);
      push(obj, fval, pri, rel, frel, dt, ft);
      for (int64_t i = 1; i <= iend; ++i) {   // for (i, sample) in enumerate(data) (iterate.jl:204-255)
        if (epoch == max_epoch && i == iend) {   // iterate.jl:219-231 (x as of this batch)
          dt = now();
          obj = fobj_of(x, &fval);
          ft = ftest_of(x);
          rel = rel_of(x);
          frel = frel_of(obj);
          push(obj, fval, pri, rel, frel, dt, ft);
        }
        hipEvent_t e0;
        tbegin(c, T_STEP, &e0);
        select_batch(c, nb > 0 ? i - 1 : -1);
        {
          BatchScope bs(c);
          const uint64_t tx = xtag_of(c, x), tp = xtag_of(c, x_prev);
          const size_t vb = sizeof(double) * m;
          if (nb == 0 && tp && tp == dev_x)   // x_prev = the previous step's x, still in c->x
            HCK(hipMemcpyAsync(c->xp, c->x, vb, hipMemcpyDeviceToDevice, c->st));
          else
            h2d(c, c->xp, x_prev, m);
          if (nb == 0 && tx && tx == dev_xn)
            HCK(hipMemcpyAsync(c->x, c->xn, vb, hipMemcpyDeviceToDevice, c->st));
          else
            h2d(c, c->x, x, m);
          dev_x = tx;
          tag_slot(x_new).v = c->xtag_next++;   // the step writes x_new
          if (c->method == SCS_PROX_LQNSCORE)
            step_lqn(c, x, x_prev, epoch, x_new, nullptr, &pri);
          else
            step_newton(c, x, epoch, x_new, nullptr, &pri);
          dev_xn = xtag_of(c, x_new);   // the step's tail wrote x_new to c->xn (and downloaded it)
        }
        c->bview = -1;
        tend(c, T_STEP, e0);
        const double nx = nrm(x, nullptr);
        const double ndx = nrm(x_new, x);
        last_nx = nx;     // the epoch-end test (:257) reads the same pair after the swap
        last_ndx = ndx;
        const bool stop = ndx < x_tol * std::max(nx, 1.0) || frel <= f_tol || pri < x_tol;
        if (stop && epoch != max_epoch) {   // iterate.jl:235-247 (f_rel_error is refreshed for the test at :257)
          dt = now();
          obj = fobj_of(x_new, &fval);
          ft = ftest_of(x_new);
          rel = rel_of(x_new);
          frel = frel_of(obj);
          push(obj, fval, pri, rel, frel, dt, ft);
        }
        std::swap(x_prev, x);
        std::memcpy(x, x_new, sizeof(double) * m);
        tag_slot(x).v = tag_slot(x_new).v;   // same content
        if (stop) {
          ++epochs;
          break;
        }
      }
      // ‖x − x_prev‖, ‖x_prev‖ = the last inner step's ‖x_new − x‖, ‖x‖ (same operands, same order)
      if (last_ndx < x_tol * std::max(last_nx, 1.0) || frel <= f_tol ||
          pri < x_tol)
        break;   // iterate.jl:257-259
      ++epochs;
    }
    std::memcpy(x_out, x, sizeof(double) * m);
    *n_hist = nh;
    *epochs_out = epochs;
    if (c->timing) tresolve(c);
  });
}

int scs_smoother_eval(scs_ctx* c, const double* x, double* gr, double* Hr) {
  if (is_group(c)) return scs_smoother_eval(c->subs[0], x, gr, Hr);   // m-space, no exchange
  return guarded(c, [&] {
    if (!c->smooth_set) fail(c, SCS_ERR_STATE, "no smoother");
    h2d(c, c->xn, x, c->m);
    HCK(launch_smoother(c->smooth, c->xn, c->m, c->mu, c->slb, c->sub, c->wel, c->gr, c->Hr, c->st));
    d2h(c, gr, c->gr, c->m);
    d2h(c, Hr, c->Hr, c->m);
    sync(c);
  });
}

int scs_prox_eval(scs_ctx* c, const double* z, const double* Hr, double lam, double alpha, double* out) {
  if (is_group(c)) return scs_prox_eval(c->subs[0], z, Hr, lam, alpha, out);
  return guarded(c, [&] {
    if (!c->reg_set) fail(c, SCS_ERR_STATE, "no regularizer");
    h2d(c, c->zb, z, c->m);
    h2d(c, c->Hr, Hr, c->m);
    ProxArgsH P = prox_args(c);
    P.lam = lam;
    HCK(launch_prox_only(P, c->zb, c->Hr, alpha, c->m, c->hinv, c->xn, c->st));
    d2h(c, out, c->xn, c->m);
    sync(c);
  });
}

int scs_gram_eval(scs_ctx* c, const double* w, double* G, int64_t ldg) {
  return guarded(c, [&] {
    if (!c->has_data || c->generic) fail(c, SCS_ERR_STATE, "no data");
    std::vector<double> wp(c->Npad, 0.0);
    std::memcpy(wp.data(), w, sizeof(double) * c->N);
    h2d(c, c->wN, wp.data(), c->Npad);
    ensure_gram(c);
    hipEvent_t e0;
    tbegin(c, T_GRAM, &e0);
    gram_main(c, c->wN, c->G, 0);
    tend(c, T_GRAM, e0);
    HCK(launch_symmetrize(c->G, c->mpad, c->m, c->st));
    HCK(hipMemcpy2DAsync(G, sizeof(double) * ldg, c->G, sizeof(double) * c->mpad, sizeof(double) * c->m, c->m,
                         hipMemcpyDeviceToHost, c->st));
    sync(c);
    if (c->timing) tresolve(c);
  });
}

// The m x m system of ProxNSCORE / ProxGGNSCORE from given weights: (Aᵀ diag(w) A + diag(dvec)) x = rhs,
// through the production path (Gram, then solve_system: Cholesky with the LU fallback, or the LU
// alone with mode 1).  G is the step's scratch, so nothing else changes.
int scs_solve_eval(scs_ctx* c, const double* w, const double* dvec, const double* rhs, int mode, double* x,
                   int* used_lu) {
  return guarded(c, [&] {
    if (!c->has_data || c->generic) fail(c, SCS_ERR_STATE, "no data");
    if (c->nranks > 1) fail(c, SCS_ERR_ARG, "scs_solve_eval runs on one rank");
    if (!w || !dvec || !rhs || !x) fail(c, SCS_ERR_ARG, "scs_solve_eval: null argument");
    HCK(hipSetDevice(c->dev));
    std::vector<double> wp(c->Npad, 0.0), v(c->mpad, 0.0);
    std::memcpy(wp.data(), w, sizeof(double) * c->N);
    h2d(c, c->wN, wp.data(), c->Npad);
    ensure_gram(c);
    hipEvent_t e0;
    tbegin(c, T_GRAM, &e0);
    gram_main(c, c->wN, c->G, 0);
    tend(c, T_GRAM, e0);
    std::memcpy(v.data(), dvec, sizeof(double) * c->m);
    h2d(c, c->gtmp2, v.data(), c->mpad);
    HCK(launch_diag_add(c->G, c->mpad, c->m, 1.0, c->gtmp2, c->st));
    std::memcpy(v.data(), rhs, sizeof(double) * c->m);
    h2d(c, c->gq, v.data(), c->mpad);
    sync(c);
    c->g_from_cache = false;
    if (mode < 0 || mode > 2) fail(c, SCS_ERR_ARG, "scs_solve_eval: mode %d (0 step path, 1 LU, 2 QR)", mode);
    solve_system(c, c->gq, mode == 1, mode == 2);
    d2h(c, x, c->gq, c->m);
    sync(c);
    if (used_lu) *used_lu = c->lu_fallback_used ? 1 : 0;
    invalidate_caches(c);
    if (c->timing) tresolve(c);
  });
}

// A x = b for a host row-major n x n A by the hand-written LU (getrf + getrs semantics); ipiv
// (0-based, LAPACK order) and info (first zero pivot, 1-based) as dgetrf reports them.  Needs a
// context only (no data).
int scs_lu_eval(scs_ctx* c, int64_t n, const double* A, const double* b, double* x, int32_t* ipiv, int* info) {
  return guarded(c, [&] {
    if (n < 1 || !A || !b || !x) fail(c, SCS_ERR_ARG, "scs_lu_eval: bad arguments");
    HCK(hipSetDevice(c->dev));
    const int64_t np = round_up(n, 128);
    if (c->lu_np != np) {
      if (c->luM) dfree_t(c, c->luM);
      if (c->lub) dfree_t(c, c->lub);
      if (c->luinfo) dfree_t(c, c->luinfo);
      c->luM = dalloc<double>(c, (size_t)np * np);
      c->lub = dalloc<double>(c, np);
      c->luinfo = dalloc<int>(c, 1);
      c->lu_np = np;
    }
    double* M = c->luM;
    double* bb = c->lub;
    auto upload = [&] {   // (also the system of a column-step redo, lu_factor_checked)
      HCK(hipMemsetAsync(M, 0, sizeof(double) * np * np, c->st));
      HCK(hipMemsetAsync(bb, 0, sizeof(double) * np, c->st));
      HCK(hipMemcpy2DAsync(M, sizeof(double) * np, A, sizeof(double) * n, sizeof(double) * n, n,
                           hipMemcpyHostToDevice, c->st));
      HCK(hipMemcpyAsync(bb, b, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
    };
    upload();
    HCK(lu_aux_init(&c->lu, np, c->st));
    hipEvent_t e0;
    tbegin(c, T_SOLVE, &e0);
    const int hinfo = lu_factor_checked(c, M, np, n, np, c->luinfo, upload);
    if (hinfo == 0) HCK(lu_solve(M, np, np, &c->lu, bb, c->st));
    tend(c, T_SOLVE, e0);
    // x only without a zero pivot; ipiv whenever the factorization completed -- dgetrf's pivots with
    // info > 0 too (the header's contract)
    if (hinfo == 0) HCK(hipMemcpyAsync(x, bb, sizeof(double) * n, hipMemcpyDeviceToHost, c->st));
    if (ipiv) HCK(hipMemcpyAsync(ipiv, c->lu.ipiv, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->st));
    sync(c);
    if (info) *info = hinfo;
    if (c->timing) tresolve(c);
  });
}

// Columns cols[0..ncols) of the local A, column-major N x ncols (ld = N).
int scs_get_columns(scs_ctx* c, const int64_t* cols, int64_t ncols, double* out) {
  return guarded(c, [&] {
    if (!c->has_data || c->generic || c->sparse) fail(c, SCS_ERR_STATE, "scs_get_columns needs a dense A");
    for (int64_t k = 0; k < ncols; ++k)
      if (cols[k] < 0 || cols[k] >= c->m) fail(c, SCS_ERR_ARG, "column %lld out of range", (long long)cols[k]);
    HCK(hipSetDevice(c->dev));
    int64_t* dc = dalloc<int64_t>(c, ncols);
    double* dout = dalloc<double>(c, (size_t)ncols * c->N);
    HCK(hipMemcpyAsync(dc, cols, sizeof(int64_t) * ncols, hipMemcpyHostToDevice, c->st));
    HCK(launch_get_columns(c->A, c->nstage, dc, ncols, c->N, dout, c->st));
    HCK(hipMemcpyAsync(out, dout, sizeof(double) * ncols * c->N, hipMemcpyDeviceToHost, c->st));
    sync(c);
    dfree_t(c, dc);
    dfree_t(c, dout);
  });
}

// The production Gram launch with weights w and -- where the step fuses it (256 x 128 tiles) --
// Aᵀv in the same pass: entries G(i_k, j_k) (ij = n pairs, 0-based) and Aᵀv (m) to the host.
int scs_gram_atv_eval(scs_ctx* c, const double* w, const double* v, const int64_t* ij, int64_t n, double* gvals,
                      double* atv, int* fused) {
  return guarded(c, [&] {
    if (!c->has_data || c->generic) fail(c, SCS_ERR_STATE, "no data");
    if (n < 0 || (n > 0 && (!ij || !gvals))) fail(c, SCS_ERR_ARG, "scs_gram_atv_eval: bad sample list");
    HCK(hipSetDevice(c->dev));
    std::vector<double> wp(c->Npad, 0.0);
    std::memcpy(wp.data(), w, sizeof(double) * c->N);
    h2d(c, c->wN, wp.data(), c->Npad);
    std::memcpy(wp.data(), v, sizeof(double) * c->N);
    h2d(c, c->vN, wp.data(), c->Npad);
    ensure_gram(c);
    const bool fuse = gram_fuse_ok(c->tall) != 0 && !c->sparse;
    hipEvent_t e0;
    tbegin(c, T_GRAM, &e0);
    gram_main(c, c->wN, c->G, 0, fuse ? c->vN : nullptr, c->gtmp);
    tend(c, T_GRAM, e0);
    if (!fuse) gemv_t_local(c, c->vN, c->gtmp);
    std::vector<int2> hij((size_t)std::max<int64_t>(n, 1));
    for (int64_t k = 0; k < n; ++k) {
      const int64_t i = ij[2 * k], j = ij[2 * k + 1];
      if (i < 0 || j < 0 || i >= c->m || j >= c->m) fail(c, SCS_ERR_ARG, "sample %lld out of range", (long long)k);
      hij[k] = make_int2((int)std::min(i, j), (int)std::max(i, j));   // the upper triangle holds G
    }
    int2* dij = dalloc<int2>(c, hij.size());
    double* dv = dalloc<double>(c, hij.size());
    HCK(hipMemcpyAsync(dij, hij.data(), sizeof(int2) * n, hipMemcpyHostToDevice, c->st));
    HCK(launch_gather_entries(c->G, c->mpad, dij, (int)n, dv, c->st));
    if (n > 0) d2h(c, gvals, dv, n);
    if (atv) d2h(c, atv, c->gtmp, c->m);
    sync(c);
    dfree_t(c, dij);
    dfree_t(c, dv);
    if (fused) *fused = fuse ? 1 : 0;
    invalidate_caches(c);
    if (c->timing) tresolve(c);
  });
}

int scs_gemv_t_eval(scs_ctx* c, const double* v, double* out) {
  return guarded(c, [&] {
    if (!c->has_data || c->generic) fail(c, SCS_ERR_STATE, "no data");
    std::vector<double> vp(c->Npad, 0.0);
    std::memcpy(vp.data(), v, sizeof(double) * c->N);
    h2d(c, c->vN, vp.data(), c->Npad);
    matvec_t(c, c->vN, c->gtmp);
    d2h(c, out, c->gtmp, c->m);
    sync(c);
  });
}

int scs_gemv_n_eval(scs_ctx* c, const double* x, double* out) {
  return guarded(c, [&] {
    if (!c->has_data || c->generic) fail(c, SCS_ERR_STATE, "no data");
    h2d(c, c->xn, x, c->m);
    const int ns = matvec_n(c, c->xn, c->nsplit);
    HCK(launch_epilogue(c->loss ? c->loss : SCS_LOSS_LEAST_SQUARES, SCS_GGN_NONE, EPI_Z, c->zpart, ns, c->Npad,
                        c->y, c->N, c->Npad, 1.0, c->z, nullptr, nullptr, nullptr, nullptr, c->valpart, c->st));
    d2h(c, out, c->z, c->N);
    sync(c);
    c->zvalid = false;
  });
}

int scs_timing_enable(scs_ctx* c, int on) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_timing_enable(s_, on); });
  return guarded(c, [&] {
    c->timing = on != 0;
    c->timing_every = on > 1 ? on : 1;
  });
}

int scs_timing_get(scs_ctx* c, scs_timing* t) {
  if (is_group(c)) return scs_timing_get(c->subs[0], t);   // device 0's accumulators
  return guarded(c, [&] {
    tresolve(c);
    t->gram_ms = c->tms[T_GRAM];
    t->gram_calls = c->tcalls[T_GRAM];
    t->gemv_ms = c->tms[T_GEMV];
    t->gemv_calls = c->tcalls[T_GEMV];
    t->solve_ms = c->tms[T_SOLVE];
    t->solve_calls = c->tcalls[T_SOLVE];
    t->step_ms = c->tms[T_STEP];
    t->step_calls = c->tcalls[T_STEP];
    t->reduce_ms = c->tms[T_REDUCE];
    t->reduce_calls = c->tcalls[T_REDUCE];
  });
}

int scs_kernel_names(scs_ctx* c, char* gram, int64_t gram_cap, char* product, int64_t product_cap) {
  if (is_group(c)) return scs_kernel_names(c->subs[0], gram, gram_cap, product, product_cap);
  return guarded(c, [&] {
    auto put = [](char* dst, int64_t cap, const std::string& v) {
      if (!dst || cap <= 0) return;
      const size_t n = std::min<size_t>(v.size(), (size_t)cap - 1);
      std::memcpy(dst, v.data(), n);
      dst[n] = 0;
    };
    put(gram, gram_cap, c->gram_kname);
    put(product, product_cap, c->prod_kname);
  });
}

int scs_timing_reset(scs_ctx* c) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_timing_reset(s_); });
  return guarded(c, [&] {
    tresolve(c);
    for (int i = 0; i < T_N; ++i) {
      c->tms[i] = 0;
      c->tcalls[i] = 0;
    }
  });
}

int scs_fallback_counts(scs_ctx* c, int64_t* counts, int n) {
  if (!c) return SCS_ERR_ARG;
  if (!counts || n < 0) {
    c->err = "scs_fallback_counts: bad arguments";
    return SCS_ERR_ARG;
  }
  for (int i = 0; i < n; ++i) counts[i] = 0;
  // a multi-device context: the sum over its devices
  std::vector<scs_ctx*> cs = is_group(c) ? c->subs : std::vector<scs_ctx*>{c};
  for (scs_ctx* s_ : cs)
    for (int i = 0; i < n && i < SCS_FB_N; ++i) counts[i] += s_->fb[i];
  return SCS_OK;
}

int scs_sync(scs_ctx* c) {
  if (is_group(c)) return group_run(c, [&](scs_ctx* s_, int) { return scs_sync(s_); });
  return guarded(c, [&] { sync(c); });
}

}  // extern "C"

// ===========================================================================
// Multi-device contexts (scs_create_multi): one process drives several GPUs
// ===========================================================================
// The reference's iterate! is one process (iterate.jl:56-76; no MPI / Distributed), so a Julia
// caller gets the node's GPUs from one DeviceProblem(...; devices): the library splits the rows
// (row_plan, the same blocks as one process per GPU), gives every device a sub-context with its
// rows and an RCCL communicator from ncclCommInitAll, and runs each supported call on all
// sub-contexts at once -- one host thread per device, since the step's exchange is a collective
// every device must enter.  Every sub-context computes the same replicated m-vectors with the same
// bits, so outputs are device 0's.

// One persistent host thread per device of a group (started by scs_create_multi, joined by
// group_destroy).  A call posts one job per device and waits for all of them.
struct scs_ctx::Workers {
  struct Slot {
    std::thread th;
    std::function<void()> job;
    bool has_job = false;
  };
  std::mutex mu;
  std::condition_variable cv_job, cv_done;
  std::vector<Slot> slots;
  int pending = 0;
  bool quit = false;

  explicit Workers(const std::vector<int>& devs) : slots(devs.size()) {
    for (size_t i = 0; i < devs.size(); ++i)
      slots[i].th = std::thread([this, i, d = devs[i]] {
        (void)hipSetDevice(d);   // once: the thread drives this device for the group's lifetime
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv_job.wait(lk, [&] { return quit || slots[i].has_job; });
            if (!slots[i].has_job) return;   // quit
            job = std::move(slots[i].job);
            slots[i].has_job = false;
          }
          job();
          {
            std::lock_guard<std::mutex> lk(mu);
            --pending;
          }
          cv_done.notify_all();
        }
      });
  }
  // run jobs[i] on worker i, all at once; returns when every job has returned
  void run(std::vector<std::function<void()>>& jobs) {
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i = 0; i < slots.size(); ++i) {
        slots[i].job = std::move(jobs[i]);
        slots[i].has_job = true;
      }
      pending = (int)slots.size();
    }
    cv_job.notify_all();
    std::unique_lock<std::mutex> lk(mu);
    cv_done.wait(lk, [&] { return pending == 0; });
  }
  ~Workers() {
    {
      std::lock_guard<std::mutex> lk(mu);
      quit = true;
    }
    cv_job.notify_all();
    for (auto& sl : slots)
      if (sl.th.joinable()) sl.th.join();
  }
};

// The exchange of a SCS_MULTI_HOST_EXCHANGE group (scs_create_multi_ex): every device's payload goes to
// a host slot, a barrier, every device sums the slots in device order (the same bits on every device),
// writes the sum back, a second barrier (no slot is rewritten before every device has read it).  It
// needs no RCCL and no distinct devices -- several sub-contexts may share one GPU -- so the group's
// fan-out, row split and exchange run on a one-GPU box; the cost is two host copies per exchange.
// abort() releases every waiter (group_run, after a device failed).
struct scs_ctx::HostExchange {
  struct Rank {
    HostExchange* ex = nullptr;
    int rank = 0;
    std::vector<double> sum;
  };
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<std::vector<double>> slot;
  std::vector<Rank> ranks;
  explicit HostExchange(int n_) : n(n_), slot((size_t)n_), ranks((size_t)n_) {
    for (int i = 0; i < n_; ++i) ranks[(size_t)i] = Rank{this, i, {}};
  }
  bool wait() {   // false once aborted, or when the others have not all arrived within 600 s
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(600), [&] { return gen != g || aborted; })) {
      aborted = true;   // a device that never arrives (diverged control flow): release everyone
      cv.notify_all();
      return false;
    }
    return gen != g;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
  static int allreduce(void* dev_buf, int64_t count, void* stream, void* user) {
    Rank* rk = static_cast<Rank*>(user);
    HostExchange* ex = rk->ex;
    hipStream_t st = static_cast<hipStream_t>(stream);
    std::vector<double>& mine = ex->slot[(size_t)rk->rank];
    mine.resize((size_t)count);
    if (hipMemcpyAsync(mine.data(), dev_buf, sizeof(double) * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return 2;
    if (!ex->wait()) return 1;
    rk->sum.assign(ex->slot[0].begin(), ex->slot[0].begin() + count);
    for (int r = 1; r < ex->n; ++r) {
      const double* o = ex->slot[(size_t)r].data();
      for (int64_t e = 0; e < count; ++e) rk->sum[(size_t)e] += o[e];
    }
    if (hipMemcpyAsync(dev_buf, rk->sum.data(), sizeof(double) * count, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return 2;
    return ex->wait() ? 0 : 1;
  }
};

scs_ctx::~scs_ctx() = default;

namespace {

// run f(sub, i) on every sub-context, each on its device's worker thread; the first failing
// device's code and message become the group's.  A device that fails while the others may be
// waiting inside a collective aborts the communicators after a grace period (ncclCommAbort unblocks
// them), so the call returns instead of hanging.  The abort only sets the shared flag and calls
// ncclCommAbort: the sub-contexts' rccl handles are cleared after every worker has returned (no
// other thread reads them then), and the flag stops any further RCCL call in the meantime.  The
// group is then unusable (SCS_ERR_COMM) and must be destroyed.  Unverified on hardware beyond one
// device (no multi-GPU box here): DESIGN.md §6.
template <class F>
int group_run(scs_ctx* g, F&& f) {
  if (g->group_broken) {
    g->err = "multi-device context: an earlier call aborted its communicators; destroy it";
    return SCS_ERR_COMM;
  }
  const int n = (int)g->subs.size();
  std::vector<int> rc(n, SCS_OK);
  std::atomic<int> done{0};
  std::atomic<bool> aborted{false};
  std::vector<std::function<void()>> jobs((size_t)n);
  for (int i = 0; i < n; ++i)
    jobs[(size_t)i] = [&, i] {
      scs_ctx* s = g->subs[i];
      rc[i] = f(s, i);
      done.fetch_add(1);
      if (rc[i] == SCS_OK || n == 1) return;
      for (int t = 0; t < 500 && done.load() < n; ++t) std::this_thread::sleep_for(std::chrono::milliseconds(10));
      if (done.load() < n && !aborted.exchange(true)) {
        g->comm_abort->store(true, std::memory_order_release);
        if (g->hx) g->hx->abort();
        for (scs_ctx* o : g->subs)
          if (o->rccl) (void)ncclCommAbort(o->rccl);
      }
    };
  g->workers->run(jobs);
  if (aborted.load()) {
    g->group_broken = true;
    for (scs_ctx* o : g->subs) o->rccl = nullptr;   // aborted (freed) by ncclCommAbort
  }
  for (int i = 0; i < n; ++i)
    if (rc[i] != SCS_OK) {
      g->err = "device " + std::to_string(g->subs[i]->dev) + ": " + g->subs[i]->err;
      return rc[i];
    }
  g->err.clear();
  return SCS_OK;
}

bool is_group(const scs_ctx* c) { return c && !c->subs.empty(); }

}  // namespace

extern "C" {

int scs_create_multi(const int* devs, int ndev, scs_ctx** out) { return scs_create_multi_ex(devs, ndev, 0, out); }

int scs_create_multi_ex(const int* devs, int ndev, int flags, scs_ctx** out) {
  if (!out || !devs || ndev < 1 || (flags & ~SCS_MULTI_HOST_EXCHANGE)) return SCS_ERR_ARG;
  *out = nullptr;
  const bool host = (flags & SCS_MULTI_HOST_EXCHANGE) != 0;
  scs_ctx* g = new scs_ctx();
  for (int i = 0; i < ndev && !host; ++i)
    for (int j = 0; j < i; ++j)
      if (devs[i] == devs[j]) {
        delete g;
        return SCS_ERR_ARG;   // RCCL takes one rank per GPU
      }
  for (int i = 0; i < ndev; ++i) {
    scs_ctx* s = nullptr;
    const int rc = scs_create(devs[i], nullptr, &s);
    if (rc != SCS_OK) {
      for (scs_ctx* o : g->subs) scs_destroy(o);
      delete g;
      return rc;
    }
    g->subs.push_back(s);
  }
  g->comm_abort = std::make_shared<std::atomic<bool>>(false);
  if (host) {
    g->hx.reset(new scs_ctx::HostExchange(ndev));
    for (int i = 0; i < ndev; ++i) {
      scs_ctx* s = g->subs[i];
      s->rank = i;
      s->nranks = ndev;
      s->ar = &scs_ctx::HostExchange::allreduce;
      s->ar_user = &g->hx->ranks[(size_t)i];
      s->comm_abort = g->comm_abort;
    }
  } else {
    std::vector<ncclComm_t> comms((size_t)ndev, nullptr);
    const ncclResult_t r = ncclCommInitAll(comms.data(), ndev, devs);
    if (r != ncclSuccess) {
      for (scs_ctx* o : g->subs) scs_destroy(o);
      delete g;
      return SCS_ERR_COMM;
    }
    for (int i = 0; i < ndev; ++i) {
      g->subs[i]->rccl = comms[(size_t)i];
      g->subs[i]->rank = i;
      g->subs[i]->nranks = ndev;
      g->subs[i]->comm_abort = g->comm_abort;
    }
  }
  g->workers.reset(new scs_ctx::Workers(std::vector<int>(devs, devs + ndev)));
  g->dev = devs[0];
  g->st = g->subs[0]->st;
  *out = g;
  return SCS_OK;
}

int scs_group_size(scs_ctx* c, int* ndev) {
  if (!c || !ndev) return SCS_ERR_ARG;
  *ndev = is_group(c) ? (int)c->subs.size() : 1;
  return SCS_OK;
}

int scs_comm_info(scs_ctx* c, int* kind, int* nranks, int* rank, int* rccl_version, char* lib, int64_t cap) {
  if (!c) return SCS_ERR_ARG;
  int k = SCS_COMM_NONE, n = 1, r = 0;
  const scs_ctx* s = is_group(c) ? c->subs[0] : c;
  if (is_group(c)) {
    k = c->hx ? SCS_COMM_GROUP_HOST : SCS_COMM_GROUP_RCCL;
    n = (int)c->subs.size();
    if (!c->hx && s->rccl) {   // the communicator's own view (ncclCommInitAll over the devices)
      int cn = 0;
      if (ncclCommCount(s->rccl, &cn) == ncclSuccess) n = cn;
    }
  } else if (s->rccl) {
    k = SCS_COMM_RCCL;
    int cn = 0, cr = 0;
    if (ncclCommCount(s->rccl, &cn) != ncclSuccess || ncclCommUserRank(s->rccl, &cr) != ncclSuccess) {
      c->err = "ncclCommCount / ncclCommUserRank failed";
      return SCS_ERR_COMM;
    }
    n = cn;
    r = cr;
  } else if (s->ar) {
    k = SCS_COMM_CALLBACK;
    n = s->nranks;
    r = s->rank;
  }
  if (kind) *kind = k;
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  if (rccl_version) {
    int v = 0;
    *rccl_version = ncclGetVersion(&v) == ncclSuccess ? v : 0;
  }
  if (lib && cap > 0) {
    Dl_info di{};
    const char* path = (dladdr((void*)&ncclAllReduce, &di) && di.dli_fname) ? di.dli_fname : "";
    char real[4096];
    if (*path && realpath(path, real)) path = real;
    std::snprintf(lib, (size_t)cap, "%s", path);
  }
  return SCS_OK;
}

}  // extern "C"

namespace {

int group_destroy(scs_ctx* g) {
  g->workers.reset();   // joins the device threads
  for (scs_ctx* s : g->subs) scs_destroy(s);
  g->subs.clear();
  delete g;
  return SCS_OK;
}

int group_set_data(scs_ctx* g, int64_t N, int64_t m, const double* A, int64_t lda, const double* y, int64_t Nglob,
                   int64_t row0) {
  const int n = (int)g->subs.size();
  if ((Nglob > 0 && Nglob != N) || row0 != 0) {
    g->err = "a multi-device context holds the whole problem: N_global = N, row0 = 0 (it splits the rows itself)";
    return SCS_ERR_ARG;
  }
  if (A && N < n) {
    g->err = "a multi-device context needs at least one row per device";
    return SCS_ERR_ARG;
  }
  g->plan = A ? row_plan(N, n) : std::vector<RowBlock>((size_t)n);
  const int rc = group_run(g, [&](scs_ctx* s, int i) {
    const RowBlock b = g->plan[(size_t)i];
    return scs_set_data(s, A ? b.rows() : 0, m, A ? A + b.r0 : nullptr, lda, y ? y + b.r0 : nullptr, A ? N : 0,
                        b.r0);
  });
  if (rc == SCS_OK) {
    g->grpN = A ? N : 0;
    g->grpm = m;
  }
  return rc;
}

int group_gen_data(scs_ctx* g, const scs_synth* sp) {
  const int n = (int)g->subs.size();
  if (!sp || sp->row0 != 0 || sp->N != sp->N_global || sp->N < n) {
    g->err = "a multi-device context generates the whole problem: spec N = N_global >= devices, row0 = 0";
    return SCS_ERR_ARG;
  }
  g->plan = row_plan(sp->N, n);
  const int rc = group_run(g, [&](scs_ctx* s, int i) {
    scs_synth q = *sp;
    q.row0 = g->plan[(size_t)i].r0;
    q.N = g->plan[(size_t)i].rows();
    return scs_gen_data(s, &q);
  });
  if (rc == SCS_OK) {
    g->grpN = sp->N;
    g->grpm = sp->m;
  }
  return rc;
}

int group_get_data(scs_ctx* g, int64_t r0, int64_t nr, double* A, int64_t lda_out, double* y) {
  if (r0 < 0 || nr < 0 || r0 + nr > g->grpN) {
    g->err = "scs_get_data: rows out of range";
    return SCS_ERR_ARG;
  }
  for (const RowPiece& p : window_pieces(g->plan, r0, nr)) {
    scs_ctx* s = g->subs[(size_t)p.dev];
    const int rc = scs_get_data(s, p.local0, p.n, A ? A + p.off : nullptr, lda_out, y ? y + p.off : nullptr);
    if (rc != SCS_OK) {
      g->err = s->err;
      return rc;
    }
  }
  return SCS_OK;
}

// the held-out rows split like the data's (row_plan; a device may hold none of them)
int group_set_test_data(scs_ctx* g, int64_t N, const double* A, int64_t lda, const double* y, int64_t Nglob,
                        int64_t row0) {
  if ((Nglob > 0 && Nglob != N) || row0 != 0) {
    g->err = "a multi-device context holds the whole test set: N_global = N, row0 = 0";
    return SCS_ERR_ARG;
  }
  const std::vector<RowBlock> plan = row_plan(std::max<int64_t>(N, 0), (int)g->subs.size());
  return group_run(g, [&](scs_ctx* s, int i) {
    const RowBlock b = plan[(size_t)i];
    return scs_set_test_data(s, b.rows(), A ? A + b.r0 : nullptr, lda, y ? y + b.r0 : nullptr, N, b.r0);
  });
}

int group_gen_test_data(scs_ctx* g, const scs_synth* sp) {
  if (!sp) {
    g->err = "null synth spec";
    return SCS_ERR_ARG;
  }
  const std::vector<RowBlock> plan = row_plan(sp->N, (int)g->subs.size());
  return group_run(g, [&](scs_ctx* s, int i) {
    scs_synth q = *sp;
    q.row0 = sp->row0 + plan[(size_t)i].r0;
    q.N = plan[(size_t)i].rows();
    q.N_global = sp->N;
    return scs_gen_test_data(s, &q);
  });
}

// one scalar / one m-vector out of a collective evaluation: every device runs it, device 0's result
int group_eval(scs_ctx* g, const double* x, double* out, int64_t nout,
               int (*fn)(scs_ctx*, const double*, double*)) {
  std::vector<std::vector<double>> o(g->subs.size(), std::vector<double>((size_t)std::max<int64_t>(nout, 1)));
  const int rc = group_run(g, [&](scs_ctx* s, int i) { return fn(s, x, o[(size_t)i].data()); });
  if (rc == SCS_OK && out) std::memcpy(out, o[0].data(), sizeof(double) * nout);
  return rc;
}

int group_step(scs_ctx* g, const double* x, const double* x_prev, int64_t iter, const double* grad_fx, double* x_new,
               double* dx, double* pri) {
  const size_t n = g->subs.size(), m = (size_t)g->grpm;
  std::vector<std::vector<double>> xn(n, std::vector<double>(m)), d(n, std::vector<double>(dx ? m : 1));
  std::vector<double> pr(n, 0.0);
  const int rc = group_run(g, [&](scs_ctx* s, int i) {
    return scs_step_grad(s, x, x_prev, iter, grad_fx, xn[(size_t)i].data(), dx ? d[(size_t)i].data() : nullptr,
                         &pr[(size_t)i]);
  });
  if (rc != SCS_OK) return rc;
  std::memcpy(x_new, xn[0].data(), sizeof(double) * m);
  if (dx) std::memcpy(dx, d[0].data(), sizeof(double) * m);
  if (pri) *pri = pr[0];
  return SCS_OK;
}

int group_iterate(scs_ctx* g, const double* x0, const double* x_star, int64_t max_epoch, double x_tol, double f_tol,
                  int rel_kind, double* x_out, const scs_history* h, int64_t* n_hist, int64_t* epochs) {
  const size_t n = g->subs.size(), m = (size_t)g->grpm;
  const size_t cap = (size_t)std::max<int64_t>(2 * max_epoch + 1, 1);
  std::vector<std::vector<double>> buf(n, std::vector<double>(7 * cap + m));
  std::vector<int64_t> nh(n, 0), ep(n, 0);
  const int rc = group_run(g, [&](scs_ctx* s, int i) {
    double* b = buf[(size_t)i].data();
    scs_history hi{b, b + cap, b + 2 * cap, b + 3 * cap, b + 4 * cap, b + 5 * cap, b + 6 * cap};
    return scs_iterate_ex(s, x0, x_star, max_epoch, x_tol, f_tol, rel_kind, b + 7 * cap, &hi, sizeof(hi),
                          &nh[(size_t)i], &ep[(size_t)i]);
  });
  if (rc != SCS_OK) return rc;
  const double* b = buf[0].data();
  const size_t k = (size_t)nh[0];
  double* dst[7] = {h ? h->obj : nullptr, h ? h->fval : nullptr, h ? h->pri_res_norm : nullptr, h ? h->rel : nullptr,
                    h ? h->objrel : nullptr, h ? h->times : nullptr, h ? h->fvaltest : nullptr};
  int has_test = 0;
  (void)scs_has_test(g->subs[0], &has_test);
  for (int a = 0; a < 7; ++a)
    if (dst[a] && (a < 6 || has_test)) std::memcpy(dst[a], b + a * cap, sizeof(double) * k);
  if (x_out) std::memcpy(x_out, b + 7 * cap, sizeof(double) * m);
  if (n_hist) *n_hist = nh[0];
  if (epochs) *epochs = ep[0];
  return SCS_OK;
}

}  // namespace
