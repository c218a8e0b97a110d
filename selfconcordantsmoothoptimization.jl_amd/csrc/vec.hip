// Feature-space (length-m) kernels of the SCORE step: smoothers, the fused
// SCORE tail (η, α, prox, primal residual), regularizer value, L-BFGS vector
// algebra and small matrix fix-ups around the m x m solve.
//
// Reductions whose value feeds a decision or the history (η, ‖x_new − x‖,
// dots of the two-loop recursion, get_reg) run in a fixed order (per-thread
// sequential strides, then a fixed wave/block tree), so repeated runs are
// bitwise identical.  Expressions follow the reference's evaluation order
// so that, on identical inputs, elementwise outputs match the oracle bit for
// bit (IEEE +,-,*,/,sqrt); pow() may differ by <= 1-2 ulp from Julia's.
// Julia evaluates a*b + c with two roundings (no @muladd / @fastmath on the reference path), and
// hipcc contracts to FMA by default: keep the roundings separate in these elementwise semantics
// kernels (it decides exact zeros, e.g. the 0/0 = NaN of the Ostrovskii-Bach gradient at x = 0).
#pragma clang fp contract(off)
#include <algorithm>
#include <utility>

#include "common.h"
#include "kernels.h"

namespace scs {

constexpr int VB = 1024;  // single-workgroup kernels: 16 waves
static inline int nblk(int64_t n, int b) { return (int)((n + b - 1) / b); }

// ---------------------------------------------------------------------------
// Smoothers  (phuber-smooth.jl, exponential-smooth.jl)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double huber_grad_d(double x, double mu) {   // phuber-smooth.jl:31-33
  return x * pow(mu * mu + x * x, -0.5);
}
__device__ __forceinline__ double huber_hess_d(double x, double mu) {   // phuber-smooth.jl:34-36
  return (mu * mu) * pow(mu * mu + x * x, -1.5);
}
__device__ __forceinline__ double pseudo_huber_d(double x, double mu) { // phuber-smooth.jl:28-30
  const double v = mu * mu + x * x;
  return (mu * mu - mu * sqrt(v) + x * x) * pow(v, -0.5);
}

// Ostrovskii & Bach (ostrovskii-bach-smooth.jl:28-36), λ = 1.  Julia literal powers: x^2,
// μ^3 are products; x^5 is the accurate Float64^Int power (pow here); (·)^(-1//2) is pow(·,-0.5).
// x = 0 gives 0/0 = NaN, propagated as the reference does.
__device__ __forceinline__ double osba_val_d(double x, double mu) {   // ostrovskii-bach-smooth.jl:28-30
  const double s = sqrt(mu * mu + 4.0 * (x * x));
  return (((s / 2.0 - mu / 2.0) + mu * log((2.0 * x - s + mu) / x) / 2.0) - 0.6931471805599453 * mu) +
         mu * log((s - mu + 2.0 * x) / x) / 2.0;
}
__device__ __forceinline__ double osba_grad_d(double x, double mu) {   // ostrovskii-bach-smooth.jl:31-33
  const double x2 = x * x, mu2 = mu * mu;
  const double s = sqrt(mu2 + 4.0 * x2);
  const double A = ((-(mu2 * mu) + mu2 * s) - 4.0 * x2 * mu) + 2.0 * x2 * s;
  const double B = (mu * s + mu2) + 4.0 * x2;
  const double C = 4.0 * mu2 * (x2 * x) + 16.0 * pow(x, 5.0);
  return A * B / C;
}
__device__ __forceinline__ double osba_hess_d(double x, double mu) {   // ostrovskii-bach-smooth.jl:34-36
  const double v = mu * mu + 4.0 * (x * x);
  return (sqrt(v) - mu) * mu / (x * x) * pow(v, -0.5) / 2.0;
}

// hμ.grad / hμ.hess of the elementwise smoothers at one coordinate (a, b: that coordinate's bounds)
__device__ __forceinline__ void smooth_elem(int kind, double xi, double ai, double bi, double mu, double& g,
                                            double& h) {
  if (kind == SCS_SMOOTH_PHUBER_L1L2) {
    g = huber_grad_d(xi, mu);
    h = huber_hess_d(xi, mu);
  } else if (kind == SCS_SMOOTH_PHUBER_INDBOX) {
    // huber_grad_indbox (phuber-smooth.jl:83-98): note the `-x < a` test.
    if (-xi < ai) {
      g = pow(ai * ai - 2.0 * xi * ai + mu * mu + xi * xi, -0.5) * (-xi + ai);
    } else if (xi == ai || xi < bi) {
      g = JL_EPS;
    } else {
      g = pow(bi * bi - 2.0 * bi * xi + mu * mu + xi * xi, -0.5) * (bi - xi);
    }
    // huber_hess_indbox (phuber-smooth.jl:99-114)
    if (xi <= ai) {
      h = (mu * mu) * pow(ai * ai - 2.0 * ai * xi + mu * mu + xi * xi, -1.5);
    } else if (ai < xi && xi < bi) {
      h = JL_EPS;
    } else if (xi >= bi) {
      h = (mu * mu) * pow(bi * bi - 2.0 * bi * xi + mu * mu + xi * xi, -1.5);
    } else {
      h = __builtin_nan("");  // NaN x: the reference leaves the entry undefined
    }
  } else if (kind == SCS_SMOOTH_LOGEXP_INDBOX) {   // log-exp-smooth.jl:45-61 (both ifelse arms, then +)
    const double g1 = (xi <= ai + mu) ? (xi - ai - 2.0 * mu) / mu : ((xi >= bi - mu) ? (xi - bi + 2.0 * mu) / mu : 0.0);
    const double g2 = (xi < ai) ? mu / (ai - xi) : ((xi > bi) ? -mu / (bi - xi) : 0.0);
    g = g1 + g2;
    const double h1 = (xi <= ai + mu) ? 1.0 / mu : ((xi >= bi - mu) ? 1.0 / mu : 0.0);
    const double h2 = (xi < ai) ? mu / ((ai - xi) * (ai - xi)) : ((xi > bi) ? mu / ((bi - xi) * (bi - xi)) : 0.0);
    h = h1 + h2;
  } else if (kind == SCS_SMOOTH_OSBA_L1L2) {   // ostrovskii-bach-smooth.jl:27
    g = osba_grad_d(xi, mu);
    h = osba_hess_d(xi, mu);
  } else {  // SCS_SMOOTH_EXP_INDBOX (exponential-smooth.jl:41-50)
    const double e = exp((-xi + ai) / mu);
    g = -e;
    h = 1.0 / mu * e;
  }
}

__global__ void smooth_elem_kernel(int kind, const double* __restrict__ x, int64_t m, double mu,
                                   const double* __restrict__ a, const double* __restrict__ b,
                                   double* __restrict__ gr, double* __restrict__ Hr) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= m) return;
  const bool box = kind == SCS_SMOOTH_PHUBER_INDBOX || kind == SCS_SMOOTH_LOGEXP_INDBOX ||
                   kind == SCS_SMOOTH_EXP_INDBOX;
  double g, h;
  smooth_elem(kind, x[i], box ? a[i] : 0.0, box && kind != SCS_SMOOTH_EXP_INDBOX ? b[i] : 0.0, mu, g, h);
  gr[i] = g;
  Hr[i] = h;
}

// PHuberSmootherGL grad/hess (phuber-smooth.jl:150-164).  Cmat for a
// contiguous partition is diag(group weight); the Hessian carries the global
// dot(Dg, Dg).  Single workgroup: the dot is one fixed-order reduction.
// OSBA = true: OsBaSmootherGL (ostrovskii-bach-smooth.jl:73-87), the same composition with the
// Ostrovskii-Bach value / grad / hess.
template <bool OSBA>
__global__ __launch_bounds__(VB) void smooth_gl_kernel(const double* __restrict__ x, int64_t m, double mu,
                                                       const double* __restrict__ wel,
                                                       double* __restrict__ gr, double* __restrict__ Hr) {
  __shared__ double sh[VB / 64];
  auto val = [&](double v) { return OSBA ? osba_val_d(v, mu) : pseudo_huber_d(v, mu); };
  auto grd = [&](double v) { return OSBA ? osba_grad_d(v, mu) : huber_grad_d(v, mu); };
  auto hes = [&](double v) { return OSBA ? osba_hess_d(v, mu) : huber_hess_d(v, mu); };
  double part = 0.0;
  for (int64_t i = threadIdx.x; i < m; i += VB) {
    const double Dg = grd(x[i]);
    part += Dg * Dg;
  }
  const double dd = block_sum<VB>(part, sh);
  for (int64_t i = threadIdx.x; i < m; i += VB) {
    const double xi = x[i];
    const double g = val(xi);
    const double Dg = grd(xi);
    const double DDg = hes(xi);
    const double Cg = wel[i] * g;
    gr[i] = grd(Cg) * Dg;
    Hr[i] = hes(Cg) * dd + grd(Cg) * DDg;
  }
}

// ---------------------------------------------------------------------------
// Prox operators (prox-operators.jl) -- elementwise parts
// ---------------------------------------------------------------------------
// h = 1 ./ Hr is passed as computed by the caller (Hdiag_inv).
__device__ __forceinline__ double prox_l1_d(double z, double hinv, double lam, double alpha) {
  const double t = (alpha * lam) / hinv;                      // prox-operators.jl:10
  return jl_sign(z) * jl_max(fabs(z) - t, 0.0);               // prox-operators.jl:11
}
__device__ __forceinline__ double prox_l2_d(double z, double hinv, double lam, double alpha) {
  const double t = (alpha * lam) / hinv;                      // prox-operators.jl:23
  return z * jl_max(1.0 - t / (z * z), 0.0);                  // prox-operators.jl:24
}
__device__ __forceinline__ double prox_box_d(double z, double lb, double ub) {
  return jl_min(jl_max(z, lb), ub);                           // prox-operators.jl:45
}

struct ProxArgs {
  int reg;            // scs_reg_kind
  int use_prox;
  double lam;         // λ (λ1 for gl)
  double lam2;        // λ2 (gl)
  const double* lb;   // C_set lower (length m, raw, may be -Inf)
  const double* ub;
  const int* gstart;  // gl groups (0-based ranges partitioning 0..m-1, any order)
  const int* gend;
  const double* gw;   // group weights (Int in the reference)
  int ngroups;
  const int* gmap;    // get_P's G (0-based) for P.matrix*x = x[G] in get_reg; null = identity
};

// Elementwise prox + the gl group pass, inside one workgroup.
// z: input (x + dx), hinv: 1/Hr, out: result.  step = α of invoke_prox.
__device__ void prox_block(const ProxArgs& P, const double* __restrict__ z, const double* __restrict__ hinv,
                           double step, int64_t m, double* __restrict__ out) {
  if (P.reg == SCS_REG_L1) {
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) out[i] = prox_l1_d(z[i], hinv[i], P.lam, step);
  } else if (P.reg == SCS_REG_L2) {
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) out[i] = prox_l2_d(z[i], hinv[i], P.lam, step);
  } else if (P.reg == SCS_REG_INDBOX) {
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) out[i] = prox_box_d(z[i], P.lb[i], P.ub[i]);
  } else {  // gl: prox-operators.jl:55-66 -> ProxL2 (prox-reg-utils.jl:84-99)
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) {
      const double t = P.lam / hinv[i];                       // λ1 ./ h (no α)
      out[i] = jl_sign(z[i]) * jl_max(fabs(z[i]) - t, 0.0);
    }
    __syncthreads();
    const double beta_scale = step * P.lam2;                  // α*λ2
    for (int g = threadIdx.x; g < P.ngroups; g += blockDim.x) {
      const int s = P.gstart[g], e = P.gend[g];
      const double beta = beta_scale * P.gw[g];
      double nrm2 = 0.0;
      for (int k = s; k <= e; ++k) nrm2 += out[k] * out[k];  // twonorm: sequential
      const double nrm = sqrt(nrm2);
      for (int k = s; k <= e; ++k) out[k] = out[k] * jl_max(1.0 - beta / (hinv[k] * nrm), 0.0);
    }
  }
  __syncthreads();
}

// Fused SCORE tail shared by the three step! methods
// (prox-N-SCORE.jl:226-246, prox-GGN-SCORE.jl:65-105, prox-L-BFGS-SCORE.jl:127-146):
//   Hinv = 1 ./ Hr;  η = sqrt(λgr' * (Hinv .* λgr));  α = step/(1 + Mg*η)
//   safe_α = min(1, α);  dx = safe_α*d;  x_new = prox(x + dx) | x + dx
//   pri = ‖x_new − x‖ | ‖dx‖
// step_dev (if non-null) overrides step_host (BB / line search results).
__global__ __launch_bounds__(VB) void score_tail_kernel(
    const double* __restrict__ x, const double* __restrict__ d, const double* __restrict__ gr,
    const double* __restrict__ Hr, int64_t m, double lam, double Mg, double step_host,
    const double* __restrict__ step_dev, ProxArgs P, double* __restrict__ hinv, double* __restrict__ zbuf,
    double* __restrict__ x_new, double* __restrict__ dx, double* __restrict__ scal) {
  __shared__ double sh[VB / 64];
  const double step = step_dev ? *step_dev : step_host;
  double part = 0.0;
  for (int64_t i = threadIdx.x; i < m; i += VB) {
    const double hi = 1.0 / Hr[i];
    hinv[i] = hi;
    const double lgr = lam * gr[i];
    part += lgr * (hi * lgr);
  }
  const double eta2 = block_sum<VB>(part, sh);
  const double eta = sqrt(eta2);
  const double alpha = step / (1.0 + Mg * eta);
  const double safe_alpha = jl_min(1.0, alpha);
  for (int64_t i = threadIdx.x; i < m; i += VB) {
    const double dxi = safe_alpha * d[i];
    dx[i] = dxi;
    zbuf[i] = x[i] + dxi;
  }
  __syncthreads();
  if (P.use_prox) {
    prox_block(P, zbuf, hinv, step, m, x_new);
  } else {
    for (int64_t i = threadIdx.x; i < m; i += VB) x_new[i] = zbuf[i];
    __syncthreads();
  }
  part = 0.0;
  for (int64_t i = threadIdx.x; i < m; i += VB) {
    const double r = P.use_prox ? (x_new[i] - x[i]) : dx[i];
    part += r * r;
  }
  const double pri2 = block_sum<VB>(part, sh);
  if (threadIdx.x == 0) {
    scal[0] = sqrt(pri2);  // pri_res_norm
    scal[1] = eta;
    scal[2] = alpha;
    scal[3] = step;
  }
}

// Multi-workgroup SCORE tail (large m, elementwise prox: l1 / l2 / indbox, or no prox): the
// same arithmetic as score_tail_kernel with the two norms reduced over TAIL_G workgroups --
// per-block partials in `part`, summed by every block in the same fixed order, so all blocks
// agree bitwise on η, α.  (gl keeps the one-workgroup kernel: its group pass is sequential.)
constexpr int TAIL_G = 256, TAIL_T = 256;

__device__ __forceinline__ double fixed_sum(const double* __restrict__ part, int n, double* sh) {
  // one wave: lane-strided partial sums, then the wave butterfly (fixed order)
  if (threadIdx.x < 64) {
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += 64) v += part[i];
    v = wave_sum(v);
    if (threadIdx.x == 0) sh[0] = v;
  }
  __syncthreads();
  const double r = sh[0];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(TAIL_T) void tail_eta_kernel(const double* __restrict__ gr, const double* __restrict__ Hr,
                                                          int64_t m, double lam, double* __restrict__ hinv,
                                                          double* __restrict__ part) {
  __shared__ double sh[TAIL_T / 64];
  double p = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)TAIL_T + threadIdx.x; i < m; i += (int64_t)TAIL_G * TAIL_T) {
    const double hi = 1.0 / Hr[i];
    hinv[i] = hi;
    const double lgr = lam * gr[i];
    p += lgr * (hi * lgr);
  }
  const double s = block_sum<TAIL_T>(p, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(TAIL_T) void tail_apply_kernel(
    const double* __restrict__ x, const double* __restrict__ d, int64_t m, double Mg, double step_host,
    const double* __restrict__ step_dev, ProxArgs P, const double* __restrict__ hinv, double* __restrict__ zbuf,
    double* __restrict__ x_new, double* __restrict__ dx, double* __restrict__ part, double* __restrict__ scal) {
  __shared__ double sh[TAIL_T / 64];
  const double step = step_dev ? *step_dev : step_host;
  const double eta = sqrt(fixed_sum(part, TAIL_G, sh));
  const double alpha = step / (1.0 + Mg * eta);
  const double safe_alpha = jl_min(1.0, alpha);
  double p = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)TAIL_T + threadIdx.x; i < m; i += (int64_t)TAIL_G * TAIL_T) {
    const double dxi = safe_alpha * d[i];
    dx[i] = dxi;
    const double z = x[i] + dxi;
    zbuf[i] = z;
    double xn = z;
    if (P.use_prox) {
      if (P.reg == SCS_REG_L1) xn = prox_l1_d(z, hinv[i], P.lam, step);
      else if (P.reg == SCS_REG_L2) xn = prox_l2_d(z, hinv[i], P.lam, step);
      else xn = prox_box_d(z, P.lb[i], P.ub[i]);
    }
    x_new[i] = xn;
    const double r = P.use_prox ? (xn - x[i]) : dxi;
    p += r * r;
  }
  const double s = block_sum<TAIL_T>(p, sh);
  if (threadIdx.x == 0) {
    part[TAIL_G + blockIdx.x] = s;
    if (blockIdx.x == 0) {
      scal[1] = eta;
      scal[2] = alpha;
      scal[3] = step;
    }
  }
}

__global__ __launch_bounds__(64) void tail_pri_kernel(const double* __restrict__ part, double* __restrict__ scal) {
  __shared__ double sh[1];
  const double s = fixed_sum(part + TAIL_G, TAIL_G, sh);
  if (threadIdx.x == 0) scal[0] = sqrt(s);
}

// prox only (kernel-level parity entry point)
__global__ __launch_bounds__(VB) void prox_only_kernel(ProxArgs P, const double* __restrict__ z,
                                                       const double* __restrict__ Hr, double step, int64_t m,
                                                       double* __restrict__ hinv, double* __restrict__ out) {
  for (int64_t i = threadIdx.x; i < m; i += VB) hinv[i] = 1.0 / Hr[i];
  __syncthreads();
  prox_block(P, z, hinv, step, m, out);
}

// get_reg (regularizers.jl:4-31); gl: λ2·fz(P.matrix*x) + λ1·Σ|x| with (P.matrix*x)_k = x[G[k]].
__global__ __launch_bounds__(VB) void reg_value_kernel(ProxArgs P, const double* __restrict__ x, int64_t m,
                                                       double* __restrict__ out) {
  __shared__ double sh[VB / 64];
  __shared__ double gsum[1];
  double part = 0.0;
  if (P.reg == SCS_REG_INDBOX) {
    for (int64_t i = threadIdx.x; i < m; i += VB) part += (x[i] < P.lb[i] || x[i] > P.ub[i]) ? 1.0 : 0.0;
    const double nout = block_sum<VB>(part, sh);
    if (threadIdx.x == 0) out[0] = nout > 0 ? __builtin_inf() : 0.0;
    return;
  }
  for (int64_t i = threadIdx.x; i < m; i += VB) part += (P.reg == SCS_REG_L2) ? x[i] * x[i] : fabs(x[i]);
  const double s = block_sum<VB>(part, sh);
  if (P.reg != SCS_REG_GL) {
    if (threadIdx.x == 0) out[0] = P.lam * s;
    return;
  }
  // fz (prox-reg-utils.jl:101-110): the group terms w_g·‖(Px)_g‖ (twonorm sequential within a
  // group) one thread per group, then their sum in group order by one thread -- the
  // reference's own order, so the value is the same as the sequential loop's bit for bit
  constexpr int GL_LDS = 4096;
  __shared__ double gterm[GL_LDS];
  double fz = 0.0;
  for (int g0 = 0; g0 < P.ngroups; g0 += GL_LDS) {
    const int ng = min(GL_LDS, P.ngroups - g0);
    for (int g = threadIdx.x; g < ng; g += VB) {
      double nrm2 = 0.0;
      for (int k = P.gstart[g0 + g]; k <= P.gend[g0 + g]; ++k) {
        const double v = P.gmap ? x[P.gmap[k]] : x[k];
        nrm2 += v * v;
      }
      gterm[g] = P.gw[g0 + g] * sqrt(nrm2);
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int g = 0; g < ng; ++g) fz += gterm[g];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    gsum[0] = fz;
    out[0] = P.lam2 * fz + P.lam * s;
  }
}

// ---------------------------------------------------------------------------
// Small helpers
// ---------------------------------------------------------------------------
// out[0] = Σ a_i b_i  (fixed order)
__global__ __launch_bounds__(VB) void dot_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                 int64_t m, double* __restrict__ out) {
  __shared__ double sh[VB / 64];
  double part = 0.0;
  for (int64_t i = threadIdx.x; i < m; i += VB) part += a[i] * b[i];
  const double s = block_sum<VB>(part, sh);
  if (threadIdx.x == 0) out[0] = s;
}

// out = a + lam*b   (∇q = ∇f + λ gr)
__global__ void axpby_kernel(const double* __restrict__ a, double lam, const double* __restrict__ b, int64_t m,
                             double* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < m) out[i] = a[i] + lam * b[i];
}

// out = a - b
__global__ void sub_kernel(const double* __restrict__ a, const double* __restrict__ b, int64_t m,
                           double* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < m) out[i] = a[i] - b[i];
}

// out = -a
__global__ void neg_kernel(const double* __restrict__ a, int64_t m, double* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < m) out[i] = -a[i];
}

// x + α d with α read from the device (line search trial point)
__global__ void trial_point_kernel(const double* __restrict__ x, const double* __restrict__ d, double alpha,
                                   int64_t m, double* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < m) out[i] = x[i] + alpha * d[i];
}

// inv_BB_step (utils.jl:43-48): (γ⋅γ)/(δ'γ), δ = x − x_prev, γ = g − g_prev
__global__ __launch_bounds__(VB) void bb_step_kernel(const double* __restrict__ x, const double* __restrict__ xp,
                                                     const double* __restrict__ g, const double* __restrict__ gp,
                                                     int64_t m, double* __restrict__ out) {
  __shared__ double sh[VB / 64];
  double gg = 0.0, dg = 0.0;
  for (int64_t i = threadIdx.x; i < m; i += VB) {
    const double dl = x[i] - xp[i];
    const double gm = g[i] - gp[i];
    gg += gm * gm;
    dg += dl * gm;
  }
  gg = block_sum<VB>(gg, sh);
  dg = block_sum<VB>(dg, sh);
  if (threadIdx.x == 0) out[0] = gg / dg;
}

// L-BFGS two-loop recursion (prox-L-BFGS-SCORE.jl:47-68) for one workgroup.
// S, Y: ring buffers [mem][ld]; order[k] = ring slot of the k-th oldest pair.
// Writes d = -r.  Dots are recomputed exactly as the reference does.
// kp / H0p (device ring, scs_iterate's pipelined loop): k = *kp and H0 = *H0p instead of the
// arguments; k = 0 gives d = -g (launch_neg's bits: the reference's `d = -∇q` branch).
// T = float: the fp32-arithmetic arm (scs_set_compute_f32; BASELINE configs[4]): every operand
// rounded to fp32 on load, dots / axpys / α, ρ, β in fp32, results stored widened (exact) in the
// fp64 buffers.  T = double is the default path, unchanged.
template <typename T>
__global__ __launch_bounds__(VB) void two_loop_kernel(const double* __restrict__ S, const double* __restrict__ Y,
                                                      int64_t ld, const int* __restrict__ order,
                                                      const int* __restrict__ kp, int k, const double* __restrict__ H0p,
                                                      double H0d, const double* __restrict__ g, int64_t m,
                                                      double* __restrict__ q, double* __restrict__ dout,
                                                      double* __restrict__ ab /*[2*k]*/) {
  __shared__ double sh[VB / 64];
  if (kp) k = *kp;
  const T H0 = (T)(H0p ? *H0p : H0d);
  if (k == 0) {
    for (int64_t i = threadIdx.x; i < m; i += VB) dout[i] = -(double)(T)g[i];
    return;
  }
  for (int64_t i = threadIdx.x; i < m; i += VB) q[i] = (double)(T)g[i];
  __syncthreads();
  for (int t = k - 1; t >= 0; --t) {           // newest -> oldest
    const double* s = S + (int64_t)order[t] * ld;
    const double* y = Y + (int64_t)order[t] * ld;
    T ys = 0, sq = 0;
    for (int64_t i = threadIdx.x; i < m; i += VB) {
      ys += (T)y[i] * (T)s[i];
      sq += (T)s[i] * (T)q[i];
    }
    ys = block_sum<VB, T>(ys, sh);
    sq = block_sum<VB, T>(sq, sh);
    const T rho = (T)1 / ys;
    const T al = rho * sq;
    for (int64_t i = threadIdx.x; i < m; i += VB) q[i] = (double)((T)q[i] - al * (T)y[i]);
    if (threadIdx.x == 0) { ab[2 * t] = (double)al; ab[2 * t + 1] = (double)rho; }
    __syncthreads();
  }
  for (int64_t i = threadIdx.x; i < m; i += VB) q[i] = (double)(H0 * (T)q[i]);   // r = H0*q (in place)
  __syncthreads();
  for (int t = 0; t < k; ++t) {                // oldest -> newest
    const double* s = S + (int64_t)order[t] * ld;
    const double* y = Y + (int64_t)order[t] * ld;
    T yr = 0;
    for (int64_t i = threadIdx.x; i < m; i += VB) yr += (T)y[i] * (T)q[i];
    yr = block_sum<VB, T>(yr, sh);
    const T al = (T)ab[2 * t], rho = (T)ab[2 * t + 1];
    const T beta = rho * yr;
    for (int64_t i = threadIdx.x; i < m; i += VB) q[i] = (double)((T)q[i] + (T)s[i] * (al - beta));
    __syncthreads();
  }
  for (int64_t i = threadIdx.x; i < m; i += VB) dout[i] = -q[i];
}

// Multi-workgroup two-loop for large m: the same recursion, with each dot
// formed as fixed-order per-chunk partials that every workgroup sums in the
// same order (so all of them agree on α, β bit for bit and runs repeat
// exactly).  One launch per recursion step; each launch applies its axpy to
// its chunk and immediately forms the next step's partial dot on the updated
// chunk, so q / r are read once per step.  The chunk partition (not the
// single-workgroup stride) sets the summation order of the dots.  T as above.
constexpr int TLB = 256;
template <typename T>
__device__ __forceinline__ T sum_parts(const double* __restrict__ p, int G) {
  T s = 0;
  for (int b = 0; b < G; ++b) s += (T)p[b];
  return s;
}

// The recursion step a launch handles is its launch index i (first loop t = k-1-i, second loop
// t = i), so with a device ring (kp) the host launches for an upper bound of k and the surplus
// launches return at once.  Partial dots live in parity buffers keyed by t (work: pys [k][G],
// then first-loop P[0], P[1] and second-loop P[2], P[3], G each), not by launch order.
// Bodies of the launches (chunk b of G).
template <typename T>
__device__ __forceinline__ void tl_init_body(const double* __restrict__ S, const double* __restrict__ Y, int64_t ld,
                                             const int* __restrict__ order, int k, const double* __restrict__ g,
                                             int64_t m, int64_t C, double* __restrict__ work, int kcap,
                                             double* __restrict__ dout, int b, int G, double* sh) {
  const int64_t i0 = b * C, i1 = min(m, i0 + C);
  if (k == 0) {   // d = -∇q
    for (int64_t i = i0 + threadIdx.x; i < i1; i += TLB) dout[i] = -(double)(T)g[i];
    return;
  }
  double* pys = work;
  double* psq = work + ((int64_t)kcap + ((k - 1) & 1)) * G;
  for (int t = 0; t < k; ++t) {
    const double* s = S + (int64_t)order[t] * ld;
    const double* y = Y + (int64_t)order[t] * ld;
    T v = 0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += TLB) v += (T)y[i] * (T)s[i];
    v = block_sum<TLB, T>(v, sh);
    if (threadIdx.x == 0) pys[t * G + b] = (double)v;
  }
  const double* s = S + (int64_t)order[k - 1] * ld;
  T v = 0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += TLB) v += (T)s[i] * (T)g[i];
  v = block_sum<TLB, T>(v, sh);
  if (threadIdx.x == 0) psq[b] = (double)v;
}

// first loop, step t (newest -> oldest): q -= α_t y_t; partial s_{t-1}·q (or, at t = 0,
// r = H0 q and the partial y_0·r of the second loop)
template <typename T>
__device__ __forceinline__ void tl_first_body(const double* __restrict__ S, const double* __restrict__ Y, int64_t ld,
                                              const int* __restrict__ order, int k, int t, T H0, int64_t m,
                                              int64_t C, const double* __restrict__ g, double* __restrict__ q,
                                              double* __restrict__ work, int kcap, double* __restrict__ ab, int b,
                                              int G, double* sh) {
  const int64_t i0 = b * C, i1 = min(m, i0 + C);
  const double* pys = work;
  const double* pin = work + ((int64_t)kcap + (t & 1)) * G;
  double* pout = work + ((int64_t)kcap + (t > 0 ? ((t - 1) & 1) : 2)) * G;
  const T ys = sum_parts<T>(pys + t * G, G), sq = sum_parts<T>(pin, G);
  const T rho = (T)1 / ys;
  const T al = rho * sq;
  const double* y = Y + (int64_t)order[t] * ld;
  const double* sn = (t > 0) ? S + (int64_t)order[t - 1] * ld : Y + (int64_t)order[0] * ld;
  const double* qin = (t == k - 1) ? g : q;   // q = ∇q before the first step
  T v = 0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += TLB) {
    T qi = (T)qin[i] - al * (T)y[i];
    if (t == 0) qi = H0 * qi;
    q[i] = (double)qi;
    v += (T)sn[i] * qi;
  }
  v = block_sum<TLB, T>(v, sh);
  if (threadIdx.x == 0) {
    pout[b] = (double)v;
    if (b == 0) { ab[2 * t] = (double)al; ab[2 * t + 1] = (double)rho; }
  }
}

// second loop, step t (oldest -> newest): r += s_t (α_t − β_t); partial y_{t+1}·r, or d = −r at the end
template <typename T>
__device__ __forceinline__ void tl_second_body(const double* __restrict__ S, const double* __restrict__ Y, int64_t ld,
                                               const int* __restrict__ order, int k, int t, int64_t m, int64_t C,
                                               double* __restrict__ r, double* __restrict__ work, int kcap,
                                               const double* __restrict__ ab, double* __restrict__ dout, int b, int G,
                                               double* sh) {
  const int64_t i0 = b * C, i1 = min(m, i0 + C);
  const double* pin = work + ((int64_t)kcap + 2 + (t & 1)) * G;
  double* pout = work + ((int64_t)kcap + 2 + ((t + 1) & 1)) * G;
  const T yr = sum_parts<T>(pin, G);
  const T al = (T)ab[2 * t], rho = (T)ab[2 * t + 1];
  const T beta = rho * yr;
  const double* s = S + (int64_t)order[t] * ld;
  const bool last = (t == k - 1);
  const double* yn = last ? s : Y + (int64_t)order[t + 1] * ld;
  T v = 0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += TLB) {
    const T ri = (T)r[i] + (T)s[i] * (al - beta);
    if (last) dout[i] = -(double)ri;
    else r[i] = (double)ri;
    v += (T)yn[i] * ri;
  }
  if (!last) {
    v = block_sum<TLB, T>(v, sh);
    if (threadIdx.x == 0) pout[b] = (double)v;
  }
}

template <typename T>
__global__ __launch_bounds__(TLB) void tl_init_kernel(const double* __restrict__ S, const double* __restrict__ Y,
                                                      int64_t ld, const int* __restrict__ order,
                                                      const int* __restrict__ kp, int k,
                                                      const double* __restrict__ g, int64_t m, int64_t C,
                                                      double* __restrict__ work, int kcap,
                                                      double* __restrict__ dout) {
  __shared__ double sh[TLB / 64];
  if (kp) k = *kp;
  tl_init_body<T>(S, Y, ld, order, k, g, m, C, work, kcap, dout, blockIdx.x, gridDim.x, sh);
}

template <typename T>
__global__ __launch_bounds__(TLB) void tl_first_kernel(const double* __restrict__ S, const double* __restrict__ Y,
                                                       int64_t ld, const int* __restrict__ order,
                                                       const int* __restrict__ kp, int k, int li,
                                                       const double* __restrict__ H0p, double H0, int64_t m,
                                                       int64_t C, const double* __restrict__ g,
                                                       double* __restrict__ q, double* __restrict__ work, int kcap,
                                                       double* __restrict__ ab) {
  __shared__ double sh[TLB / 64];
  if (kp) k = *kp;
  if (H0p) H0 = *H0p;
  const int t = k - 1 - li;
  if (t < 0) return;
  tl_first_body<T>(S, Y, ld, order, k, t, (T)H0, m, C, g, q, work, kcap, ab, blockIdx.x, gridDim.x, sh);
}

template <typename T>
__global__ __launch_bounds__(TLB) void tl_second_kernel(const double* __restrict__ S, const double* __restrict__ Y,
                                                        int64_t ld, const int* __restrict__ order,
                                                        const int* __restrict__ kp, int k, int t, int64_t m,
                                                        int64_t C, double* __restrict__ r,
                                                        double* __restrict__ work, int kcap,
                                                        const double* __restrict__ ab, double* __restrict__ dout) {
  __shared__ double sh[TLB / 64];
  if (kp) k = *kp;
  if (t >= k) return;
  tl_second_body<T>(S, Y, ld, order, k, t, m, C, r, work, kcap, ab, dout, blockIdx.x, gridDim.x, sh);
}

// L-BFGS memory update (prox-L-BFGS-SCORE.jl:148-162): γh = ∇q_new − ∇q,
// store (δh, γh) into ring slot `slot` when δhᵀγh > 1e-10.  scal[0] = δhᵀγh,
// scal[1] = γhᵀγh.  The host reads scal and advances the ring.
__global__ __launch_bounds__(VB) void lbfgs_update_kernel(const double* __restrict__ dh,
                                                          const double* __restrict__ gq_new,
                                                          const double* __restrict__ gq, int64_t m,
                                                          double* __restrict__ Sslot, double* __restrict__ Yslot,
                                                          double* __restrict__ scal) {
  __shared__ double sh[VB / 64];
  double dg = 0.0, gg = 0.0;
  for (int64_t i = threadIdx.x; i < m; i += VB) {
    const double gh = gq_new[i] - gq[i];
    Yslot[i] = gh;                 // staged; committed only if accepted (slot is free)
    Sslot[i] = dh[i];
    dg += dh[i] * gh;
    gg += gh * gh;
  }
  dg = block_sum<VB>(dg, sh);
  gg = block_sum<VB>(gg, sh);
  if (threadIdx.x == 0) { scal[0] = dg; scal[1] = gg; }
}

// ---------------------------------------------------------------------------
// ProxGGNSCORE sample-space branch (ggn_score_step, prox-GGN-SCORE.jl:124-127,
// taken when N + 1 <= m):  Jt = [Jᵀ  λgr] (m x (N+1)), J = diag(s) A,
//   M = I + Q̃ (Jtᵀ H⁻¹ Jt),  Q̃ = diag(q, 0),   M B = [r; 1],   d = -H⁻¹ Jt B.
// With P = A diag(h) Aᵀ (h = 1/Hr, the MFMA Gram on Aᵀ) and u = A (h∘λgr):
//   M[i][j] = δij + q_i s_i s_j P_ij,  M[i][N] = q_i s_i u_i,  M[N][·] = e_N.
// ---------------------------------------------------------------------------
__global__ void ggn_sample_prep_kernel(const double* __restrict__ Hr, const double* __restrict__ gr, double lam,
                                       int64_t m, int64_t mpad, double* __restrict__ hvec, double* __restrict__ hg) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f >= mpad) return;
  const double h = (f < m) ? 1.0 / Hr[f] : 0.0;   // Hdiag_inv = 1 ./ Hr_diag (prox-GGN-SCORE.jl:64)
  hvec[f] = h;
  hg[f] = (f < m) ? h * (lam * gr[f]) : 0.0;
}

__global__ void ggn_sample_assemble_kernel(const double* __restrict__ P, int64_t ldp, const double* __restrict__ s,
                                           const double* __restrict__ q, const double* __restrict__ r,
                                           const double* __restrict__ u, const double* __restrict__ kNN, int64_t N,
                                           double* __restrict__ M, int64_t ldm, double* __restrict__ b) {
  // M row-major (the LU's layout, lu.hip), row i = blockIdx.y; P is symmetric (P_ij = P_ji bitwise)
  const int64_t i = blockIdx.y;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j <= N; j += (int64_t)gridDim.x * blockDim.x) {
    double v;
    if (i == N) v = (j == N) ? 1.0 : 0.0;
    else if (j < N) v = (i == j ? 1.0 : 0.0) + q[i] * (s[i] * s[j] * P[i * ldp + j]);
    else v = q[i] * (s[i] * u[i]);
    M[i * ldm + j] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) b[i] = (i < N) ? r[i] : 1.0;
  (void)kNN;   // Q̃[N][N] = 0: the λgr·H⁻¹·λgr entry only reaches M through a zero row
}

__global__ void ggn_sample_scale_kernel(const double* __restrict__ s, const double* __restrict__ B, int64_t N,
                                        int64_t Npad, double* __restrict__ v) {
  const int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (n < Npad) v[n] = (n < N) ? s[n] * B[n] : 0.0;
}

// d = -(H⁻¹ (Jᵀ... )): d_f = -h_f (t_f + λgr_f B_N), t = Aᵀ(s∘B)
__global__ void ggn_sample_direction_kernel(const double* __restrict__ hvec, const double* __restrict__ t,
                                            const double* __restrict__ hg, const double* __restrict__ B, int64_t N,
                                            int64_t m, double* __restrict__ d) {
  const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (f < m) d[f] = -(hvec[f] * t[f] + hg[f] * B[N]);
}

hipError_t launch_ggn_sample_prep(const double* Hr, const double* gr, double lam, int64_t m, int64_t mpad,
                                  double* hvec, double* hg, hipStream_t st) {
  hipLaunchKernelGGL(ggn_sample_prep_kernel, dim3(nblk(mpad, 256)), dim3(256), 0, st, Hr, gr, lam, m, mpad, hvec, hg);
  return hipGetLastError();
}
hipError_t launch_ggn_sample_assemble(const double* P, int64_t ldp, const double* s, const double* q,
                                      const double* r, const double* u, const double* kNN, int64_t N, double* M,
                                      int64_t ldm, double* b, hipStream_t st) {
  hipLaunchKernelGGL(ggn_sample_assemble_kernel, dim3((unsigned)ceil_div(N + 1, 256), (unsigned)(N + 1)), dim3(256),
                     0, st, P, ldp, s, q, r, u, kNN, N, M, ldm, b);
  return hipGetLastError();
}
hipError_t launch_ggn_sample_scale(const double* s, const double* B, int64_t N, int64_t Npad, double* v,
                                   hipStream_t st) {
  hipLaunchKernelGGL(ggn_sample_scale_kernel, dim3(nblk(Npad, 256)), dim3(256), 0, st, s, B, N, Npad, v);
  return hipGetLastError();
}
hipError_t launch_ggn_sample_direction(const double* hvec, const double* t, const double* hg, const double* B,
                                       int64_t N, int64_t m, double* d, hipStream_t st) {
  hipLaunchKernelGGL(ggn_sample_direction_kernel, dim3(nblk(m, 256)), dim3(256), 0, st, hvec, t, hg, B, N, m, d);
  return hipGetLastError();
}

// G[i,i] += λ·Hr[i]   (H + λ.*Diagonal(Hr), prox-N-SCORE.jl:177,204; prox-GGN-SCORE.jl:129)
__global__ void diag_add_kernel(double* __restrict__ G, int64_t ldg, int64_t m, double lam,
                                const double* __restrict__ Hr) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < m) G[i * ldg + i] += lam * Hr[i];
}

// copy the strictly-upper triangle onto the lower one (the Gram stores the upper
// triangle; the LU fallback and host copies need the full matrix)
__global__ void symmetrize_kernel(double* __restrict__ G, int64_t ldg, int64_t m) {
  const int64_t j = blockIdx.y;   // column of the upper element (row i < j)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < j; i += (int64_t)gridDim.x * blockDim.x)
    G[i * ldg + j] = G[j * ldg + i];
}

// G = 0.5*(A + Aᵀ) for the quadratic loss (Hessian of 1/2 x'Ax, m x m A; A panel-blocked, S stages)
__global__ void half_sym_kernel(const double* __restrict__ A, int64_t S, int64_t m, double* __restrict__ G,
                                int64_t ldg) {
  const int64_t j = blockIdx.y;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    G[j * ldg + i] = 0.5 * (A[tiled_off(S, i, j)] + A[tiled_off(S, j, i)]);
}

// ---------------------------------------------------------------------------
// Rosenbrock (ProblemGeneric of README.md:49; chained form for m > 2)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(VB) void rosen_kernel(const double* __restrict__ x, int64_t m, int what,
                                                   double* __restrict__ out, double* __restrict__ G, int64_t ldg) {
  __shared__ double sh[VB / 64];
  if (what == 0) {  // value
    double part = 0.0;
    for (int64_t i = threadIdx.x; i + 1 < m; i += VB) {
      const double a = x[i + 1] - x[i] * x[i];
      const double b = 1.0 - x[i];
      part += 100.0 * a * a + b * b;
    }
    const double s = block_sum<VB>(part, sh);
    if (threadIdx.x == 0) out[0] = s;
  } else if (what == 1) {  // gradient
    for (int64_t i = threadIdx.x; i < m; i += VB) {
      double g = 0.0;
      if (i + 1 < m) {
        const double a = x[i + 1] - x[i] * x[i];
        g += -400.0 * x[i] * a - 2.0 * (1.0 - x[i]);
      }
      if (i > 0) g += 200.0 * (x[i] - x[i - 1] * x[i - 1]);
      out[i] = g;
    }
  } else {  // Hessian (dense, tridiagonal)
    for (int64_t j = 0; j < m; ++j)
      for (int64_t i = threadIdx.x; i < m; i += VB) G[j * ldg + i] = 0.0;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < m; i += VB) {
      double hii = 0.0;
      if (i + 1 < m) {
        hii += 1200.0 * x[i] * x[i] - 400.0 * x[i + 1] + 2.0;
        G[(i + 1) * ldg + i] = -400.0 * x[i];
        G[i * ldg + i + 1] = -400.0 * x[i];
      }
      if (i > 0) hii += 200.0;
      G[i * ldg + i] = hii;
    }
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------

hipError_t launch_smoother(int kind, const double* x, int64_t m, double mu, const double* a, const double* b,
                           const double* wel, double* gr, double* Hr, hipStream_t st) {
  if (kind == SCS_SMOOTH_PHUBER_GL)
    hipLaunchKernelGGL(smooth_gl_kernel<false>, dim3(1), dim3(VB), 0, st, x, m, mu, wel, gr, Hr);
  else if (kind == SCS_SMOOTH_OSBA_GL)
    hipLaunchKernelGGL(smooth_gl_kernel<true>, dim3(1), dim3(VB), 0, st, x, m, mu, wel, gr, Hr);
  else
    hipLaunchKernelGGL(smooth_elem_kernel, dim3(nblk(m, 256)), dim3(256), 0, st, kind, x, m, mu, a, b, gr, Hr);
  return hipGetLastError();
}

hipError_t launch_score_tail(const double* x, const double* d, const double* gr, const double* Hr, int64_t m,
                             double lam, double Mg, double step_host, const double* step_dev, const ProxArgsH& Ph,
                             double* hinv, double* zbuf, double* x_new, double* dx, double* scal, hipStream_t st) {
  ProxArgs P{Ph.reg, Ph.use_prox, Ph.lam, Ph.lam2, Ph.lb, Ph.ub, Ph.gstart, Ph.gend, Ph.gw, Ph.ngroups, Ph.gmap};
  // one workgroup is ~130 us at m = 65536 (C5); the multi-workgroup form ~10 us.  Partials live
  // in scal[64 .. 64 + 2 TAIL_G) (alloc_mspace).
  if (m >= 16384 && !(Ph.use_prox && Ph.reg == SCS_REG_GL)) {
    double* part = scal + 64;
    hipLaunchKernelGGL(tail_eta_kernel, dim3(TAIL_G), dim3(TAIL_T), 0, st, gr, Hr, m, lam, hinv, part);
    hipLaunchKernelGGL(tail_apply_kernel, dim3(TAIL_G), dim3(TAIL_T), 0, st, x, d, m, Mg, step_host, step_dev, P,
                       hinv, zbuf, x_new, dx, part, scal);
    hipLaunchKernelGGL(tail_pri_kernel, dim3(1), dim3(64), 0, st, part, scal);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(score_tail_kernel, dim3(1), dim3(VB), 0, st, x, d, gr, Hr, m, lam, Mg, step_host, step_dev, P,
                     hinv, zbuf, x_new, dx, scal);
  return hipGetLastError();
}

hipError_t launch_prox_only(const ProxArgsH& Ph, const double* z, const double* Hr, double step, int64_t m,
                            double* hinv, double* out, hipStream_t st) {
  ProxArgs P{Ph.reg, 1, Ph.lam, Ph.lam2, Ph.lb, Ph.ub, Ph.gstart, Ph.gend, Ph.gw, Ph.ngroups, Ph.gmap};
  hipLaunchKernelGGL(prox_only_kernel, dim3(1), dim3(VB), 0, st, P, z, Hr, step, m, hinv, out);
  return hipGetLastError();
}

// get_reg for l1 / l2 / indbox over TAIL_G workgroups (partials, then a fixed-order sum)
__global__ __launch_bounds__(TAIL_T) void reg_part_kernel(ProxArgs P, const double* __restrict__ x, int64_t m,
                                                          double* __restrict__ part) {
  __shared__ double sh[TAIL_T / 64];
  double p = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)TAIL_T + threadIdx.x; i < m; i += (int64_t)TAIL_G * TAIL_T) {
    if (P.reg == SCS_REG_INDBOX) p += (x[i] < P.lb[i] || x[i] > P.ub[i]) ? 1.0 : 0.0;
    else p += (P.reg == SCS_REG_L2) ? x[i] * x[i] : fabs(x[i]);
  }
  const double s = block_sum<TAIL_T>(p, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(64) void reg_final_kernel(ProxArgs P, const double* __restrict__ part,
                                                       double* __restrict__ out) {
  __shared__ double sh[1];
  const double s = fixed_sum(part, TAIL_G, sh);
  if (threadIdx.x == 0) out[0] = (P.reg == SCS_REG_INDBOX) ? (s > 0 ? __builtin_inf() : 0.0) : P.lam * s;
}

hipError_t launch_reg_value(const ProxArgsH& Ph, const double* x, int64_t m, double* out, double* part,
                            hipStream_t st) {
  ProxArgs P{Ph.reg, 1, Ph.lam, Ph.lam2, Ph.lb, Ph.ub, Ph.gstart, Ph.gend, Ph.gw, Ph.ngroups, Ph.gmap};
  if (m >= 16384 && Ph.reg != SCS_REG_GL && part) {
    hipLaunchKernelGGL(reg_part_kernel, dim3(TAIL_G), dim3(TAIL_T), 0, st, P, x, m, part);
    hipLaunchKernelGGL(reg_final_kernel, dim3(1), dim3(64), 0, st, P, part, out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(reg_value_kernel, dim3(1), dim3(VB), 0, st, P, x, m, out);
  return hipGetLastError();
}

// optim_loop!'s vector norms on the device (iterate.jl:192-197, :234): out = [Σ(x − xs)², Σx², Σ(xn − x)²]
// over G <= TAIL_G workgroups, fixed-order partial sums (xs / xn may be null: that sum is 0)
__global__ __launch_bounds__(TAIL_T) void norms_part_kernel(const double* __restrict__ x, const double* __restrict__ xs,
                                                            const double* __restrict__ xn, int64_t m,
                                                            double* __restrict__ part) {
  __shared__ double sh[TAIL_T / 64];
  double a = 0.0, b = 0.0, c = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)TAIL_T + threadIdx.x; i < m; i += (int64_t)gridDim.x * TAIL_T) {
    const double xi = x[i];
    if (xs) {
      const double t = xs[i] - xi;
      a += t * t;
    }
    b += xi * xi;
    if (xn) {
      const double t = xn[i] - xi;
      c += t * t;
    }
  }
  a = block_sum<TAIL_T>(a, sh);
  b = block_sum<TAIL_T>(b, sh);
  c = block_sum<TAIL_T>(c, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = a;
    part[TAIL_G + blockIdx.x] = b;
    part[2 * TAIL_G + blockIdx.x] = c;
  }
}

__global__ __launch_bounds__(64) void norms_final_kernel(const double* __restrict__ part, int G,
                                                         double* __restrict__ out) {
  __shared__ double sh[1];
  const double a = fixed_sum(part, G, sh);
  const double b = fixed_sum(part + TAIL_G, G, sh);
  const double c = fixed_sum(part + 2 * TAIL_G, G, sh);
  if (threadIdx.x == 0) {
    out[0] = a;
    out[1] = b;
    out[2] = c;
  }
}

hipError_t launch_norms3(const double* x, const double* xs, const double* xn, int64_t m, double* out, double* part,
                         hipStream_t st) {
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>(TAIL_G, ceil_div(m, 4 * TAIL_T)));
  hipLaunchKernelGGL(norms_part_kernel, dim3(G), dim3(TAIL_T), 0, st, x, xs, xn, m, part);
  hipLaunchKernelGGL(norms_final_kernel, dim3(1), dim3(64), 0, st, part, G, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ProxLQNSCORE epoch, fused (scs_iterate's device loop at m >= 16384; scsopt.cpp): the step's
// elementwise work runs as two passes around the two sparse/dense products --
//   lqn_tail   d = -∇q (or the two-loop's d), η from the partials the previous post pass left,
//              α, dx, the prox -> x_new, δh, pri partials            (prox-L-BFGS-SCORE.jl:102-146)
//   lqn_post   at x_new: Aᵀr = Σ of the product's partials, hμ.grad/hess, ∇q_new = Aᵀr + λ gr,
//              the memory pair (S, Y) with δhᵀγh, γhᵀγh partials (:148-162), and for the next
//              epoch η's partials, get_reg's and optim_loop!'s norms (iterate.jl:189-197, 234)
// with the same per-element arithmetic and the same TAIL_G x TAIL_T fixed-order partials as the
// separate kernels (smooth_elem, tail_eta/apply, lbfgs_update_part, reg_part), so the results
// are bitwise those of the unfused step.  R holds LQ_NPART rows of TAIL_G partials.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lqn_tail_body(const double* __restrict__ x, const double* __restrict__ d, int neg,
                                              int64_t m, double Mg, double step, const ProxArgs& P,
                                              const double* __restrict__ hinv, double* __restrict__ x_new,
                                              double* __restrict__ dx, double* __restrict__ dh,
                                              double* __restrict__ R, double* __restrict__ scal, double* sh) {
  const double eta = sqrt(fixed_sum(R + LQ_ETA * TAIL_G, TAIL_G, sh));
  const double alpha = step / (1.0 + Mg * eta);
  const double safe_alpha = jl_min(1.0, alpha);
  double p = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)TAIL_T + threadIdx.x; i < m; i += (int64_t)TAIL_G * TAIL_T) {
    const double di = neg ? -d[i] : d[i];
    const double dxi = safe_alpha * di;
    dx[i] = dxi;
    const double z = x[i] + dxi;
    double xn = z;
    if (P.use_prox) {
      if (P.reg == SCS_REG_L1) xn = prox_l1_d(z, hinv[i], P.lam, step);
      else if (P.reg == SCS_REG_L2) xn = prox_l2_d(z, hinv[i], P.lam, step);
      else xn = prox_box_d(z, P.lb[i], P.ub[i]);
    }
    x_new[i] = xn;
    const double r = P.use_prox ? (xn - x[i]) : dxi;
    dh[i] = r;
    p += r * r;
  }
  const double sp = block_sum<TAIL_T>(p, sh);
  if (threadIdx.x == 0) {
    R[LQ_PRI * TAIL_G + blockIdx.x] = sp;
    if (blockIdx.x == 0) {
      scal[1] = eta;
      scal[2] = alpha;
      scal[3] = step;
    }
  }
}

__global__ __launch_bounds__(TAIL_T) void lqn_tail_kernel(const double* __restrict__ x, const double* __restrict__ d,
                                                          int neg, int64_t m, double Mg, double step, ProxArgs P,
                                                          const double* __restrict__ hinv, double* __restrict__ x_new,
                                                          double* __restrict__ dx, double* __restrict__ dh,
                                                          double* __restrict__ R, double* __restrict__ scal) {
  __shared__ double sh[TAIL_T / 64];
  lqn_tail_body(x, d, neg, m, Mg, step, P, hinv, x_new, dx, dh, R, scal, sh);
}

// The last workgroup to finish (device-scope counter `cnt`, reset by that workgroup) forms the
// sums of the partial rows -- the fixed_sum order: lane l adds rows[l], rows[l+64], ... from 0,
// then the wave butterfly -- and, with a device ring, takes the L-BFGS memory decision
// (prox-L-BFGS-SCORE.jl:154-162, as lbfgs_accept in scsopt.cpp): accept the pair written to
// ring[mem+2] (the spare slot) when δhᵀγh > 1e-10; FIFO capped at mem; H0 = δhᵀγh / γhᵀγh.
// ring = [order[0..mem] | k | spare] on the device.
__device__ __forceinline__ void lqn_ring_accept(int* __restrict__ ring, int mem, double dg, double gg,
                                                double* __restrict__ H0) {
  if (!(dg > 1e-10)) return;
  const int k = ring[mem + 1], slot = ring[mem + 2];
  int spare = 0;
  if (k == mem) {
    spare = ring[0];
    for (int i = 0; i + 1 < k; ++i) ring[i] = ring[i + 1];
    ring[k - 1] = slot;
  } else {
    for (int j = 0; j <= mem; ++j) {   // the next unused physical slot
      bool used = (j == slot);
      for (int i = 0; i < k; ++i) used |= (ring[i] == j);
      if (!used) {
        spare = j;
        break;
      }
    }
    ring[k] = slot;
    ring[mem + 1] = k + 1;
  }
  ring[mem + 2] = spare;
  *H0 = dg / gg;
}

__global__ __launch_bounds__(TAIL_T) void lqn_post_kernel(
    const double* __restrict__ tpart, int nchunk, int64_t ldp, int64_t m, double lam, int skind, double mu,
    const double* __restrict__ sa, const double* __restrict__ sb, ProxArgs P, const double* __restrict__ xs,
    const double* __restrict__ x, const double* __restrict__ xn, const double* __restrict__ gq,
    const double* __restrict__ dh, double* __restrict__ gqn, double* __restrict__ Sbase, double* __restrict__ Ybase,
    int64_t lds, int* __restrict__ ring, int mem, int hslot, double* __restrict__ gr, double* __restrict__ Hr,
    double* __restrict__ hinv, double* __restrict__ R) {
  __shared__ double sh[TAIL_T / 64];
  const bool box = skind == SCS_SMOOTH_PHUBER_INDBOX || skind == SCS_SMOOTH_LOGEXP_INDBOX ||
                   skind == SCS_SMOOTH_EXP_INDBOX;
  const int64_t slot = ring ? ring[mem + 2] : hslot;
  double* __restrict__ Sslot = Sbase + slot * lds;
  double* __restrict__ Yslot = Ybase + slot * lds;
  double dg = 0.0, gg = 0.0, eta = 0.0, reg = 0.0, na = 0.0, nb = 0.0, nc = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)TAIL_T + threadIdx.x; i < m; i += (int64_t)TAIL_G * TAIL_T) {
    // Aᵀr: the partial rows summed as gemv_t_finalize does (4 interleaved accumulators)
    // (16 partial loads in flight per round: one load round trip per 4 adds was the kernel's time)
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int c = 0;
    for (; c + 16 <= nchunk; c += 16) {
      double t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) t[u] = tpart[(int64_t)(c + u) * ldp + i];
#pragma unroll
      for (int u = 0; u < 16; u += 4) {
        s0 += t[u];
        s1 += t[u + 1];
        s2 += t[u + 2];
        s3 += t[u + 3];
      }
    }
    for (; c + 4 <= nchunk; c += 4) {
      s0 += tpart[(int64_t)c * ldp + i];
      s1 += tpart[(int64_t)(c + 1) * ldp + i];
      s2 += tpart[(int64_t)(c + 2) * ldp + i];
      s3 += tpart[(int64_t)(c + 3) * ldp + i];
    }
    for (; c < nchunk; ++c) s0 += tpart[(int64_t)c * ldp + i];
    const double g = (s0 + s1) + (s2 + s3);
    const double xi = xn[i];
    double grn, hrn;
    smooth_elem(skind, xi, box ? sa[i] : 0.0, box && skind != SCS_SMOOTH_EXP_INDBOX ? sb[i] : 0.0, mu, grn, hrn);
    const double gqi = g + lam * grn;   // ∇q(x_new)
    gqn[i] = gqi;
    const double gh = gqi - gq[i];      // the memory pair
    Yslot[i] = gh;
    Sslot[i] = dh[i];
    dg += dh[i] * gh;
    gg += gh * gh;
    gr[i] = grn;                        // the next epoch's smoother, η, h = 1 ./ Hr
    Hr[i] = hrn;
    const double hi = 1.0 / hrn;
    hinv[i] = hi;
    const double lgr = lam * grn;
    eta += lgr * (hi * lgr);
    if (P.reg == SCS_REG_INDBOX) reg += (xi < P.lb[i] || xi > P.ub[i]) ? 1.0 : 0.0;
    else reg += (P.reg == SCS_REG_L2) ? xi * xi : fabs(xi);
    const double ta = xs[i] - xi;
    na += ta * ta;
    nb += xi * xi;
    const double tc = xi - x[i];
    nc += tc * tc;
  }
  const double v[7] = {dg, gg, eta, reg, na, nb, nc};
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const double t = block_sum<TAIL_T>(v[k], sh);
    if (threadIdx.x == 0) R[k * TAIL_G + blockIdx.x] = t;
  }
}

// The sums of lqn_post's partial rows in fixed_sum's order (lane l adds rows[l], rows[l+64], ...
// from 0, then the wave butterfly), the loss sum of the epilogue's block partials in
// sum_partials_kernel's order (1024 lane-strided accumulators, their wave sums, the 16 wave sums in
// order: thread t plays the virtual threads t + 256 j, whose waves are this thread's wave + 4 j),
// with a device ring the L-BFGS memory decision, and the epoch's scalars into pinned host memory.
__global__ __launch_bounds__(256) void lqn_post_final_kernel(ProxArgs P, const double* __restrict__ R,
                                                             const double* __restrict__ valpart, int nval,
                                                             int* __restrict__ ring, int mem,
                                                             double* __restrict__ scal, int zf_slot, int rx_slot,
                                                             int nrm_slot, int h0_slot, double* __restrict__ hmap,
                                                             int nmap) {
  __shared__ double sh[16];
  __shared__ double sr[7];
  __shared__ double sv[64];   // scal[0..nmap) as this kernel leaves it (nmap <= 64)
  if (threadIdx.x < nmap) sv[threadIdx.x] = scal[threadIdx.x];
  if (valpart) {
    double a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = 0.0;
      for (int i = threadIdx.x + 256 * j; i < nval; i += 1024) a[j] += valpart[i];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double w = wave_sum(a[j]);
      if ((threadIdx.x & 63) == 0) sh[(threadIdx.x >> 6) + 4 * j] = w;
    }
  }
  if (threadIdx.x < 64) {
    constexpr int rows[7] = {LQ_DG, LQ_GG, LQ_REG, LQ_NA, LQ_NB, LQ_NC, LQ_PRI};
    constexpr int PER = TAIL_G / 64;
    double p[7][PER];
#pragma unroll
    for (int r = 0; r < 7; ++r)
#pragma unroll
      for (int j = 0; j < PER; ++j) p[r][j] = R[rows[r] * TAIL_G + threadIdx.x + 64 * j];
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < PER; ++j) a += p[r][j];
      a = wave_sum(a);
      if (threadIdx.x == 0) sr[r] = a;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double sdg = sr[0], sgg = sr[1], rs = sr[2];
    auto put = [&](int j, double v) {
      scal[j] = v;
      if (j < nmap) sv[j] = v;
    };
    put(0, sqrt(sr[6]));
    put(16, sdg);
    put(17, sgg);
    put(rx_slot, (P.reg == SCS_REG_INDBOX) ? (rs > 0 ? __builtin_inf() : 0.0) : P.lam * rs);
    put(nrm_slot, sr[3]);
    put(nrm_slot + 1, sr[4]);
    put(nrm_slot + 2, sr[5]);
    if (valpart) {
      double r = 0.0;
#pragma unroll
      for (int i = 0; i < 16; ++i) r += sh[i];
      put(zf_slot, r);
    }
    if (ring) {
      lqn_ring_accept(ring, mem, sdg, sgg, scal + h0_slot);
      if (h0_slot < nmap) sv[h0_slot] = scal[h0_slot];
    }
  }
  __syncthreads();
  // one store per lane into the fine-grained host buffer: visible once the kernel has ended
  if (threadIdx.x < nmap) hmap[threadIdx.x] = sv[threadIdx.x];
}

hipError_t launch_lqn_eta(const double* gr, const double* Hr, int64_t m, double lam, double* hinv, double* R,
                          hipStream_t st) {
  hipLaunchKernelGGL(tail_eta_kernel, dim3(TAIL_G), dim3(TAIL_T), 0, st, gr, Hr, m, lam, hinv, R + LQ_ETA * TAIL_G);
  return hipGetLastError();
}

hipError_t launch_lqn_tail(const double* x, const double* d, int neg, int64_t m, double Mg, double step,
                           const ProxArgsH& Ph, const double* hinv, double* x_new, double* dx, double* dh, double* R,
                           double* scal, hipStream_t st) {
  ProxArgs P{Ph.reg, Ph.use_prox, Ph.lam, Ph.lam2, Ph.lb, Ph.ub, Ph.gstart, Ph.gend, Ph.gw, Ph.ngroups, Ph.gmap};
  hipLaunchKernelGGL(lqn_tail_kernel, dim3(TAIL_G), dim3(TAIL_T), 0, st, x, d, neg, m, Mg, step, P, hinv, x_new, dx,
                     dh, R, scal);
  return hipGetLastError();
}

hipError_t launch_lqn_post(const double* tpart, int nchunk, int64_t ldp, int64_t m, double lam, int skind, double mu,
                           const double* sa, const double* sb, const ProxArgsH& Ph, const double* xs, const double* x,
                           const double* xn, const double* gq, const double* dh, double* gqn, double* S, double* Y,
                           int64_t lds, int* ring, int mem, int slot, double* gr, double* Hr, double* hinv, double* R,
                           const double* valpart, int nval, double* scal, int zf_slot, int rx_slot, int nrm_slot,
                           int h0_slot, double* hmap, int nmap, hipStream_t st) {
  ProxArgs P{Ph.reg, 1, Ph.lam, Ph.lam2, Ph.lb, Ph.ub, Ph.gstart, Ph.gend, Ph.gw, Ph.ngroups, Ph.gmap};
  hipLaunchKernelGGL(lqn_post_kernel, dim3(TAIL_G), dim3(TAIL_T), 0, st, tpart, nchunk, ldp, m, lam, skind, mu, sa, sb,
                     P, xs, x, xn, gq, dh, gqn, S, Y, lds, ring, mem, slot, gr, Hr, hinv, R);
  hipLaunchKernelGGL(lqn_post_final_kernel, dim3(1), dim3(256), 0, st, P, R, valpart, nval, ring, mem, scal, zf_slot,
                     rx_slot, nrm_slot, h0_slot, hmap, nmap);
  return hipGetLastError();
}

hipError_t launch_dot(const double* a, const double* b, int64_t m, double* out, hipStream_t st) {
  hipLaunchKernelGGL(dot_kernel, dim3(1), dim3(VB), 0, st, a, b, m, out);
  return hipGetLastError();
}
hipError_t launch_axpby(const double* a, double lam, const double* b, int64_t m, double* out, hipStream_t st) {
  hipLaunchKernelGGL(axpby_kernel, dim3(nblk(m, 256)), dim3(256), 0, st, a, lam, b, m, out);
  return hipGetLastError();
}
hipError_t launch_sub(const double* a, const double* b, int64_t m, double* out, hipStream_t st) {
  hipLaunchKernelGGL(sub_kernel, dim3(nblk(m, 256)), dim3(256), 0, st, a, b, m, out);
  return hipGetLastError();
}
hipError_t launch_neg(const double* a, int64_t m, double* out, hipStream_t st) {
  hipLaunchKernelGGL(neg_kernel, dim3(nblk(m, 256)), dim3(256), 0, st, a, m, out);
  return hipGetLastError();
}
hipError_t launch_trial_point(const double* x, const double* d, double alpha, int64_t m, double* out,
                              hipStream_t st) {
  hipLaunchKernelGGL(trial_point_kernel, dim3(nblk(m, 256)), dim3(256), 0, st, x, d, alpha, m, out);
  return hipGetLastError();
}
hipError_t launch_bb_step(const double* x, const double* xp, const double* g, const double* gp, int64_t m,
                          double* out, hipStream_t st) {
  hipLaunchKernelGGL(bb_step_kernel, dim3(1), dim3(VB), 0, st, x, xp, g, gp, m, out);
  return hipGetLastError();
}
template <typename T>
static hipError_t two_loop_t(const double* S, const double* Y, int64_t ld, const int* order, int k, double H0,
                             const double* g, int64_t m, double* q, double* d, double* ab, double* work, int kcap,
                             const int* kp, const double* H0p, hipStream_t st) {
  // kp: k on the device, `k` its upper bound (launches beyond the device k return at once)
  if (m <= TWO_LOOP_SINGLE_MAX || (!kp && k < 1)) {
    hipLaunchKernelGGL(two_loop_kernel<T>, dim3(1), dim3(VB), 0, st, S, Y, ld, order, kp, k, H0p, H0, g, m, q, d, ab);
    return hipGetLastError();
  }
  const int G = (int)std::min<int64_t>(TWO_LOOP_MAX_WG, ceil_div(m, 1024));
  const int64_t C = ceil_div(m, G);
  hipLaunchKernelGGL(tl_init_kernel<T>, dim3(G), dim3(TLB), 0, st, S, Y, ld, order, kp, k, g, m, C, work, kcap, d);
  for (int i = 0; i < k; ++i)
    hipLaunchKernelGGL(tl_first_kernel<T>, dim3(G), dim3(TLB), 0, st, S, Y, ld, order, kp, k, i, H0p, H0, m, C, g, q,
                       work, kcap, ab);
  for (int t = 0; t < k; ++t)
    hipLaunchKernelGGL(tl_second_kernel<T>, dim3(G), dim3(TLB), 0, st, S, Y, ld, order, kp, k, t, m, C, q, work, kcap,
                       ab, d);
  return hipGetLastError();
}

hipError_t launch_two_loop(const double* S, const double* Y, int64_t ld, const int* order, int k, double H0,
                           const double* g, int64_t m, double* q, double* d, double* ab, double* work, int kcap,
                           const int* kp, const double* H0p, hipStream_t st, int f32) {
  return f32 ? two_loop_t<float>(S, Y, ld, order, k, H0, g, m, q, d, ab, work, kcap, kp, H0p, st)
             : two_loop_t<double>(S, Y, ld, order, k, H0, g, m, q, d, ab, work, kcap, kp, H0p, st);
}
// the same update over TAIL_G workgroups (large m): per-block partial dots, fixed-order sums
__global__ __launch_bounds__(TAIL_T) void lbfgs_update_part_kernel(const double* __restrict__ dh,
                                                                   const double* __restrict__ gq_new,
                                                                   const double* __restrict__ gq, int64_t m,
                                                                   double* __restrict__ Sslot,
                                                                   double* __restrict__ Yslot,
                                                                   double* __restrict__ part) {
  __shared__ double sh[TAIL_T / 64];
  double dg = 0.0, gg = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)TAIL_T + threadIdx.x; i < m; i += (int64_t)TAIL_G * TAIL_T) {
    const double gh = gq_new[i] - gq[i];
    Yslot[i] = gh;
    Sslot[i] = dh[i];
    dg += dh[i] * gh;
    gg += gh * gh;
  }
  dg = block_sum<TAIL_T>(dg, sh);
  gg = block_sum<TAIL_T>(gg, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = dg;
    part[TAIL_G + blockIdx.x] = gg;
  }
}

__global__ __launch_bounds__(64) void lbfgs_update_final_kernel(const double* __restrict__ part,
                                                                double* __restrict__ scal) {
  __shared__ double sh[1];
  const double dg = fixed_sum(part, TAIL_G, sh);
  const double gg = fixed_sum(part + TAIL_G, TAIL_G, sh);
  if (threadIdx.x == 0) {
    scal[0] = dg;
    scal[1] = gg;
  }
}

hipError_t launch_lbfgs_update(const double* dh, const double* gq_new, const double* gq, int64_t m, double* Sslot,
                               double* Yslot, double* scal, double* part, hipStream_t st) {
  if (m >= 16384 && part) {
    hipLaunchKernelGGL(lbfgs_update_part_kernel, dim3(TAIL_G), dim3(TAIL_T), 0, st, dh, gq_new, gq, m, Sslot, Yslot,
                       part);
    hipLaunchKernelGGL(lbfgs_update_final_kernel, dim3(1), dim3(64), 0, st, part, scal);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(lbfgs_update_kernel, dim3(1), dim3(VB), 0, st, dh, gq_new, gq, m, Sslot, Yslot, scal);
  return hipGetLastError();
}
hipError_t launch_diag_add(double* G, int64_t ldg, int64_t m, double lam, const double* Hr, hipStream_t st) {
  hipLaunchKernelGGL(diag_add_kernel, dim3(nblk(m, 256)), dim3(256), 0, st, G, ldg, m, lam, Hr);
  return hipGetLastError();
}
// flag[0] |= 1 when an m x m system (ld ldg) or its right-hand side holds a NaN / Inf
__global__ void nonfinite_kernel(const double* __restrict__ G, int64_t ldg, int64_t m, const double* __restrict__ rhs,
                                 int* __restrict__ flag) {
  const int64_t j = blockIdx.y;
  bool bad = false;
  for (int64_t i = threadIdx.x; i < m; i += blockDim.x) bad |= !isfinite(G[j * ldg + i]);
  if (j == 0)
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) bad |= !isfinite(rhs[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ void fill_kernel(double* __restrict__ a, int64_t n, double v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = v;
}

hipError_t launch_nonfinite(const double* G, int64_t ldg, int64_t m, const double* rhs, int* flag, hipStream_t st) {
  hipLaunchKernelGGL(nonfinite_kernel, dim3(1, (unsigned)m), dim3(256), 0, st, G, ldg, m, rhs, flag);
  return hipGetLastError();
}

hipError_t launch_fill(double* a, int64_t n, double v, hipStream_t st) {
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)nblk(n, 256)), dim3(256), 0, st, a, n, v);
  return hipGetLastError();
}

hipError_t launch_symmetrize(double* G, int64_t ldg, int64_t m, hipStream_t st) {
  hipLaunchKernelGGL(symmetrize_kernel, dim3(4, (unsigned)m), dim3(256), 0, st, G, ldg, m);
  return hipGetLastError();
}
hipError_t launch_half_sym(const double* A, int64_t S, int64_t m, double* G, int64_t ldg, hipStream_t st) {
  hipLaunchKernelGGL(half_sym_kernel, dim3(4, (unsigned)m), dim3(256), 0, st, A, S, m, G, ldg);
  return hipGetLastError();
}
hipError_t launch_rosen(const double* x, int64_t m, int what, double* out, double* G, int64_t ldg,
                        hipStream_t st) {
  hipLaunchKernelGGL(rosen_kernel, dim3(1), dim3(VB), 0, st, x, m, what, out, G, ldg);
  return hipGetLastError();
}

}  // namespace scs
