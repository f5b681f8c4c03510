// nls_kernels.hip -- gfx950 kernels of the Krylov/Lanczos exponential
// time-stepper (replaces device/spmv.hpp, device/lanczos{,_complex}.hpp,
// device/matfunc_{real,complex}.hpp and the pointwise kernels of
// device/{nlse,nlse_cq,sg}_solver_dev.hpp).
//
// One Lanczos iteration j is two streaming passes over HBM plus one tiny
// single-workgroup reduction:
//   k_alpha<j>   reads W_j with the 5/7-point stencil and reduces
//                a_j = W_j^H L W_j  (-> T(j,j))                 1 vector read
//   k_reduce     sums the per-workgroup partials in a fixed order and
//                computes the CGS coefficients of the next update from the
//                Gram column of W_j and the Krylov relation (no host sync)
//   k_update<j>  W_{j+1} = L W_j / s_j - sum_k H[j][k]/s_k W_k   (CGS, all k<=j)
//                and reduces g_k = W_k^H W_{j+1} and ||W_{j+1}||^2
//                                                        j+1 reads + 1 write
// The stencil is the reference's assembled CSR restated matrix-free
// (laplacians.hpp:10-105): per point, the column's z (3D) / y (2D)
// neighbours come from a register queue while the workgroup marches along the
// slowest dimension; x and (3D) y neighbours are neighbouring lanes' loads
// served from L1/L2.  The 3D "y-wrap" (i,ny-1,k)<->(i,0,k+1) falls out of
// flat-index neighbours p +- nx over contiguous plane storage.
#include <utility>

#include "nls_device.hpp"
#include "nls_kernels.hpp"

namespace nls {

template <class S> __device__ __forceinline__ S from_real(double v);
template <> __device__ __forceinline__ double from_real<double>(double v) { return v; }
template <> __device__ __forceinline__ cplx from_real<cplx>(double v) { return {v, 0.0}; }

template <int DIM> struct Tile {
  static constexpr int BX = DIM == 3 ? 64 : 256;
  static constexpr int BY = DIM == 3 ? 4 : 1;
};

// ---------------------------------------------------------------------------
// wave64 + workgroup reduction into one partial per workgroup (fixed order:
// results are bitwise reproducible run to run)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int NA>
__device__ __forceinline__ void block_store(cplx (&v)[NA], cplx *__restrict__ out) {
  __shared__ cplx red[NTHREADS / 64][NA];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    v[k].re = wave_sum(v[k].re);
    v[k].im = wave_sum(v[k].im);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NA; ++k) red[w][k] = v[k];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < NA; k += NTHREADS) {
    cplx s = red[0][k];
#pragma unroll
    for (int q = 1; q < NTHREADS / 64; ++q) s += red[q][k];
    out[k] = s;
  }
}

// ---------------------------------------------------------------------------
// The stencil march.  fn(p, cur, lap) is called for every local cell p of the
// workgroup's tiles with cur = V[p] and lap = (L V)[p].
template <class S, int DIM, class Fn>
__device__ __forceinline__ void march(const S *__restrict__ V, const Geo &g, Fn &&fn) {
  using T = Tile<DIM>;
  const int tx = threadIdx.x % T::BX, ty = threadIdx.x / T::BX;
  for (int64_t t = blockIdx.x; t < g.ntiles; t += gridDim.x) {
    const int64_t it = t % g.ntx;
    const int64_t rest = t / g.ntx;
    const int64_t jt = rest % g.nty;
    const int64_t kt = rest / g.nty;
    const int64_t x = it * T::BX + tx;
    const int64_t y = DIM == 3 ? jt * T::BY + ty : 0;
    if (x >= g.nx || y >= g.nyp) continue;
    const int64_t q0 = kt * g.kz;
    const int64_t q1 = q0 + g.kz < g.nzl ? q0 + g.kz : g.nzl;
    const int64_t r = y * g.nx + x;
    const bool bxy = (x == 0) || (x == g.nx - 1) || (DIM == 3 && (y == 0 || y == g.nyp - 1));
    S prev = zero<S>();
    if (g.z0 + q0 > 0) prev = V[(q0 - 1) * g.P + r];
    S cur = V[q0 * g.P + r];
    for (int64_t q = q0; q < q1; ++q) {
      const int64_t gq = g.z0 + q;
      const int64_t p = q * g.P + r;
      const S next = (gq + 1 < g.npl) ? V[p + g.P] : zero<S>();
      S nb = prev + next;
      if (x > 0) nb = nb + V[p - 1];
      if (x + 1 < g.nx) nb = nb + V[p + 1];
      if constexpr (DIM == 3) {
        const int64_t pg = gq * g.P + r;
        if (pg >= g.nx) nb = nb + V[p - g.nx];
        if (pg + g.nx < g.Ng) nb = nb + V[p + g.nx];
      }
      const bool bnd = bxy || gq == 0 || gq == g.npl - 1;
      const S lap = g.s * nb + (bnd ? g.sd_bd : g.sd_in) * cur;
      fn(p, cur, lap);
      prev = cur;
      cur = next;
    }
  }
}

// y = L x  (DeviceSpMV::multiply, device/spmv.hpp:65-73)
template <class S, int DIM>
__global__ __launch_bounds__(NTHREADS) void k_lap(const S *__restrict__ V, Geo g, S *__restrict__ out) {
  march<S, DIM>(V, g, [&](int64_t p, const S &, const S &lap) { out[p] = lap; });
}

// a = V^H L V and ||V||^2 per workgroup
template <class S, int DIM>
__global__ __launch_bounds__(NTHREADS) void k_alpha(const S *__restrict__ V, Geo g, cplx *__restrict__ part) {
  S a = zero<S>();
  double n2 = 0.0;
  march<S, DIM>(V, g, [&](int64_t, const S &cur, const S &lap) {
    a += cj_mul(cur, lap);
    n2 += abs2(cur);
  });
  cplx v[2] = {to_c(a), {n2, 0.0}};
  block_store<2>(v, part + (int64_t)blockIdx.x * 2);
}

// W_{J+1} = a * L W_J - sum_{k<=J} b_k W_k ;  partials g_k = W_k^H W_{J+1}, ||W_{J+1}||^2
template <class S, int DIM, int J>
__global__ __launch_bounds__(NTHREADS) void k_update(S *__restrict__ W, int64_t vs, Geo g,
                                                     const KState *__restrict__ st,
                                                     cplx *__restrict__ part) {
  constexpr int NA = J + 2;
  S acc[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) acc[k] = zero<S>();
  cplx b[J + 1];
#pragma unroll
  for (int k = 0; k <= J; ++k) b[k] = st->coef[k];
  const double a = st->coef[J + 1].re;
  const S *__restrict__ VJ = W + (int64_t)J * vs;
  S *__restrict__ out = W + (int64_t)(J + 1) * vs;
  march<S, DIM>(VJ, g, [&](int64_t p, const S &cur, const S &lap) {
    S wk[J > 0 ? J : 1];
#pragma unroll
    for (int k = 0; k < J; ++k) wk[k] = W[(int64_t)k * vs + p];
    S X = a * lap - coef_mul(b[J], cur);
#pragma unroll
    for (int k = 0; k < J; ++k) X = X - coef_mul(b[k], wk[k]);
    out[p] = X;
#pragma unroll
    for (int k = 0; k < J; ++k) acc[k] = acc[k] + cj_mul(wk[k], X);
    acc[J] = acc[J] + cj_mul(cur, X);
    acc[J + 1] = acc[J + 1] + from_real<S>(abs2(X));
  });
  cplx v[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) v[k] = to_c(acc[k]);
  block_store<NA>(v, part + (int64_t)blockIdx.x * NA);
}

// ---------------------------------------------------------------------------
// single-workgroup reductions + coefficient math + m x m eigensolve

// Deterministic sum over nb partial rows of width NA, columns [c0, c0+nc) -> dst
__device__ void sum_partials(const cplx *__restrict__ part, int nb, int NA, int c0, int nc,
                             cplx *dst) {
  __shared__ double sre[NTHREADS], sim[NTHREADS];
  const int t = threadIdx.x;
  for (int v = c0; v < c0 + nc; ++v) {
    double a = 0.0, b = 0.0;
    for (int q = t; q < nb; q += NTHREADS) {
      const cplx x = part[(int64_t)q * NA + v];
      a += x.re;
      b += x.im;
    }
    sre[t] = a;
    sim[t] = b;
    __syncthreads();
    for (int off = NTHREADS / 2; off > 0; off >>= 1) {
      if (t < off) {
        sre[t] += sre[t + off];
        sim[t] += sim[t + off];
      }
      __syncthreads();
    }
    if (t == 0) dst[v - c0] = {sre[0], sim[0]};
    __syncthreads();
  }
}

__device__ __forceinline__ double inv_or_zero(double s) { return s > 0.0 ? 1.0 / s : 0.0; }

// After k_alpha<j> (and k_update<j-1>): sums layout
//   sums[0] = a_j, sums[1] = ||W_j||^2 (A pass), sums[2 .. 2+j] = g_0..g_{j-1}, nn (U pass)
// Coefficients of k_update<j> (all from the Gram column of W_j and the
// Hessenberg columns already known; see DESIGN.md "Lanczos reformulation"):
//   H[j][j] = alpha_j = a_j / s_j^2
//   H[j][k] = sum_{l<=k} conj(H[k][l]) G[j][l] + s_{k+1} G[j][k+1]   (k < j)
//   coef[k] = H[j][k] / s_k,  coef[j+1] = 1 / s_j
__global__ __launch_bounds__(NTHREADS) void k_reduce_iter(KState *__restrict__ st,
                                                          const cplx *__restrict__ partA, int nbA,
                                                          const cplx *__restrict__ partU, int nbU,
                                                          int j, int do_sum, int do_coef) {
  if (do_sum) {
    sum_partials(partA, nbA, 2, 0, 2, st->sums);
    if (j >= 1) sum_partials(partU, nbU, j + 1, 0, j + 1, st->sums + 2);
    __syncthreads();
  }
  if (!do_coef || threadIdx.x != 0) return;
  double sj;
  if (j == 0) {
    sj = sqrt(st->sums[1].re);
    st->s[0] = sj;
    st->G[0][0] = {sj > 0.0 ? 1.0 : 0.0, 0.0};
    st->breakdown = sj > 0.0 ? 0 : 1;
  } else {
    sj = sqrt(st->sums[2 + j].re);
    st->s[j] = sj;
    st->To[j - 1] = sj;
    const double isj = inv_or_zero(sj);
    for (int k = 0; k < j; ++k) {
      const double f = inv_or_zero(st->s[k]) * isj;
      st->G[j][k] = f * st->sums[2 + k];
    }
    st->G[j][j] = {sj > 0.0 ? 1.0 : 0.0, 0.0};
    if (!(sj > 0.0) && st->breakdown == 0) st->breakdown = j + 1;
  }
  const double isj = inv_or_zero(sj);
  const cplx alpha = (isj * isj) * st->sums[0];
  st->Td[j] = alpha.re;
  st->H[j][j] = alpha;
  for (int k = 0; k < j; ++k) {
    cplx acc = {0.0, 0.0};
    for (int l = 0; l <= k; ++l) acc += cmul(cconj(st->H[k][l]), st->G[j][l]);
    acc += st->s[k + 1] * st->G[j][k + 1];
    st->H[j][k] = acc;
  }
  for (int k = 0; k <= j; ++k) st->coef[k] = inv_or_zero(st->s[k]) * st->H[j][k];
  st->coef[j + 1] = {isj, 0.0};
}

__device__ __forceinline__ double sinc_ref(double x) {  // eigen_krylov_real.hpp:95-97
  return fabs(x) < 1e-8 ? 1.0 : sin(x) / x;
}

__device__ cplx eval_f(int func, double lam, double t_re, double t_im) {
  switch (func) {
    case 0: {  // exp(t*|lambda|)
      const double a = fabs(lam);
      const double er = exp(t_re * a);
      double sn, cs;
      sincos(t_im * a, &sn, &cs);
      return {er * cs, er * sn};
    }
    case 1: {  // exp(t*lambda)
      const double er = exp(t_re * lam);
      double sn, cs;
      sincos(t_im * lam, &sn, &cs);
      return {er * cs, er * sn};
    }
    case 2: return {cos(t_re * sqrt(fabs(lam))), 0.0};
    case 3: return {sinc_ref(t_re * sqrt(fabs(lam))), 0.0};
    case 4: { const double s = sinc_ref(t_re * sqrt(fabs(lam))); return {s * s, 0.0}; }
    case 5: return {t_re * sqrt(fabs(lam)), 0.0};
    case 6: {  // eigen_krylov_real.hpp:186-191
      const double x = t_re / 2. * sqrt(fabs(lam));
      if (fabs(x) < 1e-8) return {1.0, 0.0};
      const double s = sin(x) / x;
      return {s * s, 0.0};
    }
    default: return {__builtin_nan(""), __builtin_nan("")};
  }
}

__device__ __noinline__ void eigen_phase(KState *__restrict__ st, int m, int nf, int f0, int f1,
                                         double t_re, double t_im);

// After the last k_update<m-2>: sums[0..m-1] = g_0..g_{m-2}, nn.  Completes
// T (T(m-1,m-1) = 0, eigen_krylov_complex.hpp:21), diagonalises it with
// implicit-shift QL on wave 0 (lane r owns row r of Q) and writes
//   fin[f][k] = s_0 * (Q f(Lambda) Q^T e_1)_k / s_k
// so that  f(L) W_0 = sum_k fin[f][k] W_k  (= beta V f(T) e1).
__global__ __launch_bounds__(NTHREADS) void k_reduce_final(KState *__restrict__ st,
                                                           const cplx *__restrict__ partU, int nbU,
                                                           int m, int do_sum, int do_coef, int nf,
                                                           int f0, int f1, double t_re,
                                                           double t_im) {
  if (do_sum && m >= 2) {
    sum_partials(partU, nbU, m, 0, m, st->sums);
    __syncthreads();
  }
  if (!do_coef) return;
  if (threadIdx.x == 0 && m >= 2) {
    const double s = sqrt(st->sums[m - 1].re);
    st->s[m - 1] = s;
    st->To[m - 2] = s;
    if (!(s > 0.0) && st->breakdown == 0) st->breakdown = m;
  }
  if (threadIdx.x == 0) st->Td[m - 1] = 0.0;
  __syncthreads();
  if (threadIdx.x < 64) eigen_phase(st, m, nf, f0, f1, t_re, t_im);
}

// Wave-0 part of k_reduce_final (no workgroup barriers inside: one wave's LDS
// accesses complete in program order).
__device__ __noinline__ void eigen_phase(KState *__restrict__ st, int m, int nf, int f0, int f1,
                                         double t_re, double t_im) {
  __shared__ double d[MMAX], e[MMAX], Q[MMAX][MMAX + 1];
  const int lane = threadIdx.x;
  if (lane < m) {
    d[lane] = st->Td[lane];
    e[lane] = lane < m - 1 ? st->To[lane] : 0.0;
    for (int c = 0; c < m; ++c) Q[lane][c] = lane == c ? 1.0 : 0.0;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  // implicit-shift QL on the symmetric tridiagonal (d, e); every lane runs the
  // scalar recurrence redundantly, lane r applies the rotations to row r.
  for (int l = 0; l < m; ++l) {
    int iter = 0;
    for (;;) {
      int mm;
      for (mm = l; mm < m - 1; ++mm) {
        const double dd = fabs(d[mm]) + fabs(d[mm + 1]);
        if (fabs(e[mm]) <= 2.220446049250313e-16 * dd) break;
      }
      if (mm == l) break;
      if (++iter > 64) break;
      double gg = (d[l + 1] - d[l]) / (2.0 * e[l]);
      double rr = hypot(gg, 1.0);
      gg = d[mm] - d[l] + e[l] / (gg + (gg >= 0.0 ? fabs(rr) : -fabs(rr)));
      double ss = 1.0, cc = 1.0, pp = 0.0;
      bool early = false;
      for (int i = mm - 1; i >= l; --i) {
        const double ff = ss * e[i], bb = cc * e[i];
        rr = hypot(ff, gg);
        e[i + 1] = rr;
        if (rr == 0.0) {
          d[i + 1] -= pp;
          e[mm] = 0.0;
          early = true;
          break;
        }
        ss = ff / rr;
        cc = gg / rr;
        gg = d[i + 1] - pp;
        rr = (d[i] - gg) * ss + 2.0 * cc * bb;
        pp = ss * rr;
        d[i + 1] = gg + pp;
        gg = cc * rr - bb;
        if (lane < m) {
          const double fq = Q[lane][i + 1];
          Q[lane][i + 1] = ss * Q[lane][i] + cc * fq;
          Q[lane][i] = cc * Q[lane][i] - ss * fq;
        }
      }
      if (early) continue;
      d[l] -= pp;
      e[l] = gg;
      e[mm] = 0.0;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  if (lane < m) {
    st->lam[lane] = d[lane];
    const double s0 = st->s[0];
    const double isr = inv_or_zero(st->s[lane]);
    for (int fi = 0; fi < nf; ++fi) {
      const int func = fi == 0 ? f0 : f1;
      cplx c = {0.0, 0.0};
      for (int k = 0; k < m; ++k) c += (Q[lane][k] * Q[0][k]) * eval_f(func, d[k], t_re, t_im);
      st->fin[fi][lane] = (s0 * isr) * c;
    }
  }
}

// ---------------------------------------------------------------------------
// pointwise kernels

// Nonlinear half step out = exp(-0.5*tau*rho(u)) u, tau = 1j*dt
//  cubic (nlse_solver.hpp:66-69): rho = re^2 + im^2
//  cubic-quintic (device/nlse_cq_solver.hpp:16-39): d = |u|*|u|, rho = s1 d + s2 d^2
__device__ __forceinline__ cplx nl_half(cplx u, double dt, int nonlin, cplx s1, cplx s2) {
  if (nonlin == 0) {
    const double x = u.re * u.re + u.im * u.im;
    double sn, cs;
    sincos((-0.5 * dt) * x, &sn, &cs);
    return {cs * u.re - sn * u.im, cs * u.im + sn * u.re};
  }
  const double a = hypot(u.re, u.im);
  const double d = a * a;
  const cplx rho = d * s1 + (d * d) * s2;
  const cplx z = cmul({-0.0, -0.5 * dt}, rho);
  const double er = exp(z.re);
  double sn, cs;
  sincos(z.im, &sn, &cs);
  return cmul({er * cs, er * sn}, u);
}

__global__ __launch_bounds__(NTHREADS) void k_nl_init(const cplx *__restrict__ u, cplx *__restrict__ w0,
                                                      int64_t n, double dt, int nonlin, cplx s1,
                                                      cplx s2) {
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS)
    w0[p] = nl_half(u[p], dt, nonlin, s1, s2);
}

// u = N(sum_k fin_k W_k) ; W_0 <- N(u) for the next step (fused start of step)
template <int M>
__global__ __launch_bounds__(NTHREADS) void k_final_nlse(cplx *__restrict__ W, int64_t vs, int64_t n,
                                                         const KState *__restrict__ st,
                                                         cplx *__restrict__ u, double dt,
                                                         int nonlin, cplx s1, cplx s2) {
  cplx c[M];
#pragma unroll
  for (int k = 0; k < M; ++k) c[k] = st->fin[0][k];
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    cplx y = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < M; ++k) y += cmul(c[k], W[(int64_t)k * vs + p]);
    const cplx un = nl_half(y, dt, nonlin, s1, s2);
    u[p] = un;
    W[p] = nl_half(un, dt, nonlin, s1, s2);
  }
}

// out = sum_k fin[fi][k] W_k  (one matrix-function action)
template <class S, int M>
__global__ __launch_bounds__(NTHREADS) void k_combine(const S *__restrict__ W, int64_t vs, int64_t n,
                                                      const KState *__restrict__ st,
                                                      S *__restrict__ out) {
  cplx c[M];
#pragma unroll
  for (int k = 0; k < M; ++k) c[k] = st->fin[0][k];
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    S y = zero<S>();
#pragma unroll
    for (int k = 0; k < M; ++k) y = y + coef_mul(c[k], W[(int64_t)k * vs + p]);
    out[p] = y;
  }
}

// sine-Gordon, after the Krylov basis of u (sg_solver.hpp:60-69):
//   g = m * (-sin(id(u)))  -> start vector of the second basis
//   up <- 2 cos(u) - u_past     (first half of sg_solver.hpp:71)
template <int M>
__global__ __launch_bounds__(NTHREADS) void k_sg_mid(const double *__restrict__ W, int64_t vs, int64_t n,
                                                     const KState *__restrict__ st,
                                                     const double *__restrict__ mf,
                                                     double *__restrict__ up,
                                                     double *__restrict__ g0) {
  double ci[M], cc[M];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    ci[k] = st->fin[0][k].re;
    cc[k] = st->fin[1][k].re;
  }
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    double yi = 0.0, yc = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) {
      const double w = W[(int64_t)k * vs + p];
      yi += ci[k] * w;
      yc += cc[k] * w;
    }
    g0[p] = mf[p] * (-sin(yi));
    up[p] = 2 * yc - up[p];
  }
}

//   u_new = (2 cos(u) - u_past) + tau^2 sinc2_half(g);  u_past <- u
template <int M>
__global__ __launch_bounds__(NTHREADS) void k_sg_end(const double *__restrict__ W2, int64_t vs, int64_t n,
                                                     const KState *__restrict__ st,
                                                     double *__restrict__ u,
                                                     double *__restrict__ up, double dt) {
  double c[M];
#pragma unroll
  for (int k = 0; k < M; ++k) c[k] = st->fin[0][k].re;
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    double ys = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) ys += c[k] * W2[(int64_t)k * vs + p];
    const double uo = u[p];
    u[p] = up[p] + (dt * dt) * ys;
    up[p] = uo;
  }
}

__global__ __launch_bounds__(NTHREADS) void k_sg_velocity(const double *__restrict__ u,
                                                          const double *__restrict__ up,
                                                          double *__restrict__ v, int64_t n,
                                                          double dt) {
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS)
    v[p] = (u[p] - up[p]) / dt;
}

// ---------------------------------------------------------------------------
// kernel tables (host side)

#define NLS_J_LIST(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) \
  X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) \
  X(28) X(29) X(30)
#define NLS_M_LIST(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) \
  X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) \
  X(29) X(30) X(31) X(32)

template <class S, int DIM> const void *update_fn(int J) {
  switch (J) {
#define X(J) case J: return reinterpret_cast<const void *>(&k_update<S, DIM, J>);
    NLS_J_LIST(X)
#undef X
    default: return nullptr;
  }
}

const void *kernel_update(bool cplx_, int dim, int J) {
  if (cplx_) return dim == 3 ? update_fn<cplx, 3>(J) : update_fn<cplx, 2>(J);
  return dim == 3 ? update_fn<double, 3>(J) : update_fn<double, 2>(J);
}

const void *kernel_alpha(bool cplx_, int dim) {
  if (cplx_)
    return dim == 3 ? reinterpret_cast<const void *>(&k_alpha<cplx, 3>)
                    : reinterpret_cast<const void *>(&k_alpha<cplx, 2>);
  return dim == 3 ? reinterpret_cast<const void *>(&k_alpha<double, 3>)
                  : reinterpret_cast<const void *>(&k_alpha<double, 2>);
}

const void *kernel_lap(bool cplx_, int dim) {
  if (cplx_)
    return dim == 3 ? reinterpret_cast<const void *>(&k_lap<cplx, 3>)
                    : reinterpret_cast<const void *>(&k_lap<cplx, 2>);
  return dim == 3 ? reinterpret_cast<const void *>(&k_lap<double, 3>)
                  : reinterpret_cast<const void *>(&k_lap<double, 2>);
}

const void *kernel_reduce_iter() { return reinterpret_cast<const void *>(&k_reduce_iter); }
const void *kernel_reduce_final() { return reinterpret_cast<const void *>(&k_reduce_final); }
const void *kernel_nl_init() { return reinterpret_cast<const void *>(&k_nl_init); }
const void *kernel_sg_velocity() { return reinterpret_cast<const void *>(&k_sg_velocity); }

const void *kernel_final_nlse(int M) {
  switch (M) {
#define X(M) case M: return reinterpret_cast<const void *>(&k_final_nlse<M>);
    NLS_M_LIST(X)
#undef X
    default: return nullptr;
  }
}

const void *kernel_combine(bool cplx_, int M) {
  switch (M) {
#define X(M) \
  case M: return cplx_ ? reinterpret_cast<const void *>(&k_combine<cplx, M>) \
                       : reinterpret_cast<const void *>(&k_combine<double, M>);
    NLS_M_LIST(X)
#undef X
    default: return nullptr;
  }
}

const void *kernel_sg_mid(int M) {
  switch (M) {
#define X(M) case M: return reinterpret_cast<const void *>(&k_sg_mid<M>);
    NLS_M_LIST(X)
#undef X
    default: return nullptr;
  }
}

const void *kernel_sg_end(int M) {
  switch (M) {
#define X(M) case M: return reinterpret_cast<const void *>(&k_sg_end<M>);
    NLS_M_LIST(X)
#undef X
    default: return nullptr;
  }
}

}  // namespace nls
