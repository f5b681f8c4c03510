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
// (laplacians.hpp:10-105; G2 anisotropic nlsolvers/common/include/laplacians.hpp:54-218): per point, the column's z (3D) / y (2D)
// neighbours come from a register queue while the workgroup marches along the
// slowest dimension; x and (3D) y neighbours are neighbouring lanes' loads
// served from L1/L2.  The 3D "y-wrap" (i,ny-1,k)<->(i,0,k+1) falls out of
// flat-index neighbours p +- nx over contiguous plane storage.
//
// This file holds the reductions, the eigensolve and the pointwise kernels;
// the stencil passes are in nls_stencil.hpp / nls_stencil.hip.
#include "nls_kernels.hpp"
#include "nls_reduce.hpp"
#include "nls_stencil.hpp"
#include "nls_pass2.hpp"
#include "nls_pass2d.hpp"

namespace nls {

// host-side mirror of the tiling, for grid sizes
int64_t stencil_tiles(const Geo &g, int dim, int rb) {
  int64_t a, b, c;
  if (dim == 3) {
    switch (rb) {
      case 1: tile_counts<3, 1>(g, a, b, c); break;
      case 2: tile_counts<3, 2>(g, a, b, c); break;
      default: tile_counts<3, 4>(g, a, b, c); break;
    }
  } else {
    switch (rb) {
      case 1: tile_counts<2, 1>(g, a, b, c); break;
      case 2: tile_counts<2, 2>(g, a, b, c); break;
      default: tile_counts<2, 4>(g, a, b, c); break;
    }
  }
  return a * b * c;
}
int update_rows_per_thread(int J, bool ani, bool qa) {
  if (!qa) return upd_rb(J, ani);
  return J >= NLS_QA_RB1_FROM ? 1 : (upd_rb(J, ani) > 2 ? 2 : upd_rb(J, ani));
}
int alpha_rows_per_thread() { return RB_ALPHA; }
int fused_rows_per_thread() { return FUSED_RB; }
int alpha_l2_rows_per_thread() { return RB_L2; }
int tq_words() { return NLS_TQ_XCD ? TQ_WORDS : 2; }

// ---------------------------------------------------------------------------
// single-workgroup reductions + coefficient math + m x m eigensolve

#ifndef NLS_COLSUM_U
#define NLS_COLSUM_U 8  // loads in flight per thread of k_colsum (a power of two; 2 -> 8: 512^3 small kernels 0.334 -> 0.293 ms per step, profiles/r06/ab_halo_diag_colsum_tq.txt)
#endif
// The same column sums for large partial arrays (one tile per workgroup
// grids): one workgroup per column, fixed order -> st->sums layout
// [partA columns 0..ncA) then [partU columns 0..ncU).
__device__ __forceinline__ void colsum_body(const cplx *__restrict__ partA, int nbA, int ncA,
                                            const cplx *__restrict__ partU, int nbU, cplx *__restrict__ dst,
                                            const int v) {
  const cplx *__restrict__ col = v < ncA ? partA + (int64_t)v * nbA : partU + (int64_t)(v - ncA) * nbU;
  const int nb = v < ncA ? nbA : nbU;
  // U independent loads per thread and round, one accumulator each (a chain of dependent
  // rounds over 16384 partials was the kernel's time)
  constexpr int U = NLS_COLSUM_U;
  double ac[U], bc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ac[u] = bc[u] = 0.0;
  int q = threadIdx.x;
  for (; q + (U - 1) * NTHREADS < nb; q += U * NTHREADS) {
    cplx xs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xs[u] = col[q + u * NTHREADS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ac[u] += xs[u].re;
      bc[u] += xs[u].im;
    }
  }
  for (; q < nb; q += NTHREADS) { const cplx x0 = col[q]; ac[0] += x0.re; bc[0] += x0.im; }
#pragma unroll
  for (int s = 1; s < U; s *= 2)
#pragma unroll
    for (int u = 0; u + s < U; u += 2 * s) {
      ac[u] += ac[u + s];
      bc[u] += bc[u + s];
    }
  const double a = wave_sum(ac[0]), b = wave_sum(bc[0]);
  __shared__ double ra[NTHREADS / 64], rb[NTHREADS / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { ra[w] = a; rb[w] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sa = ra[0], sb = rb[0];
    for (int i = 1; i < NTHREADS / 64; ++i) { sa += ra[i]; sb += rb[i]; }
    dst[v] = {sa, sb};
  }
}
__global__ __launch_bounds__(NTHREADS) void k_colsum(const cplx *__restrict__ partA, int nbA, int ncA,
                                                     const cplx *__restrict__ partU, int nbU,
                                                     cplx *__restrict__ dst) {
  colsum_body(partA, nbA, ncA, partU, nbU, dst, blockIdx.x);
}
const void *kernel_colsum() { return reinterpret_cast<const void *>(&k_colsum); }



__global__ __launch_bounds__(NTHREADS) void k_reduce_iter(KState *__restrict__ st,
                                                          const cplx *__restrict__ partA, int nbA,
                                                          const cplx *__restrict__ partU, int nbU,
                                                          int j, int do_sum, int do_coef, int ncA,
                                                          int qa, const cplx *__restrict__ partX, int nbX) {
  reduce_iter_body(st, partA, nbA, partU, nbU, j, do_sum, do_coef, ncA, qa, partX, nbX);
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
    case 7: {  // G2 "sinc": sinc(t*lambda), nlsolvers/device/include/matfunc_complex.hpp:293-300
      const double a = t_re * lam, b = t_im * lam;
      if (hypot(a, b) < 1e-8) return {1.0, 0.0};
      const cplx sv = {sin(a) * cosh(b), cos(a) * sinh(b)};
      const double d = a * a + b * b;
      return {(sv.re * a + sv.im * b) / d, (sv.im * a - sv.re * b) / d};
    }
    default: return {__builtin_nan(""), __builtin_nan("")};
  }
}

__device__ __noinline__ void eigen_phase_jacobi(KState *__restrict__ st, int m, int nf, int f0,
                                                int f1, double t_re, double t_im);

// After the last k_update<m-2>: sums[0..m-1] = g_0..g_{m-2}, nn (tail = 1: no
// last update, s_{m-1} already set by the last k_reduce_iter).  Completes
// T (T(m-1,m-1) = 0, eigen_krylov_complex.hpp:21), diagonalises it with
// parallel cyclic Jacobi on the whole workgroup (eigen_phase_jacobi) and writes
//   fin[f][k] = s_0 * (Q f(Lambda) Q^T e_1)_k / s_k
// so that  f(L) W_0 = sum_k fin[f][k] W_k  (= beta V f(T) e1).
__global__ __launch_bounds__(NTHREADS) void k_reduce_final(KState *__restrict__ st,
                                                           const cplx *__restrict__ partU, int nbU,
                                                           int m, int do_sum, int do_coef, int nf,
                                                           int f0, int f1, double t_re,
                                                           double t_im, int tail) {
  __shared__ cplx ssum[MMAX];
  if (tail) {
    // fused tail: s_{m-1} was set by k_reduce_iter<m-2> (ncA = 3), no sums here
  } else if (do_sum && m >= 2) {
    sum_partials(partU, nbU, m, ssum);
    __syncthreads();
    if (!do_coef) {
      for (int v = threadIdx.x; v < m; v += NTHREADS) st->sums[v] = ssum[v];
      return;
    }
  } else if (m >= 2) {
    for (int v = threadIdx.x; v < m; v += NTHREADS) ssum[v] = st->sums[v];
    __syncthreads();
  }
  if (!do_coef) return;
  if (threadIdx.x == 0 && m >= 2 && !tail) {
    const double s = sqrt(ssum[m - 1].re);
    st->s[m - 1] = s;
    st->To[m - 2] = s;
    if (!(s > 0.0) && st->breakdown == 0) st->breakdown = m;
  }
  if (threadIdx.x == 0) st->Td[m - 1] = 0.0;
  __syncthreads();
  eigen_phase_jacobi(st, m, nf, f0, f1, t_re, t_im);
}

// Cyclic Jacobi (the algorithm of the oracle, oracle/nls_oracle.cpp jacobi_eig:
// same rotation, same stopping rule off(A)^2 <= 1e-34 |A|^2, T pre-scaled to
// max|entry| = 1 like Eigen's solver) with a round-robin (circle method)
// ordering, so that the m/2 rotations of a round are disjoint and applied at
// once.  The matrices are distributed one entry per thread: thread e owns A[i][j]
// and Q[i][j] (e = i*m + j + k*NTHREADS, k < JENT) in registers.  A round is
// two phases: thread i < m computes the rotation (c_i, z_i) acting on index i
// (both members of a pair compute the same c, s: same inputs, same code), then
// every entry is rotated with plain FMAs,
//   A'[i][j] = c_i (c_j A[i][j] + z_j A[i][p_j]) + z_i (c_j A[p_i][j] + z_j A[p_i][p_j])
//   Q'[i][j] = c_j Q[i][j] + z_j Q[i][p_j]
// (p = partner index of the round, z = -s on the lower index of a pair, +s on
// the upper), reading buffer cur and writing buffer cur^1.  Partners come from
// a table built once.  The rotation is the oracle's (tan of the smaller angle,
// t = sgn(theta) / (|theta| + sqrt(theta^2 + 1)), theta = (a_qq - a_pp) / 2a_pq)
// written with one sqrt, one division and one rsqrt (its latency is the round's):
//   t = sgn(theta) |2 a_pq| / (|d| + sqrt(d^2 + 4 a_pq^2)),  d = a_qq - a_pp.
__device__ __forceinline__ void jacobi_rot(const double (*A)[MMAX + 1], int i, int pi, double &c,
                                           double &z) {
  c = 1.0;
  z = 0.0;
  if (pi == i) return;
  const int p = i < pi ? i : pi, q = i < pi ? pi : i;
  const double apq = A[p][q];
  if (apq == 0.0) return;
  const double d = A[q][q] - A[p][p], a2 = 2.0 * apq;
  const double h = sqrt(d * d + a2 * a2);
  double tt;
  if (h > 0.0 && h < 1e300) {
    const bool pos = d == 0.0 || ((d > 0.0) == (apq > 0.0));  // theta >= 0
    tt = (pos ? fabs(a2) : -fabs(a2)) / (fabs(d) + h);
  } else {  // squares under/overflowed: the direct form
    const double theta = d / a2;
    tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
  }
  c = rsqrt(tt * tt + 1.0);
  z = i == p ? -(tt * c) : tt * c;
}

__device__ __noinline__ void eigen_phase_jacobi(KState *__restrict__ st, int m, int nf, int f0,
                                                int f1, double t_re, double t_im) {
  constexpr int JENT = MMAX * MMAX / NTHREADS;
  __shared__ double A[2][MMAX][MMAX + 1];
  __shared__ double Q[2][MMAX][MMAX + 1];
  __shared__ unsigned char part[MMAX - 1][MMAX];
  __shared__ double rc[MMAX], rz[MMAX];
  __shared__ cplx fl[2][MMAX];
  __shared__ double red[2][2][NTHREADS / 64];
  __shared__ double s_scl;
  const int t = threadIdx.x;
#ifdef NLS_EIG_DEBUG
  const long long tc0 = wall_clock64();
  int nsw = 0;
#endif
  const int mp = (m + 1) & ~1;  // even number of round-robin slots (slot m is a dummy if m is odd)
  const int npair = mp / 2;
  if (t < 64) {  // T scaled to max |entry| = 1
    double v = 0.0;
    if (t < m) v = fabs(st->Td[t]);
    if (t < m - 1) v = fmax(v, fabs(st->To[t]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    if (t == 0) s_scl = v > 0.0 ? v : 1.0;
  }
  // partner table (circle method: slot 0 fixed, the others rotate); an index
  // paired with the dummy slot is its own partner (identity rotation)
  for (int e = t; e < (mp - 1) * npair; e += NTHREADS) {
    const int r = e / npair, k = e % npair;
    const int a = k == 0 ? 0 : 1 + (k - 1 + r) % (mp - 1);
    const int b = 1 + (mp - 2 - k + r) % (mp - 1);
    const bool both = a < m && b < m;
    part[r][a] = (unsigned char)(both ? b : a);
    part[r][b] = (unsigned char)(both ? a : b);
  }
  __syncthreads();
  const double iscl = 1.0 / s_scl;
  int ei[JENT], ej[JENT];
  double av[JENT], qv[JENT];
#pragma unroll
  for (int k = 0; k < JENT; ++k) {
    const int e = t + k * NTHREADS;
    ei[k] = -1;
    ej[k] = 0;
    av[k] = qv[k] = 0.0;
    if (e < m * m) {
      const int i = e / m, j = e % m;
      double a = 0.0;
      if (i == j) a = st->Td[i] * iscl;
      else if (i == j + 1) a = st->To[j] * iscl;
      else if (j == i + 1) a = st->To[i] * iscl;
      ei[k] = i;
      ej[k] = j;
      av[k] = a;
      qv[k] = i == j ? 1.0 : 0.0;
      A[0][i][j] = a;
      Q[0][i][j] = qv[k];
    }
  }
  __syncthreads();
#ifdef NLS_EIG_DEBUG
  const long long tc1 = wall_clock64();
#endif
  int cur = 0;
  for (int sweep = 0; sweep < 100; ++sweep) {
#ifdef NLS_EIG_DEBUG
    nsw = sweep;
#endif
    // convergence test on the whole matrix (oracle: off <= 1e-34 tot || off == 0)
    double off = 0.0, tot = 0.0;
#pragma unroll
    for (int k = 0; k < JENT; ++k) {
      const double a2 = av[k] * av[k];
      tot += a2;
      if (ei[k] >= 0 && ei[k] != ej[k]) off += a2;
    }
    off = wave_sum(off);
    tot = wave_sum(tot);
    if ((t & 63) == 0) {
      red[sweep & 1][0][t >> 6] = off;
      red[sweep & 1][1][t >> 6] = tot;
    }
    __syncthreads();
    double so = 0.0, sa = 0.0;
#pragma unroll
    for (int w = 0; w < NTHREADS / 64; ++w) {
      so += red[sweep & 1][0][w];
      sa += red[sweep & 1][1][w];
    }
    if (so <= 1e-34 * sa || so == 0.0) break;  // uniform across the workgroup
    for (int r = 0; r < mp - 1; ++r) {
      const double(*Ac)[MMAX + 1] = A[cur];
      const double(*Qc)[MMAX + 1] = Q[cur];
#if NLS_JAC_ONEPHASE
#pragma unroll
      for (int k = 0; k < JENT; ++k) {
        if (ei[k] < 0) continue;
        const int i = ei[k], j = ej[k];
        const int pi = part[r][i], pj = part[r][j];
        double ci, zi, cj, zj;
        jacobi_rot(Ac, i, pi, ci, zi);
        jacobi_rot(Ac, j, pj, cj, zj);
#else
      if (t < m) {
        double c, z;
        jacobi_rot(Ac, t, part[r][t], c, z);
        rc[t] = c;
        rz[t] = z;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < JENT; ++k) {
        if (ei[k] < 0) continue;
        const int i = ei[k], j = ej[k];
        const int pi = part[r][i], pj = part[r][j];
        const double ci = rc[i], zi = rz[i], cj = rc[j], zj = rz[j];
#endif
        double na = ci * (cj * av[k] + zj * Ac[i][pj]) + zi * (cj * Ac[pi][j] + zj * Ac[pi][pj]);
        if (pi == j && pi != i) na = 0.0;  // the annihilated pivot (else off(A) stalls on rounding)
        const double nq = cj * qv[k] + zj * Qc[i][pj];
        av[k] = na;
        qv[k] = nq;
        A[cur ^ 1][i][j] = na;
        Q[cur ^ 1][i][j] = nq;
      }
      __syncthreads();
      cur ^= 1;
    }
  }
#ifdef NLS_EIG_DEBUG
  const long long tc2 = wall_clock64();
#endif
  // fin[f][r] = s0 / s_r * sum_k Q[r][k] Q[0][k] f(lambda_k); f(lambda_k) once per k
  if (t < m) {
    const double lam = A[cur][t][t] * s_scl;
    st->lam[t] = lam;
    for (int fi = 0; fi < nf; ++fi) fl[fi][t] = eval_f(fi == 0 ? f0 : f1, lam, t_re, t_im);
  }
  __syncthreads();
  if (t < m) {
    const double s0 = st->s[0];
    const double isr = inv_or_zero(st->s[t]);
    for (int fi = 0; fi < nf; ++fi) {
      cplx c = {0.0, 0.0};
      for (int k = 0; k < m; ++k) c += (Q[cur][t][k] * Q[cur][0][k]) * fl[fi][k];
      st->fin[fi][t] = (s0 * isr) * c;
    }
  }
#ifdef NLS_EIG_DEBUG
  __syncthreads();
  if (t == 0)
    printf("[jacobi] m=%d sweeps=%d init %.1f us, sweeps %.1f us, fin %.1f us\n", m, nsw,
           (tc1 - tc0) * 0.01, (tc2 - tc1) * 0.01, (wall_clock64() - tc2) * 0.01);
#endif
}

// ---------------------------------------------------------------------------
// pointwise kernels

__global__ __launch_bounds__(NTHREADS) void k_nl_init(const cplx *__restrict__ u, cplx *__restrict__ w0,
                                                      const double *__restrict__ mf, int64_t n,
                                                      double dt, int nonlin, cplx s1, cplx s2) {
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS)
    w0[p] = nl_half(u[p], nonlin >= 2 ? mf[p] : 0.0, dt, nonlin, s1, s2);
}

// u = N(sum_k fin_k W_k) ; W_0 <- N(u) for the next step (fused start of step)
template <int M>
__global__ __launch_bounds__(NTHREADS) void k_final_nlse(cplx *__restrict__ W, int64_t vs, int64_t n,
                                                         const KState *__restrict__ st,
                                                         cplx *__restrict__ u,
                                                         const double *__restrict__ mf, double dt,
                                                         int nonlin, cplx s1, cplx s2) {
  // two cells per thread, all 2M basis loads issued before the first use;
  // combination coefficients broadcast from LDS
  constexpr int U = 2;
  __shared__ cplx cf[MMAX];
  for (int k = threadIdx.x; k < M; k += NTHREADS) cf[k] = st->fin[0][k];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * NTHREADS * U;
  for (int64_t base = (int64_t)blockIdx.x * NTHREADS * U + threadIdx.x; base < n; base += stride) {
    cplx w[U][M];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int64_t p = base + q * NTHREADS;
      const cplx *__restrict__ src = W + p;
#pragma unroll
      for (int k = 0; k < M; ++k) {
        w[q][k] = p < n ? ld_nt(src) : cplx{0.0, 0.0};
        src += vs;
      }
    }
    asm volatile("" ::: "memory");  // keep the coefficient reads in LDS
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int64_t p = base + q * NTHREADS;
      if (p >= n) continue;
      cplx y = {0.0, 0.0};
#pragma unroll
      for (int k = 0; k < M; ++k) y += cmul(cf[k], w[q][k]);
      const double mv = nonlin >= 2 ? mf[p] : 0.0;
      // the fused tail's N(1/2) . N(1/2) pair (nl_half2: the second phase by the
      // double-angle identity), so that the fused and unfused steps round alike
      cplx un, w0;
      nl_half2(y, mv, dt, nonlin, s1, s2, un, w0);
      st_nt(u + p, un);
      st_nt(W + p, w0);
    }
  }
}

// Neumann "copy" boundary condition of the G2 drivers (boundaries.cuh:10-19
// for 2D, :24-81 for 3D).  The reference's sequence of strided copies
// (faces of the slowest axis from their inner neighbour plane, then the next
// axis over the full extent of the previous, ...) leaves every boundary cell
// equal to the cell with all coordinates clamped into [1, n-2]; interior
// cells are never written, so the gather is race-free in place.  Only the
// boundary shell is visited: the perimeter of every local plane plus the full
// global first/last plane.  When the start vector of the next step is live
// (w0_ready), its boundary cells are refreshed with N(u) at the same time.
__host__ __device__ inline int64_t bc_perimeter(const Geo &g) {
  return g.nyp == 1 ? 2 : 2 * g.nx + 2 * (g.nyp - 2);
}
__host__ __device__ inline int64_t bc_cells(const Geo &g) {
  const int64_t full = (g.z0 == 0 ? 1 : 0) + (g.z0 + g.nzl == g.npl ? 1 : 0);
  return g.nzl * bc_perimeter(g) + full * g.P;
}
int64_t neumann_bc_cells(const Geo &g) { return bc_cells(g); }

__global__ __launch_bounds__(NTHREADS) void k_neumann_bc(cplx *__restrict__ u, cplx *__restrict__ w0,
                                                         const double *__restrict__ mf, Geo g,
                                                         int w0_ready, double dt, int nonlin,
                                                         cplx s1, cplx s2) {
  const int64_t per = bc_perimeter(g);
  const int64_t nper = g.nzl * per;
  const int64_t total = bc_cells(g);
  const int64_t nx = g.nx, nyp = g.nyp;
  for (int64_t t = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * NTHREADS) {
    int64_t q, x, y;
    if (t < nper) {  // perimeter of local plane q
      q = t / per;
      const int64_t k = t % per;
      if (nyp == 1) {
        x = k == 0 ? 0 : nx - 1;
        y = 0;
      } else if (k < nx) {
        x = k; y = 0;
      } else if (k < 2 * nx) {
        x = k - nx; y = nyp - 1;
      } else if (k < 2 * nx + nyp - 2) {
        x = 0; y = 1 + (k - 2 * nx);
      } else {
        x = nx - 1; y = 1 + (k - 2 * nx - (nyp - 2));
      }
    } else {  // full global boundary plane(s) owned by this slab
      const int64_t k = t - nper;
      const int64_t which = k / g.P, c = k % g.P;
      const bool has_first = g.z0 == 0;
      q = (which == 0 && has_first) ? 0 : g.nzl - 1;
      x = c % nx;
      y = c / nx;
    }
    const int64_t gq = g.z0 + q;
    const int64_t xs = x < 1 ? 1 : (x > nx - 2 ? nx - 2 : x);
    const int64_t ys = nyp == 1 ? 0 : (y < 1 ? 1 : (y > nyp - 2 ? nyp - 2 : y));
    const int64_t gs = gq < 1 ? 1 : (gq > g.npl - 2 ? g.npl - 2 : gq);
    const int64_t src = (gs - g.z0) * g.P + ys * nx + xs;
    const int64_t dst = q * g.P + y * nx + x;
    if (src == dst) continue;
    const cplx v = u[src];
    u[dst] = v;
    if (w0_ready) w0[dst] = nl_half(v, nonlin >= 2 ? mf[dst] : 0.0, dt, nonlin, s1, s2);
  }
}

// ---- G2 sEWI (nlsolvers/device/include/nlse_dev.hpp:205-238) ----------------
// start vector B(u) = -m |u|^2 u  (compute_B, nlse_dev.hpp:42-50)
__global__ __launch_bounds__(NTHREADS) void k_sewi_b(const cplx *__restrict__ u, const double *__restrict__ mf,
                                                     cplx *__restrict__ w0, int64_t n) {
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    const cplx v = u[p];
    const double s = -mf[p] * (v.re * v.re + v.im * v.im);
    w0[p] = s * v;
  }
}

// W_0 <- sum_k fin_k W_k in place: the result of one action becomes the start
// vector of the next (each thread reads all M values of its cell first)
template <int M>
__global__ __launch_bounds__(NTHREADS) void k_combine_w0(cplx *W, int64_t vs, int64_t n,
                                                         const KState *__restrict__ st) {
  __shared__ cplx cf[MMAX];
  for (int k = threadIdx.x; k < M; k += NTHREADS) cf[k] = st->fin[0][k];
  __syncthreads();
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    cplx w[M];
#pragma unroll
    for (int k = 0; k < M; ++k) w[k] = ld_nt(W + (int64_t)k * vs + p);
    cplx y = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < M; ++k) y += cmul(cf[k], w[k]);
    W[p] = y;
  }
}

// apply_sewi (nlse_dev.hpp:52-63):  u_new = exp(2 tau L) u_prev - 2 tau e,
// e = exp(tau L) sinc(dt L) B(u) (in `e`); u_prev <- old u.  tau = 1j*dt.
template <int M>
__global__ __launch_bounds__(NTHREADS) void k_sewi_end(const cplx *__restrict__ W, int64_t vs, int64_t n,
                                                       const KState *__restrict__ st,
                                                       cplx *__restrict__ u, cplx *__restrict__ up,
                                                       const cplx *__restrict__ e, double dt) {
  __shared__ cplx cf[MMAX];
  for (int k = threadIdx.x; k < M; k += NTHREADS) cf[k] = st->fin[0][k];
  __syncthreads();
  const cplx two_tau = {0.0, 2.0 * dt};
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    cplx y = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < M; ++k) y += cmul(cf[k], ld_nt(W + (int64_t)k * vs + p));
    const cplx uo = u[p];
    u[p] = y - cmul(two_tau, e[p]);
    up[p] = uo;
  }
}

// ---- G2 Klein-Gordon Gautschi (nlsolvers/device/include/kg_single.cuh:49-86) ----
// start vector of the sinc^2 basis: g = -m u^3  (u = slot 0 of the cos basis)
__global__ __launch_bounds__(NTHREADS) void k_kg_g(const double *__restrict__ u, const double *__restrict__ mf,
                                                   double *__restrict__ g0, int64_t n) {
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    const double x = u[p];
    g0[p] = -mf[p] * x * x * x;
  }
}

// u_new = (2 cos(t sqrt|L|) u - u_past) + (dt*dt) sinc^2(t sqrt|L|) g ;
// u_past <- u ; v = (u_new - u_past) / dt.  u is slot 0 of W (read, then overwritten
// by the same thread).
template <int M>
__global__ __launch_bounds__(NTHREADS) void k_kg_end(double *W, const double *__restrict__ W2, int64_t vs,
                                                     int64_t n, const KState *__restrict__ st,
                                                     const KState *__restrict__ st2,
                                                     double *__restrict__ up, double *__restrict__ v,
                                                     double dt) {
  __shared__ double cc[MMAX], cs[MMAX];
  for (int k = threadIdx.x; k < M; k += NTHREADS) {
    cc[k] = st->fin[0][k].re;
    cs[k] = st2->fin[0][k].re;
  }
  __syncthreads();
  const double tt = dt * dt;
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS) {
    double yc = 0.0, ys = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) {
      yc += cc[k] * ld_nt(W + (int64_t)k * vs + p);
      ys += cs[k] * ld_nt(W2 + (int64_t)k * vs + p);
    }
    const double uo = W[p];
    const double un = (yc * 2.0 - up[p]) + ys * tt;
    W[p] = un;
    up[p] = uo;
    v[p] = (un - uo) / dt;
  }
}

// Neumann copy BC on a real field (u of a Klein-Gordon handle), same clamp gather
__global__ __launch_bounds__(NTHREADS) void k_neumann_bc_r(double *__restrict__ u, Geo g) {
  const int64_t per = bc_perimeter(g);
  const int64_t nper = g.nzl * per;
  const int64_t total = bc_cells(g);
  const int64_t nx = g.nx, nyp = g.nyp;
  for (int64_t t = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * NTHREADS) {
    int64_t q, x, y;
    if (t < nper) {
      q = t / per;
      const int64_t k = t % per;
      if (nyp == 1) {
        x = k == 0 ? 0 : nx - 1;
        y = 0;
      } else if (k < nx) {
        x = k; y = 0;
      } else if (k < 2 * nx) {
        x = k - nx; y = nyp - 1;
      } else if (k < 2 * nx + nyp - 2) {
        x = 0; y = 1 + (k - 2 * nx);
      } else {
        x = nx - 1; y = 1 + (k - 2 * nx - (nyp - 2));
      }
    } else {
      const int64_t k = t - nper;
      const int64_t which = k / g.P, c = k % g.P;
      q = (which == 0 && g.z0 == 0) ? 0 : g.nzl - 1;
      x = c % nx;
      y = c / nx;
    }
    const int64_t gq = g.z0 + q;
    const int64_t xs = x < 1 ? 1 : (x > nx - 2 ? nx - 2 : x);
    const int64_t ys = nyp == 1 ? 0 : (y < 1 ? 1 : (y > nyp - 2 ? nyp - 2 : y));
    const int64_t gs = gq < 1 ? 1 : (gq > g.npl - 2 ? g.npl - 2 : gq);
    const int64_t src = (gs - g.z0) * g.P + ys * nx + xs;
    const int64_t dst = q * g.P + y * nx + x;
    if (src != dst) u[dst] = u[src];
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
                                                     double *__restrict__ g0, int gfun) {
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
      const double w = ld_nt(W + (int64_t)k * vs + p);
      yi += ci[k] * w;
      yc += cc[k] * w;
    }
    // G1 (gfun < 0): m (-sin y) (sg_solver.hpp:65-69); G2 family: -m F(y) (gg_force)
    st_nt(g0 + p, gfun < 0 ? mf[p] * (-sin(yi)) : -mf[p] * gg_force(yi, gfun));
    st_nt(up + p, 2 * yc - up[p]);
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
    for (int k = 0; k < M; ++k) ys += c[k] * ld_nt(W2 + (int64_t)k * vs + p);
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

namespace {
using Table = const void *(*)(int, bool, int);
Table table(int dim, bool ani) {
  return ani ? (dim == 3 ? &stencil_table_ani3 : &stencil_table_ani2)
             : (dim == 3 ? &stencil_table_iso3 : &stencil_table_iso2);
}
}  // namespace

const void *kernel_update(bool cplx_, int dim, int J, bool ani, bool qa) {
  return table(dim, ani)(NLS_KIND_UPDATE, cplx_, (qa ? 64 : 0) + J);
}
const void *kernel_alpha(bool cplx_, int dim, bool ani) { return table(dim, ani)(NLS_KIND_ALPHA, cplx_, 0); }
const void *kernel_lap(bool cplx_, int dim, bool ani) { return table(dim, ani)(NLS_KIND_LAP, cplx_, 0); }
const void *kernel_xpairs(bool cplx_, int dim, bool ani) { return table(dim, ani)(NLS_KIND_XPAIRS, cplx_, 0); }
int64_t xtiles(const Geo &g, int dim, int rb) { return dim == 3 ? cdiv(g.nx, 64) : cdiv(g.nx, 64 * (int64_t)rb); }
const void *kernel_reduce_qa(bool cplx_, int dim, bool ani) {
  return table(dim, ani)(NLS_KIND_REDUCE_QA, cplx_, 0);
}
const void *kernel_alpha_l2(bool cplx_, int dim, bool ani, bool pipe) {
  return table(dim, ani)(NLS_KIND_ALPHA_L2, cplx_, pipe ? 1 : 0);
}
const void *kernel_tail(bool cplx_, int dim, int mode, int M, bool ani) {
  return table(dim, ani)(NLS_KIND_FINAL, cplx_, mode * 64 + M);
}

// local-transport all-reduce: dst[v] = sum_r pub[r][parity][v] in rank order
__global__ __launch_bounds__(NTHREADS) void k_sum_ranks(cplx *__restrict__ dst, const cplx *__restrict__ pub,
                                                        int nranks, int parity, int n, int stride) {
  for (int v = threadIdx.x; v < n; v += NTHREADS) {
    cplx s = {0.0, 0.0};
    for (int r = 0; r < nranks; ++r) s += pub[((int64_t)r * 2 + parity) * stride + v];
    dst[v] = s;
  }
}
const void *kernel_sum_ranks() { return reinterpret_cast<const void *>(&k_sum_ranks); }

const void *kernel_reduce_iter() { return reinterpret_cast<const void *>(&k_reduce_iter); }
const void *kernel_reduce_final() { return reinterpret_cast<const void *>(&k_reduce_final); }
const void *kernel_nl_init() { return reinterpret_cast<const void *>(&k_nl_init); }
const void *kernel_sg_velocity() { return reinterpret_cast<const void *>(&k_sg_velocity); }
const void *kernel_neumann_bc() { return reinterpret_cast<const void *>(&k_neumann_bc); }
const void *kernel_sewi_b() { return reinterpret_cast<const void *>(&k_sewi_b); }
const void *kernel_kg_g() { return reinterpret_cast<const void *>(&k_kg_g); }
const void *kernel_neumann_bc_r() { return reinterpret_cast<const void *>(&k_neumann_bc_r); }

const void *kernel_kg_end(int M) {
  switch (M) {
#define X(M) case M: return reinterpret_cast<const void *>(&k_kg_end<M>);
    NLS_M_LIST(X)
#undef X
    default: return nullptr;
  }
}

const void *kernel_combine_w0(int M) {
  switch (M) {
#define X(M) case M: return reinterpret_cast<const void *>(&k_combine_w0<M>);
    NLS_M_LIST(X)
#undef X
    default: return nullptr;
  }
}

const void *kernel_sewi_end(int M) {
  switch (M) {
#define X(M) case M: return reinterpret_cast<const void *>(&k_sewi_end<M>);
    NLS_M_LIST(X)
#undef X
    default: return nullptr;
  }
}

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

// two-vectors-per-pass Lanczos (nls_pass2.hpp, nls_pass2d.hpp): the LDS-DMA pass
// k_p2d at even J <= P2D_JMAX; d2: a 2D grid as planes of 4 rows; pr: a real 2D
// field as pairs of cells
bool pass2_jreg(int J, int akind) { return p2d_jreg(J, akind); }
const void *kernel_pass2(int J, bool hz, bool d2, bool pr, bool peer) {
  if (peer) return (d2 || pr) ? nullptr : kernel_pass2_peer(J, hz);
  switch (J) {
#define X(J)                                                                                       \
  case J:                                                                                          \
    if (pr)                                                                                        \
      return hz ? reinterpret_cast<const void *>(&k_p2d<J, true, true, true>)                      \
                : reinterpret_cast<const void *>(&k_p2d<J, false, true, true>);                    \
    return d2 ? (hz ? reinterpret_cast<const void *>(&k_p2d<J, true, true>)                        \
                    : reinterpret_cast<const void *>(&k_p2d<J, false, true>))                      \
              : (hz ? reinterpret_cast<const void *>(&k_p2d<J, true>) : reinterpret_cast<const void *>(&k_p2d<J, false>));
    X(0) X(2) X(4) X(6) X(8) X(10) X(12) X(14)
#undef X
    default: return nullptr;
  }
}
static_assert(offsetof(P2State, bZ2) == offsetof(P2State, bZ1) + sizeof(cplx) &&
                  offsetof(P2State, bY2) == offsetof(P2State, bY1) + sizeof(cplx) &&
                  offsetof(P2State, bY3) == offsetof(P2State, bY2) + sizeof(cplx),
              "k_p2coef writes the b coefficients of a vector as an array");
const void *kernel_p2tail() { return reinterpret_cast<const void *>(&k_p2tail); }
const void *kernel_p2tfin() { return reinterpret_cast<const void *>(&k_p2tfin); }
const void *kernel_p2coef() { return reinterpret_cast<const void *>(&k_p2coef); }

// A pass's column sums and its k_p2coef in one launch (single-rank handles; the collective
// path all-reduces between the two): workgroup v sums column v as k_colsum does, and the
// workgroup that finishes last -- the counter's acquire-release at agent scope publishes
// every other workgroup's column to it -- runs the coefficient step.  The column sums are
// the same bits as k_colsum's (same per-column order); only a launch and a kernel
// boundary per pass go.  cnt: a zeroed device word, reset by the last workgroup.
__global__ __launch_bounds__(NTHREADS) void k_colsum_p2coef(const cplx *__restrict__ partU, int nbU,
                                                            cplx *__restrict__ dst, int32_t *__restrict__ cnt,
                                                            P2State *__restrict__ ps, KState *__restrict__ st,
                                                            int J, int mode, int ns, int nsn, int real) {
  colsum_body(nullptr, 0, 0, partU, nbU, dst, blockIdx.x);
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    // thread 0 wrote dst[v]: its release orders that store before the count
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (int)gridDim.x - 1;
    if (s_last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;  // uniform
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every thread: no stale line of the sums
  p2coef_body(ps, st, J, mode, ns, nsn, real);
}
const void *kernel_colsum_p2coef() { return reinterpret_cast<const void *>(&k_colsum_p2coef); }

// The end of a fused-tail basis in one launch (single-rank handles): k_alpha_l2's three
// column sums (one workgroup each), then on the last workgroup k_p2tail, the eigensolve
// (k_reduce_final with tail = 1) and k_p2tfin -- four launches and three kernel
// boundaries fewer per basis, the same bits (k_colsum_p2coef's counter protocol).
__global__ __launch_bounds__(NTHREADS) void k_tail_chain(const cplx *__restrict__ partA, int nbA,
                                                         cplx *__restrict__ dst, int32_t *__restrict__ cnt,
                                                         P2State *__restrict__ ps, KState *__restrict__ st, int m,
                                                         int nf, int f0, int f1, double t_re, double t_im) {
  colsum_body(partA, nbA, 3, nullptr, 0, dst, blockIdx.x);
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (int)gridDim.x - 1;
    if (s_last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;  // uniform
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  p2tail_body(ps, st, dst, m);
  __syncthreads();
  if (threadIdx.x == 0) st->Td[m - 1] = 0.0;  // k_reduce_final, tail = 1
  __syncthreads();
  eigen_phase_jacobi(st, m, nf, f0, f1, t_re, t_im);
  __syncthreads();
  p2tfin_body(ps, st, m, nf);
}
const void *kernel_tail_chain() { return reinterpret_cast<const void *>(&k_tail_chain); }
size_t p2state_bytes() { return sizeof(P2State); }
size_t p2state_sums_offset() { return offsetof(P2State, sums); }
size_t p2state_peer_offset() { return offsetof(P2State, pdn); }
int p2state_peer_slots() { return P2M + 1; }

}  // namespace nls
