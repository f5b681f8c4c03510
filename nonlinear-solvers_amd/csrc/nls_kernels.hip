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

// ---------------------------------------------------------------------------
// single-workgroup reductions + coefficient math + m x m eigensolve

// The same column sums for large partial arrays (one tile per workgroup
// grids): one workgroup per column, fixed order -> st->sums layout
// [partA columns 0..ncA) then [partU columns 0..ncU).
__global__ __launch_bounds__(NTHREADS) void k_colsum(const cplx *__restrict__ partA, int nbA, int ncA,
                                                     const cplx *__restrict__ partU, int nbU,
                                                     cplx *__restrict__ dst) {
  const int v = blockIdx.x;
  const cplx *__restrict__ col = v < ncA ? partA + (int64_t)v * nbA : partU + (int64_t)(v - ncA) * nbU;
  const int nb = v < ncA ? nbA : nbU;
  double a0 = 0.0, b0 = 0.0, a1 = 0.0, b1 = 0.0;
  int q = threadIdx.x;
  for (; q + NTHREADS < nb; q += 2 * NTHREADS) {
    const cplx x0 = col[q], x1 = col[q + NTHREADS];
    a0 += x0.re; b0 += x0.im;
    a1 += x1.re; b1 += x1.im;
  }
  if (q < nb) { const cplx x0 = col[q]; a0 += x0.re; b0 += x0.im; }
  const double a = wave_sum(a0 + a1), b = wave_sum(b0 + b1);
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

__device__ __noinline__ void eigen_phase(KState *__restrict__ st, int m, int nf, int f0, int f1,
                                         double t_re, double t_im);
#ifndef NLS_EIGEN_JACOBI
#define NLS_EIGEN_JACOBI 1
#endif
__device__ __noinline__ void eigen_phase_jacobi(KState *__restrict__ st, int m, int nf, int f0,
                                                int f1, double t_re, double t_im);

// After the last k_update<m-2>: sums[0..m-1] = g_0..g_{m-2}, nn (tail = 1: no
// last update, s_{m-1} already set by the last k_reduce_iter).  Completes
// T (T(m-1,m-1) = 0, eigen_krylov_complex.hpp:21), diagonalises it with
// implicit-shift QL on wave 0 (lane r owns row r of Q) and writes
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
#if NLS_EIGEN_JACOBI
  eigen_phase_jacobi(st, m, nf, f0, f1, t_re, t_im);
#else
  if (threadIdx.x < 64) eigen_phase(st, m, nf, f0, f1, t_re, t_im);
#endif
}

// Parallel cyclic Jacobi on the whole workgroup (the algorithm of the oracle,
// oracle/nls_oracle.cpp jacobi_eig, with a round-robin ordering so that the
// m/2 rotations of a round are disjoint and applied at once).  Per round: one
// thread per pair computes (c, s); then all threads rotate the column pairs of
// A and Q, then the row pairs of A.  Sweeps until off(A)^2 <= 1e-34 |A|^2.
__device__ __noinline__ void eigen_phase_jacobi(KState *__restrict__ st, int m, int nf, int f0,
                                                int f1, double t_re, double t_im) {
  __shared__ double A[MMAX][MMAX + 1];
  __shared__ double Q[MMAX][MMAX + 1];
  __shared__ double rc[MMAX / 2], rs[MMAX / 2];
  __shared__ int rp[MMAX / 2], rq[MMAX / 2];
  __shared__ double red[2][NTHREADS / 64];
  __shared__ double s_scl;
  const int t = threadIdx.x;
  const int mp = (m + 1) & ~1;  // even number of round-robin slots (slot m is a dummy if m is odd)
  const int npair = mp / 2;
  // T scaled to max |entry| = 1 (as the QL path and Eigen's solver)
  if (t < 64) {
    double v = 0.0;
    if (t < m) v = fabs(st->Td[t]);
    if (t < m - 1) v = fmax(v, fabs(st->To[t]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    if (t == 0) s_scl = v > 0.0 ? v : 1.0;
  }
  __syncthreads();
  const double iscl = 1.0 / s_scl;
  for (int e = t; e < m * m; e += NTHREADS) {
    const int i = e / m, j = e % m;
    double a = 0.0;
    if (i == j) a = st->Td[i] * iscl;
    else if (i == j + 1) a = st->To[j] * iscl;
    else if (j == i + 1) a = st->To[i] * iscl;
    A[i][j] = a;
    Q[i][j] = i == j ? 1.0 : 0.0;
  }
  __syncthreads();
  int sweep = 0;
  for (; sweep < 100; ++sweep) {
    // convergence test on the whole matrix (oracle: off <= 1e-34 tot || off == 0)
    double off = 0.0, tot = 0.0;
    for (int e = t; e < m * m; e += NTHREADS) {
      const int i = e / m, j = e % m;
      const double a2 = A[i][j] * A[i][j];
      tot += a2;
      if (i != j) off += a2;
    }
    off = wave_sum(off);
    tot = wave_sum(tot);
    if ((t & 63) == 0) {
      red[0][t >> 6] = off;
      red[1][t >> 6] = tot;
    }
    __syncthreads();
    double so = 0.0, sa = 0.0;
#pragma unroll
    for (int w = 0; w < NTHREADS / 64; ++w) {
      so += red[0][w];
      sa += red[1][w];
    }
    __syncthreads();
    if (so <= 1e-34 * sa || so == 0.0) break;  // uniform across the workgroup
    for (int r = 0; r < mp - 1; ++r) {
      if (t < npair) {  // circle method: slot 0 fixed, the others rotate
        const int a = t == 0 ? 0 : 1 + (t - 1 + r) % (mp - 1);
        const int b = 1 + (mp - 2 - t + r) % (mp - 1);
        const int p = a < b ? a : b, q = a < b ? b : a;
        double c = 1.0, sn = 0.0;
        if (q < m) {
          const double apq = A[p][q];
          if (apq != 0.0) {
            const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
            const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            c = 1.0 / sqrt(tt * tt + 1.0);
            sn = tt * c;
          }
        }
        rp[t] = p;
        rq[t] = q < m ? q : p;  // dummy pair: identity rotation on p
        rc[t] = c;
        rs[t] = q < m ? sn : 0.0;
      }
      __syncthreads();
      // A <- J^T A J and Q <- Q J in one phase: the pairs are disjoint, so each
      // 2x2 block A[{pa,qa}][{pb,qb}] (and each Q row segment) has one owner.
      // The annihilated entry of a diagonal block is set to exactly zero (else
      // rounding keeps off(A) above the stopping threshold for ever).
      for (int e = t; e < npair * npair + m * npair; e += NTHREADS) {
        if (e < npair * npair) {
          const int a = e / npair, b = e % npair;
          const int pa = rp[a], qa = rq[a], pb = rp[b], qb = rq[b];
          const double ca = rc[a], sa = rs[a], cb = rc[b], sb = rs[b];
          const bool va = pa != qa, vb = pb != qb;
          const double b00 = A[pa][pb], b01 = vb ? A[pa][qb] : 0.0;
          const double b10 = va ? A[qa][pb] : 0.0, b11 = (va && vb) ? A[qa][qb] : 0.0;
          // rows: [[ca, -sa], [sa, ca]] * B
          const double r00 = ca * b00 - sa * b10, r01 = ca * b01 - sa * b11;
          const double r10 = sa * b00 + ca * b10, r11 = sa * b01 + ca * b11;
          // columns: * [[cb, sb], [-sb, cb]]
          double n00 = r00 * cb - r01 * sb, n01 = r00 * sb + r01 * cb;
          double n10 = r10 * cb - r11 * sb, n11 = r10 * sb + r11 * cb;
          if (a == b && va) n01 = n10 = 0.0;
          A[pa][pb] = n00;
          if (vb) A[pa][qb] = n01;
          if (va) A[qa][pb] = n10;
          if (va && vb) A[qa][qb] = n11;
        } else {
          const int e2 = e - npair * npair;
          const int k = e2 / npair, b = e2 % npair;
          const int p = rp[b], q = rq[b];
          if (p == q) continue;
          const double c = rc[b], sn = rs[b];
          const double qkp = Q[k][p], qkq = Q[k][q];
          Q[k][p] = c * qkp - sn * qkq;
          Q[k][q] = sn * qkp + c * qkq;
        }
      }
      __syncthreads();
    }
  }
#ifdef NLS_EIG_DEBUG
  if (t == 0) printf("[jacobi] m=%d sweeps=%d\n", m, sweep);
#endif
  // fin[f][r] = s0 / s_r * sum_k Q[r][k] Q[0][k] f(lambda_k)
  if (t < m) {
    st->lam[t] = A[t][t] * s_scl;
    const double s0 = st->s[0];
    const double isr = inv_or_zero(st->s[t]);
    for (int fi = 0; fi < nf; ++fi) {
      const int func = fi == 0 ? f0 : f1;
      cplx c = {0.0, 0.0};
      for (int k = 0; k < m; ++k) c += (Q[t][k] * Q[0][k]) * eval_f(func, A[k][k] * s_scl, t_re, t_im);
      st->fin[fi][t] = (s0 * isr) * c;
    }
  }
}

// Wave-0 part of k_reduce_final.  Lane k holds d[k] and e[k] in registers; the
// implicit-shift QL recurrence (uniform across lanes) reads them with
// v_readlane and writes them back with a lane-select, so its dependency chain
// never waits on LDS.  Lane r applies every Givens rotation to row r of Q (LDS).
__device__ __forceinline__ double rdlane(double v, int i) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), i);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), i);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __noinline__ void eigen_phase(KState *__restrict__ st, int m, int nf, int f0, int f1,
                                         double t_re, double t_im) {
  __shared__ double Q[MMAX][MMAX + 1];
  const int lane = threadIdx.x;
  // scale T to max|entry| = 1 (as Eigen's SelfAdjointEigenSolver does)
  double dl = lane < m ? st->Td[lane] : 0.0;
  double el = lane < m - 1 ? st->To[lane] : 0.0;
  double scl = fmax(fabs(dl), fabs(el));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) scl = fmax(scl, __shfl_xor(scl, off, 64));
  const double iscl = scl > 0.0 ? 1.0 / scl : 1.0;
  if (scl == 0.0) scl = 1.0;
  dl *= iscl;
  el *= iscl;
  if (lane < m)
    for (int c = 0; c < m; ++c) Q[lane][c] = lane == c ? 1.0 : 0.0;
  auto setd = [&](int i, double v) { if (lane == i) dl = v; };
  auto sete = [&](int i, double v) { if (lane == i) el = v; };
#ifdef NLS_EIG_DEBUG
  int tot_iter = 0, tot_rot = 0;
#endif
  for (int l = 0; l < m; ++l) {
    int iter = 0;
    for (;;) {
      int mm;
      for (mm = l; mm < m - 1; ++mm) {
        const double dd = fabs(rdlane(dl, mm)) + fabs(rdlane(dl, mm + 1));
        if (fabs(rdlane(el, mm)) <= 2.220446049250313e-16 * dd) break;
      }
      if (mm == l) break;
      if (++iter > 64) break;
#ifdef NLS_EIG_DEBUG
      ++tot_iter;
      tot_rot += mm - l;
#endif
      const double dlv = rdlane(dl, l), el_l = rdlane(el, l);
      double gg = (rdlane(dl, l + 1) - dlv) / (2.0 * el_l);
      double rr = hypot(gg, 1.0);
      gg = rdlane(dl, mm) - dlv + el_l / (gg + (gg >= 0.0 ? fabs(rr) : -fabs(rr)));
      double ss = 1.0, cc = 1.0, pp = 0.0;
      bool early = false;
      for (int i = mm - 1; i >= l; --i) {
        const double ei = rdlane(el, i);
        const double ff = ss * ei, bb = cc * ei;
        rr = sqrt(ff * ff + gg * gg);
        sete(i + 1, rr);
        if (rr == 0.0) {
          setd(i + 1, rdlane(dl, i + 1) - pp);
          sete(mm, 0.0);
          early = true;
          break;
        }
        const double irr = 1.0 / rr;
        ss = ff * irr;
        cc = gg * irr;
        gg = rdlane(dl, i + 1) - pp;
        rr = (rdlane(dl, i) - gg) * ss + 2.0 * cc * bb;
        pp = ss * rr;
        setd(i + 1, gg + pp);
        gg = cc * rr - bb;
        if (lane < m) {
          const double fq = Q[lane][i + 1];
          Q[lane][i + 1] = ss * Q[lane][i] + cc * fq;
          Q[lane][i] = cc * Q[lane][i] - ss * fq;
        }
      }
      if (early) continue;
      setd(l, rdlane(dl, l) - pp);
      sete(l, gg);
      sete(mm, 0.0);
    }
  }
#ifdef NLS_EIG_DEBUG
  if (lane == 0) printf("[ql] m=%d iters=%d rotations=%d\n", m, tot_iter, tot_rot);
#endif
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  const double lam_l = dl * scl;
  if (lane < m) {
    st->lam[lane] = lam_l;
    const double s0 = st->s[0];
    const double isr = inv_or_zero(st->s[lane]);
    for (int fi = 0; fi < nf; ++fi) {
      const int func = fi == 0 ? f0 : f1;
      cplx c = {0.0, 0.0};
      for (int k = 0; k < m; ++k) c += (Q[lane][k] * Q[0][k]) * eval_f(func, rdlane(lam_l, k), t_re, t_im);
      st->fin[fi][lane] = (s0 * isr) * c;
    }
  }
}

// ---------------------------------------------------------------------------
// pointwise kernels

__global__ __launch_bounds__(NTHREADS) void k_nl_init(const cplx *__restrict__ u, cplx *__restrict__ w0,
                                                      const double *__restrict__ mf, int64_t n,
                                                      double dt, int nonlin, cplx s1, cplx s2) {
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS)
    w0[p] = nl_half(u[p], nonlin == 2 ? mf[p] : 0.0, dt, nonlin, s1, s2);
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
      const double mv = nonlin == 2 ? mf[p] : 0.0;
      const cplx un = nl_half(y, mv, dt, nonlin, s1, s2);
      st_nt(u + p, un);
      st_nt(W + p, nl_half(un, mv, dt, nonlin, s1, s2));
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
    if (w0_ready) w0[dst] = nl_half(v, nonlin == 2 ? mf[dst] : 0.0, dt, nonlin, s1, s2);
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
      const double w = ld_nt(W + (int64_t)k * vs + p);
      yi += ci[k] * w;
      yc += cc[k] * w;
    }
    st_nt(g0 + p, mf[p] * (-sin(yi)));
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
const void *kernel_alpha_l2(bool cplx_, int dim, bool ani) {
  return table(dim, ani)(NLS_KIND_ALPHA_L2, cplx_, 0);
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

}  // namespace nls

