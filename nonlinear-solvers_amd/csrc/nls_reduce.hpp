// nls_reduce.hpp -- the single-workgroup reduction that follows every alpha
// pass: fixed-order column sums of the per-workgroup partials and the CGS
// coefficients of the next update (k_reduce_iter).  (Running it in the last
// workgroup of k_alpha instead was measured slower: the device-scope release
// fence every workgroup needs across the XCDs' L2s costs more than the launch.)
#pragma once
#include "nls_common.hpp"

namespace nls {

// Deterministic column sums of column-major partials: dst[v] = sum_q part[v*nb + q],
// v < nc.  One wave per column, fixed order (bitwise reproducible).
__device__ inline void sum_partials(const cplx *__restrict__ part, int nb, int nc, cplx *dst) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int v = w; v < nc; v += NTHREADS / 64) {
    const cplx *__restrict__ col = part + (int64_t)v * nb;
    double a0 = 0.0, b0 = 0.0, a1 = 0.0, b1 = 0.0;
    int q = lane;
    for (; q + 64 < nb; q += 128) {
      const cplx x0 = col[q], x1 = col[q + 64];
      a0 += x0.re; b0 += x0.im;
      a1 += x1.re; b1 += x1.im;
    }
    if (q < nb) { const cplx x0 = col[q]; a0 += x0.re; b0 += x0.im; }
    const double a = wave_sum(a0 + a1), b = wave_sum(b0 + b1);
    if (lane == 0) dst[v] = {a, b};
  }
}

__device__ __forceinline__ double inv_or_zero(double s) { return s > 0.0 ? 1.0 / s : 0.0; }

// After k_alpha<j> (and k_update<j-1>): sums layout
//   sums[0] = a_j, sums[1] = ||W_j||^2 (A pass), [sums[2] = ||L W_j||^2 if ncA == 3],
//   sums[ncA .. ncA+j] = g_0..g_{j-1}, nn (U pass)
// Coefficients of k_update<j> (all from the Gram column of W_j and the
// Hessenberg columns already known; see DESIGN.md "Lanczos reformulation"):
//   H[j][j] = alpha_j = a_j / s_j^2
//   H[j][k] = sum_{l<=k} conj(H[k][l]) G[j][l] + s_{k+1} G[j][k+1]   (k < j)
//   coef[k] = H[j][k] / s_k,  coef[j+1] = 1 / s_j
// ncA == 3 (fused tail, j = m-2: W_{j+1} is never stored): the norm of the last
// vector from the Krylov relation of the orthonormal basis,
//   s_{j+1}^2 = ||L v_j||^2 - sum_{k<=j} |H[j][k]|^2,
// exact up to rounding of order eps ||L||^2 / s_{j+1}^2; s_{j+1} only enters the
// last (smallest) coefficient of f(T) e_1, so that error is far below the
// tolerance of the path.  A non-positive value is a breakdown (column zero).
__device__ inline void reduce_iter_body(KState *__restrict__ st, const cplx *__restrict__ partA,
                                        int nbA, const cplx *__restrict__ partU, int nbU, int j,
                                        int do_sum, int do_coef, int ncA) {
  __shared__ cplx ssum[2 * MMAX + 8];
  const int ncols = ncA + (j >= 1 ? j + 1 : 0);
  if (do_sum) {
    sum_partials(partA, nbA, ncA, ssum);
    if (j >= 1) sum_partials(partU, nbU, j + 1, ssum + ncA);
    __syncthreads();
    if (!do_coef) {
      for (int v = threadIdx.x; v < ncols; v += NTHREADS) st->sums[v] = ssum[v];
      return;
    }
  } else {
    for (int v = threadIdx.x; v < ncols; v += NTHREADS) ssum[v] = st->sums[v];
    __syncthreads();
  }
  if (!do_coef) return;
  // Coefficient math, parallel over k: the previous Hessenberg columns, norms
  // and the new Gram column are staged in LDS (one coalesced read of the state)
  // instead of a serial chain of dependent global loads.
  __shared__ double s_s[MMAX + 1];
  __shared__ cplx s_G[MMAX];
  __shared__ cplx s_H[MMAX][MMAX];
  const int t = threadIdx.x;
  for (int k = t; k < j; k += NTHREADS) s_s[k] = st->s[k];
  for (int e = t; e < j * MMAX; e += NTHREADS) {
    const int k = e / MMAX, l = e % MMAX;
    if (l <= k) s_H[k][l] = st->H[k][l];
  }
  const double sj = sqrt(j == 0 ? ssum[1].re : ssum[ncA + j].re);
  const double isj = inv_or_zero(sj);
  if (t == 0) s_s[j] = sj;
  __syncthreads();
  for (int k = t; k < j; k += NTHREADS) s_G[k] = (inv_or_zero(s_s[k]) * isj) * ssum[ncA + k];
  if (t == 0) s_G[j] = {sj > 0.0 ? 1.0 : 0.0, 0.0};
  __syncthreads();
  const cplx alpha = (isj * isj) * ssum[0];
  for (int k = t; k <= j; k += NTHREADS) {
    cplx h;
    if (k == j) {
      h = alpha;
    } else {
      //   H[j][k] = sum_{l<=k} conj(H[k][l]) G[j][l] + s_{k+1} G[j][k+1]
      cplx acc = {0.0, 0.0};
      for (int l = 0; l <= k; ++l) acc += cmul(cconj(s_H[k][l]), s_G[l]);
      acc += s_s[k + 1] * s_G[k + 1];
      h = acc;
    }
    st->H[j][k] = h;
    st->G[j][k] = s_G[k];
    st->coef[k] = inv_or_zero(s_s[k]) * h;
    if (ncA == 3) s_H[j][k] = h;
  }
  if (t == 0) {
    st->s[j] = sj;
    st->Td[j] = alpha.re;
    st->coef[j + 1] = {isj, 0.0};
    if (j == 0) {
      st->breakdown = sj > 0.0 ? 0 : 1;
    } else {
      st->To[j - 1] = sj;
      if (!(sj > 0.0) && st->breakdown == 0) st->breakdown = j + 1;
    }
  }
  if (ncA == 3) {
    __syncthreads();
    if (t == 0) {
      double h2 = 0.0;
      for (int k = 0; k <= j; ++k) h2 += abs2(s_H[j][k]);
      const double r2 = ssum[2].re * (isj * isj) - h2;
      const double sn = r2 > 0.0 && sj > 0.0 ? sqrt(r2) : 0.0;
      st->s[j + 1] = sn;
      st->To[j] = sn;
      if (!(sn > 0.0) && st->breakdown == 0) st->breakdown = j + 2;
    }
  }
}

}  // namespace nls
