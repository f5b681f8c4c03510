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
//
// qa = 1 (no alpha pass: ncA = 0; the update pass i = j-1 also reduced
// q = y^H L y, y = L W_i, and the measured W_i^H L W_i as columns j+1, j+2;
// k_xpairs the x-tile seam part of q as nbX partials in partX, summed here).
// With Y = y / s_i = L v_i, the coefficients c_k = H[i][k] the pass used
// (W_j = Y - sum_k c_k v_k exactly, up to the kernel's rounding) and the exact
// projections A(k,l) = v_k^H L v_l -- off-diagonal H entries (Krylov relation +
// Gram), diagonal the MEASURED Rayleigh quotients T_d (not the alpha used as a
// coefficient: that one carries the rounding of its own formula, which would
// otherwise be amplified ~6x per iteration) --
//   a_j = W_j^H L W_j = Y^H L Y - 2 Re sum_k conj(c_k) B_k + sum_{k,l} conj(c_k) c_l A(k,l),
//   B_k = v_k^H L Y = sum_{l<=k} conj(H[k][l]) A(l,i) + s_{k+1} (k < i ? A(k+1,i) : conj(H[j][i])),
//   H[j][i] = v_i^H L v_j = s_j + sum_{l<=i} conj(c_l) G[j][l]       (Krylov relation of L v_i).
// The measured diagonal also replaces T_d[i] (the reference's alpha is the
// Rayleigh quotient v^H L v, eigen_krylov_complex.hpp:27-38).
// Conditioning: the terms are O(||L||^3) while a_j = s_j^2 alpha_j; near a
// breakdown (s_j -> 0) the cancellation loses everything.  When the sum of the
// terms' magnitudes exceeds 1e4 s_j^2 (|alpha_i| + s_i + s_j) (relative error of
// alpha_j ~1e-12 and worse), need_alpha is set: the conditional alpha pass
// (k_reduce_qa, the kernel around this body) then reduces a_j directly from W_j and
// redoes the coefficients (the U sums are kept at sums[2..j+2] for that).
__device__ inline void reduce_iter_body(KState *__restrict__ st, const cplx *__restrict__ partA,
                                        int nbA, const cplx *__restrict__ partU, int nbU, int j,
                                        int do_sum, int do_coef, int ncA, int qa,
                                        const cplx *__restrict__ partX = nullptr, int nbX = 0) {
  __shared__ cplx ssum[2 * MMAX + 8];
  __shared__ cplx sx;  // x-seam pairs of q (qa)
  const int ncols = ncA + (j >= 1 ? j + 1 + 2 * qa : 0);
  if (qa && do_coef) sum_partials(partX, nbX, 1, &sx);  // wave 0
  if (do_sum) {
    if (ncA > 0) sum_partials(partA, nbA, ncA, ssum);
    if (j >= 1) sum_partials(partU, nbU, j + 1 + 2 * qa, ssum + ncA);
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
  __shared__ double s_a;  // a_j (qa) -- ssum[0] is a Gram entry when ncA = 0
  if (qa) {
    __shared__ double s_term[MMAX];
    __shared__ double s_tm[MMAX];  // measured diagonal A(l,l), l <= i
    const int i = j - 1;
    const double isi = inv_or_zero(s_s[i]);
    for (int l = t; l < i; l += NTHREADS) s_tm[l] = st->Td[l];
    if (t == 0) s_tm[i] = ssum[j + 2].re * (isi * isi);
    __syncthreads();  // s_G, s_tm
    // A(k,l) = v_k^H L v_l
    auto A = [&](int k, int l) -> cplx {
      if (k == l) return {s_tm[k], 0.0};
      return k < l ? s_H[l][k] : cconj(s_H[k][l]);
    };
    for (int k = t; k <= i; k += NTHREADS) {
      cplx bk = {0.0, 0.0}, row = {0.0, 0.0};
      for (int l = 0; l <= k; ++l) bk += cmul(cconj(s_H[k][l]), A(l, i));
      if (k < i) {
        bk += s_s[k + 1] * A(k + 1, i);
      } else {
        cplx hji = {sj, 0.0};  // H[j][i]
        for (int l = 0; l <= i; ++l) hji += cmul(cconj(s_H[i][l]), s_G[l]);
        bk += sj * cconj(hji);
      }
      for (int l = 0; l <= i; ++l) row += cmul(s_H[i][l], A(k, l));
      const cplx ck = s_H[i][k];
      s_term[k] = -2.0 * cj_mul(ck, bk).re + cj_mul(ck, row).re;
    }
    __syncthreads();
    if (t == 0) {
      const double q = (ssum[j + 1].re + sx.re) * (isi * isi);  // + x-seam pairs
      double a = q, mag = fabs(q);
      for (int k = 0; k <= i; ++k) {  // fixed order
        a += s_term[k];
        mag += fabs(s_term[k]);
      }
      s_a = a;
      st->Td[i] = s_tm[i];
      st->need_alpha = (sj > 0.0 && mag > 1e4 * (sj * sj) * (fabs(s_tm[i]) + s_s[i] + sj)) ? 1 : 0;
    }
    for (int v = t; v <= j; v += NTHREADS) st->sums[2 + v] = ssum[v];  // for the fallback
  }
  __syncthreads();
  const cplx alpha = (isj * isj) * (qa ? cplx{s_a, 0.0} : ssum[0]);
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
