// nls_pass2.hpp -- two new Lanczos vectors per basis pass (3D isotropic NLSE,
// single-rank handles; NLS_PASS2=1).  The scheme and its numerics are in
// DESIGN.md §3 "two new vectors per basis pass" and tests/sstep_model.py.
//
// Stored raw vectors S_0..S_J (S_0 = the start vector), orthonormal basis
// W = S C (C upper triangular), D = C^{-1} (S_l = sum_{i<=l} W_i D[i][l]),
// Arnoldi matrix H[k][i] = W_k^H L W_i.  One pass k_pass2<J> reads S_0..S_J once
// and the stencils L S_J, L^2 S_J of the last one (radius-2 tile march through
// LDS), and writes
//   X = bX1 L S_J + sum_l aX[l] S_l               (-> S_{J+1})
//   Z = bZ2 L^2 S_J + bZ1 L S_J + sum_l aZ[l] S_l  (-> S_{J+2}, unless the last pass)
// with X = L W_J - sigma W_J - sum_{k<J} conj(H[J][k]) W_k and Z = (L - sigma) X,
// reducing S_l^H X, S_l^H Z, X^H X, X^H Z, Z^H Z.  k_p2coef turns those into the
// new columns of C, D, H and the coefficients of the next pass.
#pragma once
#include "nls_common.hpp"

namespace nls {

constexpr int P2M = MMAX + 2;
struct P2State {
  cplx C[P2M][P2M];  // C[l][i]: W_i = sum_l S_l C[l][i]
  cplx D[P2M][P2M];  // D[i][l]: S_l = sum_i W_i D[i][l]
  cplx H[P2M][P2M];  // H[k][i] = W_k^H L W_i
  cplx aX[P2M], aZ[P2M], aY[P2M], aW[P2M];  // S coefficients of V_1 (X), V_2 (Z), V_3 (Y), V_4 (W)
  cplx bX1, bZ1, bZ2, bY1, bY2, bY3;  // stencil coefficients: b_i[p] of L^p S_J (bZ1, bZ2 = b_2[1..2])
  cplx bW[4];                         // b_4[1..4] (the four-vector first pass, k_p4d0)
  double sigma, beta;
  cplx sums[3 * P2M + 8];
  cplx tk[P2M];   // fused tail: t_k = W_k^H L S_{m-2} (k_p2tail)
  double beta_t;  // fused tail: beta_{m-1}
  int32_t blind;  // the J = 0 pass ran on the raw start vector (mode 2), beta from its sums
  // peer stores (NLS_PEER=1, multi-rank k_p2d): where stored vector k's local planes 0, 1
  // (pdn: the neighbour below's upper ghost planes) and nzl-2, nzl-1 (pup: the neighbour
  // above's lower ones) also go; written once by the host, nullptr = no such neighbour.
  // Read by k_p2d after its march loop (a kernel argument would be loaded at entry and
  // held in SGPRs across the loop)
  void *pdn[P2M + 1], *pup[P2M + 1];
};

#ifndef NLS_NO_P2_KERNELS  // (defined by translation units that only need the types)
// Coefficient kernel (one workgroup).  A pass at J writes ns = 1 .. 4 new
// vectors V_1 = L W_J - sigma W_J - sum_{k<J} conj(H[J][k]) W_k, V_{i+1} = (L - sigma) V_i
// (k_p2d: ns <= 2; k_p4d0: ns = 4 at J = 0; the recurrences hold for any ns,
// tests/sstep_model.py) and reduces, in this order, S_l^H V_i (l <= J, per i)
// and the Gram V_a^H V_b (a <= b, row by row); J = 0 of a blind start also ||S_0||^2.
// mode 0: start (after the alpha pass and reduction of W_0: s[0] = beta, H[0][0] =
// alpha_0); mode 2: blind start, no alpha pass: the J = 0 pass runs on the raw start
// vector (C00 = 1) with the previous step's alpha_0 as its shift; mode 1 at J = 0 then
// takes beta from ||S_0||^2, rescales the sums to the normalised scheme and the new
// rows of C (columns of D) by 1/beta (beta); mode 1: after the pass at J (sums = its
// columns, summed).  Computes the new columns of C, D, H (tests/sstep_model.py
// coef_update) and, for a next pass of nsn > 0 vectors at J' = J + ns, its
// coefficients (pass_coefficients); nsn = 0: T into the KState for k_reduce_final
// (s[] = 1, so fin is in the W basis; k_p2tfin converts it).  real: the sums come
// from a real field marched as cell pairs; their imaginary parts are dropped.
__device__ __forceinline__ void p2coef_body(P2State *__restrict__ ps, KState *__restrict__ st, int J, int mode, int ns,
                                            int nsn, int real) {
  __shared__ cplx q[4][P2M], sv[P2M], lw[P2M], w[2][P2M];
  __shared__ cplx bb[2][6];
  __shared__ double nu[4];
  __shared__ double s_prev, s_beta;
  // C, D, H staged in LDS for the kernel's lifetime (its loops are chains of dependent
  // reads), written back at the end
  __shared__ cplx sC[P2M][P2M], sD[P2M][P2M], sH[P2M][P2M];
  const int t = threadIdx.x;
  int Jn;  // J of the next pass
  // mode 1 touches rows / columns < J + ns + 2 only (the start modes zero and write back
  // the whole matrices, so everything beyond stays zero): stage that block
  const int nb = (mode == 1) ? min(J + ns + 2, P2M) : P2M;
  for (int e = t; e < nb * nb; e += NTHREADS) {
    const int r = e / nb, c = e % nb;
    sC[r][c] = ps->C[r][c];
    sD[r][c] = ps->D[r][c];
    sH[r][c] = ps->H[r][c];
  }
  if (t == 0) s_prev = ps->H[0][0].re;  // mode 2's shift: the previous step's alpha_0
  __syncthreads();
  if (mode == 0 || mode == 2) {
    for (int e = t; e < P2M * P2M; e += NTHREADS) {
      const int i = e / P2M, k = e % P2M;
      sC[i][k] = {0.0, 0.0};
      sD[i][k] = {0.0, 0.0};
      sH[i][k] = {0.0, 0.0};
    }
    __syncthreads();
    if (t == 0) {
      if (mode == 0) {
        const double b = st->s[0];
        ps->beta = b;
        sC[0][0] = {b > 0.0 ? 1.0 / b : 0.0, 0.0};
        sD[0][0] = {b, 0.0};
        ps->sigma = st->H[0][0].re;
        ps->blind = 0;
      } else {
        ps->beta = 1.0;
        sC[0][0] = {1.0, 0.0};
        sD[0][0] = {1.0, 0.0};
        ps->sigma = s_prev;
        ps->blind = 1;
      }
    }
    __syncthreads();
    Jn = 0;
  } else {
    cplx *sw = ps->sums;
    const int ng = ns * (ns + 1) / 2, og = ns * (J + 1);  // Gram entries, their offset
    if (real) {
      // a real field marched as cell pairs (k_p2d PR): the real parts are the dots
      for (int e = t; e <= og + ng; e += NTHREADS) sw[e].im = 0.0;
      __syncthreads();
    }
    // Gram entry (a, b), a <= b
    auto gidx = [ns, og](int a, int b) { return og + a * ns - a * (a - 1) / 2 + (b - a); };
    if (J == 0 && ps->blind) {
      // the J = 0 pass ran on the raw S_0 (C00 = 1): its S-dots are beta, its Gram
      // beta^2 times those of the normalised scheme; ||S_0||^2 follows them
      if (t == 0) {
        const double b = sqrt(sw[og + ng].re);
        const double ib = b > 0.0 ? 1.0 / b : 0.0;
        s_beta = b;
        for (int e = 0; e < og; ++e) sw[e] = ib * sw[e];
        for (int e = og; e < og + ng; ++e) sw[e] = (ib * ib) * sw[e];
        ps->beta = b;
        sC[0][0] = {ib, 0.0};
        sD[0][0] = {b, 0.0};
      }
      __syncthreads();
    }
    const double sig = ps->sigma;
    for (int i = 0; i < ns; ++i) {
      const int n = J + 1 + i;  // the new vector's index
      // S_l^H V_i for l < n: the pass's S-dots (l <= J), the Gram (l = J + 1 + a)
      for (int l = t; l < n; l += NTHREADS) sv[l] = l <= J ? sw[i * (J + 1) + l] : sw[gidx(l - J - 1, i)];
      __syncthreads();
      // q_k = W_k^H V_i = sum_{l <= k} conj(C[l][k]) S_l^H V_i
      for (int k = t; k < n; k += NTHREADS) {
        cplx v = {0.0, 0.0};
        for (int l = 0; l <= k; ++l) v += cj_mul(sC[l][k], sv[l]);
        q[i][k] = v;
      }
      __syncthreads();
      if (t == 0) {
        double n2 = sw[gidx(i, i)].re;
        for (int k = 0; k < n; ++k) n2 -= abs2(q[i][k]);
        nu[i] = n2 > 0.0 ? sqrt(n2) : 0.0;
      }
      __syncthreads();
      const double nui = nu[i], inu = nui > 0.0 ? 1.0 / nui : 0.0;
      // C[:, n] = (e_n - C q) / nu ; D[:, n] = (q, nu)
      for (int r = t; r <= n; r += NTHREADS) {
        cplx v = {r == n ? 1.0 : 0.0, 0.0};
        for (int k = r; k < n; ++k) v = v - cmul(sC[r][k], q[i][k]);
        sC[r][n] = inu * v;
        sD[r][n] = r < n ? q[i][r] : cplx{nui, 0.0};
      }
      __syncthreads();
    }
    // H column J: q1_k + sigma delta_kJ + conj(H[J][k]) (k < J); H[J+1][J] = nu_1
    for (int r = t; r <= J + 1; r += NTHREADS) {
      cplx h = r <= J ? q[0][r] : cplx{nu[0], 0.0};
      if (r == J) h.re += sig;
      if (r < J) h += cconj(sH[J][r]);
      sH[r][J] = h;
    }
    __syncthreads();
    // H column c = J + i (i >= 1), L W_c = (V_{i+1} + sigma V_i - sum_{k<c} q^(i-1)_k L W_k) / nu_{i-1}:
    //   (wv_i + sigma wv_{i-1} - sum_{k<c} q^(i-1)_k H[:, k]) / nu_{i-1},  wv_i = (q^(i), nu_i)
    for (int i = 1; i < ns; ++i) {
      const int c = J + i;
      const double inp = nu[i - 1] > 0.0 ? 1.0 / nu[i - 1] : 0.0;
      for (int r = t; r <= c + 1; r += NTHREADS) {
        cplx v = r <= c ? q[i][r] : cplx{nu[i], 0.0};
        const cplx wp = r < c ? q[i - 1][r] : (r == c ? cplx{nu[i - 1], 0.0} : cplx{0.0, 0.0});
        v += sig * wp;
        for (int k = (r > 0 ? r - 1 : 0); k < c; ++k) v = v - cmul(q[i - 1][k], sH[r][k]);
        sH[r][c] = inp * v;
      }
      __syncthreads();
    }
    if (t == 0 && ns > 1) ps->sigma = sH[J + ns - 1][J + ns - 1].re;
    Jn = J + ns;
    __syncthreads();
    if (J == 0 && ps->blind) {
      // the stored S_1..S_ns are beta times the normalised scheme's: their C rows scale
      // by 1/beta, their D columns by beta (C = D^-1 stays consistent)
      const double b = s_beta, ib = b > 0.0 ? 1.0 / b : 0.0;
      for (int e = t; e < ns * nb; e += NTHREADS) {
        const int l = 1 + e / nb, k = e % nb;
        sC[l][k] = ib * sC[l][k];
        sD[k][l] = b * sD[k][l];
      }
      __syncthreads();
      if (t == 0) ps->blind = 0;
    }
  }
  if (nsn > 0) {
    // coefficients of the pass at j = Jn: V_i = sum_l a_i[l] S_l + sum_p b_i[p] L^p S_j
    // through the W coefficients w of V_i (tests/sstep_model.py pass_coefficients):
    //   lw = -C_jj H[:, :j] D[:j, j]   (L W_j = C_jj L S_j + lw)
    //   w_1 = lw - sigma e_j - conj(H[j][:j]),  b_1 = (C_jj)
    //   w_{i+1} = H[:, :j] w_i[:j] + w_i[j] lw - sigma w_i
    //   b_{i+1}[1] = w_i[j] C_jj - sigma b_i[1],  b_{i+1}[p+1] = b_i[p] - sigma b_i[p+1]
    const int j = Jn;
    const double sig = ps->sigma;
    const cplx cjj = sC[j][j];
    for (int k = t; k <= j; k += NTHREADS) {
      cplx v = {0.0, 0.0};
      for (int i = (k > 0 ? k - 1 : 0); i < j; ++i) v += cmul(sH[k][i], sD[i][j]);
      v = cmul(cjj, v);
      lw[k] = {-v.re, -v.im};
      cplx x = lw[k];
      if (k == j) x.re -= sig;
      if (k < j) x = x - cconj(sH[j][k]);
      w[0][k] = x;
    }
    if (t == 0) bb[0][0] = bb[0][1] = bb[0][2] = bb[0][3] = bb[0][4] = {0.0, 0.0};
    if (t == 0) bb[0][1] = cjj;
    __syncthreads();
    cplx *adst[4] = {ps->aX, ps->aZ, ps->aY, ps->aW};
    cplx *bdst[4] = {&ps->bX1, &ps->bZ1, &ps->bY1, ps->bW};
    for (int i = 0; i < nsn; ++i) {
      const int cu = i & 1, nx = cu ^ 1;
      // S-basis coefficients a_i = C w_i
      for (int l = t; l <= j; l += NTHREADS) {
        cplx a = {0.0, 0.0};
        for (int k = l; k <= j; ++k) a += cmul(sC[l][k], w[cu][k]);
        adst[i][l] = a;
      }
      if (t == 0)
        for (int p = 1; p <= i + 1; ++p) bdst[i][p - 1] = bb[cu][p];
      if (i + 1 < nsn) {
        for (int k = t; k <= j; k += NTHREADS) {
          cplx v = {0.0, 0.0};
          for (int i2 = (k > 0 ? k - 1 : 0); i2 < j; ++i2) v += cmul(sH[k][i2], w[cu][i2]);
          v += cmul(w[cu][j], lw[k]);
          w[nx][k] = v - sig * w[cu][k];
        }
        if (t == 0) {
          bb[nx][0] = {0.0, 0.0};
          bb[nx][1] = cmul(w[cu][j], cjj) - sig * bb[cu][1];
          for (int p = 1; p < 4; ++p) bb[nx][p + 1] = bb[cu][p] - sig * bb[cu][p + 1];
        }
      }
      __syncthreads();
    }
  } else if (t < MMAX) {
    // T as the reference builds it (alpha_j, j < Jn; norms; T[Jn][Jn] = 0 set by
    // k_reduce_final), s[] = 1 so that k_reduce_final's fin is c = Q f(Lambda) Q^T e_1
    if (t < Jn) {
      st->Td[t] = sH[t][t].re;
      st->To[t] = sH[t + 1][t].re;
    }
    st->s[t] = 1.0;
  }
  __syncthreads();
  for (int e = t; e < nb * nb; e += NTHREADS) {
    const int r = e / nb, c = e % nb;
    ps->C[r][c] = sC[r][c];
    ps->D[r][c] = sD[r][c];
    ps->H[r][c] = sH[r][c];
  }
}
__global__ __launch_bounds__(NTHREADS) void k_p2coef(P2State *__restrict__ ps, KState *__restrict__ st,
                                                     int J, int mode, int ns, int nsn, int real) {
  p2coef_body(ps, st, J, mode, ns, nsn, real);
}

#endif  // NLS_NO_P2_KERNELS

}  // namespace nls
