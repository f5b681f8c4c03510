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
  cplx aX[P2M], aZ[P2M];
  cplx bX1, bZ1, bZ2;
  double sigma, beta;
  cplx sums[2 * P2M + 8];
  cplx tk[P2M];   // fused tail: t_k = W_k^H L S_{m-2} (k_p2tail)
  double beta_t;  // fused tail: beta_{m-1}
  int32_t blind;  // the J = 0 pass ran on the raw start vector (mode 2), beta from its sums
};

// Register-march form of the same pass (the LDS-DMA form k_p2d, nls_pass2d.hpp, is the default).  Each
// wave owns a column of 64 lanes x P2R_RB rows and marches z on its own, no LDS,
// no barriers: lanes hold x = 60 xt - 2 + lane, of which lanes 2..61 are outputs
// and lanes 0,1,62,63 the x halo (x neighbours by lane shuffles; L S_J is valid
// on lanes 1..62, L^2 S_J on 2..61).  Register queues: S_J on rows -2..RB+1 for
// planes k-1..k+1, L S_J on rows -1..RB for planes k-2..k.  Step k loads
// S_J(k+1) and the J other streams of plane k-1, forms L S_J(k), then
// L^2 S_J(k-1) and the outputs of plane k-1.
constexpr int p2r_rb(int J) { return P2R_ROWS(J); }  // rows per wave (registers; measured per J)
constexpr int P2R_XO = 60;  // output x per wave
template <int J, bool HZ>
__global__ __launch_bounds__(NTHREADS) void k_pass2r(cplx *__restrict__ W, int64_t vs, Geo g,
                                                     const P2State *__restrict__ ps,
                                                     cplx *__restrict__ part, int nb) {
  constexpr int RB = p2r_rb(J), SR = RB + 4, LR = RB + 2;
  // columns: gX[0..J], then HZ: gZ[0..J], X^H X, X^H Z, Z^H Z; else X^H X.  (Deriving
  // S_l^H Z, l < J, from gX through the Arnoldi relation instead loses ~1e-7 absolute
  // at ||L|| ~ 1e2 -- the relation's rounding times ||L|| ||X|| -- measured, not kept.)
  constexpr int NC = HZ ? 2 * (J + 1) + 3 : J + 2;
  __shared__ cplx red[NTHREADS / 64][NC];
  __shared__ cplx cX[J + 1], cZ[J + 1];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nx = (int)g.nx, ny = (int)g.nyp, P = (int)g.P, nz = (int)g.npl;
  const int ntx = (nx + P2R_XO - 1) / P2R_XO, nry = ny / RB;
  const int nzc = (nz + g.kz - 1) / g.kz;
  for (int l = t; l <= J; l += NTHREADS) {
    cX[l] = ps->aX[l];
    cZ[l] = ps->aZ[l];
  }
  __syncthreads();
  const cplx bX1 = ps->bX1, bZ1 = ps->bZ1, bZ2 = ps->bZ2;
  const double s = g.s, sdi = g.sd_in, sdb = g.sd_bd;
  const cplx *__restrict__ SJ = W + (int64_t)J * vs;
  cplx *__restrict__ Xo = W + (int64_t)(J + 1) * vs;
  cplx *__restrict__ Zo = W + (int64_t)(J + 2) * vs;
  const volatile cplx *vX = cX, *vZ = cZ;
  auto ldc = [](const volatile cplx *p) { return cplx{p->re, p->im}; };
  cplx acc[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) acc[i] = {0.0, 0.0};
  const int wid = blockIdx.x * (NTHREADS / 64) + w;
  if (wid < ntx * nry * nzc) {  // uniform per wave
    const int xt = wid % ntx, yt = (wid / ntx) % nry, zc = wid / (ntx * nry);
    const int x = xt * P2R_XO - 2 + lane, y0 = yt * RB;
    const int k0 = zc * g.kz, k1 = min(k0 + g.kz, nz);
    const bool xin = x >= 0 && x < nx;
    const bool out = lane >= 2 && lane < 62 && x < nx;
    // true plane / row of row yy (-2..ny+1) of plane k; diagonal of a cell
    auto plane_of = [&](int k, int yy) { return yy < 0 ? k - 1 : (yy >= ny ? k + 1 : k); };
    auto row_of = [&](int yy) { return yy < 0 ? yy + ny : (yy >= ny ? yy - ny : yy); };
    auto dg = [&](int j, int kk) {
      const bool bd = x == 0 || x == nx - 1 || j == 0 || j == ny - 1 || kk == 0 || kk == nz - 1;
      return bd ? sdb : sdi;
    };
    auto ldS = [&](int k, int yy) {
      const int kk = plane_of(k, yy);
      cplx v = {0.0, 0.0};
      if (xin && kk >= 0 && kk < nz) v = SJ[k * P + yy * nx + x];
      return v;
    };
    cplx sq[3][SR], lq[3][LR];
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      sq[0][r] = ldS(k0 - 2, y0 - 2 + r);
      sq[1][r] = ldS(k0 - 1, y0 - 2 + r);
      sq[2][r] = {0.0, 0.0};
    }
#pragma unroll
    for (int r = 0; r < LR; ++r) lq[0][r] = lq[1][r] = lq[2][r] = {0.0, 0.0};
    // step k: sq[0] = plane k-1, sq[1] = plane k, load sq[2] = plane k+1;
    //         lq[1..2] = L1 planes k-2, k-1 -> shifted, lq[2] = L1(k); outputs at plane k-1
#pragma unroll 1
    for (int k = k0 - 1; k <= k1; ++k) {
#pragma unroll
      for (int r = 0; r < SR; ++r) sq[2][r] = ldS(k + 1, y0 - 2 + r);
      const bool emit = k - 1 >= k0;
      // the J other streams of the first output row, in flight during the L1 step
      cplx sv[J + 1];
      {
        const int flat = (k - 1) * P + y0 * nx + x;
#pragma unroll
        for (int l = 0; l < J; ++l) sv[l] = (emit && out) ? ld_nt(W + l * vs + flat) : cplx{0.0, 0.0};
      }
      // L1 at plane k, rows y0-1 .. y0+RB (S rows 1 .. RB+2)
#pragma unroll
      for (int r = 0; r < LR; ++r) {
        const cplx c = sq[1][r + 1];
        cplx xm = shfl_up1(c), xp = shfl_dn1(c);
        if (x == 0) xm = {0.0, 0.0};
        if (x == nx - 1) xp = {0.0, 0.0};
        const int yy = y0 - 1 + r, kk = plane_of(k, yy);
        cplx v = {0.0, 0.0};
        if (xin && kk >= 0 && kk < nz) {
          const cplx nbs = xm + xp + sq[1][r] + sq[1][r + 2] + sq[0][r + 1] + sq[2][r + 1];
          v = dg(row_of(yy), kk) * c + s * nbs;
        }
        lq[0][r] = lq[1][r];
        lq[1][r] = lq[2][r];
        lq[2][r] = v;
      }
      // lq[0] = L1(k-2), lq[1] = L1(k-1), lq[2] = L1(k): outputs at plane k-1
      if (emit) {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int flat = (k - 1) * P + (y0 + r) * nx + x;
          if (r > 0) {
#pragma unroll
            for (int l = 0; l < J; ++l) sv[l] = out ? ld_nt(W + l * vs + flat) : cplx{0.0, 0.0};
          }
          sv[J] = sq[0][r + 2];
          const cplx l1 = lq[1][r + 1];
          cplx X = cmul(bX1, l1);
#pragma unroll
          for (int l = 0; l <= J; ++l) X += cmul(ldc(vX + l), sv[l]);
          cplx Z = {0.0, 0.0};
          if constexpr (HZ) {
            cplx xm = shfl_up1(l1), xp = shfl_dn1(l1);
            if (x == 0) xm = {0.0, 0.0};
            if (x == nx - 1) xp = {0.0, 0.0};
            const cplx nbs = xm + xp + lq[1][r] + lq[1][r + 2] + lq[0][r + 1] + lq[2][r + 1];
            const cplx l2 = dg(y0 + r, k - 1) * l1 + s * nbs;
            Z = cmul(bZ2, l2) + cmul(bZ1, l1);
#pragma unroll
            for (int l = 0; l <= J; ++l) Z += cmul(ldc(vZ + l), sv[l]);
          }
          if (out) {
#pragma unroll
            for (int l = 0; l <= J; ++l) acc[l] += cj_mul(sv[l], X);
            st_nt(Xo + flat, X);
            if constexpr (HZ) {
#pragma unroll
              for (int l = 0; l <= J; ++l) acc[J + 1 + l] += cj_mul(sv[l], Z);
              acc[2 * J + 2].re += abs2(X);
              acc[2 * J + 3] += cj_mul(X, Z);
              acc[2 * J + 4].re += abs2(Z);
              st_nt(Zo + flat, Z);
            } else {
              acc[J + 1].re += abs2(X);
            }
          }
        }
      }
#pragma unroll
      for (int r = 0; r < SR; ++r) {
        sq[0][r] = sq[1][r];
        sq[1][r] = sq[2][r];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const double a = wave_sum(acc[i].re), b = wave_sum(acc[i].im);
    if (lane == 0) red[w][i] = {a, b};
  }
  __syncthreads();
  for (int i = t; i < NC; i += NTHREADS) {
    cplx v = red[0][i];
    for (int q = 1; q < NTHREADS / 64; ++q) v += red[q][i];
    part[(int64_t)i * nb + blockIdx.x] = v;
  }
}

// Coefficient kernel (one workgroup).  mode 0: start (after the alpha pass and
// reduction of W_0: s[0] = beta, H[0][0] = alpha_0); mode 2: blind start, no
// alpha pass: the J = 0 pass runs on the raw start vector (C00 = 1) with the
// previous step's alpha_0 as its shift and also reduces ||S_0||^2; mode 1 at
// J = 0 then takes beta from it, rescales the sums to the normalised scheme and
// the stored S_1, S_2 columns of C (and D) by 1/beta (beta); mode 1: after the
// pass at J (sums = the pass's columns, summed).  Computes the new columns of C, D, H
// and, if another pass follows (J' + 1 < m), its coefficients; otherwise T into
// the KState for k_reduce_final (s[] = 1, so fin is in the W basis; k_p2fin
// converts it).
__global__ __launch_bounds__(NTHREADS) void k_p2coef(P2State *__restrict__ ps, KState *__restrict__ st,
                                                     int J, int m, int mode) {
  __shared__ cplx p[P2M], q[P2M], lw[P2M], xw[P2M], zw[P2M];
  __shared__ cplx gz[P2M];
  __shared__ double nu[2];
  __shared__ double s_prev, s_beta;
  const int t = threadIdx.x;
  int Jn;  // J of the next pass
  if (t == 0) s_prev = ps->H[0][0].re;  // mode 2's shift: the previous step's alpha_0
  __syncthreads();
  if (mode == 0 || mode == 2) {
    for (int e = t; e < P2M * P2M; e += NTHREADS) {
      const int i = e / P2M, k = e % P2M;
      ps->C[i][k] = {0.0, 0.0};
      ps->D[i][k] = {0.0, 0.0};
      ps->H[i][k] = {0.0, 0.0};
    }
    __syncthreads();
    if (t == 0) {
      if (mode == 0) {
        const double b = st->s[0];
        ps->beta = b;
        ps->C[0][0] = {b > 0.0 ? 1.0 / b : 0.0, 0.0};
        ps->D[0][0] = {b, 0.0};
        ps->sigma = st->H[0][0].re;
        ps->blind = 0;
      } else {
        ps->beta = 1.0;
        ps->C[0][0] = {1.0, 0.0};
        ps->D[0][0] = {1.0, 0.0};
        ps->sigma = s_prev;
        ps->blind = 1;
      }
    }
    __syncthreads();
    Jn = 0;
  } else {
    const int hz = J + 2 < m;  // the pass also produced Z
    if (J == 0 && ps->blind) {
      // the J = 0 pass ran on the raw S_0 (C00 = 1): its sums are beta (gX, gZ) and
      // beta^2 (xx, xz, zz) times those of the normalised scheme; ||S_0||^2 follows them
      cplx *sw = ps->sums;
      const int ns = hz ? 5 : 2;
      if (t == 0) {
        const double b = sqrt(sw[ns].re);
        const double ib = b > 0.0 ? 1.0 / b : 0.0;
        s_beta = b;
        sw[0] = ib * sw[0];
        if (hz) {
          sw[1] = ib * sw[1];
          sw[2] = (ib * ib) * sw[2];
          sw[3] = (ib * ib) * sw[3];
          sw[4] = (ib * ib) * sw[4];
        } else {
          sw[1] = (ib * ib) * sw[1];
        }
        ps->beta = b;
        ps->C[0][0] = {ib, 0.0};
        ps->D[0][0] = {b, 0.0};
      }
      __syncthreads();
    }
    const cplx *sm = ps->sums;
    // sums: hz: gX[0..J], gZ[0..J], xx, xz, zz; else gX[0..J], xx
    const int o = 2 * J + 2;
    const cplx xx = hz ? sm[o] : sm[J + 1];
    const cplx xz = hz ? sm[o + 1] : cplx{0.0, 0.0}, zz = hz ? sm[o + 2] : cplx{0.0, 0.0};
    if (hz)
      for (int l = t; l <= J; l += NTHREADS) gz[l] = sm[J + 1 + l];
    __syncthreads();
#ifdef NLS_P2_DEBUG
    if (t == 0 && hz)
      for (int l = 0; l <= J; ++l)
        printf("[p2 J=%d] gz[%d] = %.15e %.15e  gX = %.15e sigma %.15e\n", J, l, gz[l].re, gz[l].im, sm[l].re, ps->sigma);
#endif
    // p_k = W_k^H X = sum_l conj(C[l][k]) (S_l^H X)
    for (int k = t; k <= J; k += NTHREADS) {
      cplx v = {0.0, 0.0};
      for (int l = 0; l <= k; ++l) v += cj_mul(ps->C[l][k], sm[l]);
      p[k] = v;
    }
    __syncthreads();
    if (t == 0) {
      double n2 = xx.re;
      for (int k = 0; k <= J; ++k) n2 -= abs2(p[k]);
      nu[0] = n2 > 0.0 ? sqrt(n2) : 0.0;
    }
    __syncthreads();
    const double nu1 = nu[0], inu1 = nu1 > 0.0 ? 1.0 / nu1 : 0.0;
    const double sig = ps->sigma;
    for (int i = t; i <= J + 1; i += NTHREADS) {
      // C[:, J+1] = (e_{J+1} - C p) / nu1 ; D[:, J+1] = (p, nu1)
      cplx v = {i == J + 1 ? 1.0 : 0.0, 0.0};
      for (int k = i; k <= J; ++k) v = v - cmul(ps->C[i][k], p[k]);
      ps->C[i][J + 1] = inu1 * v;
      ps->D[i][J + 1] = i <= J ? p[i] : cplx{nu1, 0.0};
      // H column J: p_k + sigma delta_kJ + conj(H[J][k]) (k < J); H[J+1][J] = nu1
      cplx h = i <= J ? p[i] : cplx{nu1, 0.0};
      if (i == J) h.re += sig;
      if (i < J) h += cconj(ps->H[J][i]);
      ps->H[i][J] = h;
    }
    __syncthreads();
    if (hz) {
      // q_k = W_k^H Z (k <= J+1): S-dots gZ (l <= J) and S_{J+1}^H Z = xz
      for (int k = t; k <= J + 1; k += NTHREADS) {
        cplx v = {0.0, 0.0};
        for (int l = 0; l <= k && l <= J; ++l) v += cj_mul(ps->C[l][k], gz[l]);
        if (k == J + 1) v += cj_mul(ps->C[J + 1][J + 1], xz);
        q[k] = v;
      }
      __syncthreads();
      if (t == 0) {
        double n2 = zz.re;
        for (int k = 0; k <= J + 1; ++k) n2 -= abs2(q[k]);
        nu[1] = n2 > 0.0 ? sqrt(n2) : 0.0;
      }
      __syncthreads();
      const double nu2 = nu[1], inu2 = nu2 > 0.0 ? 1.0 / nu2 : 0.0;
      for (int i = t; i <= J + 2; i += NTHREADS) {
        cplx v = {i == J + 2 ? 1.0 : 0.0, 0.0};
        for (int k = i; k <= J + 1; ++k) v = v - cmul(ps->C[i][k], q[k]);
        ps->C[i][J + 2] = inu2 * v;
        ps->D[i][J + 2] = i <= J + 1 ? q[i] : cplx{nu2, 0.0};
      }
      // H column J+1 = (wz + sigma wx - p_J (wx + sigma e_J + conj(H[J][:J])) - sum_{k<J} p_k H[:,k]) / nu1
      //   wx = (p, nu1, 0), wz = (q, nu2)
      for (int i = t; i <= J + 2; i += NTHREADS) {
        const cplx wxi = i <= J ? p[i] : (i == J + 1 ? cplx{nu1, 0.0} : cplx{0.0, 0.0});
        const cplx wzi = i <= J + 1 ? q[i] : cplx{nu2, 0.0};
        cplx lwj = wxi;
        if (i == J) lwj.re += sig;
        if (i < J) lwj += cconj(ps->H[J][i]);
        cplx v = wzi + sig * wxi - cmul(p[J], lwj);
        if (i <= J)
          for (int k = (i > 0 ? i - 1 : 0); k < J; ++k) v = v - cmul(p[k], ps->H[i][k]);
        ps->H[i][J + 1] = inu1 * v;
      }
      __syncthreads();
      if (t == 0) ps->sigma = ps->H[J + 1][J + 1].re;
      Jn = J + 2;
    } else {
      Jn = J + 1;  // W_{m-1} done
    }
    __syncthreads();
    if (J == 0 && ps->blind) {
      // the stored S_1 (and S_2) are beta times the normalised scheme's: their C rows
      // scale by 1/beta, their D columns by beta (C = D^-1 stays consistent)
      const double b = s_beta, ib = b > 0.0 ? 1.0 / b : 0.0;
      const int nl = hz ? 2 : 1;
      for (int e = t; e < nl * P2M; e += NTHREADS) {
        const int l = 1 + e / P2M, k = e % P2M;
        ps->C[l][k] = ib * ps->C[l][k];
        ps->D[k][l] = b * ps->D[k][l];
      }
      __syncthreads();
      if (t == 0) ps->blind = 0;
    }
  }
  if (Jn + 1 < m) {
    // coefficients of the pass at Jn
    const int j = Jn;
    const double sig = ps->sigma;
    const cplx cjj = ps->C[j][j];
    // lw = -C[j][j] H[:, :j] D[:j, j]   (the W part of L W_j besides C[j][j] L S_j)
    for (int k = t; k <= j; k += NTHREADS) {
      cplx v = {0.0, 0.0};
      for (int i = (k > 0 ? k - 1 : 0); i < j; ++i) v += cmul(ps->H[k][i], ps->D[i][j]);
      v = cmul(cjj, v);
      lw[k] = {-v.re, -v.im};
    }
    __syncthreads();
    for (int k = t; k <= j; k += NTHREADS) {
      cplx v = lw[k];
      if (k == j) v.re -= sig;
      if (k < j) v = v - cconj(ps->H[j][k]);
      xw[k] = v;
    }
    __syncthreads();
    // zw = H[:, :j] xw[:j] + xw[j] lw - sigma xw
    for (int k = t; k <= j; k += NTHREADS) {
      cplx v = {0.0, 0.0};
      for (int i = (k > 0 ? k - 1 : 0); i < j; ++i) v += cmul(ps->H[k][i], xw[i]);
      v += cmul(xw[j], lw[k]);
      v = v - sig * xw[k];
      zw[k] = v;
    }
    __syncthreads();
    // S-basis coefficients a = C w
    for (int l = t; l <= j; l += NTHREADS) {
      cplx ax = {0.0, 0.0}, az = {0.0, 0.0};
      for (int k = l; k <= j; ++k) {
        ax += cmul(ps->C[l][k], xw[k]);
        az += cmul(ps->C[l][k], zw[k]);
      }
      ps->aX[l] = ax;
      ps->aZ[l] = az;
    }
    if (t == 0) {
      ps->bX1 = cjj;
      ps->bZ1 = cmul(xw[j], cjj) - sig * cjj;
      ps->bZ2 = cjj;
    }
  } else if (t < MMAX) {
    // T as the reference builds it (alpha_j, j < m-1; norms; T[m-1][m-1] = 0 set by
    // k_reduce_final), s[] = 1 so that k_reduce_final's fin is c = Q f(Lambda) Q^T e_1
    if (t < m - 1) {
      st->Td[t] = ps->H[t][t].re;
      st->To[t] = ps->H[t + 1][t].re;
    }
    st->s[t] = 1.0;
  }
}

// fin (W basis, from k_reduce_final) -> S basis: fin_S = beta C fin_W
__global__ __launch_bounds__(NTHREADS) void k_p2fin(const P2State *__restrict__ ps,
                                                    KState *__restrict__ st, int m, int nf) {
  __shared__ cplx fw[2][MMAX];
  const int t = threadIdx.x;
  for (int e = t; e < nf * m; e += NTHREADS) fw[e / m][e % m] = st->fin[e / m][e % m];
  __syncthreads();
  for (int e = t; e < nf * m; e += NTHREADS) {
    const int f = e / m, l = e % m;
    cplx v = {0.0, 0.0};
    for (int i = l; i < m; ++i) v += cmul(ps->C[l][i], fw[f][i]);
    st->fin[f][l] = ps->beta * v;
  }
}

}  // namespace nls
