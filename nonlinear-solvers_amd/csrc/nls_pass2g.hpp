// nls_pass2g.hpp -- the two-vector basis pass without LDS staging (k_p2m): the form for
// the operators and shapes the LDS-DMA pass k_p2d does not take -- the G2
// anisotropic operator div(c grad) (nlsolvers/common/include/laplacians.hpp:54-103,
// 158-218) of the G2 NLSE drivers (m = 25 in 3D, nlse_cubic_driver_3d.cpp:112-114;
// 20 in 2D), whose J ring would exceed the LDS, and isotropic grids with ny % 4 != 0
// or m > 18.  The scheme, coefficients and per-cell formulas are k_p2d's
// (nls_pass2.hpp); the pass is two launches:
//
//   k_lap  : y = L S_J at local planes [-1, nzl] (the neighbour slabs' first planes
//            from the two-plane halo) into lbuf
//   k_p2m  : the register-queue march over y, which gives every cell y and L y =
//            L^2 S_J; X = bX1 y + sum_l aX[l] S_l, Z = bZ2 L y + bZ1 y + sum_l aZ[l]
//            S_l, their stores and the pass's dots in k_p2d's column layout.
//
// Per pass that moves y once more than k_p2d (written, then marched) and, for
// div(c grad), c twice: at m = 25 a G2 step moves ~236 vectors instead of the
// one-vector passes' ~374 (bench.py moved_bytes_per_cell_step).  (A per-cell form
// with the stencils of y through L1/L2 ran at ~3.5 TB/s, the march at ~5.3 TB/s;
// measured in round 3 and removed.)
#pragma once
#include "nls_pass2d.hpp"
#include "nls_stencil.hpp"

namespace nls {

// The per-workgroup partials of a pass whose accumulators are split over wave pairs
// (HZ: X set on even waves, Z set on odd ones; k_p2m, k_p2b) in k_p2d's column order:
// [S_l^H X (l <= J)] [S_l^H Z] [X^H X] [X^H Z] [Z^H Z] [||S_0||^2 (J = 0)], without Z
// [S_l^H X] [X^H X] [||S_0||^2] summed over all four waves.
template <int J, bool HZ, int NC, int NH>
__device__ __forceinline__ void p2_split_store(cplx (&acc)[NH], cplx (&red)[NTHREADS / 64][NH],
                                               cplx *__restrict__ part, int nb, int poff) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < NH; ++c) {
    const double a = wave_sum(acc[c].re), b = wave_sum(acc[c].im);
    if (lane == 0) red[w][c] = {a, b};
  }
  __syncthreads();
  for (int c = threadIdx.x; c < NC; c += NTHREADS) {
    cplx v;
    if constexpr (HZ) {
      int par, a;
      if (c <= J) { par = 0; a = c; }                      // S_l^H X
      else if (c <= 2 * J + 1) { par = 1; a = c - J - 1; }  // S_l^H Z
      else if (c == 2 * J + 2) { par = 0; a = J + 1; }      // X^H X
      else if (c == 2 * J + 3) { par = 1; a = J + 1; }      // X^H Z
      else if (c == 2 * J + 4) { par = 1; a = J + 2; }      // Z^H Z
      else { par = 0; a = J + 2; }                          // ||S_0||^2 (J = 0)
      v = red[par][a] + red[par + 2][a];
    } else {
      v = red[0][c];
#pragma unroll
      for (int q = 1; q < NTHREADS / 64; ++q) v += red[q][c];
    }
    part[(int64_t)c * nb + poff + blockIdx.x] = v;
  }
}

// The pass marches y = L S_J (lbuf, written by k_lap over planes [-1, nzl] on the same
// tiles) with nls_stencil.hpp's register-queue
// tile march, which hands each cell y and L y (z neighbours from registers, x from
// the neighbouring lane, y from the thread's rows; only tile-edge values through
// L1/L2), then streams S_0..S_J as k_update does: every load of every row first,
// then X, Z, their stores and the dots.  All NC accumulators per lane (one wave per
// SIMD from J ~ 14); the coefficients are broadcast from LDS at every use.
template <int J> struct P2mRB { static constexpr int v = J <= 4 ? 2 : 1; };
template <int DIM, int J, bool HZ, bool ANI>
__global__ __launch_bounds__(NTHREADS) void k_p2m(cplx *__restrict__ W, int64_t vs, Geo g,
                                                  const P2State *__restrict__ ps, cplx *__restrict__ part,
                                                  int nb, const cplx *__restrict__ lbuf, int poff) {
  constexpr int NC = (HZ ? 2 * (J + 1) + 3 : J + 2) + (J == 0 ? 1 : 0);
  constexpr int RB = P2mRB<J>::v;
  __shared__ cplx cX[J + 1], cZ[J + 1];
  for (int l = threadIdx.x; l <= J; l += NTHREADS) {
    cX[l] = ps->aX[l];
    cZ[l] = ps->aZ[l];
  }
  __syncthreads();
  const cplx bX1 = ps->bX1, bZ1 = ps->bZ1, bZ2 = ps->bZ2;
  cplx *__restrict__ Xo = W + (int64_t)(J + 1) * vs;
  cplx *__restrict__ Zo = W + (int64_t)(J + 2) * vs;
  const cplx zero = {0.0, 0.0};
  cplx acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = zero;
  const cplx *L0 = lbuf + g.P;  // y at local plane 0 (planes -1 .. nzl)
  auto body = [&](const int *p, const cplx *cur, const cplx *lap, const bool *ok) {
    cplx sv[RB][J + 1];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const cplx *__restrict__ src = W + p[r];
#pragma unroll
      for (int l = 0; l < J; ++l) {
        sv[r][l] = ok[r] ? ld_nt(src) : zero;
        src += vs;
      }
      sv[r][J] = ok[r] ? *src : zero;
    }
    asm volatile("" ::: "memory");  // keep the coefficient LDS reads at their use
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (!ok[r]) continue;
      cplx Xa = cmul(bX1, cur[r]), Xb = zero;
#pragma unroll
      for (int l = 0; l <= J; ++l) cmac((l & 1) ? Xb : Xa, cX[l], sv[r][l]);
      const cplx X = Xa + Xb;
      st_nt(Xo + p[r], X);
#pragma unroll
      for (int l = 0; l <= J; ++l) cjmac(acc[l], sv[r][l], X);
      if constexpr (HZ) {
        cplx Za = cmul(bZ2, lap[r]) + cmul(bZ1, cur[r]), Zb = zero;
#pragma unroll
        for (int l = 0; l <= J; ++l) cmac((l & 1) ? Zb : Za, cZ[l], sv[r][l]);
        const cplx Z = Za + Zb;
        st_nt(Zo + p[r], Z);
#pragma unroll
        for (int l = 0; l <= J; ++l) cjmac(acc[J + 1 + l], sv[r][l], Z);
        acc[2 * J + 2].re = fma(X.re, X.re, fma(X.im, X.im, acc[2 * J + 2].re));
        cjmac(acc[2 * J + 3], X, Z);
        acc[2 * J + 4].re = fma(Z.re, Z.re, fma(Z.im, Z.im, acc[2 * J + 4].re));
      } else {
        acc[J + 1].re = fma(X.re, X.re, fma(X.im, X.im, acc[J + 1].re));
      }
      if constexpr (J == 0)
        acc[NC - 1].re = fma(sv[r][0].re, sv[r][0].re, fma(sv[r][0].im, sv[r][0].im, acc[NC - 1].re));
    }
  };
  march<cplx, DIM, RB, true, ANI>(L0, g, body);
  block_store<NC>(acc, part, nb, poff);
}

}  // namespace nls
