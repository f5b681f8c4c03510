// nls_pass2b.hpp -- the boundary planes of a split multi-rank two-vector pass.
//
// A collective handle overlaps the halo exchange of the pass's new stencil vector
// with the pass itself: the slab's first two and last two planes are computed
// first, on the halo stream, which then sends them, while the interior planes
// [2, nzl-2) run as the LDS-DMA pass k_p2d on the compute stream (nls_api.cpp
// run_lanczos2).  Computing those four planes with k_p2d itself (tiles of depth 2)
// cost ~10 % per rank at the 8-GPU slab (512 x 512 x 64, tools/slab_probe.py):
// k_p2d needs ~150 KB of LDS at J >= 6, so each short, latency-bound boundary tile
// held a whole CU.  These two kernels do the same arithmetic with registers only
// (a few KB of LDS for the final reduction), so the dispatcher can place their
// waves beside the interior pass's on the same CUs:
//
//   k_p2b_lap : L S_J at local planes {-1, 0, 1, 2, nzl-3, .., nzl} into lbuf
//               (8 planes; the ghost planes -1 and nzl from the two-plane halo)
//   k_p2b     : per cell of planes {0, 1, nzl-2, nzl-1}: L^2 S_J from lbuf, then
//               X = bX1 L S_J + sum_l aX[l] S_l, Z = bZ2 L^2 S_J + bZ1 L S_J +
//               sum_l aZ[l] S_l (nls_pass2.hpp), their stores and the pass's dot
//               products, in k_p2d's column layout and evaluation order.
#pragma once
#include "nls_pass2g.hpp"  // p2_split_store

namespace nls {

constexpr int P2B_LPLANES = 8;  // planes of L S_J the boundary planes' L^2 needs
constexpr int P2B_OPLANES = 4;  // output planes per boundary launch
// local plane of lbuf slot i, of output plane i, and the lbuf slot of local plane k
__device__ __forceinline__ int p2b_lplane(int i, int nzl) { return i < 4 ? i - 1 : nzl - 7 + i; }
__device__ __forceinline__ int p2b_oplane(int i, int nzl) { return i < 2 ? i : nzl - 4 + i; }
__device__ __forceinline__ int p2b_slot(int k, int nzl) { return k <= 2 ? k + 1 : k - nzl + 7; }

// (L S_J) at local plane k, row y, column x of the slab (laplacians.hpp:55-105: the
// 3D flat-index operator incl. the y-wrap, diagonal -5/-6); 0 outside the grid, as
// k_p2d's P2D_LAP.  S_J's two ghost planes per side hold the neighbours' planes.
struct P2bGeo {
  int nx, ny, P, nz, z0;
  double s, sdi, sdb;
};
__device__ __forceinline__ cplx p2b_lap_at(const cplx *__restrict__ SJ, const P2bGeo &g, int k, int y, int x) {
  const int nx = g.nx, ny = g.ny, P = g.P, nz = g.nz;
  const int kk = g.z0 + k;
  if (x < 0 || x >= nx || kk < 0 || kk >= nz) return {0.0, 0.0};
  const cplx *c = SJ + (k * P + y * nx + x);
  const cplx zero = {0.0, 0.0};
  const cplx xm = x > 0 ? c[-1] : zero, xp = x + 1 < nx ? c[1] : zero;
  const cplx ym = (kk > 0 || y > 0) ? c[-nx] : zero;            // idx - nx >= 0
  const cplx yp = (kk < nz - 1 || y < ny - 1) ? c[nx] : zero;   // idx + nx < N
  const cplx zm = kk > 0 ? c[-P] : zero, zp = kk < nz - 1 ? c[P] : zero;
  const bool bd = x == 0 || x == nx - 1 || y == 0 || y == ny - 1 || kk == 0 || kk == nz - 1;
  return (bd ? g.sdb : g.sdi) * c[0] + g.s * (((zm + zp) + (xm + xp)) + (ym + yp));
}

__global__ __launch_bounds__(NTHREADS) void k_p2b_lap(const cplx *__restrict__ SJ, Geo g,
                                                      cplx *__restrict__ lbuf) {
  const P2bGeo pg = {(int)g.nx, (int)g.nyp, (int)g.P, (int)g.npl, (int)g.z0, g.s, g.sd_in, g.sd_bd};
  const int P = pg.P, nx = pg.nx, nzl = (int)g.nzl;
  const int total = P2B_LPLANES * P;
  for (int e = blockIdx.x * NTHREADS + threadIdx.x; e < total; e += gridDim.x * NTHREADS) {
    const int i = e / P, r = e - i * P, y = r / nx, x = r - y * nx;
    lbuf[e] = p2b_lap_at(SJ, pg, p2b_lplane(i, nzl), y, x);
  }
}

// Partials at part[c * nb + poff + blockIdx.x], the columns of k_p2d<J, HZ>:
// [S_l^H X (l <= J)] [S_l^H Z (l <= J)] [X^H X] [X^H Z] [Z^H Z] (HZ) or [S_l^H X] [X^H X],
// then ||S_0||^2 at J = 0.  Registers are what lets these waves sit beside k_p2d's
// (<= ~248 VGPRs next to a 257-VGPR k_p2d<12> wave), so with Z the work of a cell is
// split over two waves: both form X and Z, the "X" wave (even wave index) stores them
// and accumulates the X column set, the "Z" wave the Z set -- half the accumulators
// each; the combination coefficients are read as wave-uniform (scalar) loads, not
// hoisted into VGPRs.  A workgroup covers 128 cells (waves 0/1: cells 0..63, waves
// 2/3: 64..127).
template <int J, bool HZ>
__global__ __launch_bounds__(NTHREADS) void k_p2b(cplx *__restrict__ W, int64_t vs, Geo g,
                                                  const P2State *__restrict__ ps, cplx *__restrict__ part,
                                                  int nb, const cplx *__restrict__ lbuf, int poff) {
  constexpr int NC = (HZ ? 2 * (J + 1) + 3 : J + 2) + (J == 0 ? 1 : 0);
  constexpr int NH = HZ ? J + 3 : NC;  // accumulators per wave (X set: J+1 dots, xx, s0 | Z set: J+1, xz, zz)
  constexpr int CPB = HZ ? 128 : 256;  // cells per workgroup pass
  __shared__ cplx red[NTHREADS / 64][NH];
  const cplx *__restrict__ cX = ps->aX, *__restrict__ cZ = ps->aZ;
  const cplx bX1 = ps->bX1, bZ1 = ps->bZ1, bZ2 = ps->bZ2;
  const int P = (int)g.P, nx = (int)g.nx, ny = (int)g.nyp, nz = (int)g.npl, nzl = (int)g.nzl;
  const int z0 = (int)g.z0;
  const double s = g.s, sdi = g.sd_in, sdb = g.sd_bd;
  cplx *__restrict__ Xo = W + (int64_t)(J + 1) * vs;
  cplx *__restrict__ Zo = W + (int64_t)(J + 2) * vs;
  const cplx zero = {0.0, 0.0};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool zw = HZ && (w & 1);  // the Z-set wave (uniform)
  const int cell0 = HZ ? (w >> 1) * 64 + lane : threadIdx.x;
  cplx acc[NH];
#pragma unroll
  for (int c = 0; c < NH; ++c) acc[c] = zero;
  const int total = P2B_OPLANES * P;
  for (int e = blockIdx.x * CPB + cell0; e < total; e += gridDim.x * CPB) {
    const int i = e / P, r = e - i * P, y = r / nx, x = r - y * nx;
    const int k = p2b_oplane(i, nzl), kk = z0 + k;
    const cplx *Lc = lbuf + (int64_t)p2b_slot(k, nzl) * P;
    const cplx l1 = Lc[r];
    const int64_t flat = (int64_t)k * P + r;
    cplx sv[J + 1];
#pragma unroll
    for (int l = 0; l <= J; ++l) sv[l] = W[l * vs + flat];
    cplx Xa = cmul(bX1, l1), Xb = zero;
#pragma unroll
    for (int l = 0; l <= J; ++l) cmac((l & 1) ? Xb : Xa, cX[l], sv[l]);
    const cplx X = Xa + Xb;
    if constexpr (HZ) {
      // L^2 S_J as k_p2d: z from planes k-1, k+1, x within the row, y in flat form
      // (row -1 = row ny-1 of plane k-1, row ny = row 0 of plane k+1; lbuf holds 0
      // outside the grid)
      const cplx *Lm = lbuf + (int64_t)p2b_slot(k - 1, nzl) * P;
      const cplx *Lp = lbuf + (int64_t)p2b_slot(k + 1, nzl) * P;
      const cplx xm = x > 0 ? Lc[r - 1] : zero, xp = x + 1 < nx ? Lc[r + 1] : zero;
      const cplx ym = y > 0 ? Lc[r - nx] : Lm[(ny - 1) * nx + x];
      const cplx yp = y + 1 < ny ? Lc[r + nx] : Lp[x];
      const cplx zz = Lm[r] + Lp[r];
      const bool bd = x == 0 || x == nx - 1 || y == 0 || y == ny - 1 || kk == 0 || kk == nz - 1;
      const cplx l2 = (bd ? sdb : sdi) * l1 + s * ((zz + (xm + xp)) + (ym + yp));
      cplx Za = cmul(bZ2, l2) + cmul(bZ1, l1), Zb = zero;
#pragma unroll
      for (int l = 0; l <= J; ++l) cmac((l & 1) ? Zb : Za, cZ[l], sv[l]);
      const cplx Z = Za + Zb;
      if (zw) {
#pragma unroll
        for (int l = 0; l <= J; ++l) cjmac(acc[l], sv[l], Z);
        cjmac(acc[J + 1], X, Z);
        acc[J + 2].re = fma(Z.re, Z.re, fma(Z.im, Z.im, acc[J + 2].re));
      } else {
        st_nt(Xo + flat, X);
        st_nt(Zo + flat, Z);
#pragma unroll
        for (int l = 0; l <= J; ++l) cjmac(acc[l], sv[l], X);
        acc[J + 1].re = fma(X.re, X.re, fma(X.im, X.im, acc[J + 1].re));
        if constexpr (J == 0) acc[J + 2].re = fma(sv[0].re, sv[0].re, fma(sv[0].im, sv[0].im, acc[J + 2].re));
      }
    } else {
      st_nt(Xo + flat, X);
#pragma unroll
      for (int l = 0; l <= J; ++l) cjmac(acc[l], sv[l], X);
      acc[J + 1].re = fma(X.re, X.re, fma(X.im, X.im, acc[J + 1].re));
      if constexpr (J == 0) acc[NC - 1].re = fma(sv[0].re, sv[0].re, fma(sv[0].im, sv[0].im, acc[NC - 1].re));
    }
  }
  p2_split_store<J, HZ, NC, NH>(acc, red, part, nb, poff);
}

}  // namespace nls
