// nls_pass2g.hpp -- the two-vector basis pass without LDS staging: the form for
// the operators and shapes the LDS-DMA pass k_p2d does not take -- the G2
// anisotropic operator div(c grad) (nlsolvers/common/include/laplacians.hpp:54-103,
// 158-218) of the G2 NLSE drivers (m = 25 in 3D, nlse_cubic_driver_3d.cpp:112-114;
// 20 in 2D), whose J ring would exceed the LDS, and isotropic grids with ny % 4 != 0
// or m > 18.  The scheme, coefficients and per-cell formulas are k_p2d's
// (nls_pass2.hpp); the pass is split in two launches:
//
//   k_p2g_lap : y = L S_J at local planes [-1, nzl] into lbuf (nzl + 2 planes; the
//               ghost planes from the two-plane halo, 0 outside the grid)
//   k_p2g     : per cell of the slab: L^2 S_J = L y from lbuf, then
//               X = bX1 y + sum_l aX[l] S_l, Z = bZ2 L y + bZ1 y + sum_l aZ[l] S_l,
//               their stores and the pass's dots S_l^H X, S_l^H Z, X^H X, X^H Z,
//               Z^H Z (+ ||S_0||^2 at J = 0) in k_p2d's column layout.
//
// Per pass that moves lbuf once more than k_p2d (written, then read with the
// stencil) and, for div(c grad), c twice: at m = 25 a G2 step moves ~236 vectors
// instead of the one-vector passes' ~374 (bench.py moved_bytes_per_cell_step).
#pragma once
#include "nls_pass2d.hpp"

namespace nls {

struct LGeo {
  int nx, ny, P, nz, z0;  // ny: rows per plane (3D), 1 (2D: "planes" are grid rows)
  double s, sdi, sdb;
};
__device__ __forceinline__ LGeo lgeo(const Geo &g) {
  return {(int)g.nx, (int)g.nyp, (int)g.P, (int)g.npl, (int)g.z0, g.s, g.sd_in, g.sd_bd};
}

// (L V) at local plane k, row y, column x (laplacians.hpp:10-105 isotropic, incl.
// the 3D flat-index y-wrap; ANI: face weights (c_a + c_b)/2, diagonal -sum of the
// weights, as nls_stencil.hpp march); 0 outside the grid.  V and C point at local
// plane 0; their ghost planes hold the neighbouring slabs' planes.
template <int DIM, bool ANI>
__device__ __forceinline__ cplx lap_cell(const cplx *__restrict__ V, const double *__restrict__ C,
                                         const LGeo &g, int k, int y, int x) {
  const cplx zero = {0.0, 0.0};
  const int kk = g.z0 + k;
  if (x < 0 || x >= g.nx || kk < 0 || kk >= g.nz) return zero;
  const int p = k * g.P + y * g.nx + x;
  const bool exm = x > 0, exp_ = x + 1 < g.nx, ezm = kk > 0, ezp = kk + 1 < g.nz;
  const cplx cur = V[p];
  const cplx xm = exm ? V[p - 1] : zero, xp = exp_ ? V[p + 1] : zero;
  const cplx prev = ezm ? V[p - g.P] : zero, next = ezp ? V[p + g.P] : zero;
  if constexpr (DIM == 3) {
    const bool eym = kk > 0 || y > 0, eyp = kk < g.nz - 1 || y < g.ny - 1;  // idx -/+ nx in range
    const cplx ym = eym ? V[p - g.nx] : zero, yp = eyp ? V[p + g.nx] : zero;
    if constexpr (ANI) {
      const double cc = C[p];
      const double wxm = exm ? 0.5 * (cc + C[p - 1]) : 0.0, wxp = exp_ ? 0.5 * (cc + C[p + 1]) : 0.0;
      const double wym = eym ? 0.5 * (cc + C[p - g.nx]) : 0.0, wyp = eyp ? 0.5 * (cc + C[p + g.nx]) : 0.0;
      const double wzm = ezm ? 0.5 * (cc + C[p - g.P]) : 0.0, wzp = ezp ? 0.5 * (cc + C[p + g.P]) : 0.0;
      return g.s * ((((wzm * prev + wzp * next) + (wxm * xm + wxp * xp)) + (wym * ym + wyp * yp)) -
                    (((wzm + wzp) + (wxm + wxp)) + (wym + wyp)) * cur);
    } else {
      const bool bd = !exm || !exp_ || y == 0 || y == g.ny - 1 || !ezm || !ezp;
      return (bd ? g.sdb : g.sdi) * cur + g.s * (((prev + next) + (xm + xp)) + (ym + yp));
    }
  } else {
    if constexpr (ANI) {
      const double cc = C[p];
      const double wxm = exm ? 0.5 * (cc + C[p - 1]) : 0.0, wxp = exp_ ? 0.5 * (cc + C[p + 1]) : 0.0;
      const double wzm = ezm ? 0.5 * (cc + C[p - g.P]) : 0.0, wzp = ezp ? 0.5 * (cc + C[p + g.P]) : 0.0;
      return g.s * (((wzm * prev + wzp * next) + (wxm * xm + wxp * xp)) - ((wzm + wzp) + (wxm + wxp)) * cur);
    } else {
      const bool bd = !exm || !exp_ || !ezm || !ezp;
      return g.s * ((prev + next) + (xm + xp)) + (bd ? g.sdb : g.sdi) * cur;
    }
  }
}

template <int DIM, bool ANI>
__global__ __launch_bounds__(NTHREADS) void k_p2g_lap(const cplx *__restrict__ SJ, Geo g,
                                                      cplx *__restrict__ lbuf) {
  const LGeo lg = lgeo(g);
  const double *C = g.cf;
  const int P = lg.P, nx = lg.nx;
  const int total = ((int)g.nzl + 2) * P;
  for (int e = blockIdx.x * NTHREADS + threadIdx.x; e < total; e += gridDim.x * NTHREADS) {
    const int k = e / P - 1, r = e - (k + 1) * P;
    const int y = DIM == 3 ? r / nx : 0, x = DIM == 3 ? r - y * nx : r;
    lbuf[e] = lap_cell<DIM, ANI>(SJ, C, lg, k, y, x);
  }
}

// Cells of local planes [g.qa, g.qb); partials at part[c * nb + poff + blockIdx.x].
template <int DIM, int J, bool HZ, bool ANI>
__global__ __launch_bounds__(NTHREADS) void k_p2g(cplx *__restrict__ W, int64_t vs, Geo g,
                                                  const P2State *__restrict__ ps, cplx *__restrict__ part,
                                                  int nb, const cplx *__restrict__ lbuf, int poff) {
  constexpr int NC = (HZ ? 2 * (J + 1) + 3 : J + 2) + (J == 0 ? 1 : 0);
  // the combination coefficients by wave-uniform (scalar) loads at their use: staged in
  // LDS, the compiler hoisted them into 8 (J + 1) VGPRs
  const cplx *__restrict__ cX = ps->aX, *__restrict__ cZ = ps->aZ;
  const cplx bX1 = ps->bX1, bZ1 = ps->bZ1, bZ2 = ps->bZ2;
  const LGeo lg = lgeo(g);
  const double *C = g.cf;
  const int P = lg.P, nx = lg.nx;
  const cplx *L0 = lbuf + P;  // y at local plane 0
  cplx *__restrict__ Xo = W + (int64_t)(J + 1) * vs;
  cplx *__restrict__ Zo = W + (int64_t)(J + 2) * vs;
  const cplx zero = {0.0, 0.0};
  cplx acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = zero;
  const int e0 = g.qa * P, total = (g.qb - g.qa) * P;
  for (int e = blockIdx.x * NTHREADS + threadIdx.x; e < total; e += gridDim.x * NTHREADS) {
    const int flat = e0 + e, k = flat / P, r = flat - k * P;
    const int y = DIM == 3 ? r / nx : 0, x = DIM == 3 ? r - y * nx : r;
    const cplx l1 = L0[flat];
    cplx sv[J + 1];
#pragma unroll
    for (int l = 0; l < J; ++l) sv[l] = ld_nt(W + l * vs + flat);
    sv[J] = W[J * vs + flat];
    cplx Xa = cmul(bX1, l1), Xb = zero;
#pragma unroll
    for (int l = 0; l <= J; ++l) cmac((l & 1) ? Xb : Xa, cX[l], sv[l]);
    const cplx X = Xa + Xb;
    st_nt(Xo + flat, X);
#pragma unroll
    for (int l = 0; l <= J; ++l) cjmac(acc[l], sv[l], X);
    if constexpr (HZ) {
      const cplx l2 = lap_cell<DIM, ANI>(L0, C, lg, k, y, x);
      cplx Za = cmul(bZ2, l2) + cmul(bZ1, l1), Zb = zero;
#pragma unroll
      for (int l = 0; l <= J; ++l) cmac((l & 1) ? Zb : Za, cZ[l], sv[l]);
      const cplx Z = Za + Zb;
      st_nt(Zo + flat, Z);
#pragma unroll
      for (int l = 0; l <= J; ++l) cjmac(acc[J + 1 + l], sv[l], Z);
      acc[2 * J + 2].re = fma(X.re, X.re, fma(X.im, X.im, acc[2 * J + 2].re));
      cjmac(acc[2 * J + 3], X, Z);
      acc[2 * J + 4].re = fma(Z.re, Z.re, fma(Z.im, Z.im, acc[2 * J + 4].re));
    } else {
      acc[J + 1].re = fma(X.re, X.re, fma(X.im, X.im, acc[J + 1].re));
    }
    if constexpr (J == 0) acc[NC - 1].re = fma(sv[0].re, sv[0].re, fma(sv[0].im, sv[0].im, acc[NC - 1].re));
  }
  block_store<NC>(acc, part, nb, poff);
}

}  // namespace nls
