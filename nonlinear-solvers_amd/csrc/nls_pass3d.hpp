// nls_pass3d.hpp -- the three-vector basis pass k_p3d<J>: one read of S_0..S_J
// writes S_{J+1..J+3} (tests/sstep_model.py, the s-step schedule: J = 2 and 5 at
// m >= 10, single-rank handles).  It is k_p2d (nls_pass2d.hpp) one stencil level
// deeper; the coefficients come from k_p2coef with ns = 3:
//   X = bX1 L S_J + sum_l aX[l] S_l
//   Z = bZ2 L^2 S_J + bZ1 L S_J + sum_l aZ[l] S_l
//   Y = bY3 L^3 S_J + bY2 L^2 S_J + bY1 L S_J + sum_l aY[l] S_l
// and the sums S_l^H {X, Z, Y} and the Gram X^H X, X^H Z, X^H Y, Z^H Z, Z^H Y, Y^H Y.
//
// Tile and rings (one workgroup of 4 waves per CU, 64 x-cells x 4 rows, marching z):
//   S ring  S_J rows y0-3 .. y0+6 (10), 64 cells + 6 x-halo cells, NSL planes;
//           each wave DMAs 3 rows per plane (2w, 2w+1, and 8 + (w & 1), which
//           waves w and w+2 both load: same data, uniform op counts)
//   L ring  L S_J rows y0-2 .. y0+5 (8), 64 cells + 4 x-halo cells, 4 planes: step p
//           writes L(p+3) while it reads L(p .. p+2) for L^2(p+1), so one barrier
//           per step covers every ring
//   M ring  L^2 S_J rows y0-1 .. y0+4 (6), 2 planes (the y neighbours of L^3)
//   J ring  the J other stored vectors of the wave's row, NP planes (as k_p2d)
// Step p (outputs at plane p) computes L(p+3) (rows 2w, 2w+1 and their halo cells),
// L^2(p+1) (own row in a register queue with its two x-halo values, the edge rows
// for the M ring), and L^3(p) of the own row from the queue, the M ring and DPP
// lane shifts.  The pipeline starts P3_WU = 5 planes before the tile (no outputs;
// their J DMAs load the zero row), so every step issues the same ops and the
// s_waitcnt counts come from a compile-time replay of the issue order (p3_after).
#pragma once
#include "nls_pass2d.hpp"

namespace nls {

constexpr int P3_SR = 10;             // staged S_J rows (y0-3 .. y0+6)
constexpr int P3_SRW = 70;            // cells per staged S row: x0..x0+63, x0-3, x0-2, x0-1, x0+64, x0+65, x0+66
constexpr int P3_LR = 8;              // L S_J rows (y0-2 .. y0+5)
constexpr int P3_LRW = 68;            // cells per L row: x0..x0+63, x0-2, x0-1, x0+64, x0+65
constexpr int P3_MR = 6;              // L^2 S_J rows (y0-1 .. y0+4)
constexpr int P3_WU = 5;              // pipeline steps before the first output plane
constexpr int P3_NSD = 6;             // S DMAs per wave and plane (3 rows: main + halo)
constexpr int P3_STW = 3;             // stores per output step
#ifndef NLS_P3_DSA
#define NLS_P3_DSA 2                  // S look-ahead planes beyond the step's need
#endif
#ifndef NLS_P3_NP_MAX
#define NLS_P3_NP_MAX 5
#endif
constexpr int P3_DSP = NLS_P3_DSA + 2;                   // step i issues S plane i + DSP
constexpr int P3_NSL = NLS_P3_DSA + 4;                   // S slots (early issue)
constexpr int P3_SBYTES = P3_NSL * P3_SR * P3_SRW * 16;  // S ring
constexpr int P3_OFF_L = P3_SBYTES;
constexpr int P3_OFF_M = P3_OFF_L + 4 * P3_LR * P3_LRW * 16;
constexpr int P3_OFF_J = P3_OFF_M + 2 * P3_MR * 64 * 16;
__host__ __device__ constexpr int p3_avail(int J) { return P2D_LDS - P3_OFF_J - 3 * (J + 1) * 16; }
__host__ __device__ constexpr int p3_np(int J) {
  return p3_avail(J) / (P2D_TR * 1024 * J) < NLS_P3_NP_MAX ? p3_avail(J) / (P2D_TR * 1024 * J) : NLS_P3_NP_MAX;
}
__host__ __device__ constexpr int p3_off_c(int J) { return P3_OFF_J + p3_np(J) * J * P2D_TR * 1024; }
__host__ __device__ constexpr int p3_lds_bytes(int J) { return p3_off_c(J) + 3 * (J + 1) * 16; }
__host__ __device__ constexpr bool p3_rings_ok(int J) {
  return J >= 1 && p3_np(J) >= 2 && p3_lds_bytes(J) <= P2D_LDS;
}
static_assert(p3_rings_ok(2) && p3_rings_ok(5), "k_p3d rings do not fit the LDS");

// Replay of one wave's VMEM issue order: the prologue's S groups 0 .. DSP-1 and J
// groups 0 .. NP-2, then per step i: S group i+DSP, J group i+NP-1, WAIT(i), the
// stores (output steps only).  WAIT(i) needs S group i+2 and J group i; returns the
// ops issued after the last of them.
__host__ __device__ constexpr int p3_after(int J, int i) {
  const int NP = p3_np(J);
  int cnt = 0, lastS = 0, lastJ = 0;
  for (int n = 0; n < P3_DSP; ++n) {
    cnt += P3_NSD;
    if (n == i + 2) lastS = cnt;
  }
  for (int nj = 0; nj + 1 < NP; ++nj) {
    cnt += J;
    if (nj == i) lastJ = cnt;
  }
  for (int s = 0; s <= i; ++s) {
    cnt += P3_NSD;
    if (s + P3_DSP == i + 2) lastS = cnt;
    cnt += J;
    if (s + NP - 1 == i) lastJ = cnt;
    if (s == i) break;
    cnt += s >= P3_WU ? P3_STW : 0;
  }
  return cnt - (lastS > lastJ ? lastS : lastJ);
}
constexpr int P3_I0 = P3_WU + P3_DSP + NLS_P3_NP_MAX + 2;  // periodic from here
static_assert(p3_after(2, P3_I0) == p3_after(2, P3_I0 + 7) && p3_after(5, P3_I0) == p3_after(5, P3_I0 + 7),
              "k_p3d wait counts not periodic");
template <int J, int I = 0> __device__ __forceinline__ void p3_wait(int i) {
  if constexpr (I >= P3_I0) {
    wait_vm<p3_after(J, I)>();
  } else {
    if (i == I) {
      wait_vm<p3_after(J, I)>();
      return;
    }
    p3_wait<J, I + 1>(i);
  }
}

// L of one cell from three staged planes (row stride rw cells): centre ci, x
// neighbours mi / pi (absent at the grid's x edges), y neighbours ci -/+ rw
__device__ __forceinline__ cplx p3_lap(const cplx *Pm, const cplx *Pc, const cplx *Pp, int rw, int ci, int mi,
                                       int pi, bool hm, bool hp, double dg, double s, bool ok) {
  const cplx c = Pc[ci];
  const cplx xm = hm ? Pc[mi] : cplx{0.0, 0.0};
  const cplx xp = hp ? Pc[pi] : cplx{0.0, 0.0};
  const cplx ym = Pc[ci - rw], yp = Pc[ci + rw];
  const cplx zm = Pm[ci], zp = Pp[ci];
  const cplx v = dg * c + s * (((zm + zp) + (xm + xp)) + (ym + yp));
  return ok ? v : cplx{0.0, 0.0};
}

template <int J>
__global__ __launch_bounds__(NTHREADS, 1) void k_p3d(cplx *__restrict__ W, int64_t vs, Geo g,
                                                     const P2State *__restrict__ ps, cplx *__restrict__ part,
                                                     int nb, const cplx *__restrict__ zbuf, int poff) {
  static_assert(p3_rings_ok(J), "rings exceed LDS");
  constexpr int NP = p3_np(J);
  constexpr int NC = 3 * (J + 1) + 6;
  __shared__ __attribute__((aligned(16))) char smem[p3_lds_bytes(J)];
  const cplx *Sr = reinterpret_cast<const cplx *>(smem);         // [NSL][10][70]
  cplx *Lr = reinterpret_cast<cplx *>(smem + P3_OFF_L);          // [4][8][68]
  cplx *Mr = reinterpret_cast<cplx *>(smem + P3_OFF_M);          // [2][6][64]
  cplx *cX = reinterpret_cast<cplx *>(smem + p3_off_c(J));       // [J+1] x 3
  cplx *cZ = cX + (J + 1), *cY = cZ + (J + 1);
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nx = (int)g.nx, ny = (int)g.nyp, P = (int)g.P, nz = (int)g.npl;
  const int ntx = (nx + P2D_XO - 1) / P2D_XO, nty = ny / P2D_TR;
  const int qa = g.qa, qb = g.qb;
  const int nzc = (qb - qa + g.kz - 1) / g.kz;
  const int ntiles = ntx * nty * nzc;
  const int b = blockIdx.x, T8 = ntiles / 8;
  const int tile = b < 8 * T8 ? (b % 8) * T8 + b / 8 : b;  // XCD-banded (as k_p2d)
  const int yt = tile % nty, rest = tile / nty, xt = rest % ntx, zc = rest / ntx;
  const int x0 = xt * P2D_XO, y0 = yt * P2D_TR;
  const int k0 = qa + zc * g.kz, k1 = min(k0 + g.kz, qb);
  const int x = x0 + lane;
  const bool xin = x < nx;
  const bool full = x0 + P2D_XO <= nx;
  const int src_lane = xin ? lane : nx - 1 - x0;
  const int y = y0 + w;
  for (int l = t; l <= J; l += NTHREADS) {
    cX[l] = ps->aX[l];
    cZ[l] = ps->aZ[l];
    cY[l] = ps->aY[l];
  }
  const cplx bX1 = ps->bX1, bZ1 = ps->bZ1, bZ2 = ps->bZ2, bY1 = ps->bY1, bY2 = ps->bY2, bY3 = ps->bY3;
  const double s = g.s, sdi = g.sd_in, sdb = g.sd_bd;
  const int64_t P16 = (int64_t)P * 16;
  const char *__restrict__ SJb = reinterpret_cast<const char *>(W + (int64_t)J * vs);
  cplx *__restrict__ Xo = W + (int64_t)(J + 1) * vs;
  cplx *__restrict__ Zo = W + (int64_t)(J + 2) * vs;
  cplx *__restrict__ Yo = W + (int64_t)(J + 3) * vs;
  __syncthreads();

  auto clampx = [nx](int v) { return v < 0 ? 0 : (v >= nx ? nx - 1 : v); };
  const uint32_t xoff = (uint32_t)clampx(x) * 16u;
  // halo piece of a staged S row: lanes 0..23, dword lane&3 of cell hc = lane>>2 of
  // x0-3, x0-2, x0-1, x0+64, x0+65, x0+66
  const int hc = (lane >> 2) < 6 ? (lane >> 2) : 5;
  const uint32_t hoff = (uint32_t)clampx(hc < 3 ? x0 - 3 + hc : x0 + 61 + hc) * 16u + (uint32_t)(lane & 3) * 4u;
  // L from S (main lanes): x neighbours lane-1 / lane+1, the tile edges from the halo
  const int smi = lane > 0 ? lane - 1 : 66, spi = lane < 63 ? lane + 1 : 67;
  // L halo cells (extra pass, lanes 0..7: L row 2w + (lane >> 2), cell lane & 3 of
  // x0-2, x0-1, x0+64, x0+65; S row indices: centre / minus / plus)
  const int lh = lane & 3;
  const int lhx = lh == 0 ? x0 - 2 : (lh == 1 ? x0 - 1 : (lh == 2 ? x0 + 64 : x0 + 65));
  const int lhc = 65 + lh, lhm = lh == 0 ? 64 : (lh == 1 ? 65 : (lh == 2 ? 63 : 67));
  const int lhp = lh == 0 ? 66 : (lh == 1 ? 0 : (lh == 2 ? 68 : 69));
  // L^2 from L (main lanes): x neighbours, tile edges from the L halo (x0-1 at 65, x0+64 at 66)
  const int lmi = lane > 0 ? lane - 1 : 65, lpi = lane < 63 ? lane + 1 : 66;
  // L^2 halo values of the own row (lanes 0 / 1: x0-1 / x0+64)
  const int ex = lane == 1 ? x0 + 64 : x0 - 1;
  const int eci = lane == 1 ? 66 : 65, emi = lane == 1 ? 63 : 64, epi = lane == 1 ? 67 : 0;
#define P3_PLANE(p, yy) ((yy) < 0 ? (p) - 1 : ((yy) >= ny ? (p) + 1 : (p)))
#define P3_ROW(yy) ((yy) < 0 ? (yy) + ny : ((yy) >= ny ? (yy) - ny : (yy)))
#define P3_DIAG(xx, j, kk) \
  ((((xx) == 0) | ((xx) == nx - 1) | ((j) == 0) | ((j) == ny - 1) | ((kk) == 0) | ((kk) == nz - 1)) ? sdb : sdi)
  // DMA S_J rows 2w, 2w+1, 8 + (w & 1) of plane p into S slot sl (zero row outside
  // the grid and past the last plane a tile needs, k1 + 2)
#define P3_ISSUE_S(p, sl)                                                                  \
  do {                                                                                     \
    const int p_ = (p);                                                                    \
    _Pragma("unroll") for (int r_ = 0; r_ < 3; ++r_) {                                     \
      const int tr_ = r_ < 2 ? 2 * w + r_ : 8 + (w & 1);                                   \
      const int yy_ = y0 - 3 + tr_, kk_ = P3_PLANE(p_, yy_);                               \
      const bool ok_ = kk_ >= 0 && kk_ < nz && p_ <= k1 + 2;                               \
      const char *b_ = ok_ ? SJb + (p_ * P16 + (int64_t)yy_ * nx * 16)                     \
                           : reinterpret_cast<const char *>(zbuf);                         \
      char *dst_ = smem + (((sl) * P3_SR + tr_) * P3_SRW) * 16;                            \
      dma16(b_, xoff, dst_, 0);                                                            \
      if (lane < 24) dma4(b_, hoff, dst_ + 1024);                                          \
    }                                                                                      \
  } while (0)
  const char *sb[J];
#pragma unroll
  for (int l = 0; l < J; ++l) sb[l] = reinterpret_cast<const char *>(W + l * vs) + (int64_t)y * nx * 16;
#define P3_ISSUE_J(p, sl)                                                                  \
  do {                                                                                     \
    const int p_ = (p);                                                                    \
    const int64_t po_ = p_ * P16;                                                          \
    char *dst_ = smem + P3_OFF_J + (((sl) * J) * P2D_TR + w) * 1024;                       \
    _Pragma("unroll") for (int l_ = 0; l_ < J; ++l_) {                                     \
      const void *b_ = (p_ >= k0 && p_ < k1) ? (const void *)(sb[l_] + po_) : (const void *)zbuf; \
      dma16(b_, xoff, dst_ + l_ * P2D_TR * 1024, 1);                                       \
    }                                                                                      \
  } while (0)

  cplx acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = {0.0, 0.0};
  const int kw = k0 - P3_WU;  // plane of step 0
  // S plane n (global kw + n - 1... ): step i reads S planes p+2 .. p+4 = n i .. i+2
#define P3_SPLANE(n) (kw + 2 + (n))
#pragma unroll
  for (int n = 0; n < P3_DSP; ++n) P3_ISSUE_S(P3_SPLANE(n), n);
#pragma unroll
  for (int d = 0; d + 1 < NP; ++d) P3_ISSUE_J(kw + d, d);
  int sa = 0;                       // S slot of step i's first plane (n = i)
  int sis = P3_DSP % P3_NSL;        // S slot of the next issued plane
  int jr = 0, jis = NP - 1;         // J slots: plane p, next issued
  int lb = 0;                       // L ring slot of L(p)
  int mb = 0;                       // M ring slot of L^2(p)
  cplx mq0 = {0.0, 0.0}, mq1 = {0.0, 0.0}, me1 = {0.0, 0.0};  // L^2(p-1), L^2(p) own row; L^2(p) halo
  cplx sq0 = {0.0, 0.0}, sq1 = {0.0, 0.0}, sq2 = {0.0, 0.0}, sq3 = {0.0, 0.0};  // S_J(p .. p+3) own row
  const int nsteps = k1 - kw;
  for (int i = 0; i < nsteps; ++i) {
    const int p = kw + i;
    P3_ISSUE_S(P3_SPLANE(i + P3_DSP), sis);
    P3_ISSUE_J(p + NP - 1, jis);
    p3_wait<J>(i);
    raw_barrier();
    const int sb1 = sa + 1 == P3_NSL ? 0 : sa + 1, sb2 = sb1 + 1 == P3_NSL ? 0 : sb1 + 1;
    const cplx *S0 = Sr + sa * P3_SR * P3_SRW, *S1 = Sr + sb1 * P3_SR * P3_SRW, *S2 = Sr + sb2 * P3_SR * P3_SRW;
    // ---- L(p+3): L rows 2w, 2w+1 (S centre rows 2w+1, 2w+2) and their halo cells
    {
      const int pl = p + 3;
      cplx *Ld = Lr + ((lb + 3) & 3) * P3_LR * P3_LRW;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int lr = 2 * w + r, yy = y0 - 2 + lr, kk = P3_PLANE(pl, yy);
        const int so = (lr + 1) * P3_SRW;
        const cplx v = p3_lap(S0 + so, S1 + so, S2 + so, P3_SRW, lane, smi, spi, x > 0, x + 1 < nx,
                              P3_DIAG(x, P3_ROW(yy), kk), s, xin && kk >= 0 && kk < nz);
        Ld[lr * P3_LRW + lane] = v;
      }
      if (lane < 8) {
        const int lr = 2 * w + (lane >> 2), yy = y0 - 2 + lr, kk = P3_PLANE(pl, yy);
        const int so = (lr + 1) * P3_SRW;
        const cplx v = p3_lap(S0 + so, S1 + so, S2 + so, P3_SRW, lhc, lhm, lhp, lhx > 0, lhx + 1 < nx,
                              P3_DIAG(lhx, P3_ROW(yy), kk), s, lhx >= 0 && lhx < nx && kk >= 0 && kk < nz);
        Ld[lr * P3_LRW + 64 + lh] = v;
      }
    }
    // the own row of S_J(p+4) (S centre row w+3 of plane n = i+2) into the queue
    const cplx snew = S2[(w + 3) * P3_SRW + lane];
    // ---- L^2(p+1) from L(p), L(p+1), L(p+2): own row (register + M ring), halo values,
    // the edge rows (wave 0: y0-1, wave 3: y0+4)
    cplx mn, men;
    {
      const int pl = p + 1;
      const cplx *L0 = Lr + lb * P3_LR * P3_LRW, *L1 = Lr + ((lb + 1) & 3) * P3_LR * P3_LRW,
                 *L2 = Lr + ((lb + 2) & 3) * P3_LR * P3_LRW;
      cplx *Md = Mr + (mb ^ 1) * P3_MR * 64;
      {
        const int lo = (w + 2) * P3_LRW;
        mn = p3_lap(L0 + lo, L1 + lo, L2 + lo, P3_LRW, lane, lmi, lpi, x > 0, x + 1 < nx,
                    P3_DIAG(x, y, pl), s, xin && pl >= 0 && pl < nz);
        Md[(w + 1) * 64 + lane] = mn;
        men = {0.0, 0.0};
        if (lane < 2)
          men = p3_lap(L0 + lo, L1 + lo, L2 + lo, P3_LRW, eci, emi, epi, ex > 0, ex + 1 < nx,
                       P3_DIAG(ex, y, pl), s, ex >= 0 && ex < nx && pl >= 0 && pl < nz);
      }
      if (w == 0 || w == P2D_TR - 1) {
        const int q = w == 0 ? 0 : P3_MR - 1, yy = y0 - 1 + q, kk = P3_PLANE(pl, yy);
        const int lo = (q + 1) * P3_LRW;
        Md[q * 64 + lane] = p3_lap(L0 + lo, L1 + lo, L2 + lo, P3_LRW, lane, lmi, lpi, x > 0, x + 1 < nx,
                                   P3_DIAG(x, P3_ROW(yy), kk), s, xin && kk >= 0 && kk < nz);
      }
    }
    // ---- outputs at plane p
    if (i >= P3_WU) {
      const cplx l1 = Lr[(lb * P3_LR + w + 2) * P3_LRW + lane];  // L S_J(p), own row
      const cplx l2 = mq1;                                       // L^2 S_J(p)
      cplx xm = lane_prev(l2), xp = lane_next(l2);
      const cplx er = {__hiloint2double(__builtin_amdgcn_readlane(__double2hiint(me1.re), 1),
                                        __builtin_amdgcn_readlane(__double2loint(me1.re), 1)),
                       __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(me1.im), 1),
                                        __builtin_amdgcn_readlane(__double2loint(me1.im), 1))};
      if (lane == 0) xm = me1;
      if (lane == 63) xp = er;
      const cplx ym = Mr[(mb * P3_MR + w) * 64 + lane], yp = Mr[(mb * P3_MR + w + 2) * 64 + lane];
      const cplx l3 = P3_DIAG(x, y, p) * l2 + s * (((mq0 + mn) + (xm + xp)) + (ym + yp));
      cplx sv[J + 1];
      {
        const cplx *jv = reinterpret_cast<const cplx *>(smem + P3_OFF_J + ((jr * J) * P2D_TR + w) * 1024);
#pragma unroll
        for (int l = 0; l < J; ++l) sv[l] = jv[l * P2D_TR * 64 + lane];
      }
      sv[J] = sq0;
      cplx Xa = cmul(bX1, l1), Xb = {0.0, 0.0};
      cplx Za = cmul(bZ2, l2) + cmul(bZ1, l1), Zb = {0.0, 0.0};
      cplx Ya = cmul(bY3, l3) + cmul(bY2, l2), Yb = cmul(bY1, l1);
#pragma unroll
      for (int l = 0; l <= J; ++l) {
        cmac((l & 1) ? Xb : Xa, cX[l], sv[l]);
        cmac((l & 1) ? Zb : Za, cZ[l], sv[l]);
        cmac((l & 1) ? Yb : Ya, cY[l], sv[l]);
      }
      const cplx X = Xa + Xb, Z = Za + Zb, Y = Ya + Yb;
      const int flat = p * P + y * nx + x0 + src_lane;
      if (full) {
        st_nt(Xo + flat, X);
        st_nt(Zo + flat, Z);
        st_nt(Yo + flat, Y);
      } else {
        st_nt(Xo + flat, cplx{__shfl(X.re, src_lane, 64), __shfl(X.im, src_lane, 64)});
        st_nt(Zo + flat, cplx{__shfl(Z.re, src_lane, 64), __shfl(Z.im, src_lane, 64)});
        st_nt(Yo + flat, cplx{__shfl(Y.re, src_lane, 64), __shfl(Y.im, src_lane, 64)});
      }
      if (xin) {
#pragma unroll
        for (int l = 0; l <= J; ++l) {
          cjmac(acc[l], sv[l], X);
          cjmac(acc[J + 1 + l], sv[l], Z);
          cjmac(acc[2 * J + 2 + l], sv[l], Y);
        }
        constexpr int o = 3 * J + 3;
        acc[o].re = fma(X.re, X.re, fma(X.im, X.im, acc[o].re));
        cjmac(acc[o + 1], X, Z);
        cjmac(acc[o + 2], X, Y);
        acc[o + 3].re = fma(Z.re, Z.re, fma(Z.im, Z.im, acc[o + 3].re));
        cjmac(acc[o + 4], Z, Y);
        acc[o + 5].re = fma(Y.re, Y.re, fma(Y.im, Y.im, acc[o + 5].re));
      }
    }
    mq0 = mq1;
    mq1 = mn;
    me1 = men;
    sq0 = sq1;
    sq1 = sq2;
    sq2 = sq3;
    sq3 = snew;
    sa = sb1;
    sis = sis + 1 == P3_NSL ? 0 : sis + 1;
    jr = jr + 1 == NP ? 0 : jr + 1;
    jis = jis + 1 == NP ? 0 : jis + 1;
    lb = (lb + 1) & 3;
    mb ^= 1;
  }
#undef P3_PLANE
#undef P3_ROW
#undef P3_DIAG
#undef P3_ISSUE_S
#undef P3_ISSUE_J
#undef P3_SPLANE
  wait_vm<0>();
  raw_barrier();
  cplx *red = reinterpret_cast<cplx *>(smem);  // [4][NC]
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const double a = wave_sum(acc[c].re), bb = wave_sum(acc[c].im);
    if (lane == 0) red[w * NC + c] = {a, bb};
  }
  __syncthreads();
  for (int c = t; c < NC; c += NTHREADS) {
    cplx v = red[c];
#pragma unroll
    for (int q = 1; q < P2D_TR; ++q) v += red[q * NC + c];
    part[(int64_t)c * nb + poff + blockIdx.x] = v;
  }
}

}  // namespace nls
