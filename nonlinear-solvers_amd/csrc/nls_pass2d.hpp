// nls_pass2d.hpp -- the two-vector basis pass with LDS-DMA staging (k_p2d), the
// form the two-vectors-per-pass Lanczos runs by default.  Scheme, coefficients
// and the per-cell formulas: nls_pass2.hpp (P2State, k_p2coef) and DESIGN.md §3.
//
// Why a new form: the pass holds 2(J+1)+3 complex accumulators per lane, so
// with the streamed S_l in VGPRs it runs at one wave per SIMD with too few
// bytes in flight (the register-march k_pass2r streamed at ~55 % of the
// pattern's rate).  Here every byte the pass reads moves HBM -> LDS by
// global_load_lds_dwordx4 (1 KiB per wave-instruction, no VGPR destination),
// issued D planes ahead of its use, so the in-flight bytes no longer compete
// with the accumulators for registers:
//
//   workgroup = 4 waves = one tile of 60 x-cells x 4 rows (one row per wave),
//               marched over kz planes; one workgroup per CU (LDS-bound).
//   S ring:     S_J rows y0-2 .. y0+5 of D+3 planes (shared by the 4 waves;
//               each wave DMAs 2 rows of each plane).  L S_J of the next plane
//               is computed from it for the wave's rows -1, 0, +1 and kept in a
//               register queue (3 planes), L^2 S_J of the current plane from
//               that queue (x neighbours by lane shuffles).
//   J ring:     the J other stored vectors S_0..S_{J-1} of the wave's row,
//               D+1 planes per wave (private to the wave).
//   lanes:      x = x0 - 2 + lane; lanes 2..61 are outputs (L S_J valid on
//               1..62, L^2 S_J on 2..61).
//
// Completion is counted by hand (hipcc does not track LDS-DMA writes): every
// wave issues, per step, exactly one group of J + 2 DMAs (its 2 S rows of
// plane k+D+2, its J rows of plane k+D) followed by STW (1 or 2) stores, so
// the group a step needs is retired by a constant s_waitcnt vmcnt(N_i)
// (N_i below); groups beyond the tile's planes DMA a zero block instead, and
// stores from non-output lanes duplicate an output lane's store (same value,
// same address), so no instruction is ever skipped by an all-false branch.
// A raw s_barrier after the wait publishes the other waves' S rows.
#pragma once
#include "nls_pass2.hpp"

namespace nls {

constexpr int P2D_XO = 60;            // output x per wave
constexpr int P2D_TR = 4;             // rows per tile (one per wave)
constexpr int P2D_SR = P2D_TR + 4;    // S_J rows staged per plane (y0-2 .. y0+5)
constexpr int P2D_JMAX = 14;          // largest J whose rings fit 160 KiB of LDS
__host__ __device__ constexpr int p2d_depth(int J) {  // planes of DMA lookahead
  return J >= 8 ? 1 : J >= 6 ? 2 : J >= 4 ? 3 : J >= 2 ? 4 : 6;
}
__host__ __device__ constexpr int p2d_nsl(int J) { return p2d_depth(J) + 3; }
__host__ __device__ constexpr int p2d_nj(int J) { return p2d_depth(J) + 1; }
// byte offsets inside the one LDS array
__host__ __device__ constexpr int p2d_off_j(int J) { return p2d_nsl(J) * P2D_SR * 64 * 16; }
__host__ __device__ constexpr int p2d_off_c(int J) { return p2d_off_j(J) + p2d_nj(J) * P2D_TR * (J > 0 ? J : 1) * 64 * 16; }
__host__ __device__ constexpr int p2d_lds_bytes(int J) { return p2d_off_c(J) + 2 * (J + 1) * 16; }

__device__ __forceinline__ void dma16(const cplx *g, char *lds, unsigned aux) {
  if (aux) __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 16, 0, 2);
  else __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}
template <int N> __device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait for the group issued for step i: N_i = NB + STW * min(i, D)
template <int NB, int STW, int D, int I = 0> __device__ __forceinline__ void wait_group(int i) {
  if constexpr (I >= D) {
    wait_vm<NB + STW * D>();
  } else {
    if (i == I) {
      wait_vm<NB + STW * I>();
      return;
    }
    wait_group<NB, STW, D, I + 1>(i);
  }
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int J, bool HZ>
__global__ __launch_bounds__(NTHREADS, 1) void k_p2d(cplx *__restrict__ W, int64_t vs, Geo g,
                                                     const P2State *__restrict__ ps,
                                                     cplx *__restrict__ part, int nb,
                                                     const cplx *__restrict__ zbuf) {
  static_assert(J <= P2D_JMAX, "rings exceed LDS");
  constexpr int D = p2d_depth(J), NSL = p2d_nsl(J), NJ = p2d_nj(J);
  constexpr int STW = HZ ? 2 : 1;           // stores per step
  constexpr int NB = (D - 1) * (J + 2);     // DMAs of the groups issued after the awaited one
  constexpr int NC = HZ ? 2 * (J + 1) + 3 : J + 2;
  constexpr int JS = J > 0 ? J : 1;
  __shared__ __attribute__((aligned(16))) char smem[p2d_lds_bytes(J)];
  cplx *Sr = reinterpret_cast<cplx *>(smem);                    // [NSL][P2D_SR][64]
  cplx *Jr = reinterpret_cast<cplx *>(smem + p2d_off_j(J));     // [NJ][4][JS][64]
  cplx *cX = reinterpret_cast<cplx *>(smem + p2d_off_c(J));     // [J+1]
  cplx *cZ = cX + (J + 1);                                      // [J+1]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nx = (int)g.nx, ny = (int)g.nyp, P = (int)g.P, nz = (int)g.npl;
  const int ntx = (nx + P2D_XO - 1) / P2D_XO, nty = ny / P2D_TR;
  const int nzc = (nz + g.kz - 1) / g.kz;
  const int ntiles = ntx * nty * nzc;
  // XCD-banded order: the 8 XCDs take contiguous tile ranges, so the y-adjacent
  // tiles sharing S_J halo rows run on one XCD (its L2) at the same time
  const int b = blockIdx.x, T8 = ntiles / 8;
  const int tile = b < 8 * T8 ? (b % 8) * T8 + b / 8 : b;
  const int yt = tile % nty, rest = tile / nty, xt = rest % ntx, zc = rest / ntx;
  const int x0 = xt * P2D_XO, y0 = yt * P2D_TR;
  const int k0 = zc * g.kz, k1 = min(k0 + g.kz, nz);
  const int x = x0 - 2 + lane;
  const bool xin = x >= 0 && x < nx;
  const int nvalid = min(P2D_XO, nx - x0);  // output lanes 2 .. nvalid+1
  const bool out = lane >= 2 && lane < 2 + nvalid;
  const int src_lane = lane < 2 ? 2 : (lane >= 2 + nvalid ? 1 + nvalid : lane);
  const int y = y0 + w;  // this wave's row (ny % 4 == 0: always a real row)

  for (int l = t; l <= J; l += NTHREADS) {
    cX[l] = ps->aX[l];
    cZ[l] = ps->aZ[l];
  }
  const cplx bX1 = ps->bX1, bZ1 = ps->bZ1, bZ2 = ps->bZ2;
  const double s = g.s, sdi = g.sd_in, sdb = g.sd_bd;
  const cplx *__restrict__ SJ = W + (int64_t)J * vs;
  cplx *__restrict__ Xo = W + (int64_t)(J + 1) * vs;
  cplx *__restrict__ Zo = W + (int64_t)(J + 2) * vs;
  __syncthreads();  // coefficients in LDS (no DMA in flight yet)

  // (no lambdas capturing by reference here: hipcc kept their captures on the
  // stack, and every scratch access is a VMEM op that breaks the vmcnt counting)
#define P2D_PLANE(p, yy) ((yy) < 0 ? (p) - 1 : ((yy) >= ny ? (p) + 1 : (p)))
#define P2D_ROW(yy) ((yy) < 0 ? (yy) + ny : ((yy) >= ny ? (yy) - ny : (yy)))
#define P2D_DIAG(j, kk) \
  ((xedge || (j) == 0 || (j) == ny - 1 || (kk) == 0 || (kk) == nz - 1) ? sdb : sdi)
#define P2D_SSLOT(p) (((p) - k0 + 2) % NSL)
  const bool xedge = x == 0 || x == nx - 1;
  // DMA this wave's two S_J rows of plane p (zero block past the tile's last needed plane)
#define P2D_ISSUE_S(p)                                                                  \
  do {                                                                                  \
    const int p_ = (p);                                                                 \
    char *dst_ = smem + (P2D_SSLOT(p_) * P2D_SR + 2 * w) * 1024;                        \
    _Pragma("unroll") for (int r_ = 0; r_ < 2; ++r_) {                                  \
      const int yy_ = y0 - 2 + 2 * w + r_, kk_ = P2D_PLANE(p_, yy_);                    \
      const bool ok_ = xin && kk_ >= 0 && kk_ < nz && p_ <= k1 + 1;                     \
      dma16(ok_ ? SJ + (p_ * P + yy_ * nx + x) : zbuf + lane, dst_ + r_ * 1024, 0);     \
    }                                                                                   \
  } while (0)
  // DMA the J stored vectors of this wave's row of plane p into J slot (i % NJ)
#define P2D_ISSUE_J(p, i)                                                               \
  do {                                                                                  \
    const int p_ = (p);                                                                 \
    char *dst_ = smem + p2d_off_j(J) + ((((i) % NJ) * P2D_TR + w) * JS) * 1024;          \
    const bool ok_ = out && p_ < k1;                                                    \
    const int off_ = ok_ ? p_ * P + y * nx + x : 0;                                     \
    _Pragma("unroll") for (int l_ = 0; l_ < J; ++l_)                                    \
      dma16(ok_ ? W + (l_ * vs + off_) : zbuf + lane, dst_ + l_ * 1024, 1);             \
  } while (0)
  const int lm = lane > 0 ? lane - 1 : 0, lp = lane < 63 ? lane + 1 : 63;
  // L S_J at plane p for S tile row tr (yy = y0 - 2 + tr), from ring planes p-1, p, p+1
#define P2D_LAP(dst, p, tr)                                                             \
  do {                                                                                  \
    const int p_ = (p), tr_ = (tr);                                                     \
    const cplx *Sm_ = Sr + P2D_SSLOT(p_ - 1) * (P2D_SR * 64);                           \
    const cplx *Sc_ = Sr + P2D_SSLOT(p_) * (P2D_SR * 64);                               \
    const cplx *Sp_ = Sr + P2D_SSLOT(p_ + 1) * (P2D_SR * 64);                           \
    const int yy_ = y0 - 2 + tr_, kk_ = P2D_PLANE(p_, yy_);                             \
    const cplx c_ = Sc_[tr_ * 64 + lane];                                               \
    const cplx xm_ = Sc_[tr_ * 64 + lm], xp_ = Sc_[tr_ * 64 + lp];                      \
    const cplx ym_ = Sc_[(tr_ - 1) * 64 + lane], yp_ = Sc_[(tr_ + 1) * 64 + lane];      \
    const cplx zm_ = Sm_[tr_ * 64 + lane], zp_ = Sp_[tr_ * 64 + lane];                  \
    const double dg_ = P2D_DIAG(P2D_ROW(yy_), kk_);                                     \
    const bool ok_ = xin && kk_ >= 0 && kk_ < nz;                                       \
    const cplx v_ = dg_ * c_ + s * (((zm_ + zp_) + (xm_ + xp_)) + (ym_ + yp_));         \
    dst = ok_ ? v_ : cplx{0.0, 0.0};                                                    \
  } while (0)

  cplx acc[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) acc[i] = {0.0, 0.0};

  // prologue: S planes k0-2 .. k0+1, L S_J of planes k0-1 (centre row) and k0
  for (int p = k0 - 2; p <= k0 + 1; ++p) P2D_ISSUE_S(p);
  wait_vm<0>();
  raw_barrier();
  cplx lq0;      // L S_J(k-1), centre row
  cplx lq1[3];   // L S_J(k), rows -1, 0, +1
  P2D_LAP(lq0, k0 - 1, w + 2);
#pragma unroll
  for (int r = 0; r < 3; ++r) P2D_LAP(lq1[r], k0, w + 1 + r);
  raw_barrier();  // every wave is done with the slot of plane k0-2
#pragma unroll
  for (int i = 0; i < D; ++i) {
    P2D_ISSUE_S(k0 + 2 + i);
    P2D_ISSUE_J(k0 + i, i);
  }

  for (int k = k0; k < k1; ++k) {
    const int i = k - k0;
    wait_group<NB, STW, D>(i);
    raw_barrier();
    P2D_ISSUE_S(k + D + 2);
    P2D_ISSUE_J(k + D, i + D);
    // L S_J of plane k+1, rows -1, 0, +1
    cplx ln[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) P2D_LAP(ln[r], k + 1, w + 1 + r);
    // the J stored vectors of this cell and S_J itself
    const cplx *jr = Jr + (((i % NJ) * P2D_TR + w) * JS) * 64;
    cplx sv[J + 1];
#pragma unroll
    for (int l = 0; l < J; ++l) sv[l] = jr[l * 64 + lane];
    sv[J] = Sr[(P2D_SSLOT(k) * P2D_SR + w + 2) * 64 + lane];
    const cplx l1 = lq1[1];
    cplx X = cmul(bX1, l1);
#pragma unroll
    for (int l = 0; l <= J; ++l) X += cmul(cX[l], sv[l]);
    cplx Z = {0.0, 0.0};
    if constexpr (HZ) {
      const cplx xm = shfl_up1(l1), xp = shfl_dn1(l1);  // zero outside [0, nx): L S_J = 0 there
      const cplx l2 = P2D_DIAG(y, k) * l1 + s * (((lq0 + ln[1]) + (xm + xp)) + (lq1[0] + lq1[2]));
      Z = cmul(bZ2, l2) + cmul(bZ1, l1);
#pragma unroll
      for (int l = 0; l <= J; ++l) Z += cmul(cZ[l], sv[l]);
    }
    // stores from every lane: non-output lanes repeat an output lane's store
    const int flat = k * P + y * nx + (x0 - 2 + src_lane);
    {
      const cplx Xs = {__shfl(X.re, src_lane, 64), __shfl(X.im, src_lane, 64)};
      st_nt(Xo + flat, Xs);
    }
    if constexpr (HZ) {
      const cplx Zs = {__shfl(Z.re, src_lane, 64), __shfl(Z.im, src_lane, 64)};
      st_nt(Zo + flat, Zs);
    }
    if (out) {
#pragma unroll
      for (int l = 0; l <= J; ++l) acc[l] += cj_mul(sv[l], X);
      if constexpr (HZ) {
#pragma unroll
        for (int l = 0; l <= J; ++l) acc[J + 1 + l] += cj_mul(sv[l], Z);
        acc[2 * J + 2].re += abs2(X);
        acc[2 * J + 3] += cj_mul(X, Z);
        acc[2 * J + 4].re += abs2(Z);
      } else {
        acc[J + 1].re += abs2(X);
      }
    }
    lq0 = lq1[1];
#pragma unroll
    for (int r = 0; r < 3; ++r) lq1[r] = ln[r];
  }
#undef P2D_PLANE
#undef P2D_ROW
#undef P2D_DIAG
#undef P2D_SSLOT
#undef P2D_ISSUE_S
#undef P2D_ISSUE_J
#undef P2D_LAP
  wait_vm<0>();  // the look-ahead DMAs land before the LDS is reused
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
    part[(int64_t)c * nb + blockIdx.x] = v;
  }
}

// ---- fused tail of the two-vector scheme ----------------------------------
// After the last basis pass the stored vectors are S_0..S_j (j = m-2) with
// W = S C orthonormal and the H columns < j known.  One k_alpha_l2 pass over
// S_j reduces a = S_j^H L S_j and l2 = ||L S_j||^2 (sums[0], sums[2]); with
// y = L S_j and D = C^-1 (ps->D):
//   t_k = W_k^H y = sum_i conj(H[i][k]) D[i][j]        (k < j)
//   t_j = conj(C_jj) (a - sum_{i<j} conj(D[i][j]) t_i)
//   lw  = -C_jj H[:, :j] D[:j, j]        (L W_j = C_jj y + sum_k lw_k W_k)
//   alpha_j = C_jj t_j + lw_j,  beta_{j+1} = |C_jj| sqrt(l2 - sum_k |t_k|^2)
//   W_{j+1} = C_jj (y - sum_k t_k W_k) / beta_{j+1}
// (tests/sstep_model.py tail_coefficients; 20-step trajectories at the
// headline stiffness within 1e-14 of the MGS oracle).  k_p2tail completes T
// (s[] = 1: k_reduce_final's fin is then f(T) e_1 in the W basis) and keeps
// t, beta in the P2State; k_p2tfin maps fin to the coefficients k_tail reads:
// fin'[k] over the stored S_k (k <= j), fin'[j+1] for y, coef = e_{j+1}.
__global__ __launch_bounds__(NTHREADS) void k_p2tail(P2State *__restrict__ ps, KState *__restrict__ st,
                                                     const cplx *__restrict__ sums, int m) {
  __shared__ cplx tk[P2M];
  const int j = m - 2, t = threadIdx.x;
  for (int k = t; k < j; k += NTHREADS) {
    cplx v = {0.0, 0.0};
    for (int i = 0; i <= k + 1 && i <= j; ++i) v += cj_mul(ps->H[i][k], ps->D[i][j]);
    tk[k] = v;
  }
  __syncthreads();
  if (t == 0) {
    const cplx cjj = ps->C[j][j];
    cplx r = sums[0];
    for (int i = 0; i < j; ++i) r = r - cj_mul(ps->D[i][j], tk[i]);
    const cplx tj = cj_mul(cjj, r);
    tk[j] = tj;
    cplx lwj = {0.0, 0.0};
    for (int i = (j > 0 ? j - 1 : 0); i < j; ++i) lwj += cmul(ps->H[j][i], ps->D[i][j]);
    lwj = cmul(cjj, lwj);
    const double alpha = cmul(cjj, tj).re - lwj.re;
    double n2 = sums[2].re;
    for (int k = 0; k <= j; ++k) n2 -= abs2(tk[k]);
    const double b = sqrt(abs2(cjj)) * (n2 > 0.0 ? sqrt(n2) : 0.0);
    ps->beta_t = b;
    st->Td[j] = alpha;
    st->To[j] = b;
    if (!(b > 0.0) && st->breakdown == 0) st->breakdown = m;
  }
  __syncthreads();
  for (int k = t; k <= j; k += NTHREADS) ps->tk[k] = tk[k];
  if (t < MMAX) {
    if (t < j) {
      st->Td[t] = ps->H[t][t].re;
      st->To[t] = ps->H[t + 1][t].re;
    }
    st->s[t] = 1.0;
  }
}

__global__ __launch_bounds__(NTHREADS) void k_p2tfin(const P2State *__restrict__ ps,
                                                     KState *__restrict__ st, int m, int nf) {
  __shared__ cplx fw[2][MMAX];
  const int j = m - 2, t = threadIdx.x;
  for (int e = t; e < nf * m; e += NTHREADS) fw[e / m][e % m] = st->fin[e / m][e % m];
  __syncthreads();
  const cplx cjj = ps->C[j][j];
  const double b = ps->beta_t, ib = b > 0.0 ? 1.0 / b : 0.0;
  for (int e = t; e < nf * (j + 2); e += NTHREADS) {
    const int f = e / (j + 2), l = e % (j + 2);
    const cplx cl = fw[f][j + 1];  // coefficient of W_{j+1}
    const cplx g = ib * cmul(cl, cjj);
    cplx v = {0.0, 0.0};
    if (l <= j) {
      // sum_{k >= l} C[l][k] (fin_k - g t_k)
      for (int k = l; k <= j; ++k) v += cmul(ps->C[l][k], fw[f][k] - cmul(g, ps->tk[k]));
    } else {
      v = g;
    }
    st->fin[f][l] = ps->beta * v;
  }
  for (int l = t; l <= j + 1; l += NTHREADS) st->coef[l] = {l == j + 1 ? 1.0 : 0.0, 0.0};
}

}  // namespace nls
