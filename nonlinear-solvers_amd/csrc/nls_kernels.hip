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
// (laplacians.hpp:10-105): per point, the column's z (3D) / y (2D)
// neighbours come from a register queue while the workgroup marches along the
// slowest dimension; x and (3D) y neighbours are neighbouring lanes' loads
// served from L1/L2.  The 3D "y-wrap" (i,ny-1,k)<->(i,0,k+1) falls out of
// flat-index neighbours p +- nx over contiguous plane storage.
#include <utility>

#include "nls_device.hpp"
#include "nls_kernels.hpp"

namespace nls {

template <class S> __device__ __forceinline__ S from_real(double v);
template <> __device__ __forceinline__ double from_real<double>(double v) { return v; }
template <> __device__ __forceinline__ cplx from_real<cplx>(double v) { return {v, 0.0}; }

// ---------------------------------------------------------------------------
// wave64 + workgroup reduction into one partial per workgroup (fixed order:
// results are bitwise reproducible run to run)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// partials are stored column-major: out[k * gridDim.x + blockIdx.x], so the
// single-workgroup reduction reads each column with coalesced 1 KiB wave loads.
template <int NA>
__device__ __forceinline__ void block_store(cplx (&v)[NA], cplx *__restrict__ out) {
  __shared__ cplx red[NTHREADS / 64][NA];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    v[k].re = wave_sum(v[k].re);
    v[k].im = wave_sum(v[k].im);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NA; ++k) red[w][k] = v[k];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < NA; k += NTHREADS) {
    cplx s = red[0][k];
#pragma unroll
    for (int q = 1; q < NTHREADS / 64; ++q) s += red[q][k];
    out[(int64_t)k * gridDim.x + blockIdx.x] = s;
  }
}

// ---------------------------------------------------------------------------
// memory helpers: basis vectors streamed once per pass use non-temporal
// loads/stores (measured +5-10 % on 16-stream passes, tools/bw_probe.hip);
// the stencil vector keeps default policy (its neighbours are re-read).
typedef double v2d __attribute__((ext_vector_type(2)));
__device__ __forceinline__ cplx ld_nt(const cplx *p) {
  const v2d v = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p));
  return {v.x, v.y};
}
__device__ __forceinline__ double ld_nt(const double *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_nt(cplx *p, cplx v) {
  v2d t;
  t.x = v.re;
  t.y = v.im;
  __builtin_nontemporal_store(t, reinterpret_cast<v2d *>(p));
}
__device__ __forceinline__ void st_nt(double *p, double v) { __builtin_nontemporal_store(v, p); }

// wave64 cross-lane moves (ds_bpermute)
__device__ __forceinline__ double shfl_up1(double v) { return __shfl_up(v, 1, 64); }
__device__ __forceinline__ cplx shfl_up1(cplx v) { return {__shfl_up(v.re, 1, 64), __shfl_up(v.im, 1, 64)}; }
__device__ __forceinline__ double shfl_dn1(double v) { return __shfl_down(v, 1, 64); }
__device__ __forceinline__ cplx shfl_dn1(cplx v) { return {__shfl_down(v.re, 1, 64), __shfl_down(v.im, 1, 64)}; }
__device__ __forceinline__ double bcast(double v, int l) { return __shfl(v, l, 64); }
__device__ __forceinline__ cplx bcast(cplx v, int l) { return {__shfl(v.re, l, 64), __shfl(v.im, l, 64)}; }

// ---------------------------------------------------------------------------
// Tiling of the stencil kernels (256 threads = 4 wave64 per workgroup):
//   3D: tile = 64 x  *  4*RB y-rows  *  kz z-planes; wave w owns RB consecutive
//       rows, lane = x.  y-neighbours inside the wave's rows come from
//       registers, x-neighbours from the neighbouring lane (ds_bpermute).
//   2D: tile = 64*RB x  *  4*kz rows; wave w marches its own kz rows, each lane
//       owns RB x-positions 64 apart (x-neighbours across the 64-chunk seam
//       from the neighbouring chunk's lane 0/63).
// Both march along the slowest dimension with a (prev, cur, next) register
// queue, so every cell of the stencil vector is fetched from HBM once; only
// tile-edge neighbours (1 lane of 64, wave-boundary rows) use L1/L2 loads.
__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

template <int DIM, int RB> __host__ __device__ inline void tile_counts(const Geo &g, int64_t &ntx,
                                                                        int64_t &nty, int64_t &ntz) {
  if (DIM == 3) {
    ntx = cdiv(g.nx, 64);
    nty = cdiv(g.nyp, 4 * RB);
    ntz = cdiv(g.nzl, g.kz);
  } else {
    ntx = cdiv(g.nx, 64 * RB);
    nty = 1;
    ntz = cdiv(g.nzl, 4 * (int64_t)g.kz);
  }
}

// fn(p, cur, lap) for every local cell p of the workgroup's tiles, with
// cur = V[p] and lap = (L V)[p] (laplacians.hpp:10-105, flat-index form).
// Local indices are 32-bit (the host guarantees (nzl+2)*P < 2^31); the flat
// range tests of the reference (idx-nx >= 0, idx+nx < N) are evaluated on
// (plane, row) coordinates so they never need 64-bit global indices.
//
// PLANE = true: fn(p[RB], cur[RB], lap[RB], ok[RB]) is called once per plane
// with all rows of the thread, so the caller can issue every streamed load of
// all its rows before the first use (more loads in flight per accumulator set).
template <class S, int DIM, int RB, bool PLANE = false, class Fn>
__device__ __forceinline__ void march(const S *__restrict__ V, const Geo &g, Fn &&fn) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t ntx64, nty64, ntz64;
  tile_counts<DIM, RB>(g, ntx64, nty64, ntz64);
  const int ntx = (int)ntx64, nty = (int)nty64;
  const int tiles = (int)(ntx64 * nty64 * ntz64);
  const int T8 = tiles / 8;
  const int P = (int)g.P, nx = (int)g.nx, nyp = (int)g.nyp, nzl = (int)g.nzl, kz = g.kz;
  const int z0 = (int)g.z0, npl = (int)g.npl;
  for (int t0 = blockIdx.x; t0 < tiles; t0 += gridDim.x) {
    // optional XCD-banded order (workgroups b, b+8 share an XCD): speed only
    const int t = (g.remap && t0 < 8 * T8) ? (t0 % 8) * T8 + t0 / 8 : t0;
    const int it = t % ntx;
    const int rest = t / ntx;
    const int jt = rest % nty;
    const int kt = rest / nty;
    if constexpr (DIM == 3) {
      const int x = it * 64 + lane;
      const bool xin = x < nx;
      const int yb = jt * (4 * RB) + w * RB;
      if (yb >= nyp) continue;  // wave-uniform
      const int q0 = kt * kz;
      const int q1 = q0 + kz < nzl ? q0 + kz : nzl;
      bool rv[RB];
      int off[RB];
      S prev[RB], cur[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        rv[r] = yb + r < nyp;
        off[r] = (yb + r) * nx + x;
        const bool ld = xin && rv[r];
        prev[r] = (ld && z0 + q0 > 0) ? V[(q0 - 1) * P + off[r]] : zero<S>();
        cur[r] = ld ? V[q0 * P + off[r]] : zero<S>();
      }
      const bool bx = (x == 0) || (x == nx - 1);
      for (int q = q0; q < q1; ++q) {
        const int gq = z0 + q;
        const bool bz = gq == 0 || gq == npl - 1;
        const bool has_next = gq + 1 < npl;
        S next[RB], lapv[RB];
        int pv[RB];
        bool okv[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r)
          next[r] = (xin && rv[r] && has_next) ? V[(q + 1) * P + off[r]] : zero<S>();
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          pv[r] = q * P + off[r];
          okv[r] = false;
          lapv[r] = zero<S>();
          if (!rv[r]) continue;  // wave-uniform
          const int p = q * P + off[r];
          const int y = yb + r;
          S ym, yp;
          if (r > 0) ym = cur[r - 1];
          else ym = (xin && (gq > 0 || y > 0)) ? V[p - nx] : zero<S>();            // idx - nx >= 0
          if (r + 1 < RB && rv[r + 1 < RB ? r + 1 : r]) yp = cur[r + 1 < RB ? r + 1 : r];
          else yp = (xin && (gq < npl - 1 || y < nyp - 1)) ? V[p + nx] : zero<S>();  // idx + nx < N
          S xm = shfl_up1(cur[r]), xp = shfl_dn1(cur[r]);
          const S xe = ((lane == 0 && x > 0) || (lane == 63 && x + 1 < nx)) && xin
                           ? V[p + (lane == 0 ? -1 : 1)] : zero<S>();
          if (lane == 0) xm = xe;
          if (lane == 63) xp = xe;
          if (!(x > 0)) xm = zero<S>();
          if (!(x + 1 < nx)) xp = zero<S>();
          const bool bnd = bx || bz || y == 0 || y == nyp - 1;
          const S lap = g.s * (((prev[r] + next[r]) + (xm + xp)) + (ym + yp)) +
                        (bnd ? g.sd_bd : g.sd_in) * cur[r];
          if constexpr (PLANE) {
            okv[r] = xin;
            lapv[r] = lap;
          } else {
            if (xin) fn(p, cur[r], lap);
          }
        }
        if constexpr (PLANE) fn(pv, cur, lapv, okv);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          prev[r] = cur[r];
          cur[r] = next[r];
        }
      }
    } else {
      const int q0 = (kt * 4 + w) * kz;
      if (q0 >= nzl) continue;  // wave-uniform
      const int q1 = q0 + kz < nzl ? q0 + kz : nzl;
      int xr[RB];
      S prev[RB], cur[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        xr[r] = it * 64 * RB + 64 * r + lane;
        const bool ld = xr[r] < nx;
        prev[r] = (ld && z0 + q0 > 0) ? V[(q0 - 1) * P + xr[r]] : zero<S>();
        cur[r] = ld ? V[q0 * P + xr[r]] : zero<S>();
      }
      for (int q = q0; q < q1; ++q) {
        const int gq = z0 + q;
        const bool bz = gq == 0 || gq == npl - 1;
        const bool has_next = gq + 1 < npl;
        S next[RB], lapv[RB];
        int pv[RB];
        bool okv[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r)
          next[r] = (xr[r] < nx && has_next) ? V[(q + 1) * P + xr[r]] : zero<S>();
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int x = xr[r];
          const int p = q * P + x;
          pv[r] = p;
          S xm = shfl_up1(cur[r]), xp = shfl_dn1(cur[r]);
          const S cm = bcast(cur[r > 0 ? r - 1 : 0], 63);
          const S cp = bcast(cur[r + 1 < RB ? r + 1 : r], 0);
          const bool edge_ld = (lane == 0 && r == 0 && x < nx && x > 0) ||
                               (lane == 63 && r + 1 == RB && x + 1 < nx);
          const S xe = edge_ld ? V[p + (lane == 0 ? -1 : 1)] : zero<S>();
          if (lane == 0) xm = r > 0 ? cm : xe;
          if (lane == 63) xp = r + 1 < RB ? cp : xe;
          if (!(x > 0)) xm = zero<S>();
          if (!(x + 1 < nx)) xp = zero<S>();
          const bool bnd = x == 0 || x == nx - 1 || bz;
          const S lap = g.s * ((prev[r] + next[r]) + (xm + xp)) + (bnd ? g.sd_bd : g.sd_in) * cur[r];
          if constexpr (PLANE) {
            okv[r] = x < nx;
            lapv[r] = lap;
          } else {
            if (x < nx) fn(p, cur[r], lap);
          }
        }
        if constexpr (PLANE) fn(pv, cur, lapv, okv);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          prev[r] = cur[r];
          cur[r] = next[r];
        }
      }
    }
  }
}

#ifndef NLS_UPD_RB_MODE
#define NLS_UPD_RB_MODE 1
#endif
#ifndef NLS_COEF_LDS
#define NLS_COEF_LDS 1
#endif
__host__ __device__ constexpr int upd_rb(int J) {
  return NLS_UPD_RB_MODE == 0 ? (J <= 2 ? 4 : (J <= 6 ? 2 : 1))
       : NLS_UPD_RB_MODE == 1 ? (J <= 2 ? 4 : 2)
       : NLS_UPD_RB_MODE == 2 ? (J <= 6 ? 4 : 2)
                              : (J <= 2 ? 4 : (J <= 6 ? 2 : (J <= 18 ? 2 : 1)));
}
template <int J> struct UpdRB { static constexpr int v = upd_rb(J); };
constexpr int RB_ALPHA = 4;

// y = L x  (DeviceSpMV::multiply, device/spmv.hpp:65-73)
template <class S, int DIM>
__global__ __launch_bounds__(NTHREADS) void k_lap(const S *__restrict__ V, Geo g, S *__restrict__ out) {
  march<S, DIM, RB_ALPHA>(V, g, [&](int p, const S &, const S &lap) { out[p] = lap; });
}

// a = V^H L V and ||V||^2 per workgroup, in the symmetric forward-edge form
//   V^H L V = sum_p d_p |v_p|^2 + 2 s sum_p Re(conj(v_p) (v_{p+1} + v_{p+nx} + v_{p+P}))
// (each off-diagonal pair of the reference matrix visited once; the matrix is
// real symmetric, laplacians.hpp:32-37, 89-97, so the form is real).  Only the
// forward neighbours are needed: x+1 from the next lane, y+1 from the thread's
// next row, z+1 from the register queue; plane q+2 is prefetched while plane q
// is reduced.
template <class S, int DIM, int RB>
__device__ __forceinline__ void alpha_tiles(const S *__restrict__ V, const Geo &g, double &a, double &n2) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t ntx, nty, ntz;
  tile_counts<DIM, RB>(g, ntx, nty, ntz);
  const int64_t tiles = ntx * nty * ntz;
  const int64_t P = g.P, nx = g.nx;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t it = t % ntx;
    const int64_t rest = t / ntx;
    const int64_t jt = rest % nty;
    const int64_t kt = rest / nty;
    int64_t q0, q1, yb = 0;
    int64_t off[RB];
    bool rv[RB], xin[RB];
    if constexpr (DIM == 3) {
      yb = jt * (4 * RB) + (int64_t)w * RB;
      if (yb >= g.nyp) continue;
      q0 = kt * g.kz;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        rv[r] = yb + r < g.nyp;
        off[r] = (yb + r) * nx + it * 64 + lane;
        xin[r] = it * 64 + lane < nx;
      }
    } else {
      q0 = (kt * 4 + w) * (int64_t)g.kz;
      if (q0 >= g.nzl) continue;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        rv[r] = true;
        off[r] = it * 64 * RB + 64 * r + lane;
        xin[r] = off[r] < nx;
      }
    }
    q1 = q0 + g.kz < g.nzl ? q0 + g.kz : g.nzl;
    S cur[RB], nxt[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const bool ld = xin[r] && rv[r];
      cur[r] = ld ? V[q0 * P + off[r]] : zero<S>();
      nxt[r] = (ld && g.z0 + q0 + 1 < g.npl) ? V[(q0 + 1) * P + off[r]] : zero<S>();
    }
    for (int64_t q = q0; q < q1; ++q) {
      const int64_t gq = g.z0 + q;
      // forward neighbours that live outside this wave's registers
      S xe[RB], ye = zero<S>();
#pragma unroll
      for (int r = 0; r < RB; ++r) xe[r] = shfl_dn1(cur[r]);
      if constexpr (DIM == 3) {
        const int rl = RB - 1;
        // y+1 of the wave's last valid row: flat p + nx (covers the 3D y-wrap)
        int rlast = 0;
#pragma unroll
        for (int r = 0; r < RB; ++r) if (rv[r]) rlast = r;
        const int64_t p = q * P + off[rlast];
        const int64_t pg = gq * P + off[rlast];
        (void)rl;
        ye = (xin[rlast] && pg + nx < g.Ng) ? V[p + nx] : zero<S>();
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int64_t x = it * 64 + lane;
          if (lane == 63) xe[r] = (rv[r] && x + 1 < nx) ? V[q * P + off[r] + 1] : zero<S>();
        }
      } else {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const S c0 = bcast(cur[r + 1 < RB ? r + 1 : r], 0);
          if (lane == 63) {
            if (r + 1 < RB) xe[r] = c0;
            else xe[r] = (off[r] + 1 < nx) ? V[q * P + off[r] + 1] : zero<S>();
          }
        }
      }
      // prefetch plane q+2
      S nn[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r)
        nn[r] = (xin[r] && rv[r] && gq + 2 < g.npl && q + 2 < q1 + 1) ? V[(q + 2) * P + off[r]]
                                                                        : zero<S>();
      const bool bz = gq == 0 || gq == g.npl - 1;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (!rv[r]) continue;
        const int64_t x = DIM == 3 ? it * 64 + lane : off[r];
        if (!xin[r]) continue;
        const S c = cur[r];
        S f = (x + 1 < nx) ? xe[r] : zero<S>();
        if constexpr (DIM == 3) {
          const bool last = !(r + 1 < RB && rv[r + 1 < RB ? r + 1 : r]);
          f = f + (last ? ye : cur[r + 1 < RB ? r + 1 : r]);
        }
        f = f + nxt[r];
        const bool bnd = x == 0 || x == nx - 1 || bz ||
                         (DIM == 3 && (yb + r == 0 || yb + r == g.nyp - 1));
        const double c2 = abs2(c);
        n2 += c2;
        a += (bnd ? g.sd_bd : g.sd_in) * c2 + 2.0 * g.s * to_c(cj_mul(c, f)).re;
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        cur[r] = nxt[r];
        nxt[r] = nn[r];
      }
    }
  }
}

template <class S, int DIM>
__global__ __launch_bounds__(NTHREADS) void k_alpha(const S *__restrict__ V, Geo g, cplx *__restrict__ part) {
  double a = 0.0, n2 = 0.0;
  alpha_tiles<S, DIM, RB_ALPHA>(V, g, a, n2);
  cplx v[2] = {{a, 0.0}, {n2, 0.0}};
  block_store<2>(v, part);
}

// W_{J+1} = a * L W_J - sum_{k<=J} b_k W_k ;  partials g_k = W_k^H W_{J+1}, ||W_{J+1}||^2
template <class S, int DIM, int J>
__global__ __launch_bounds__(NTHREADS) void k_update(const S *__restrict__ W, S *__restrict__ out,
                                                     int64_t vs, Geo g,
                                                     const KState *__restrict__ st,
                                                     cplx *__restrict__ part) {
  constexpr int NA = J + 2;
  S acc[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) acc[k] = zero<S>();
#if NLS_COEF_LDS
  // Coefficients broadcast from LDS at every use (ds_read_b128, one address per
  // wave): keeps 4(J+1) SGPRs free, which otherwise spill to VGPR lanes and cost
  // ~90 v_readlane per cell row in the hot loop.  The empty asm with a memory
  // clobber stops the compiler from hoisting the LDS reads back into registers.
  __shared__ cplx cfs[MMAX + 2];
  for (int k = threadIdx.x; k <= J + 1; k += NTHREADS) cfs[k] = st->coef[k];
  __syncthreads();
  const double a = cfs[J + 1].re;
#define NLS_B(k) cfs[k]
#define NLS_RELOAD() asm volatile("" ::: "memory")
#else
  cplx b[J + 1];
#pragma unroll
  for (int k = 0; k <= J; ++k) b[k] = st->coef[k];
  const double a = st->coef[J + 1].re;
#define NLS_B(k) b[k]
#define NLS_RELOAD() ((void)0)
#endif
  const S *__restrict__ VJ = W + (int64_t)J * vs;
  constexpr int RB = UpdRB<J>::v;
  march<S, DIM, RB, true>(VJ, g, [&](const int *p, const S *cur, const S *lap, const bool *ok) {
    // every streamed load of every row first ...
    S wk[RB][J > 0 ? J : 1];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const S *__restrict__ src = W + p[r];
#pragma unroll
      for (int k = 0; k < J; ++k) {
        wk[r][k] = ok[r] ? ld_nt(src) : zero<S>();
        src += vs;
      }
    }
    NLS_RELOAD();
    // ... then the CGS update, the store and the Gram / norm partial sums
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (!ok[r]) continue;
      S X = a * lap[r] - coef_mul(NLS_B(J), cur[r]);
#pragma unroll
      for (int k = 0; k < J; ++k) X = X - coef_mul(NLS_B(k), wk[r][k]);
      st_nt(out + p[r], X);
#pragma unroll
      for (int k = 0; k < J; ++k) acc[k] = acc[k] + cj_mul(wk[r][k], X);
      acc[J] = acc[J] + cj_mul(cur[r], X);
      acc[J + 1] = acc[J + 1] + from_real<S>(abs2(X));
    }
  });
  cplx v[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) v[k] = to_c(acc[k]);
  block_store<NA>(v, part);
#undef NLS_B
#undef NLS_RELOAD
}

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
int update_rows_per_thread(int J) { return upd_rb(J); }
int alpha_rows_per_thread() { return RB_ALPHA; }

// ---------------------------------------------------------------------------
// single-workgroup reductions + coefficient math + m x m eigensolve

// Deterministic column sums of column-major partials: dst[v] = sum_q part[v*nb + q],
// v < nc.  One wave per column, fixed order (bitwise reproducible).
__device__ void sum_partials(const cplx *__restrict__ part, int nb, int nc, cplx *dst) {
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
//   sums[0] = a_j, sums[1] = ||W_j||^2 (A pass), sums[2 .. 2+j] = g_0..g_{j-1}, nn (U pass)
// Coefficients of k_update<j> (all from the Gram column of W_j and the
// Hessenberg columns already known; see DESIGN.md "Lanczos reformulation"):
//   H[j][j] = alpha_j = a_j / s_j^2
//   H[j][k] = sum_{l<=k} conj(H[k][l]) G[j][l] + s_{k+1} G[j][k+1]   (k < j)
//   coef[k] = H[j][k] / s_k,  coef[j+1] = 1 / s_j
__global__ __launch_bounds__(NTHREADS) void k_reduce_iter(KState *__restrict__ st,
                                                          const cplx *__restrict__ partA, int nbA,
                                                          const cplx *__restrict__ partU, int nbU,
                                                          int j, int do_sum, int do_coef) {
  __shared__ cplx ssum[2 * MMAX + 8];
  const int ncols = 2 + (j >= 1 ? j + 1 : 0);
  if (do_sum) {
    sum_partials(partA, nbA, 2, ssum);
    if (j >= 1) sum_partials(partU, nbU, j + 1, ssum + 2);
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
  const double sj = sqrt(j == 0 ? ssum[1].re : ssum[2 + j].re);
  const double isj = inv_or_zero(sj);
  if (t == 0) s_s[j] = sj;
  __syncthreads();
  for (int k = t; k < j; k += NTHREADS) s_G[k] = (inv_or_zero(s_s[k]) * isj) * ssum[2 + k];
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
    default: return {__builtin_nan(""), __builtin_nan("")};
  }
}

__device__ __noinline__ void eigen_phase(KState *__restrict__ st, int m, int nf, int f0, int f1,
                                         double t_re, double t_im);

// After the last k_update<m-2>: sums[0..m-1] = g_0..g_{m-2}, nn.  Completes
// T (T(m-1,m-1) = 0, eigen_krylov_complex.hpp:21), diagonalises it with
// implicit-shift QL on wave 0 (lane r owns row r of Q) and writes
//   fin[f][k] = s_0 * (Q f(Lambda) Q^T e_1)_k / s_k
// so that  f(L) W_0 = sum_k fin[f][k] W_k  (= beta V f(T) e1).
__global__ __launch_bounds__(NTHREADS) void k_reduce_final(KState *__restrict__ st,
                                                           const cplx *__restrict__ partU, int nbU,
                                                           int m, int do_sum, int do_coef, int nf,
                                                           int f0, int f1, double t_re,
                                                           double t_im) {
  __shared__ cplx ssum[MMAX];
  if (do_sum && m >= 2) {
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
  if (threadIdx.x == 0 && m >= 2) {
    const double s = sqrt(ssum[m - 1].re);
    st->s[m - 1] = s;
    st->To[m - 2] = s;
    if (!(s > 0.0) && st->breakdown == 0) st->breakdown = m;
  }
  if (threadIdx.x == 0) st->Td[m - 1] = 0.0;
  __syncthreads();
  if (threadIdx.x < 64) eigen_phase(st, m, nf, f0, f1, t_re, t_im);
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

// Nonlinear half step out = exp(-0.5*tau*rho(u)) u, tau = 1j*dt
//  cubic (nlse_solver.hpp:66-69): rho = re^2 + im^2
//  cubic-quintic (device/nlse_cq_solver.hpp:16-39): d = |u|*|u|, rho = s1 d + s2 d^2
__device__ __forceinline__ cplx nl_half(cplx u, double dt, int nonlin, cplx s1, cplx s2) {
  if (nonlin == 0) {
    const double x = u.re * u.re + u.im * u.im;
    double sn, cs;
    sincos((-0.5 * dt) * x, &sn, &cs);
    return {cs * u.re - sn * u.im, cs * u.im + sn * u.re};
  }
  const double a = hypot(u.re, u.im);
  const double d = a * a;
  const cplx rho = d * s1 + (d * d) * s2;
  const cplx z = cmul({-0.0, -0.5 * dt}, rho);
  const double er = exp(z.re);
  double sn, cs;
  sincos(z.im, &sn, &cs);
  return cmul({er * cs, er * sn}, u);
}

__global__ __launch_bounds__(NTHREADS) void k_nl_init(const cplx *__restrict__ u, cplx *__restrict__ w0,
                                                      int64_t n, double dt, int nonlin, cplx s1,
                                                      cplx s2) {
  for (int64_t p = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * NTHREADS)
    w0[p] = nl_half(u[p], dt, nonlin, s1, s2);
}

// u = N(sum_k fin_k W_k) ; W_0 <- N(u) for the next step (fused start of step)
template <int M>
__global__ __launch_bounds__(NTHREADS) void k_final_nlse(cplx *__restrict__ W, int64_t vs, int64_t n,
                                                         const KState *__restrict__ st,
                                                         cplx *__restrict__ u, double dt,
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
      const cplx un = nl_half(y, dt, nonlin, s1, s2);
      st_nt(u + p, un);
      st_nt(W + p, nl_half(un, dt, nonlin, s1, s2));
    }
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

#define NLS_J_LIST(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) \
  X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) \
  X(28) X(29) X(30)
#define NLS_M_LIST(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) \
  X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) \
  X(29) X(30) X(31) X(32)

template <class S, int DIM> const void *update_fn(int J) {
  switch (J) {
#define X(J) case J: return reinterpret_cast<const void *>(&k_update<S, DIM, J>);
    NLS_J_LIST(X)
#undef X
    default: return nullptr;
  }
}

const void *kernel_update(bool cplx_, int dim, int J) {
  if (cplx_) return dim == 3 ? update_fn<cplx, 3>(J) : update_fn<cplx, 2>(J);
  return dim == 3 ? update_fn<double, 3>(J) : update_fn<double, 2>(J);
}

const void *kernel_alpha(bool cplx_, int dim) {
  if (cplx_)
    return dim == 3 ? reinterpret_cast<const void *>(&k_alpha<cplx, 3>)
                    : reinterpret_cast<const void *>(&k_alpha<cplx, 2>);
  return dim == 3 ? reinterpret_cast<const void *>(&k_alpha<double, 3>)
                  : reinterpret_cast<const void *>(&k_alpha<double, 2>);
}

const void *kernel_lap(bool cplx_, int dim) {
  if (cplx_)
    return dim == 3 ? reinterpret_cast<const void *>(&k_lap<cplx, 3>)
                    : reinterpret_cast<const void *>(&k_lap<cplx, 2>);
  return dim == 3 ? reinterpret_cast<const void *>(&k_lap<double, 3>)
                  : reinterpret_cast<const void *>(&k_lap<double, 2>);
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
