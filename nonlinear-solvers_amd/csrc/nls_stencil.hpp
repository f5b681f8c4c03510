// nls_stencil.hpp -- device-side building blocks of the stencil kernels
// (included by nls_stencil.hip, which is compiled once per operator variant
// and dimension, and by nls_kernels.hip for the shared helpers).
//
// Two operators share one tiled march:
//   iso  (G1, laplacians.hpp:10-105): constant 5/7-point stencil, diagonal
//        -4/-3 (2D) or -6/-5 (3D) times the scale.
//   ani  (G2, nlsolvers/common/include/laplacians.hpp:54-103, 158-218):
//        div(c grad u) with face weights w = (c_a + c_b)/2 on every coupling
//        of the same flat-index pattern (incl. the 3D y-wrap) and diagonal
//        -sum(w), i.e.  (L v)_p = s * sum_{q ~ p} w_pq (v_q - v_p).
//        c is marched alongside the vector (one extra f64 stream per pass).
#pragma once
#include <type_traits>
#include <utility>

#include "nls_common.hpp"

namespace nls {

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

// Timing diagnostic only (wrong results; never a product build): the 3D march skips the
// loads from outside its tile -- bit 1 the x-edge cells of lanes 0 / 63, bit 2 the y rows
// above / below the tile, bit 4 the plane below the tile's first -- so a variant library
// shows what each kind of halo load costs k_alpha_l2 and k_tail (profiles/r06/ab_halo_diag_colsum_tq.txt)
#ifndef NLS_DIAG_HALO
#define NLS_DIAG_HALO 0
#endif

template <int DIM, int RB> __host__ __device__ inline void tile_counts(const Geo &g, int64_t &ntx,
                                                                        int64_t &nty, int64_t &ntz) {
  const int64_t nq = g.qb - g.qa;  // local planes [qa, qb) covered by this launch
  if (DIM == 3) {
    ntx = cdiv(g.nx, 64);
    nty = cdiv(g.nyp, 4 * RB);
    ntz = cdiv(nq, g.kz);
  } else {
    ntx = cdiv(g.nx, 64 * RB);
    nty = 1;
    ntz = cdiv(nq, 4 * (int64_t)g.kz);
  }
}

// weight of one anisotropic coupling, (c_a + c_b) / 2 (laplacians.hpp:181-209),
// zero when the neighbour is not coupled
__device__ __forceinline__ double face_w(bool e, double ca, double cb) { return e ? 0.5 * (ca + cb) : 0.0; }

// fn(p, cur, lap) for every local cell p of the workgroup's tiles, with
// cur = V[p] and lap = (L V)[p] (laplacians.hpp:10-105, flat-index form).
// Local indices are 32-bit (the host guarantees (nzl+4)*P + pad < 2^31); the flat
// range tests of the reference (idx-nx >= 0, idx+nx < N) are evaluated on
// (plane, row) coordinates so they never need 64-bit global indices.
//
// PLANE = true: fn(p[RB], cur[RB], lap[RB], ok[RB]) is called once per plane
// with all rows of the thread, so the caller can issue every streamed load of
// all its rows before the first use (more loads in flight per accumulator set).
// ANI = true: the G2 operator; the coefficient field g.cf (same layout and
// ghost planes as a basis vector) is marched with the same register queue.
template <class S, int DIM, int RB, bool PLANE = false, bool ANI = false, class Fn>
__device__ __forceinline__ void march(const S *__restrict__ V, const Geo &g, Fn &&fn) {
  const double *__restrict__ C = g.cf;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t ntx64, nty64, ntz64;
  tile_counts<DIM, RB>(g, ntx64, nty64, ntz64);
  const int ntx = (int)ntx64, nty = (int)nty64;
  const int tiles = (int)(ntx64 * nty64 * ntz64);
  const int T8 = tiles / 8;
  const int P = (int)g.P, nx = (int)g.nx, nyp = (int)g.nyp, qa = g.qa, qb = g.qb, kz = g.kz;
  const int z0 = (int)g.z0, npl = (int)g.npl;
  int32_t *const tq = g.tq;
#define NLS_TQ_NEXT() (NLS_TQ_XCD ? tq_next_xcd(tq, ntx, nty, (int)ntz64) : tq_next(tq))
  for (int t0 = tq ? NLS_TQ_NEXT() : (int)blockIdx.x; t0 < tiles; t0 = tq ? NLS_TQ_NEXT() : t0 + (int)gridDim.x) {
    // optional XCD-banded order (workgroups b, b+8 share an XCD): speed only.  (In-plane
    // y-bands per XCD, x fastest, so that a tile's x- and y-neighbours share its L2, made
    // k_alpha_l2 slower at 512^3: 0.512 against 0.500 ms, profiles/r06/envab_fuse_l2remap.txt)
    const int t = (g.remap && t0 < 8 * T8) ? (t0 % 8) * T8 + t0 / 8 : t0;
    const int it = t % ntx;
    const int rest = t / ntx;
    const int jt = rest % nty;
    const int kt = rest / nty;
    if constexpr (DIM == 3) {
      const int x = it * 64 + lane;
      const bool xin = x < nx;
      const int yb = jt * (4 * RB) + w * RB;
      // wave-uniform; guarded rather than skipped with continue, so the tile queue's
      // barrier (tq_next) is reached from one point of uniform control flow
      if (yb < nyp) {
        const int q0 = qa + kt * kz;
        const int q1 = q0 + kz < qb ? q0 + kz : qb;
        bool rv[RB];
        int off[RB];
        S prev[RB], cur[RB];
        double cprv[RB], ccur[RB];
  #pragma unroll
        for (int r = 0; r < RB; ++r) {
          rv[r] = yb + r < nyp;
          off[r] = (yb + r) * nx + x;
          const bool ld = xin && rv[r];
          prev[r] = (ld && z0 + q0 > 0 && !(NLS_DIAG_HALO & 4)) ? V[(q0 - 1) * P + off[r]] : zero<S>();
          cur[r] = ld ? V[q0 * P + off[r]] : zero<S>();
          if constexpr (ANI) {
            cprv[r] = (ld && z0 + q0 > 0) ? C[(q0 - 1) * P + off[r]] : 0.0;
            ccur[r] = ld ? C[q0 * P + off[r]] : 0.0;
          }
        }
        const bool bx = (x == 0) || (x == nx - 1);
        for (int q = q0; q < q1; ++q) {
          const int gq = z0 + q;
          const bool bz = gq == 0 || gq == npl - 1;
          const bool has_next = gq + 1 < npl;
          S next[RB], lapv[RB];
          double cnxt[RB];
          int pv[RB];
          bool okv[RB];
  #pragma unroll
          for (int r = 0; r < RB; ++r) {
            const bool ld = xin && rv[r] && has_next;
            next[r] = ld ? V[(q + 1) * P + off[r]] : zero<S>();
            if constexpr (ANI) cnxt[r] = ld ? C[(q + 1) * P + off[r]] : 0.0;
          }
  #pragma unroll
          for (int r = 0; r < RB; ++r) {
            pv[r] = q * P + off[r];
            okv[r] = false;
            lapv[r] = zero<S>();
            if (!rv[r]) continue;  // wave-uniform
            const int p = q * P + off[r];
            const int y = yb + r;
            const bool eym = gq > 0 || y > 0;            // idx - nx >= 0
            const bool eyp = gq < npl - 1 || y < nyp - 1;  // idx + nx < N
            const bool inner_yp = r + 1 < RB && rv[r + 1 < RB ? r + 1 : r];
            S ym, yp;
            constexpr bool noyh = (NLS_DIAG_HALO & 2) != 0;
            if (r > 0) ym = cur[r - 1];
            else ym = (xin && eym && !(noyh && w == 0)) ? V[p - nx] : zero<S>();
            if (inner_yp) yp = cur[r + 1 < RB ? r + 1 : r];
            else yp = (xin && eyp && !(noyh && w == 3)) ? V[p + nx] : zero<S>();
            S xm = shfl_up1(cur[r]), xp = shfl_dn1(cur[r]);
            const bool edge_ld =
                ((lane == 0 && x > 0) || (lane == 63 && x + 1 < nx)) && xin && !(NLS_DIAG_HALO & 1);
            const S xe = edge_ld ? V[p + (lane == 0 ? -1 : 1)] : zero<S>();
            if (lane == 0) xm = xe;
            if (lane == 63) xp = xe;
            if (!(x > 0)) xm = zero<S>();
            if (!(x + 1 < nx)) xp = zero<S>();
            S lap;
            if constexpr (ANI) {
              const double cc = ccur[r];
              double cym, cyp;
              if (r > 0) cym = ccur[r - 1];
              else cym = (xin && eym) ? C[p - nx] : 0.0;
              if (inner_yp) cyp = ccur[r + 1 < RB ? r + 1 : r];
              else cyp = (xin && eyp) ? C[p + nx] : 0.0;
              double cxm = shfl_up1(cc), cxp = shfl_dn1(cc);
              const double cxe = edge_ld ? C[p + (lane == 0 ? -1 : 1)] : 0.0;
              if (lane == 0) cxm = cxe;
              if (lane == 63) cxp = cxe;
              const double wxm = face_w(x > 0, cc, cxm), wxp = face_w(x + 1 < nx, cc, cxp);
              const double wym = face_w(eym, cc, cym), wyp = face_w(eyp, cc, cyp);
              const double wzm = face_w(gq > 0, cc, cprv[r]), wzp = face_w(has_next, cc, cnxt[r]);
              lap = g.s * ((((wzm * prev[r] + wzp * next[r]) + (wxm * xm + wxp * xp)) +
                            (wym * ym + wyp * yp)) -
                           (((wzm + wzp) + (wxm + wxp)) + (wym + wyp)) * cur[r]);
            } else {
              const bool bnd = bx || bz || y == 0 || y == nyp - 1;
              lap = g.s * (((prev[r] + next[r]) + (xm + xp)) + (ym + yp)) +
                    (bnd ? g.sd_bd : g.sd_in) * cur[r];
            }
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
            if constexpr (ANI) {
              cprv[r] = ccur[r];
              ccur[r] = cnxt[r];
            }
          }
        }
      }
    } else {
      const int q0 = qa + (kt * 4 + w) * kz;
      if (q0 < qb) {  // wave-uniform (see the 3D branch)
        const int q1 = q0 + kz < qb ? q0 + kz : qb;
        int xr[RB];
        S prev[RB], cur[RB];
        double cprv[RB], ccur[RB];
  #pragma unroll
        for (int r = 0; r < RB; ++r) {
          xr[r] = it * 64 * RB + 64 * r + lane;
          const bool ld = xr[r] < nx;
          prev[r] = (ld && z0 + q0 > 0) ? V[(q0 - 1) * P + xr[r]] : zero<S>();
          cur[r] = ld ? V[q0 * P + xr[r]] : zero<S>();
          if constexpr (ANI) {
            cprv[r] = (ld && z0 + q0 > 0) ? C[(q0 - 1) * P + xr[r]] : 0.0;
            ccur[r] = ld ? C[q0 * P + xr[r]] : 0.0;
          }
        }
        for (int q = q0; q < q1; ++q) {
          const int gq = z0 + q;
          const bool bz = gq == 0 || gq == npl - 1;
          const bool has_next = gq + 1 < npl;
          S next[RB], lapv[RB];
          double cnxt[RB];
          int pv[RB];
          bool okv[RB];
  #pragma unroll
          for (int r = 0; r < RB; ++r) {
            const bool ld = xr[r] < nx && has_next;
            next[r] = ld ? V[(q + 1) * P + xr[r]] : zero<S>();
            if constexpr (ANI) cnxt[r] = ld ? C[(q + 1) * P + xr[r]] : 0.0;
          }
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
            S lap;
            if constexpr (ANI) {
              const double cc = ccur[r];
              double cxm = shfl_up1(cc), cxp = shfl_dn1(cc);
              const double ccm = bcast(ccur[r > 0 ? r - 1 : 0], 63);
              const double ccp = bcast(ccur[r + 1 < RB ? r + 1 : r], 0);
              const double cxe = edge_ld ? C[p + (lane == 0 ? -1 : 1)] : 0.0;
              if (lane == 0) cxm = r > 0 ? ccm : cxe;
              if (lane == 63) cxp = r + 1 < RB ? ccp : cxe;
              const double wxm = face_w(x > 0, cc, cxm), wxp = face_w(x + 1 < nx, cc, cxp);
              const double wzm = face_w(gq > 0, cc, cprv[r]), wzp = face_w(has_next, cc, cnxt[r]);
              lap = g.s * (((wzm * prev[r] + wzp * next[r]) + (wxm * xm + wxp * xp)) -
                           ((wzm + wzp) + (wxm + wxp)) * cur[r]);
            } else {
              const bool bnd = x == 0 || x == nx - 1 || bz;
              lap = g.s * ((prev[r] + next[r]) + (xm + xp)) + (bnd ? g.sd_bd : g.sd_in) * cur[r];
            }
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
            if constexpr (ANI) {
              cprv[r] = ccur[r];
              ccur[r] = cnxt[r];
            }
          }
        }
      }
    }
  }
  if (tq) tq_done(tq);
#undef NLS_TQ_NEXT
}

// march3p: the 3D isotropic march with one row per thread (march<S, 3, 1>'s cells,
// couplings, arithmetic order and tile order, so its callers' sums are bit-identical),
// software-pipelined: the stencil vector's own row is loaded two planes ahead and the
// plane's side values (rows y-1, y+1 and the wave's x-edge cell) one plane ahead, so no
// load is consumed in the iteration that issues it.  (march loads the y and x-edge values
// of a plane in the iteration that uses them: their L2 latency is exposed once per plane,
// k_alpha_l2 at 512^3 waited on memory 0.59 of its cycles with 0.21 issuing,
// profiles/r05/sq2_nlse3d_512.txt.)  No barrier inside: no tile queue.
template <class S, bool ANI, class Fn>
__device__ __forceinline__ void march3p(const S *__restrict__ V, const Geo &g, Fn &&fn) {
  const double *__restrict__ C = g.cf;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t ntx64, nty64, ntz64;
  tile_counts<3, 1>(g, ntx64, nty64, ntz64);
  const int ntx = (int)ntx64, nty = (int)nty64;
  const int tiles = (int)(ntx64 * nty64 * ntz64);
  const int P = (int)g.P, nx = (int)g.nx, nyp = (int)g.nyp, qa = g.qa, qb = g.qb, kz = g.kz;
  const int z0 = (int)g.z0, npl = (int)g.npl;
  // the per-plane values of one row: the vector and (ANI) the coefficient field
  struct Row {
    S v;
    double c;
  };
  struct Side {
    S ym, yp, xe;
    double cym, cyp, cxe;
  };
  for (int t = (int)blockIdx.x; t < tiles; t += (int)gridDim.x) {
    const int it = t % ntx;
    const int rest = t / ntx;
    const int jt = rest % nty;
    const int kt = rest / nty;
    const int x = it * 64 + lane;
    const bool xin = x < nx;
    const int y = jt * 4 + w;
    if (y >= nyp) continue;  // wave-uniform
    const int q0 = qa + kt * kz;
    const int q1 = q0 + kz < qb ? q0 + kz : qb;
    const int off = y * nx + x;
    const bool edge_ld = ((lane == 0 && x > 0) || (lane == 63 && x + 1 < nx)) && xin;
    const int eo = lane == 0 ? -1 : 1;
    const bool bxy = x == 0 || x == nx - 1 || y == 0 || y == nyp - 1;
    // the own row of plane q: zero outside the global grid (march's prev / next rules)
    auto own = [&](int q) -> Row {
      const int gq = z0 + q;
      const bool ld = xin && gq >= 0 && gq < npl;
      Row r;
      r.v = ld ? V[q * P + off] : zero<S>();
      r.c = 0.0;
      if constexpr (ANI) r.c = ld ? C[q * P + off] : 0.0;
      return r;
    };
    auto side = [&](int q) -> Side {
      const int gq = z0 + q, p = q * P + off;
      const bool lm = xin && (gq > 0 || y > 0);            // idx - nx >= 0
      const bool lp = xin && (gq < npl - 1 || y < nyp - 1);  // idx + nx < N
      Side sd;
      sd.ym = lm ? V[p - nx] : zero<S>();
      sd.yp = lp ? V[p + nx] : zero<S>();
      sd.xe = edge_ld ? V[p + eo] : zero<S>();
      sd.cym = sd.cyp = sd.cxe = 0.0;
      if constexpr (ANI) {
        sd.cym = lm ? C[p - nx] : 0.0;
        sd.cyp = lp ? C[p + nx] : 0.0;
        sd.cxe = edge_ld ? C[p + eo] : 0.0;
      }
      return sd;
    };
    const Side zs{zero<S>(), zero<S>(), zero<S>(), 0.0, 0.0, 0.0};
    const Row zr{zero<S>(), 0.0};
    Row am = own(q0 - 1), a0 = own(q0), a1 = own(q0 + 1);
    Row a2 = q0 + 2 <= q1 ? own(q0 + 2) : zr;
    Side sc = side(q0);
    for (int q = q0; q < q1; ++q) {
      // issue: the side values of plane q+1, the own row of plane q+3 (uniform guards)
      const Side sn = q + 1 < q1 ? side(q + 1) : zs;
      const Row a3 = q + 3 <= q1 ? own(q + 3) : zr;
      const int gq = z0 + q;
      S xm = shfl_up1(a0.v), xp = shfl_dn1(a0.v);
      if (lane == 0) xm = sc.xe;
      if (lane == 63) xp = sc.xe;
      if (!(x > 0)) xm = zero<S>();
      if (!(x + 1 < nx)) xp = zero<S>();
      S lap;
      if constexpr (ANI) {
        const double cc = a0.c;
        const bool eym = gq > 0 || y > 0, eyp = gq < npl - 1 || y < nyp - 1;
        double cxm = shfl_up1(cc), cxp = shfl_dn1(cc);
        if (lane == 0) cxm = sc.cxe;
        if (lane == 63) cxp = sc.cxe;
        const double wxm = face_w(x > 0, cc, cxm), wxp = face_w(x + 1 < nx, cc, cxp);
        const double wym = face_w(eym, cc, sc.cym), wyp = face_w(eyp, cc, sc.cyp);
        const double wzm = face_w(gq > 0, cc, am.c), wzp = face_w(gq + 1 < npl, cc, a1.c);
        lap = g.s * ((((wzm * am.v + wzp * a1.v) + (wxm * xm + wxp * xp)) + (wym * sc.ym + wyp * sc.yp)) -
                     (((wzm + wzp) + (wxm + wxp)) + (wym + wyp)) * a0.v);
      } else {
        const bool bnd = bxy || gq == 0 || gq == npl - 1;
        lap = g.s * (((am.v + a1.v) + (xm + xp)) + (sc.ym + sc.yp)) + (bnd ? g.sd_bd : g.sd_in) * a0.v;
      }
      if (xin) fn(q * P + off, a0.v, lap);
      am = a0;
      a0 = a1;
      a1 = a2;
      a2 = a3;
      sc = sn;
    }
  }
}

#include "nls_march_q.hpp"

#ifndef NLS_UPD_RB_MODE
#define NLS_UPD_RB_MODE 1
#endif
#ifndef NLS_COEF_LDS
#define NLS_COEF_LDS 1
#endif
#ifndef NLS_ANI_RB1_FROM
#define NLS_ANI_RB1_FROM 13  // anisotropic passes with J >= this: one row per thread (G2 256^3 m=25: -5 % update time)
#endif
__host__ __device__ constexpr int upd_rb(int J, bool ani = false) {
  return (ani && J >= NLS_ANI_RB1_FROM) ? 1
       : NLS_UPD_RB_MODE == 0 ? (J <= 2 ? 4 : (J <= 6 ? 2 : 1))
       : NLS_UPD_RB_MODE == 1 ? (J <= 2 ? 4 : 2)
       : NLS_UPD_RB_MODE == 2 ? (J <= 6 ? 4 : 2)
                              : (J <= 2 ? 4 : (J <= 6 ? 2 : (J <= 18 ? 2 : 1)));
}
template <int J, bool ANI> struct UpdRB { static constexpr int v = upd_rb(J, ANI); };
#ifndef NLS_QA_RB1_FROM
#define NLS_QA_RB1_FROM 99  // update passes with the folded alpha: one row per thread from this J (RB = 1 measured slower)
#endif
template <int J, bool ANI> struct UpdRBQ {
  static constexpr int v = J >= NLS_QA_RB1_FROM ? 1 : (upd_rb(J, ANI) > 2 ? 2 : upd_rb(J, ANI));
};
constexpr int RB_ALPHA = 4;
#ifndef NLS_RB_L2
#define NLS_RB_L2 1  // measured at 512^3: RB 1 / kz 32 0.50 ms vs RB 4 / kz 8 0.58 ms (tools/exp_l2.sh)
#endif
constexpr int RB_L2 = NLS_RB_L2;  // rows per thread of k_alpha_l2
#ifndef NLS_FUSED_RB
#define NLS_FUSED_RB 1
#endif
constexpr int FUSED_RB = NLS_FUSED_RB;  // rows per thread of k_tail


// y = L x  (DeviceSpMV::multiply, device/spmv.hpp:65-73)
template <class S, int DIM, bool ANI>
__global__ __launch_bounds__(NTHREADS) void k_lap(const S *__restrict__ V, Geo g, S *__restrict__ out) {
  march<S, DIM, RB_ALPHA, false, ANI>(V, g, [&](int p, const S &, const S &lap) { out[p] = lap; });
}

// a = V^H L V and ||V||^2 per workgroup, from forward couplings only (each
// off-diagonal pair of the reference matrix visited once; the matrices are
// real symmetric, laplacians.hpp:32-37, 89-97, 181-209, so the form is real):
//   iso:  V^H L V = sum_p d_p |v_p|^2 + 2 s sum_p Re(conj(v_p) (v_{p+1} + v_{p+nx} + v_{p+P}))
//   ani:  V^H L V = -s sum_{forward pairs (p,q)} w_pq |v_p - v_q|^2   (diag = -sum w)
// Only the forward neighbours are needed: x+1 from the next lane, y+1 from the
// thread's next row, z+1 from the register queue; plane q+2 is prefetched
// while plane q is reduced.
template <class S, int DIM, int RB, bool ANI>
__device__ __forceinline__ void alpha_tiles(const S *__restrict__ V, const Geo &g, double &a, double &n2) {
  const double *__restrict__ C = g.cf;
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
      q0 = g.qa + kt * g.kz;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        rv[r] = yb + r < g.nyp;
        off[r] = (yb + r) * nx + it * 64 + lane;
        xin[r] = it * 64 + lane < nx;
      }
    } else {
      q0 = g.qa + (kt * 4 + w) * (int64_t)g.kz;
      if (q0 >= g.qb) continue;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        rv[r] = true;
        off[r] = it * 64 * RB + 64 * r + lane;
        xin[r] = off[r] < nx;
      }
    }
    q1 = q0 + g.kz < g.qb ? q0 + g.kz : g.qb;
    S cur[RB], nxt[RB];
    double ccu[RB], cnx[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const bool ld = xin[r] && rv[r];
      const bool ldn = ld && g.z0 + q0 + 1 < g.npl;
      cur[r] = ld ? V[q0 * P + off[r]] : zero<S>();
      nxt[r] = ldn ? V[(q0 + 1) * P + off[r]] : zero<S>();
      if constexpr (ANI) {
        ccu[r] = ld ? C[q0 * P + off[r]] : 0.0;
        cnx[r] = ldn ? C[(q0 + 1) * P + off[r]] : 0.0;
      }
    }
    for (int64_t q = q0; q < q1; ++q) {
      const int64_t gq = g.z0 + q;
      // forward neighbours that live outside this wave's registers
      S xe[RB], ye = zero<S>();
      double cxe[RB], cye = 0.0;
      bool eye = false;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        xe[r] = shfl_dn1(cur[r]);
        if constexpr (ANI) cxe[r] = shfl_dn1(ccu[r]);
      }
      if constexpr (DIM == 3) {
        // y+1 of the wave's last valid row: flat p + nx (covers the 3D y-wrap)
        int rlast = 0;
#pragma unroll
        for (int r = 0; r < RB; ++r) if (rv[r]) rlast = r;
        const int64_t p = q * P + off[rlast];
        const int64_t pg = gq * P + off[rlast];
        eye = xin[rlast] && pg + nx < g.Ng;
        ye = eye ? V[p + nx] : zero<S>();
        if constexpr (ANI) cye = eye ? C[p + nx] : 0.0;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int64_t x = it * 64 + lane;
          if (lane == 63) {
            const bool e = rv[r] && x + 1 < nx;
            xe[r] = e ? V[q * P + off[r] + 1] : zero<S>();
            if constexpr (ANI) cxe[r] = e ? C[q * P + off[r] + 1] : 0.0;
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const S c0 = bcast(cur[r + 1 < RB ? r + 1 : r], 0);
          double cc0 = 0.0;
          if constexpr (ANI) cc0 = bcast(ccu[r + 1 < RB ? r + 1 : r], 0);
          if (lane == 63) {
            if (r + 1 < RB) {
              xe[r] = c0;
              if constexpr (ANI) cxe[r] = cc0;
            } else {
              const bool e = off[r] + 1 < nx;
              xe[r] = e ? V[q * P + off[r] + 1] : zero<S>();
              if constexpr (ANI) cxe[r] = e ? C[q * P + off[r] + 1] : 0.0;
            }
          }
        }
      }
      // prefetch plane q+2
      S nn[RB];
      double cnn[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const bool ld = xin[r] && rv[r] && gq + 2 < g.npl && q + 2 < q1 + 1;
        nn[r] = ld ? V[(q + 2) * P + off[r]] : zero<S>();
        if constexpr (ANI) cnn[r] = ld ? C[(q + 2) * P + off[r]] : 0.0;
      }
      const bool bz = gq == 0 || gq == g.npl - 1;
      const bool ez = gq + 1 < g.npl;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (!rv[r]) continue;
        const int64_t x = DIM == 3 ? it * 64 + lane : off[r];
        if (!xin[r]) continue;
        const S c = cur[r];
        const bool last = !(r + 1 < RB && rv[r + 1 < RB ? r + 1 : r]);
        if constexpr (ANI) {
          const double cc = ccu[r];
          double acc = 0.0;
          if (x + 1 < nx) acc += face_w(true, cc, cxe[r]) * abs2(c - xe[r]);
          if constexpr (DIM == 3) {
            const S yv = last ? ye : cur[r + 1 < RB ? r + 1 : r];
            const double cy = last ? cye : ccu[r + 1 < RB ? r + 1 : r];
            if (!last || eye) acc += face_w(true, cc, cy) * abs2(c - yv);
          }
          if (ez) acc += face_w(true, cc, cnx[r]) * abs2(c - nxt[r]);
          n2 += abs2(c);
          a -= g.s * acc;
        } else {
          S f = (x + 1 < nx) ? xe[r] : zero<S>();
          if constexpr (DIM == 3) f = f + (last ? ye : cur[r + 1 < RB ? r + 1 : r]);
          f = f + nxt[r];
          const bool bnd = x == 0 || x == nx - 1 || bz ||
                           (DIM == 3 && (yb + r == 0 || yb + r == g.nyp - 1));
          const double c2 = abs2(c);
          n2 += c2;
          a += (bnd ? g.sd_bd : g.sd_in) * c2 + 2.0 * g.s * to_c(cj_mul(c, f)).re;
        }
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        cur[r] = nxt[r];
        nxt[r] = nn[r];
        if constexpr (ANI) {
          ccu[r] = cnx[r];
          cnx[r] = cnn[r];
        }
      }
    }
  }
}

template <class S, int DIM, bool ANI>
__global__ __launch_bounds__(NTHREADS) void k_alpha(const S *__restrict__ V, Geo g, cplx *__restrict__ part) {
  double a = 0.0, n2 = 0.0;
  alpha_tiles<S, DIM, RB_ALPHA, ANI>(V, g, a, n2);
  cplx v[2] = {{a, 0.0}, {n2, 0.0}};
  block_store<2>(v, part, gridDim.x, 0);
}

// The reduction after a folded-alpha update pass (k_reduce_iter with qa = 1), with
// its own fallback: when the folded alpha is ill-conditioned (need_alpha, near a
// breakdown) this one workgroup reduces W_j^H L W_j itself (alpha_tiles over every
// tile of the slab: slow, but only near a breakdown) and redoes the coefficients
// from the direct value -- no extra launches in the common case.
template <class S, int DIM, bool ANI>
__global__ __launch_bounds__(NTHREADS) void k_reduce_qa(KState *__restrict__ st, const cplx *__restrict__ partU,
                                                        int nbU, int j, int do_sum,
                                                        const cplx *__restrict__ partX, int nbX,
                                                        const S *__restrict__ Wj, Geo ga) {
  reduce_iter_body(st, nullptr, 0, partU, nbU, j, do_sum, 1, 0, 1, partX, nbX);
  __syncthreads();
  if (st->need_alpha == 0) return;  // uniform (thread 0's global write, after the barrier)
  double a = 0.0, n2 = 0.0;
  alpha_tiles<S, DIM, RB_ALPHA, ANI>(Wj, ga, a, n2);
  __shared__ double ra[NTHREADS / 64], rn[NTHREADS / 64];
  a = wave_sum(a);
  n2 = wave_sum(n2);
  if ((threadIdx.x & 63) == 0) {
    ra[threadIdx.x >> 6] = a;
    rn[threadIdx.x >> 6] = n2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sa = ra[0], sn = rn[0];
    for (int w = 1; w < NTHREADS / 64; ++w) {
      sa += ra[w];
      sn += rn[w];
    }
    st->sums[0] = {sa, 0.0};
    st->sums[1] = {sn, 0.0};
  }
  __syncthreads();
  reduce_iter_body(st, nullptr, 0, nullptr, 0, j, 0, 1, 2, 0);
}

// W_{J+1} = a * L W_J - sum_{k<=J} b_k W_k ;  partials g_k = W_k^H W_{J+1}, ||W_{J+1}||^2
// QA: also q = (L W_J)^H L (L W_J) (march_q), from which the reduction gets the
// next alpha (no separate alpha pass over W_{J+1}), and the measured
// W_J^H L W_J (every cell has W_J and L W_J in registers): partial columns J+2, J+3.
// QA also stores the x-tile seam values of L W_J in E (see march_q, k_xpairs).
template <class S, int DIM, int J, bool ANI, bool QA = false>
__global__ __launch_bounds__(NTHREADS) void k_update(const S *__restrict__ W, S *__restrict__ out,
                                                     int64_t vs, Geo g,
                                                     const KState *__restrict__ st,
                                                     cplx *__restrict__ part, int pstride, int poff,
                                                     S *__restrict__ E) {
  constexpr int NA = J + 2;
  S acc[NA];
  double qacc = 0.0, ameas = 0.0;
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
  constexpr int RB = QA ? UpdRBQ<J, ANI>::v : UpdRB<J, ANI>::v;
  auto body = [&](const int *p, const S *cur, const S *lap, const bool *ok) {
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
      if constexpr (QA) ameas += to_c(cj_mul(cur[r], lap[r])).re;
    }
  };
  if constexpr (QA) march_q<S, DIM, RB, ANI>(VJ, g, qacc, E, body);
  else march<S, DIM, RB, true, ANI>(VJ, g, body);
  cplx v[NA + (QA ? 2 : 0)];
#pragma unroll
  for (int k = 0; k < NA; ++k) v[k] = to_c(acc[k]);
  if constexpr (QA) {
    v[NA] = {qacc, 0.0};
    v[NA + 1] = {ameas, 0.0};
  }
  block_store<NA + (QA ? 2 : 0)>(v, part, pstride, poff);
#undef NLS_B
#undef NLS_RELOAD
}

// Last alpha pass of a fused-tail Lanczos (see k_final_fused): full stencil per
// cell, so besides a = V^H L V and ||V||^2 it also reduces ||L V||^2, from which
// the norm of the never-stored last vector follows (k_reduce_iter, ncA = 3).
template <class S, int DIM, bool ANI, bool PIPE = false>
__global__ __launch_bounds__(NTHREADS) void k_alpha_l2(const S *__restrict__ V, Geo g,
                                                       cplx *__restrict__ part) {
  double a = 0.0, n2 = 0.0, l2 = 0.0;
  auto body = [&](int, const S &c, const S &lap) {
    a += to_c(cj_mul(c, lap)).re;
    n2 += abs2(c);
    l2 += abs2(lap);
  };
  // 3D isotropic, NLS_L2_PIPE=1: the pipelined march (512^3, same box, two rounds: 0.52-0.54 ms
  // against 0.50 through march, profiles/r06/ab_alpha_l2_pipe.txt; off)
  if constexpr (PIPE && DIM == 3 && RB_L2 == 1) march3p<S, ANI>(V, g, body);
  else march<S, DIM, RB_L2, false, ANI>(V, g, body);
  cplx v[3] = {{a, 0.0}, {n2, 0.0}, {l2, 0.0}};
  block_store<3>(v, part, gridDim.x, 0);
}

// Fused tail of a Krylov basis (M >= 3): the last Lanczos vector is never
// stored.  With J = M-2, the pass marches W_J with the stencil and streams
// W_0..W_{J-1}.  The last vector k_update<J> would have written,
//   W_{M-1} = a L W_J - sum_{k<=J} b_k W_k      (a = 1/s_J, b_k = H[J][k]/s_k),
// enters each final combination  y_f = sum_{k<M} fin_f[k] W_k  only linearly, so
// the pass evaluates
//   y_f = (fin_f[M-1] a) L W_J + sum_{k<=J} (fin_f[k] - fin_f[M-1] b_k) W_k
// with the coefficients folded once per workgroup, and hands y_f to the step's
// epilogue (MODE).  This replaces k_update<M-2> plus the combination kernel of
// the step: M+1 (NLSE) streams instead of 2M+2.  The norm s_{M-1} the eigensolve
// needs comes from the last alpha pass, ||W_{M-1}||^2 = ||L v_J||^2 - sum_k
// |H[J][k]|^2 (orthonormal basis; k_alpha_l2 + k_reduce_iter with ncA = 3).
// Modes and arguments: TailMode / TailArgs (nls_device.hpp).
// Writes go to the thread's own cell only; W_0 of the tail basis may be
// updated in place (it is read only at that cell, the stencil vector is W_J).
// sin via the register-light reduction of nl_sincos (sine-Gordon's -sin(id u))
__device__ __forceinline__ double sin_rl(double x) {
  double sn, cs;
  nl_sincos(x, sn, cs);
  return sn;
}

#ifndef NLS_TAIL_LDS_PAD
#define NLS_TAIL_LDS_PAD 0
#endif
#ifndef NLS_TAIL_WPE
#define NLS_TAIL_WPE 1  // waves per SIMD the fused tail's registers must allow (launch bound; 1: unconstrained)
#endif
template <class S, int DIM, int M, bool ANI, int MODE>
__global__ __launch_bounds__(NTHREADS, NLS_TAIL_WPE) void k_tail(TailArgs ta, Geo g) {
  static_assert(M >= 3, "the stencil vector must not be W_0 (updated in place)");
  constexpr int J = M - 2;
  constexpr int NF = tail_nf(MODE);
  constexpr bool KG = MODE == TAIL_KG_END || MODE == TAIL_KG_END1;
  constexpr int M2 = MODE == TAIL_KG_END ? M : 1;
  __shared__ S cf[NF][MMAX + 1];  // cf[f][k] for W_k (k <= J), cf[f][J+1] for L W_J
  __shared__ double c2[MMAX];     // KG: combination of the stored basis
#if NLS_TAIL_LDS_PAD
  // (occupancy experiment: LDS that caps the workgroups per CU)
  __shared__ volatile char lds_pad[NLS_TAIL_LDS_PAD];
  if (threadIdx.x == 0 && g.nx < 0) lds_pad[0] = 1;
#endif
  const KState *__restrict__ st = ta.st;
  if (threadIdx.x <= J + 1) {
    const int k = threadIdx.x;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const cplx fl = st->fin[f][J + 1];
      const cplx c = k <= J ? st->fin[f][k] - cmul(fl, st->coef[k]) : st->coef[J + 1].re * fl;
      if constexpr (std::is_same<S, cplx>::value) cf[f][k] = c;
      else cf[f][k] = c.re;
    }
  }
  if constexpr (MODE == TAIL_KG_END) {
    for (int k = threadIdx.x; k < M; k += NTHREADS) c2[k] = ta.st2->fin[0][k].re;
  }
  __syncthreads();
  S *__restrict__ W = static_cast<S *>(ta.W);
  const double *__restrict__ W2 = static_cast<const double *>(ta.W2);
  const int64_t vs = ta.vs;
  const S *__restrict__ VJ = W + (int64_t)J * vs;
  // the per-cell inputs besides the stencil vector: the J streamed basis vectors, the
  // KG sinc^2 basis, and the epilogue's own reads (e0, e1 of the state type, d0 f64)
  struct TBuf {
    S wk[J];
    double w2[M2];
    S e0, e1;
    double d0;
  };
  auto load = [&](int q, TBuf &b) {
    const S *__restrict__ src = W + q;
#pragma unroll
    for (int k = 0; k < J; ++k) {
      b.wk[k] = ld_nt(src);
      src += vs;
    }
    if constexpr (KG) {
      const double *__restrict__ s2 = W2 + q;
#pragma unroll
      for (int k = 0; k < M2; ++k) {
        b.w2[k] = ld_nt(s2);
        s2 += vs;
      }
    }
    b.e0 = b.e1 = zero<S>();
    b.d0 = 0.0;
    if constexpr (MODE == TAIL_NLSE) {
      if (ta.nonlin >= 2) b.d0 = ta.mf[q];
    } else if constexpr (MODE == TAIL_SG_MID || MODE == TAIL_GG_MID) {
      b.d0 = ta.mf[q];
      b.e0 = static_cast<const S *>(ta.up)[q];
    } else if constexpr (MODE == TAIL_SG_END) {
      b.e0 = static_cast<const S *>(ta.u)[q];
      b.e1 = static_cast<const S *>(ta.up)[q];
    } else if constexpr (KG) {
      b.e0 = static_cast<const S *>(ta.up)[q];
    } else if constexpr (MODE == TAIL_SEWI_END) {
      b.e0 = static_cast<const S *>(ta.u)[q];
      b.e1 = static_cast<const S *>(ta.e)[q];
    }
  };
  // y_f = sum_k cf[f][k] W_k + cf[f][J+1] L W_J, then the step's epilogue at cell q.
  // Four partial sums (term k into sum k mod 4): one chain of 2(J+2) dependent f64 FMAs
  // per component left the waves stalled on the chain (512^3, m = 16: tail 6.02 ->
  // 5.92 ms with four, same box, profiles/r04/ab_tail.txt)
  auto finish = [&](int q, const S &cur, const S &lap, const TBuf &b) {
    S y[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      S a4[4] = {zero<S>(), zero<S>(), zero<S>(), zero<S>()};
#pragma unroll
      for (int k = 0; k < J; ++k) smac(a4[k & 3], cf[f][k], b.wk[k]);
      smac(a4[J & 3], cf[f][J], cur);
      smac(a4[(J + 1) & 3], cf[f][J + 1], lap);
      y[f] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    }
    if constexpr (MODE == TAIL_NLSE) {
      cplx un, w0;
      nl_half2(to_c(y[0]), b.d0, ta.dt, ta.nonlin, ta.s1, ta.s2, un, w0);  // u = N(y), W_0 = N(u)
      if (ta.u) st_nt(static_cast<cplx *>(ta.u) + q, un);  // NULL: another step follows
      st_nt(reinterpret_cast<cplx *>(W) + q, w0);
    } else if constexpr (MODE == TAIL_SG_MID) {
      st_nt(static_cast<double *>(ta.out) + q, b.d0 * (-sin_rl(to_c(y[0]).re)));
      st_nt(static_cast<double *>(ta.up) + q, 2 * to_c(y[1]).re - to_c(b.e0).re);
    } else if constexpr (MODE == TAIL_GG_MID) {  // e.g. phi4_single.cuh:38-45
      st_nt(static_cast<double *>(ta.out) + q, -b.d0 * gg_force(to_c(y[0]).re, ta.nonlin));
      st_nt(static_cast<double *>(ta.up) + q, 2 * to_c(y[1]).re - to_c(b.e0).re);
    } else if constexpr (MODE == TAIL_SG_END) {
      const double uo = to_c(b.e0).re;
      static_cast<double *>(ta.u)[q] = to_c(b.e1).re + (ta.dt * ta.dt) * to_c(y[0]).re;
      static_cast<double *>(ta.up)[q] = uo;
    } else if constexpr (KG) {
      double ys = 0.0;
      if constexpr (MODE == TAIL_KG_END1) {
        ys = b.w2[0];
      } else {
#pragma unroll
        for (int k = 0; k < M2; ++k) ys += c2[k] * b.w2[k];
      }
      const double uo = to_c(b.wk[0]).re;  // u is W_0 of the tail (cos) basis
      const double un = (to_c(y[0]).re * 2.0 - to_c(b.e0).re) + ys * (ta.dt * ta.dt);
      reinterpret_cast<double *>(W)[q] = un;
      static_cast<double *>(ta.up)[q] = uo;
      static_cast<double *>(ta.v)[q] = (un - uo) / ta.dt;
    } else if constexpr (MODE == TAIL_COMBINE_W0) {
      W[q] = y[0];
    } else if constexpr (MODE == TAIL_COMBINE) {
      static_cast<S *>(ta.out)[q] = y[0];
    } else {  // TAIL_SEWI_END
      static_cast<cplx *>(ta.u)[q] = to_c(y[0]) - cmul({0.0, 2.0 * ta.dt}, to_c(b.e1));
      static_cast<cplx *>(ta.up)[q] = to_c(b.e0);
    }
  };
  // one row per thread: with the epilogue at the end of the combination, two
  // rows no longer fit in the 256 registers of two waves per SIMD
  constexpr int RB = FUSED_RB;
  march<S, DIM, RB, true, ANI>(VJ, g, [&](const int *p, const S *cur, const S *lap, const bool *ok) {
    TBuf b[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r)
      if (ok[r]) load(p[r], b[r]);
    asm volatile("" ::: "memory");  // keep the coefficient reads in LDS
#pragma unroll
    for (int r = 0; r < RB; ++r)
      if (ok[r]) finish(p[r], cur[r], lap[r], b[r]);
  });
}

#define NLS_J_LIST(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) \
  X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) \
  X(28) X(29) X(30)
#define NLS_MF_LIST(X) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) \
  X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) \
  X(29) X(30) X(31) X(32)
#define NLS_M_LIST(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) \
  X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) \
  X(29) X(30) X(31) X(32)

}  // namespace nls
