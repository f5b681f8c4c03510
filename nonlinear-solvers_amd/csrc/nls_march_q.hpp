// nls_march_q.hpp -- the stencil march of the update passes with the next
// alpha folded in (included by nls_stencil.hpp inside namespace nls, after march()).
//
// march_q<...>(V, g, q, fn) is march<..., PLANE = true, ...>(V, g, fn) that
// additionally accumulates
//     q += Y^H L Y,   Y = L V   (the stencil result handed to fn),
// in the symmetric forward-coupling form of the alpha pass (each off-diagonal
// pair of the reference matrix once; laplacians.hpp:10-105 / G2 :54-218):
//   iso:  sum_p d_p |Y_p|^2 + 2 s sum_p Re(conj(Y_p) (Y_{p+1} + Y_{p+nx} + Y_{p+P}))
//   ani:  -s sum_{forward pairs (p,q)} w_pq |Y_p - Y_q|^2
// From q the reduction recovers the diagonal entry alpha_{j+1} of the NEXT
// Lanczos vector without reading it again (nls_reduce.hpp, "qa"), so the update
// pass j replaces the separate alpha pass j+1.
//
// Forward partners that are not in the thread's registers:
//   x+1 of lane 63        -> across the x-tile seam: lane 63 and lane 0 store their
//                            L V values in a side buffer E (1/32 of a vector) and
//                            k_xpairs adds those pairs (in-kernel alternatives --
//                            gathering, or a register queue of the x+1 column --
//                            cost a full alpha pass in single-lane memory
//                            instructions and remote-XCD latency)
//   y+1 of the last row   -> (3D) a halo row marched with its own register
//                            queue: the flat row after the wave's last row
//                            (row 0 of the next plane when that is the y-wrap)
//   z+1 of the last plane -> one extra "peek" plane per tile (L V only)
// Single-rank handles only: on a z-slab the peek of the last local plane would
// need a second ghost plane (multi-rank handles keep the alpha pass).
#pragma once

// one forward pair of the quadratic form: iso 2 s Re(conj(a) b) (the diagonal
// part d_p |a|^2 is added per cell), ani -s w |a - b|^2
template <class S, bool ANI>
__device__ __forceinline__ double qpair(const Geo &g, const S &a, const S &b, double w) {
  if constexpr (ANI) return -g.s * w * abs2(a - b);
  else return 2.0 * g.s * to_c(cj_mul(a, b)).re;
}

// Edge buffer layout: E[side][t][y][q], side 0 = the first x of x-tile t (lane 0 of
// chunk 0), side 1 = its last x (lane 63 of the last chunk); y = row (3D) or 0 (2D).
// A wave stages its seam values for the planes of a tile in LDS and writes them at
// the end of the tile as runs along q (single-lane 16-B stores per plane went to
// HBM as partial-line writes: +2.5 ms per 512^3 step).
__host__ __device__ inline int64_t xedge_index(const Geo &g, int64_t ntx, int side, int64_t q, int64_t y,
                                               int64_t t) {
  return ((side * ntx + t) * g.nyp + y) * g.nzl + q;
}
constexpr int SEAM_KZ = 64;  // planes per tile the LDS seam staging holds (else direct stores)

template <class S, int DIM, int RB, bool ANI, class Fn>
__device__ __forceinline__ void march_q(const S *__restrict__ V, const Geo &g, double &qacc,
                                        S *__restrict__ E, Fn &&fn) {
  const double *__restrict__ C = g.cf;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t ntx64, nty64, ntz64;
  tile_counts<DIM, RB>(g, ntx64, nty64, ntz64);
  const int ntx = (int)ntx64, nty = (int)nty64;
  const int tiles = (int)(ntx64 * nty64 * ntz64);
  const int T8 = tiles / 8;
  const int P = (int)g.P, nx = (int)g.nx, nyp = (int)g.nyp, qa = g.qa, qb = g.qb, kz = g.kz;
  const int z0 = (int)g.z0, npl = (int)g.npl;
  for (int t0 = blockIdx.x; t0 < tiles; t0 += gridDim.x) {
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
      const int q0 = qa + kt * kz;
      const int q1 = q0 + kz < qb ? q0 + kz : qb;
      bool rv[RB];
      int off[RB];
      S prev[RB], cur[RB], lprev[RB];
      double cprv[RB], ccur[RB];
      int rlast = 0;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        rv[r] = yb + r < nyp;
        if (rv[r]) rlast = r;
        off[r] = (yb + r) * nx + x;
        const bool ld = xin && rv[r];
        prev[r] = (ld && z0 + q0 > 0) ? V[(q0 - 1) * P + off[r]] : zero<S>();
        cur[r] = ld ? V[q0 * P + off[r]] : zero<S>();
        lprev[r] = zero<S>();
        if constexpr (ANI) {
          cprv[r] = (ld && z0 + q0 > 0) ? C[(q0 - 1) * P + off[r]] : 0.0;
          ccur[r] = ld ? C[q0 * P + off[r]] : 0.0;
        }
      }
      // halo row: the flat row after the last valid row (y-wrap: row 0 of plane q+1).
      // In tiles whose 4*RB rows are all valid, waves 0..2 take L V of their halo row
      // (the next wave's first row) from LDS; only wave 3 marches its own halo row.
      const bool shy = (jt + 1) * (4 * RB) <= nyp;  // workgroup-uniform
      const bool own_halo = !shy || w == 3;         // wave-uniform
      __shared__ S hls[2][4][64];
      __shared__ S seam[4][2][RB][SEAM_KZ];  // per wave: [side][row][plane - q0]
      const bool stage = q1 - q0 <= SEAM_KZ;
      const int yl = yb + rlast;
      const int hw = yl + 1 >= nyp ? 1 : 0;
      const int hy = hw ? 0 : yl + 1;
      const int hoff = hy * nx + x;
      S hprv, hcur;
      double chprv = 0.0, chcur = 0.0;
      {
        const int hq = q0 + hw;
        const bool hl = own_halo && xin;
        hprv = (hl && z0 + hq - 1 >= 0 && z0 + hq - 1 < npl) ? V[(hq - 1) * P + hoff] : zero<S>();
        hcur = (hl && z0 + hq < npl) ? V[hq * P + hoff] : zero<S>();
        if constexpr (ANI) {
          chprv = (hl && z0 + hq - 1 >= 0 && z0 + hq - 1 < npl) ? C[(hq - 1) * P + hoff] : 0.0;
          chcur = (hl && z0 + hq < npl) ? C[hq * P + hoff] : 0.0;
        }
      }
      const bool bx = (x == 0) || (x == nx - 1);
      for (int q = q0; q <= q1; ++q) {
        const int gq = z0 + q;
        const bool peek = q == q1;
        if (peek && !(gq < npl)) break;  // wave-uniform: no plane above the tile
        const bool bz = gq == 0 || gq == npl - 1;
        const bool has_next = gq + 1 < npl;
        S next[RB], lapv[RB];
        double cnxt[RB], wxpv[RB], wypv[RB], wzmv[RB];
        int pv[RB];
        bool okv[RB], exv[RB];
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
          wxpv[r] = wypv[r] = wzmv[r] = 0.0;
          exv[r] = false;
          if (!rv[r]) continue;  // wave-uniform
          const int p = q * P + off[r];
          const int y = yb + r;
          const bool eym = gq > 0 || y > 0;
          const bool eyp = gq < npl - 1 || y < nyp - 1;
          const bool inner_yp = r + 1 < RB && rv[r + 1 < RB ? r + 1 : r];
          S ym, yp;
          if (r > 0) ym = cur[r - 1];
          else ym = (xin && eym) ? V[p - nx] : zero<S>();
          if (inner_yp) yp = cur[r + 1 < RB ? r + 1 : r];
          else yp = (xin && eyp) ? V[p + nx] : zero<S>();
          S xm = shfl_up1(cur[r]), xp = shfl_dn1(cur[r]);
          const bool edge_ld = ((lane == 0 && x > 0) || (lane == 63 && x + 1 < nx)) && xin;
          const S xe = edge_ld ? V[p + (lane == 0 ? -1 : 1)] : zero<S>();
          if (lane == 0) xm = xe;
          if (lane == 63) xp = xe;
          if (!(x > 0)) xm = zero<S>();
          if (!(x + 1 < nx)) xp = zero<S>();
          exv[r] = eyp;
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
            wxpv[r] = wxp;
            wypv[r] = wyp;
            wzmv[r] = wzm;
          } else {
            const bool bnd = bx || bz || y == 0 || y == nyp - 1;
            lap = g.s * (((prev[r] + next[r]) + (xm + xp)) + (ym + yp)) +
                  (bnd ? g.sd_bd : g.sd_in) * cur[r];
          }
          okv[r] = xin;
          lapv[r] = lap;
        }
        if (!peek) {
          fn(pv, cur, lapv, okv);
          // L V on the halo row (its y-1 neighbour is the last row; flat p + nx wraps)
          S hlap = zero<S>();
          double wyl = 0.0;  // ani weight of the (last row, halo) pair
          if constexpr (ANI) wyl = wypv[rlast];
          S hnext = zero<S>();
          double chnext = 0.0;
          if (shy) {  // publish this wave's first row, take the next wave's
            hls[q & 1][w][lane] = lapv[0];
            __syncthreads();
            if (w < 3) hlap = hls[q & 1][w + 1][lane];
          }
          if (own_halo) {
            const int hq = q + hw;  // local plane of the halo cell
            const int ghq = z0 + hq;
            const bool hexists = ghq < npl;
            const bool hnext_ok = ghq + 1 < npl;
            hnext = (xin && hnext_ok) ? V[(hq + 1) * P + hoff] : zero<S>();
            if constexpr (ANI) chnext = (xin && hnext_ok) ? C[(hq + 1) * P + hoff] : 0.0;
            const int ph = hq * P + hoff;
            const bool heyp = ghq < npl - 1 || hy < nyp - 1;
            const S hyp = (xin && hexists && heyp) ? V[ph + nx] : zero<S>();
            S hxm = shfl_up1(hcur), hxp = shfl_dn1(hcur);
            const bool hedge = ((lane == 0 && x > 0) || (lane == 63 && x + 1 < nx)) && xin && hexists;
            const S hxe = hedge ? V[ph + (lane == 0 ? -1 : 1)] : zero<S>();
            if (lane == 0) hxm = hxe;
            if (lane == 63) hxp = hxe;
            if (!(x > 0)) hxm = zero<S>();
            if (!(x + 1 < nx)) hxp = zero<S>();
            if constexpr (ANI) {
              const double cc = chcur;
              const double cym = ccur[rlast];
              const double cyp = (xin && hexists && heyp) ? C[ph + nx] : 0.0;
              double cxm = shfl_up1(cc), cxp = shfl_dn1(cc);
              const double cxe = hedge ? C[ph + (lane == 0 ? -1 : 1)] : 0.0;
              if (lane == 0) cxm = cxe;
              if (lane == 63) cxp = cxe;
              const double wxm = face_w(x > 0, cc, cxm), wxp = face_w(x + 1 < nx, cc, cxp);
              const double wym = face_w(true, cc, cym), wyp = face_w(heyp, cc, cyp);
              const double wzm = face_w(ghq > 0, cc, chprv), wzp = face_w(hnext_ok, cc, chnext);
              hlap = g.s * ((((wzm * hprv + wzp * hnext) + (wxm * hxm + wxp * hxp)) +
                             (wym * cur[rlast] + wyp * hyp)) -
                            (((wzm + wzp) + (wxm + wxp)) + (wym + wyp)) * hcur);
            } else {
              const bool hbnd = bx || ghq == 0 || ghq == npl - 1 || hy == 0 || hy == nyp - 1;
              hlap = g.s * (((hprv + hnext) + (hxm + hxp)) + (cur[rlast] + hyp)) +
                     (hbnd ? g.sd_bd : g.sd_in) * hcur;
            }
          }
          // forward pairs of plane q: x+1 (inside the tile) and y+1
#pragma unroll
          for (int r = 0; r < RB; ++r) {
            const S yx = shfl_dn1(lapv[r]);
            if (!rv[r] || !xin) continue;
            const S yv = lapv[r];
            double acc = 0.0;
            if constexpr (!ANI) {
              const bool bnd = bx || bz || yb + r == 0 || yb + r == nyp - 1;
              acc += (bnd ? g.sd_bd : g.sd_in) * abs2(yv);
            }
            if (x + 1 < nx && lane != 63) acc += qpair<S, ANI>(g, yv, yx, wxpv[r]);
            // x-tile seam: the pair (lane 63, next tile's lane 0) is added by k_xpairs
            if (lane == 0 || lane == 63) {
              const int side = lane == 0 ? 0 : 1;
              if (stage) seam[w][side][r][q - q0] = yv;
              else E[xedge_index(g, ntx, side, q, yb + r, it)] = yv;
            }
            if (r < rlast) acc += qpair<S, ANI>(g, yv, lapv[r + 1 < RB ? r + 1 : r], wypv[r]);
            else if (exv[r]) acc += qpair<S, ANI>(g, yv, hlap, wyl);
            qacc += acc;
          }
          hprv = hcur;
          hcur = hnext;
          if constexpr (ANI) {
            chprv = chcur;
            chcur = chnext;
          }
        }
        // z pair (plane q-1, plane q); its ani weight is wzm of plane q
        if (q > q0) {
#pragma unroll
          for (int r = 0; r < RB; ++r)
            if (rv[r] && xin) qacc += qpair<S, ANI>(g, lprev[r], lapv[r], wzmv[r]);
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          lprev[r] = lapv[r];
          prev[r] = cur[r];
          cur[r] = next[r];
          if constexpr (ANI) {
            cprv[r] = ccur[r];
            ccur[r] = cnxt[r];
          }
        }
      }
      if (stage) {  // the tile's seam values, one run along q per side and row
        __builtin_amdgcn_wave_barrier();
        for (int i = lane; i < q1 - q0; i += 64) {
#pragma unroll
          for (int r = 0; r < RB; ++r) {
            if (!rv[r]) continue;
            E[xedge_index(g, ntx, 0, q0 + i, yb + r, it)] = seam[w][0][r][i];
            if (it * 64 + 63 < nx) E[xedge_index(g, ntx, 1, q0 + i, yb + r, it)] = seam[w][1][r][i];
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    } else {
      const int q0 = qa + (kt * 4 + w) * kz;
      if (q0 >= qb) continue;  // wave-uniform
      const int q1 = q0 + kz < qb ? q0 + kz : qb;
      __shared__ S seam2[4][2][SEAM_KZ];  // per wave: [side][row - q0]
      const bool stage = q1 - q0 <= SEAM_KZ;
      int xr[RB];
      S prev[RB], cur[RB], lprev[RB];
      double cprv[RB], ccur[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        xr[r] = it * 64 * RB + 64 * r + lane;
        const bool ld = xr[r] < nx;
        prev[r] = (ld && z0 + q0 > 0) ? V[(q0 - 1) * P + xr[r]] : zero<S>();
        cur[r] = ld ? V[q0 * P + xr[r]] : zero<S>();
        lprev[r] = zero<S>();
        if constexpr (ANI) {
          cprv[r] = (ld && z0 + q0 > 0) ? C[(q0 - 1) * P + xr[r]] : 0.0;
          ccur[r] = ld ? C[q0 * P + xr[r]] : 0.0;
        }
      }
      for (int q = q0; q <= q1; ++q) {
        const int gq = z0 + q;
        const bool peek = q == q1;
        if (peek && !(gq < npl)) break;  // wave-uniform
        const bool bz = gq == 0 || gq == npl - 1;
        const bool has_next = gq + 1 < npl;
        S next[RB], lapv[RB];
        double cnxt[RB], wxpv[RB], wzmv[RB];
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
          wxpv[r] = wzmv[r] = 0.0;
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
            wxpv[r] = wxp;
            wzmv[r] = wzm;
          } else {
            const bool bnd = x == 0 || x == nx - 1 || bz;
            lap = g.s * ((prev[r] + next[r]) + (xm + xp)) + (bnd ? g.sd_bd : g.sd_in) * cur[r];
          }
          okv[r] = x < nx;
          lapv[r] = lap;
        }
        if (!peek) {
          fn(pv, cur, lapv, okv);
          // forward x pairs of row q: within the chunk and across chunk seams
#pragma unroll
          for (int r = 0; r < RB; ++r) {
            const S yx = shfl_dn1(lapv[r]);
            const S ys = bcast(lapv[r + 1 < RB ? r + 1 : r], 0);
            const int x = xr[r];
            if (!(x < nx)) continue;
            const S yv = lapv[r];
            double acc = 0.0;
            if constexpr (!ANI) {
              const bool bnd = x == 0 || x == nx - 1 || bz;
              acc += (bnd ? g.sd_bd : g.sd_in) * abs2(yv);
            }
            if (x + 1 < nx && !(lane == 63 && r + 1 == RB))
              acc += qpair<S, ANI>(g, yv, lane == 63 ? ys : yx, wxpv[r]);
            // x-tile seam: the pair (last chunk's lane 63, next tile's lane 0) -> k_xpairs
            if ((lane == 0 && r == 0) || (lane == 63 && r + 1 == RB)) {
              const int side = lane == 0 ? 0 : 1;
              if (stage) seam2[w][side][q - q0] = yv;
              else E[xedge_index(g, ntx, side, q, 0, it)] = yv;
            }
            qacc += acc;
          }
        }
        // row pair (q-1, q); its ani weight is wzm of row q
        if (q > q0) {
#pragma unroll
          for (int r = 0; r < RB; ++r)
            if (xr[r] < nx) qacc += qpair<S, ANI>(g, lprev[r], lapv[r], wzmv[r]);
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          lprev[r] = lapv[r];
          prev[r] = cur[r];
          cur[r] = next[r];
          if constexpr (ANI) {
            cprv[r] = ccur[r];
            ccur[r] = cnxt[r];
          }
        }
      }
      if (stage) {  // the tile's seam values as runs along q
        __builtin_amdgcn_wave_barrier();
        const bool rgt = it * 64 * RB + 64 * RB - 1 < nx;
        for (int i = lane; i < q1 - q0; i += 64) {
          E[xedge_index(g, ntx, 0, q0 + i, 0, it)] = seam2[w][0][i];
          if (rgt) E[xedge_index(g, ntx, 1, q0 + i, 0, it)] = seam2[w][1][i];
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
}


// The x-tile seam pairs of march_q's quadratic form: (last x of tile t, first x
// of tile t+1) for every row and plane, from the edge buffer; one partial per
// workgroup into column `col` of the update pass's partial array.
template <class S, int DIM, bool ANI>
__global__ __launch_bounds__(NTHREADS) void k_xpairs(const S *__restrict__ E, Geo g, int ntx, int tw,
                                                     cplx *__restrict__ part) {
  const double *__restrict__ C = g.cf;
  const int64_t npair = g.nzl * g.nyp * (ntx - 1);
  double acc = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; e < npair; e += (int64_t)gridDim.x * NTHREADS) {
    const int64_t q = e % g.nzl, rest = e / g.nzl;  // q fastest: runs of the E layout
    const int64_t y = rest % g.nyp, t = rest / g.nyp;
    const S a = E[xedge_index(g, ntx, 1, q, y, t)];
    const S b = E[xedge_index(g, ntx, 0, q, y, t + 1)];
    double w = 0.0;
    if constexpr (ANI) {
      const int64_t p = q * g.P + y * g.nx + (t + 1) * tw - 1;
      w = face_w(true, C[p], C[p + 1]);
    }
    acc += qpair<S, ANI>(g, a, b, w);
  }
  cplx v[1] = {{acc, 0.0}};
  block_store<1>(v, part, gridDim.x, 0);
}
