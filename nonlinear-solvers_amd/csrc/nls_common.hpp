// nls_common.hpp -- device helpers shared by the stencil, reduction and
// pointwise kernels: wave64 / workgroup reductions, non-temporal memory
// operations, cross-lane moves.
#pragma once
#include "nls_device.hpp"

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

// partials are stored column-major: out[k * stride + off + blockIdx.x] (stride =
// gridDim.x, off = 0 unless several launches share one partial array), so the
// single-workgroup reduction reads each column with coalesced 1 KiB wave loads.
template <int NA>
__device__ __forceinline__ void block_store(cplx (&v)[NA], cplx *__restrict__ out, int stride, int off) {
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
    out[(int64_t)k * stride + off + blockIdx.x] = s;
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


// Dynamic tile queue (Geo::tq, the fused tail's march): a resident grid whose workgroups take
// the next tile index from a global counter, so the tiles being streamed at any moment
// are the next ones in order -- a compact address window, which streams faster than
// long per-workgroup marches that drift apart (DESIGN.md section 4, round 3;
// tools/bw_probe6.hip: 15 reads + 1 write at 6.59 TB/s with 4-plane tiles against
// 5.82-5.90 for one 256-plane march per workgroup).  Only for kernels without
// per-workgroup partial sums: the tile -> workgroup assignment varies run to run.
__device__ __forceinline__ int tq_next(int32_t *tq) {
  __shared__ int s_tile;
  __syncthreads();  // every thread has read the previous index
  if (threadIdx.x == 0) s_tile = atomicAdd(tq, 1);
  __syncthreads();
  return s_tile;
}
// XCD-banded tile queue (NLS_TQ_XCD): eight heads, one per band of tiles; workgroup b
// takes the tiles of band b % 8 (blocks b, b + 8 share an XCD -- which XCD does not
// matter) and, once its band is empty, helps the next bands.  A band is a range of tile
// rows jt (all x tiles, all z chunks; 2D or ny < 8 tiles: a range of chunks kt), dealt
// x-fastest, then jt, then kt: the y-neighbour tiles whose edge rows a tile's stencil
// re-reads run at the same time on the same XCD (its L2), and every band moves through
// the z chunks at the same pace (one compact streamed window, as the single queue).
// Heads at tq[TQ_STRIDE * h] (own 128-B lines), the done counter at tq[TQ_STRIDE * 8].
// Off: the 512^3 tail took 6.04-6.06 ms against 5.75 with the single queue (same box,
// profiles/r05/ab_r5d.txt) -- the band's shared L2 does not pay for losing the chip-wide
// dispatch order of the single head
#ifndef NLS_TQ_XCD
#define NLS_TQ_XCD 0
#endif
#ifndef NLS_TQ_XCD_PHASE
#define NLS_TQ_XCD_PHASE 0
#endif
constexpr int TQ_STRIDE = 32;
constexpr int TQ_WORDS = TQ_STRIDE * 9;
__device__ __forceinline__ int tq_next_xcd(int32_t *tq, int ntx, int nty, int ntz) {
  __shared__ int s_tile;
  __syncthreads();  // every thread has read the previous index
  if (threadIdx.x == 0) {
    const bool yb = nty >= 8;  // band over tile rows, else over z chunks
    const int nb = yb ? nty : ntz, h0 = (int)(blockIdx.x & 7);
    int tile = ntx * nty * ntz;  // none left
    for (int d = 0; d < 8; ++d) {
      const int h = (h0 + d) & 7, lo = h * nb / 8, hi = (h + 1) * nb / 8;
      const int cnt = ntx * (hi - lo) * (yb ? ntz : nty);
      if (cnt == 0) continue;
      const int t = atomicAdd(tq + TQ_STRIDE * h, 1);
      if (t >= cnt) continue;
      const int it = t % ntx, r = t / ntx;
      // NLS_TQ_XCD_PHASE: band h starts h * PHASE tile rows into its range (the bands'
      // concurrent rows then sit (band + h * PHASE) rows apart, not a power of two of rows)
      const int jt = yb ? lo + (r % (hi - lo) + h * NLS_TQ_XCD_PHASE) % (hi - lo) : r % nty;
      const int kt = yb ? r / (hi - lo) : lo + r / nty;
      tile = (kt * nty + jt) * ntx + it;
      break;
    }
    s_tile = tile;
  }
  __syncthreads();
  return s_tile;
}
// the last workgroup to finish (every other one has taken its last index) resets the queue
__device__ __forceinline__ void tq_done(int32_t *tq) {
  if (NLS_TQ_XCD) {
    if (threadIdx.x == 0 && atomicAdd(tq + TQ_STRIDE * 8, 1) == (int)gridDim.x - 1) {
      for (int h = 0; h < 8; ++h) atomicExch(tq + TQ_STRIDE * h, 0);
      atomicExch(tq + TQ_STRIDE * 8, 0);
    }
    return;
  }
  if (threadIdx.x == 0 && atomicAdd(tq + 1, 1) == (int)gridDim.x - 1) {
    atomicExch(tq, 0);
    atomicExch(tq + 1, 0);
  }
}

// ---------------------------------------------------------------------------
// Nonlinear half step, tau = 1j*dt
//  0 cubic (nlse_solver.hpp:66-69): out = exp(-0.5*tau*rho) u, rho = re^2 + im^2
//  1 cubic-quintic (device/nlse_cq_solver.hpp:16-39): d = |u|*|u|, rho = s1 d + s2 d^2
//  2 G2 cubic with focusing field (nlsolvers/device/include/nlse_dev.hpp:20-40):
//    out = u * exp(0.5*tau * m|u|^2)   (note the sign: G2 integrates with +tau)
//  3 G2 cubic-quintic (nlsolvers/device/include/nlse_cubic_quintic.cuh:9-40):
//    out = u * exp(-0.5*tau * m (s1 d + s2 d^2)), real s1, s2
//
// sin/cos of the phase without OCML's sincos, whose large-argument (Payne-Hanek)
// path needs so many registers that it sets the register budget of every
// streaming kernel ending in this step (k_final_fused: 1 wave/SIMD instead of 2).
// Cody-Waite reduction r = x - n pi/2 with a two-term FMA split of pi/2 (absolute
// error ~1e-16 for every |x| < 2^53), then Taylor polynomials on |r| <= pi/4 to
// r^17 / r^18 (truncation < 1e-19); ~1 ulp against libm in the common case of a
// small phase (dt |u|^2 / 2), where n = 0 and r = x exactly.
__device__ __forceinline__ void nl_sincos(double x, double &sn, double &cs) {
  const double n = rint(x * 0.63661977236758134308);
  double r = fma(-n, 1.5707963267948966, x);
  r = fma(-n, 6.123233995736766e-17, r);
  const double z = r * r;
  double ps = 1.0 / 355687428096000.0;            //  1/17!
  ps = fma(ps, z, -1.0 / 1307674368000.0);        // -1/15!
  ps = fma(ps, z, 1.0 / 6227020800.0);            //  1/13!
  ps = fma(ps, z, -1.0 / 39916800.0);             // -1/11!
  ps = fma(ps, z, 1.0 / 362880.0);                //  1/9!
  ps = fma(ps, z, -1.0 / 5040.0);                 // -1/7!
  ps = fma(ps, z, 1.0 / 120.0);                   //  1/5!
  ps = fma(ps, z, -1.0 / 6.0);                    // -1/3!
  const double s = fma(r * z, ps, r);
  double pc = 1.0 / 6402373705728000.0;           //  1/18!
  pc = fma(pc, z, -1.0 / 20922789888000.0);       // -1/16!
  pc = fma(pc, z, 1.0 / 87178291200.0);           //  1/14!
  pc = fma(pc, z, -1.0 / 479001600.0);            // -1/12!
  pc = fma(pc, z, 1.0 / 3628800.0);               //  1/10!
  pc = fma(pc, z, -1.0 / 40320.0);                // -1/8!
  pc = fma(pc, z, 1.0 / 720.0);                   //  1/6!
  pc = fma(pc, z, -1.0 / 24.0);                   // -1/4!  (times -z^2 below)
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;                      // fdlibm-style split of 1 - z/2
  const double c = w + (((1.0 - w) - hz) - (z * z) * pc);
  const int q = (int)(n - 4.0 * floor(0.25 * n));  // quadrant, 0..3
  sn = q == 0 ? s : q == 1 ? c : q == 2 ? -s : -c;
  cs = q == 0 ? c : q == 1 ? -s : q == 2 ? -c : s;
}

// g = -m F(y) of the G2 Gautschi family (GautschiForce, nls_device.hpp):
// sg_single.cuh:18, sg_double.cuh:19, sg_hyperbolic.cuh:18, phi4_single.cuh:18.
// sin via the register-light nl_sincos; sinh from one exp (|y| >= 2^-5) or its
// Taylor series (below, where exp(y) - exp(-y) would cancel).
__device__ __forceinline__ double gg_force(double y, int kind) {
  double sn, cs;
  switch (kind) {
    case 1: {
      double s2, c2;
      nl_sincos(y, sn, cs);
      nl_sincos(0.5 * y, s2, c2);
      return sn + s2;
    }
    case 2: {
      const double a = fabs(y);
      if (a < 0.03125) {
        const double z = y * y;
        return y + y * z * (1.0 / 6.0 + z * (1.0 / 120.0 + z * (1.0 / 5040.0 + z * (1.0 / 362880.0))));
      }
      const double e = exp(a);
      return copysign(0.5 * (e - 1.0 / e), y);
    }
    case 3: return y + y * y * y;
    default: nl_sincos(y, sn, cs); return sn;
  }
}

__device__ __forceinline__ cplx nl_half(cplx u, double mval, double dt, int nonlin, cplx s1, cplx s2) {
  if (nonlin == 3) {  // G2 cubic-quintic: rho = m (s1 d + s2 d^2), real s (nlse_cubic_quintic.cuh:21-22)
    const double d = u.re * u.re + u.im * u.im;
    const double ph = (-0.5 * dt) * (mval * (s1.re * d + s2.re * (d * d)));
    double sn, cs;
    nl_sincos(ph, sn, cs);
    return {cs * u.re - sn * u.im, cs * u.im + sn * u.re};
  }
  if (nonlin == 0 || nonlin == 2) {
    const double x = u.re * u.re + u.im * u.im;
    const double ph = nonlin == 0 ? (-0.5 * dt) * x : (0.5 * dt) * (mval * x);
    double sn, cs;
    nl_sincos(ph, sn, cs);
    return {cs * u.re - sn * u.im, cs * u.im + sn * u.re};
  }
  const double a = hypot(u.re, u.im);
  const double d = a * a;
  const cplx rho = d * s1 + (d * d) * s2;
  const cplx z = cmul({-0.0, -0.5 * dt}, rho);
  const double er = exp(z.re);
  double sn, cs;
  nl_sincos(z.im, sn, cs);
  return cmul({er * cs, er * sn}, u);
}

// Both half steps of the fused tail's epilogue: u = N(y) and the next start vector
// N(u) = N(N(y)).  For the unit-modulus phases (nonlin 0, 2, 3: rho depends on |u|
// only and |N(y)| = |y|) N(N(y)) = y exp(2 i ph): the second phase comes from the
// first by the double-angle identities instead of a second sin/cos evaluation (one
// rounding away from applying N twice, far below every parity tolerance).  The
// complex-sigma cubic-quintic (nonlin 1) changes |u| and applies N twice.
#ifndef NLS_NL_HALF2
#define NLS_NL_HALF2 1
#endif
__device__ __forceinline__ void nl_half2(cplx y, double mval, double dt, int nonlin, cplx s1, cplx s2, cplx &u,
                                         cplx &u2) {
  if (nonlin == 1 || !NLS_NL_HALF2) {
    u = nl_half(y, mval, dt, nonlin, s1, s2);
    u2 = nl_half(u, mval, dt, nonlin, s1, s2);
    return;
  }
  const double d = y.re * y.re + y.im * y.im;
  const double ph = nonlin == 3 ? (-0.5 * dt) * (mval * (s1.re * d + s2.re * (d * d)))
                  : nonlin == 0 ? (-0.5 * dt) * d
                                : (0.5 * dt) * (mval * d);
  double sn, cs;
  nl_sincos(ph, sn, cs);
  u = {cs * y.re - sn * y.im, cs * y.im + sn * y.re};
  const double c2 = fma(cs, cs, -sn * sn), s2n = 2.0 * sn * cs;
  u2 = {c2 * y.re - s2n * y.im, c2 * y.im + s2n * y.re};
}

}  // namespace nls
