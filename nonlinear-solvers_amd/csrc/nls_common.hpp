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


}  // namespace nls
