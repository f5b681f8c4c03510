// bw_probe2.hip -- K-stream read + 1 write, varying the contiguous chunk per wave
// and the work distribution (persistent grid-stride vs one block per chunk).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe2 tools/bw_probe2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

struct __align__(16) c2 { double x, y; };
typedef double v2d __attribute__((ext_vector_type(2)));
#define CHECK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(_e), __LINE__); exit(1);} } while (0)

__device__ inline c2 ldnt(const c2* p) { v2d v = __builtin_nontemporal_load((const v2d*)p); return {v.x, v.y}; }

// Each wave owns one 64-element (1 KiB) chunk per "row"; a block's 4 waves take
// rows spaced by ROWSTRIDE elements (ROWSTRIDE = 64: contiguous 4 KiB per block;
// = 512: 3D-tile-like 8 KiB apart).  Each wave marches PL planes (stride P).
template <int K, int ROWSTRIDE, int PL>
__global__ __launch_bounds__(256) void kT(const c2* __restrict__ W, long vs, long P, long ntiles,
                                          long tiles_per_plane_row, c2* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    // tile -> (x chunk, row group, plane chunk)
    long xr = t % tiles_per_plane_row, zc = t / tiles_per_plane_row;
    long base = (xr / (ROWSTRIDE / 64)) * (4 * ROWSTRIDE) + (xr % (ROWSTRIDE / 64)) * 64 + w * ROWSTRIDE + lane;
    for (int q = 0; q < PL; ++q) {
      long p = (zc * PL + q) * P + base;
      c2 s = {0, 0};
#pragma unroll
      for (int k = 0; k < K; ++k) { c2 v = ldnt(W + k * vs + p); s.x += v.x * (k + 1); s.y += v.y; }
      out[p] = s;
    }
  }
}

template <class F> float timeit(F f, int reps) {
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  f(); CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a)); for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

int main() {
  const long P = 512L * 512, nz = 512, n = P * nz, vs = n + 256;
  const int K = 15;
  c2 *W, *out;
  CHECK(hipMalloc(&W, (size_t)K * vs * sizeof(c2)));
  CHECK(hipMalloc(&out, (size_t)n * sizeof(c2)));
  CHECK(hipMemset(W, 0, (size_t)K * vs * sizeof(c2)));
  auto rep = [&](const char* nm, float ms) {
    printf("%-44s %7.3f ms %7.1f GB/s\n", nm, ms, (K + 1) * n * 16.0 / 1e9 / (ms * 1e-3));
  };
  const long tpr = P / 256;  // tiles per plane (each tile = 256 cells per plane)
  for (int grid : {512, 1024, 2048, 8192}) {
    char buf[128];
    long nt16 = tpr * (nz / 16), nt4 = tpr * (nz / 4), nt1 = tpr * nz;
    snprintf(buf, 128, "contig4K  PL=16 grid=%d", grid);
    rep(buf, timeit([&] { kT<K, 64, 16><<<grid, 256>>>(W, vs, P, nt16, tpr, out); }, 3));
    snprintf(buf, 128, "rows8K    PL=16 grid=%d", grid);
    rep(buf, timeit([&] { kT<K, 512, 16><<<grid, 256>>>(W, vs, P, nt16, tpr, out); }, 3));
    snprintf(buf, 128, "contig4K  PL=4  grid=%d", grid);
    rep(buf, timeit([&] { kT<K, 64, 4><<<grid, 256>>>(W, vs, P, nt4, tpr, out); }, 3));
    snprintf(buf, 128, "contig4K  PL=1  grid=%d", grid);
    rep(buf, timeit([&] { kT<K, 64, 1><<<grid, 256>>>(W, vs, P, nt1, tpr, out); }, 3));
  }
  long nt1 = tpr * nz;
  rep("contig4K PL=1 full grid", timeit([&] { kT<K, 64, 1><<<nt1, 256>>>(W, vs, P, nt1, tpr, out); }, 3));
  rep("rows8K   PL=1 full grid", timeit([&] { kT<K, 512, 1><<<nt1, 256>>>(W, vs, P, nt1, tpr, out); }, 3));
  return 0;
}
