// bw_probe3.hip -- K read streams + 1 write: separate vectors (vector-major)
// vs chunk-interleaved (AoSoA: the K vectors of one 64-cell chunk contiguous).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe3 tools/bw_probe3.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

struct __align__(16) c2 { double x, y; };
typedef double v2d __attribute__((ext_vector_type(2)));
#define CHECK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(_e), __LINE__); exit(1);} } while (0)
__device__ inline c2 ldnt(const c2* p) { v2d v = __builtin_nontemporal_load((const v2d*)p); return {v.x, v.y}; }
__device__ inline void stnt(c2* p, c2 v) { v2d t; t.x = v.x; t.y = v.y; __builtin_nontemporal_store(t, (v2d*)p); }

// vector-major: W[k*vs + p]; output out[p]
template <int K, bool NTS>
__global__ __launch_bounds__(256) void kV(const c2* __restrict__ W, long vs, long n, c2* __restrict__ out) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long)gridDim.x * 256) {
    c2 s = {0, 0};
#pragma unroll
    for (int k = 0; k < K; ++k) { c2 v = ldnt(W + k * vs + p); s.x += v.x * (k + 1); s.y += v.y; }
    if (NTS) stnt(out + p, s); else out[p] = s;
  }
}
// chunk-interleaved: chunk c (64 cells) holds M vectors contiguously: W[(c*M + k)*64 + l];
// reads k < K, writes slot K of the same chunk
template <int K, int M, bool NTS>
__global__ __launch_bounds__(256) void kI(c2* __restrict__ W, long n) {
  const int lane = threadIdx.x & 63;
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long)gridDim.x * 256) {
    const long c = p >> 6;
    const c2* base = W + c * M * 64 + lane;
    c2 s = {0, 0};
#pragma unroll
    for (int k = 0; k < K; ++k) { c2 v = ldnt(base + k * 64); s.x += v.x * (k + 1); s.y += v.y; }
    if (NTS) stnt(W + (c * M + K) * 64 + lane, s); else W[(c * M + K) * 64 + lane] = s;
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
  const long n = 1L << 27, vs = n + 256;
  const int M = 16;
  c2 *W, *out;
  CHECK(hipMalloc(&W, (size_t)M * vs * sizeof(c2)));
  CHECK(hipMalloc(&out, (size_t)n * sizeof(c2)));
  CHECK(hipMemset(W, 0, (size_t)M * vs * sizeof(c2)));
  auto rep = [&](const char* nm, int K, float ms) {
    printf("%-36s K=%2d %7.3f ms %7.1f GB/s\n", nm, K, ms, (K + 1) * n * 16.0 / 1e9 / (ms * 1e-3));
  };
  for (int grid : {1024, 2048, 8192, (int)(n / 256)}) {
    printf("grid %d\n", grid);
    rep("vector-major plainST", 15, timeit([&] { kV<15, false><<<grid, 256>>>(W, vs, n, out); }, 3));
    rep("vector-major ntST", 15, timeit([&] { kV<15, true><<<grid, 256>>>(W, vs, n, out); }, 3));
    rep("interleaved plainST", 15, timeit([&] { kI<15, M, false><<<grid, 256>>>(W, n); }, 3));
    rep("interleaved ntST", 15, timeit([&] { kI<15, M, true><<<grid, 256>>>(W, n); }, 3));
    rep("vector-major ntST", 4, timeit([&] { kV<4, true><<<grid, 256>>>(W, vs, n, out); }, 3));
    rep("interleaved ntST", 4, timeit([&] { kI<4, M, true><<<grid, 256>>>(W, n); }, 3));
    rep("vector-major ntST", 8, timeit([&] { kV<8, true><<<grid, 256>>>(W, vs, n, out); }, 3));
    rep("interleaved ntST", 8, timeit([&] { kI<8, M, true><<<grid, 256>>>(W, n); }, 3));
  }
  return 0;
}
