// bw_probe.hip -- HBM bandwidth probe for the access patterns of the Lanczos
// update pass: K read streams + 1 write stream of complex<double>.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe tools/bw_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct __align__(16) c2 { double x, y; };

#define CHECK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(_e), __LINE__); exit(1);} } while (0)

// pattern A: lane-contiguous 16 B, grid-stride, K streams
template <int K>
__global__ __launch_bounds__(256) void kA(const c2* __restrict__ W, long vs, long n, c2* __restrict__ out) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long)gridDim.x * 256) {
    c2 s = {0, 0};
#pragma unroll
    for (int k = 0; k < K; ++k) { c2 w = W[k * vs + p]; s.x += w.x * (k + 1); s.y += w.y; }
    out[p] = s;
  }
}

// pattern B: each thread does U consecutive chunks (strided by 256 elements) per iteration
template <int K, int U>
__global__ __launch_bounds__(256) void kB(const c2* __restrict__ W, long vs, long n, c2* __restrict__ out) {
  const long step = (long)gridDim.x * 256 * U;
  for (long base = (long)blockIdx.x * 256 * U + threadIdx.x; base < n; base += step) {
    c2 s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = {0, 0};
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long p = base + u * 256;
        if (p < n) { c2 w = W[k * vs + p]; s[u].x += w.x * (k + 1); s[u].y += w.y; }
      }
#pragma unroll
    for (int u = 0; u < U; ++u) { long p = base + u * 256; if (p < n) out[p] = s[u]; }
  }
}

// pattern C: non-temporal loads/stores
template <int K>
__global__ __launch_bounds__(256) void kC(const c2* __restrict__ W, long vs, long n, c2* __restrict__ out) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long)gridDim.x * 256) {
    c2 s = {0, 0};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double* q = reinterpret_cast<const double*>(&W[k * vs + p]);
      double a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1);
      s.x += a * (k + 1); s.y += b;
    }
    double* o = reinterpret_cast<double*>(&out[p]);
    __builtin_nontemporal_store(s.x, o); __builtin_nontemporal_store(s.y, o + 1);
  }
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  f(); CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : (1L << 27);  // 134M cells = 512^3
  const long pad = argc > 2 ? atol(argv[2]) : 0;
  const long vs = n + pad;
  const int Kmax = 16;
  c2 *W, *out;
  CHECK(hipMalloc(&W, (size_t)Kmax * vs * sizeof(c2)));
  CHECK(hipMalloc(&out, (size_t)n * sizeof(c2)));
  CHECK(hipMemset(W, 0, (size_t)Kmax * vs * sizeof(c2)));
  int ncu; CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto report = [&](const char* name, int K, float ms) {
    double gb = (double)(K + 1) * n * 16 / 1e9;
    printf("%-28s K=%2d  %8.3f ms  %7.1f GB/s\n", name, K, ms, gb / (ms * 1e-3));
  };
  for (int grid : {ncu * 4, ncu * 8, ncu * 16, (int)((n + 255) / 256)}) {
    printf("grid %d\n", grid);
    report("A lane16B", 1, timeit([&] { kA<1><<<grid, 256>>>(W, vs, n, out); }, 5));
    report("A lane16B", 4, timeit([&] { kA<4><<<grid, 256>>>(W, vs, n, out); }, 5));
    report("A lane16B", 15, timeit([&] { kA<15><<<grid, 256>>>(W, vs, n, out); }, 5));
    report("B U=2", 15, timeit([&] { kB<15, 2><<<grid, 256>>>(W, vs, n, out); }, 5));
    report("B U=4", 4, timeit([&] { kB<4, 4><<<grid, 256>>>(W, vs, n, out); }, 5));
    report("B U=4", 1, timeit([&] { kB<1, 4><<<grid, 256>>>(W, vs, n, out); }, 5));
    report("C nontemporal", 1, timeit([&] { kC<1><<<grid, 256>>>(W, vs, n, out); }, 5));
    report("C nontemporal", 15, timeit([&] { kC<15><<<grid, 256>>>(W, vs, n, out); }, 5));
  }
  return 0;
}
