// bw_probe4.hip -- access-pattern probe for the Lanczos update pass: K read
// streams + 1 write, (a) grid-stride over the flat vector (the best case of
// bw_probe3) vs (b) the 3D tile march of k_update (64 x * R rows per wave, 4
// waves, kz planes per tile, plane by plane), no stencil, no arithmetic beyond
// a sum.  Tells whether the march order itself costs bandwidth.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe4 tools/bw_probe4.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>

struct __align__(16) c2 { double x, y; };
typedef double v2d __attribute__((ext_vector_type(2)));
#define CHECK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(_e), __LINE__); exit(1);} } while (0)
__device__ inline c2 ldnt(const c2* p) { v2d v = __builtin_nontemporal_load((const v2d*)p); return {v.x, v.y}; }
__device__ inline void stnt(c2* p, c2 v) { v2d t; t.x = v.x; t.y = v.y; __builtin_nontemporal_store(t, (v2d*)p); }

template <int K>
__global__ __launch_bounds__(256) void kflat(const c2* __restrict__ W, long vs, long n, c2* __restrict__ out) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long)gridDim.x * 256) {
    c2 s = {0, 0};
#pragma unroll
    for (int k = 0; k < K; ++k) { c2 v = ldnt(W + k * vs + p); s.x += v.x; s.y += v.y; }
    stnt(out + p, s);
  }
}

// tile march: nx = 512 (8 x-tiles of 64), rows per wave R, 4 waves -> 4R rows per tile
template <int K, int R>
__global__ __launch_bounds__(256) void ktile(const c2* __restrict__ W, long vs, int nx, int ny, int nz, int kz,
                                              c2* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ntx = nx / 64, nty = ny / (4 * R), ntz = nz / kz;
  const int tiles = ntx * nty * ntz;
  const long P = (long)nx * ny;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int it = t % ntx, jt = (t / ntx) % nty, kt = t / (ntx * nty);
    const int x = it * 64 + lane, y0 = jt * 4 * R + w * R;
    for (int q = kt * kz; q < kt * kz + kz; ++q) {
      c2 v[R][K];
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int k = 0; k < K; ++k) v[r][k] = ldnt(W + k * vs + q * P + (long)(y0 + r) * nx + x);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        c2 s = {0, 0};
#pragma unroll
        for (int k = 0; k < K; ++k) { s.x += v[r][k].x; s.y += v[r][k].y; }
        stnt(out + q * P + (long)(y0 + r) * nx + x, s);
      }
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
  const int nx = 512, ny = 512, nz = 512;
  const long n = (long)nx * ny * nz, vs = n + 256;
  constexpr int K = 15;
  c2 *W, *out;
  CHECK(hipMalloc(&W, (size_t)K * vs * sizeof(c2)));
  CHECK(hipMalloc(&out, (size_t)n * sizeof(c2)));
  CHECK(hipMemset(W, 0, (size_t)K * vs * sizeof(c2)));
  auto rep = [&](const char* nm, float ms) {
    printf("%-44s %7.3f ms %7.1f GB/s\n", nm, ms, (K + 1) * n * 16.0 / 1e9 / (ms * 1e-3));
  };
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  for (int g : {ncu * 2, ncu * 4, (int)(n / 256)})
    rep((std::string("flat grid ") + std::to_string(g)).c_str(),
        timeit([&] { kflat<K><<<g, 256>>>(W, vs, n, out); }, 3));
  for (int kz : {4, 16, 32}) {
    const int tiles1 = (nx / 64) * (ny / 4) * (nz / kz), tiles2 = (nx / 64) * (ny / 8) * (nz / kz);
    for (int g : {ncu * 2, 1 << 30}) {
      char nm[96];
      snprintf(nm, sizeof nm, "tile R=1 kz=%d grid %s", kz, g == 1 << 30 ? "tiles" : "2/CU");
      rep(nm, timeit([&] { ktile<K, 1><<<g == 1 << 30 ? tiles1 : g, 256>>>(W, vs, nx, ny, nz, kz, out); }, 3));
      snprintf(nm, sizeof nm, "tile R=2 kz=%d grid %s", kz, g == 1 << 30 ? "tiles" : "2/CU");
      rep(nm, timeit([&] { ktile<K, 2><<<g == 1 << 30 ? tiles2 : g, 256>>>(W, vs, nx, ny, nz, kz, out); }, 3));
    }
  }
  return 0;
}
