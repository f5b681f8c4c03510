// bw_probe5.hip -- does the basis layout limit the many-stream update passes?
// K read streams + 1 write in the 3D tile march of k_update (64 x * 2 rows per
// wave, 4 waves, kz = 32 planes per tile), 512^3 complex<double>, three layouts
// of the Krylov basis (K+1 vectors):
//   sep   : vector-major, one padded array per vector (the library's layout)
//   row   : [plane][row][vector][x]  -- the K+1 rows of one (plane,row) adjacent
//   plane : [plane][vector][row][x]  -- the K+1 planes adjacent
// no stencil, no arithmetic beyond a sum.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe5 tools/bw_probe5.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

struct __align__(16) c2 { double x, y; };
typedef double v2d __attribute__((ext_vector_type(2)));
#define CHECK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(_e), __LINE__); exit(1);} } while (0)
__device__ inline c2 ldnt(const c2* p) { v2d v = __builtin_nontemporal_load((const v2d*)p); return {v.x, v.y}; }
__device__ inline void stnt(c2* p, c2 v) { v2d t; t.x = v.x; t.y = v.y; __builtin_nontemporal_store(t, (v2d*)p); }

// address of (vector k, plane q, row y, x) for layout L (0 sep, 1 row, 2 plane); NV = K+1 vectors
template <int L>
__device__ inline long addr(int k, int q, int y, int x, int nx, int ny, int NV, long vs) {
  if (L == 0) return k * vs + ((long)q * ny + y) * nx + x;
  if (L == 1) return (((long)q * ny + y) * NV + k) * nx + x;
  return (((long)q * NV + k) * ny + y) * nx + x;
}

template <int K, int L>
__global__ __launch_bounds__(256) void ktile(c2* __restrict__ W, long vs, int nx, int ny, int nz, int kz) {
  constexpr int R = 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ntx = nx / 64, nty = ny / (4 * R), ntz = nz / kz;
  const int tiles = ntx * nty * ntz;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int it = t % ntx, jt = (t / ntx) % nty, kt = t / (ntx * nty);
    const int x = it * 64 + lane, y0 = jt * 4 * R + w * R;
    for (int q = kt * kz; q < kt * kz + kz; ++q) {
      c2 v[R][K];
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int k = 0; k < K; ++k) v[r][k] = ldnt(W + addr<L>(k, q, y0 + r, x, nx, ny, K + 1, vs));
#pragma unroll
      for (int r = 0; r < R; ++r) {
        c2 s = {0, 0};
#pragma unroll
        for (int k = 0; k < K; ++k) { s.x += v[r][k].x; s.y += v[r][k].y; }
        stnt(W + addr<L>(K, q, y0 + r, x, nx, ny, K + 1, vs), s);
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

template <int K> void run(c2* W, long n, int nx, int ny, int nz, int ncu) {
  const long vs = n + 256;
  const int kz = 32, tiles = (nx / 64) * (ny / 8) * (nz / kz);
  const char* nm[3] = {"sep", "row", "plane"};
  for (int L = 0; L < 3; ++L)
    for (int g : {ncu * 2, tiles}) {
      float ms = timeit([&] {
        if (L == 0) ktile<K, 0><<<g, 256>>>(W, vs, nx, ny, nz, kz);
        if (L == 1) ktile<K, 1><<<g, 256>>>(W, vs, nx, ny, nz, kz);
        if (L == 2) ktile<K, 2><<<g, 256>>>(W, vs, nx, ny, nz, kz);
      }, 3);
      printf("K=%2d %-6s grid %6d  %7.3f ms %7.1f GB/s\n", K, nm[L], g, ms, (K + 1) * n * 16.0 / 1e9 / (ms * 1e-3));
    }
}

int main() {
  const int nx = 512, ny = 512, nz = 512;
  const long n = (long)nx * ny * nz;
  c2* W;
  CHECK(hipMalloc(&W, (size_t)16 * (n + 256) * sizeof(c2)));
  CHECK(hipMemset(W, 0, (size_t)16 * (n + 256) * sizeof(c2)));
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  run<3>(W, n, nx, ny, nz, ncu);
  run<8>(W, n, nx, ny, nz, ncu);
  run<15>(W, n, nx, ny, nz, ncu);
  return 0;
}
