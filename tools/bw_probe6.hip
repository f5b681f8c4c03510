// bw_probe6.hip -- why does a one-cell-per-thread stream (bw_probe5 kflat1) beat the
// tile march of the fused tail and the basis passes at equal bytes?  K read streams
// + NW writes of a 512^3 grid of c128, register loads, one tile per workgroup:
//   tile = 64 x * 4 rows (one per wave) * KZ planes, marched plane by plane;
//   order: x-fastest (the 8 x tiles of a row group are consecutive workgroups, so
//   every 8 KiB row is read whole at about the same time) or y-fastest (k_p2d's);
//   FMA: a dependent chain of that many FMAs per cell between the loads and the
//   store (the compute phase of the real kernels, with no loads in flight);
//   LDS: dynamic LDS per workgroup, only to cap the resident workgroups per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe6 tools/bw_probe6.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

struct __align__(16) c2 { double x, y; };
typedef double v2d __attribute__((ext_vector_type(2)));
#define CHECK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(_e), __LINE__); exit(1);} } while (0)
__device__ inline c2 ldnt(const c2* p) { v2d v = __builtin_nontemporal_load((const v2d*)p); return {v.x, v.y}; }
__device__ inline void stnt(c2* p, c2 v) { v2d t; t.x = v.x; t.y = v.y; __builtin_nontemporal_store(t, (v2d*)p); }

template <int K, int NW, int FMA>
__device__ __forceinline__ void cell(const c2* __restrict__ W, long vs, long p, c2* __restrict__ out, double a) {
  c2 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ldnt(W + k * vs + p);
  c2 s = {0, 0}, t = {0, 0};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    s.x += v[k].x; s.y += v[k].y;
    t.x += (k + 1) * v[k].x; t.y -= v[k].y;
  }
#pragma unroll
  for (int f = 0; f < FMA; ++f) { s.x = fma(s.x, a, s.y); s.y = fma(s.y, a, s.x); }
  stnt(out + p, s);
  if (NW > 1) stnt(out + vs + p, t);
}

template <int K, int NW, int FMA>
__global__ __launch_bounds__(256) void kflat1(const c2* __restrict__ W, long vs, long n, c2* __restrict__ out, double a) {
  extern __shared__ char dyn[];
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  if (a == 12345.0) dyn[threadIdx.x] = 1;
  cell<K, NW, FMA>(W, vs, p, out, a);
}

// one tile per workgroup: 64 x * 4 rows * KZ planes of an nx * ny * nz grid
template <int K, int NW, int FMA>
__global__ __launch_bounds__(256) void ktile(const c2* __restrict__ W, long vs, int nx, int ny, int nz, int kz,
                                              int xfast, c2* __restrict__ out, double a) {
  extern __shared__ char dyn[];
  if (a == 12345.0) dyn[threadIdx.x] = 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ntx = nx / 64, nty = ny / 4;
  const int t = blockIdx.x;
  int xt, yt;
  if (xfast) { xt = t % ntx; yt = (t / ntx) % nty; }
  else { yt = t % nty; xt = (t / nty) % ntx; }
  const int zt = t / (ntx * nty);
  const long P = (long)nx * ny;
  const long base = (long)(yt * 4 + w) * nx + xt * 64 + lane;
  for (int q = zt * kz; q < zt * kz + kz; ++q) cell<K, NW, FMA>(W, vs, q * P + base, out, a);
}

// the same tiles, but a persistent grid: workgroup b takes tiles b, b + G, b + 2G, ...
template <int K, int NW, int FMA>
__global__ __launch_bounds__(256) void kpers(const c2* __restrict__ W, long vs, int nx, int ny, int nz, int kz,
                                              c2* __restrict__ out, double a) {
  extern __shared__ char dyn[];
  if (a == 12345.0) dyn[threadIdx.x] = 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ntx = nx / 64, nty = ny / 4, tiles = ntx * nty * (nz / kz);
  const long P = (long)nx * ny;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int xt = t % ntx, yt = (t / ntx) % nty, zt = t / (ntx * nty);
    const long base = (long)(yt * 4 + w) * nx + xt * 64 + lane;
    for (int q = zt * kz; q < zt * kz + kz; ++q) cell<K, NW, FMA>(W, vs, q * P + base, out, a);
  }
}

// persistent grid with dynamic tile assignment: each workgroup takes the next tile
// index from a global counter (vector atomic by one lane), so the tiles in flight
// stay the next ones in order, as with one tile per workgroup
template <int K, int NW, int FMA>
__global__ __launch_bounds__(256) void kdyn(const c2* __restrict__ W, long vs, int nx, int ny, int nz, int kz,
                                             c2* __restrict__ out, double a, int* ctr) {
  extern __shared__ char dyn[];
  __shared__ int s_t;
  if (a == 12345.0) dyn[threadIdx.x] = 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ntx = nx / 64, nty = ny / 4, tiles = ntx * nty * (nz / kz);
  const long P = (long)nx * ny;
  for (;;) {
    if (threadIdx.x == 0) s_t = atomicAdd(ctr, 1);
    __syncthreads();
    const int t = s_t;
    __syncthreads();
    if (t >= tiles) break;
    const int xt = t % ntx, yt = (t / ntx) % nty, zt = t / (ntx * nty);
    const long base = (long)(yt * 4 + w) * nx + xt * 64 + lane;
    for (int q = zt * kz; q < zt * kz + kz; ++q) cell<K, NW, FMA>(W, vs, q * P + base, out, a);
  }
}

template <class F> float timeit(F f, int reps) {
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  f(); CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0)); for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); return ms / reps;
}

static const int NX = 512;
static long g_n, g_vs;
static c2 *g_W, *g_out;
static int* g_ctr;

template <int K, int NW, int FMA> void run(int lds) {
  if (lds > 64 * 1024) {
    CHECK(hipFuncSetAttribute((const void*)kdyn<K, NW, FMA>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CHECK(hipFuncSetAttribute((const void*)kpers<K, NW, FMA>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CHECK(hipFuncSetAttribute((const void*)kflat1<K, NW, FMA>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CHECK(hipFuncSetAttribute((const void*)ktile<K, NW, FMA>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  }
  const double gb = (K + NW) * g_n * 16.0 / 1e9;
  float ms = timeit([&] { kflat1<K, NW, FMA><<<(int)(g_n / 256), 256, lds>>>(g_W, g_vs, g_n, g_out, 1.0000001); }, 5);
  printf("K=%2d NW=%d FMA=%3d LDS %3d KiB  flat1                 %7.3f ms %7.1f GB/s\n", K, NW, FMA, lds / 1024, ms, gb / ms * 1e3);
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int per_cu = lds ? ((160 * 1024) / (lds + 1024) < 4 ? (160 * 1024) / (lds + 1024) : 4) : 4;
  for (int kz : {4, 16, 64}) {
    ms = timeit([&] {
      CHECK(hipMemsetAsync(g_ctr, 0, sizeof(int)));
      kdyn<K, NW, FMA><<<ncu * per_cu, 256, lds>>>(g_W, g_vs, NX, NX, NX, kz, g_out, 1.0000001, g_ctr);
    }, 5);
    printf("K=%2d NW=%d FMA=%3d LDS %3d KiB  dynamic    kz=%-3d x-fast %7.3f ms %7.1f GB/s\n", K, NW, FMA, lds / 1024, kz, ms,
           gb / ms * 1e3);
  }
  for (int kz : {4, 16}) {
    ms = timeit([&] { kpers<K, NW, FMA><<<ncu * per_cu, 256, lds>>>(g_W, g_vs, NX, NX, NX, kz, g_out, 1.0000001); }, 5);
    printf("K=%2d NW=%d FMA=%3d LDS %3d KiB  persistent kz=%-3d x-fast %7.3f ms %7.1f GB/s\n", K, NW, FMA, lds / 1024, kz, ms,
           gb / ms * 1e3);
  }
  for (int kz : {4, 32, 256}) {
    for (int xf : {1, 0}) {
      const int grid = (NX / 64) * (NX / 4) * (NX / kz);
      ms = timeit([&] { ktile<K, NW, FMA><<<grid, 256, lds>>>(g_W, g_vs, NX, NX, NX, kz, xf, g_out, 1.0000001); }, 5);
      printf("K=%2d NW=%d FMA=%3d LDS %3d KiB  tile kz=%-3d %s     %7.3f ms %7.1f GB/s\n", K, NW, FMA, lds / 1024, kz,
             xf ? "x-fast" : "y-fast", ms, gb / ms * 1e3);
    }
  }
}

int main() {
  g_n = (long)NX * NX * NX;
  g_vs = g_n + 4096;
  CHECK(hipMalloc(&g_W, (size_t)15 * g_vs * sizeof(c2)));
  CHECK(hipMalloc(&g_out, (size_t)2 * g_vs * sizeof(c2)));
  CHECK(hipMemset(g_W, 0, (size_t)15 * g_vs * sizeof(c2)));
  CHECK(hipMalloc(&g_ctr, sizeof(int)));
  // the fused tail (15 reads + 1 write) at the tail's occupancy (2 workgroups per CU)
  // and unlimited, without and with a compute phase
  run<15, 1, 0>(80 * 1024);
  // the J = 12 pass pattern (13 reads + 2 writes), one workgroup per CU (the dynamic
  // LDS request leaves room for the kernels' static LDS: 160 KiB in all failed with
  // "invalid argument" in round 3)
  run<13, 2, 0>(156 * 1024);
  // the J = 0 pass pattern (1 read + 2 writes) at three workgroups per CU
  run<1, 2, 0>(52 * 1024);
  return 0;
}
