// bw_probe5.hip -- what can an LDS-DMA stream reach against register loads?  K read
// streams + NW write streams per cell (the fused tail: K = 15, NW = 1; the J = 12
// two-vector pass: K = 13, NW = 2; the J = 0 pass: K = 1, NW = 2), no stencil, a sum
// per output.  (a) register loads, grid-stride over the flat vectors (bw_probe4's
// best case); (b) every read moved HBM -> LDS by global_load_lds_dwordx4 (1 KiB per
// wave-instruction, non-temporal), each wave marching its own contiguous run of
// 64-cell rows with a private ring of NP rows per stream, completion counted by hand
// (no barriers: a wave reads only what it DMA'd itself).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe5 tools/bw_probe5.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

struct __align__(16) c2 { double x, y; };
typedef double v2d __attribute__((ext_vector_type(2)));
#define CHECK(e) do { hipError_t _e = (e); if (_e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(_e), __LINE__); exit(1);} } while (0)
__device__ inline c2 ldnt(const c2* p) { v2d v = __builtin_nontemporal_load((const v2d*)p); return {v.x, v.y}; }
__device__ inline void stnt(c2* p, c2 v) { v2d t; t.x = v.x; t.y = v.y; __builtin_nontemporal_store(t, (v2d*)p); }

template <int K, int NW>
__global__ __launch_bounds__(256) void kflat(const c2* __restrict__ W, long vs, long n, c2* __restrict__ out) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long)gridDim.x * 256) {
    c2 s = {0, 0}, t = {0, 0};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      c2 v = ldnt(W + k * vs + p);
      s.x += v.x; s.y += v.y;
      t.x += (k + 1) * v.x; t.y -= v.y;
    }
    stnt(out + p, s);
    if (NW > 1) stnt(out + vs + p, t);
  }
}

// one cell per thread, one short-lived workgroup per 256 cells (bw_probe3's best case);
// dynamic LDS only to cap the resident workgroups per CU (occupancy of the real kernels)
template <int K, int NW>
__global__ __launch_bounds__(256) void kflat1(const c2* __restrict__ W, long vs, long n, c2* __restrict__ out) {
  extern __shared__ char dyn[];
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  c2 s = {0, 0}, t = {0, 0};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    c2 v = ldnt(W + k * vs + p);
    s.x += v.x; s.y += v.y;
    t.x += (k + 1) * v.x; t.y -= v.y;
  }
  if (s.x == 12345.0) dyn[threadIdx.x] = 1;
  stnt(out + p, s);
  if (NW > 1) stnt(out + vs + p, t);
}

template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 0 ? 0 : (N > 63 ? 63 : N)) : "memory");
}
// ops issued after row i's group, up to the wait of step i: NP-1 later groups and
// min(i, NP-1) stores groups of NW
template <int K, int NW, int NP> __host__ __device__ constexpr int after(int i) {
  return (NP - 1) * K + (i < NP - 1 ? i : NP - 1) * NW;
}
template <int K, int NW, int NP, int I = 0> __device__ __forceinline__ void wait_step(int i) {
  if constexpr (I >= NP - 1) {
    wait_vm<after<K, NW, NP>(I)>();
  } else {
    if (i == I) { wait_vm<after<K, NW, NP>(I)>(); return; }
    wait_step<K, NW, NP, I + 1>(i);
  }
}

template <int K, int NW, int NP, int NWV, int OCC>
__global__ __launch_bounds__(64 * NWV, OCC) void kdma(const c2* __restrict__ W, long vs, long nrows, int R,
                                                    c2* __restrict__ out) {
  static_assert(after<K, NW, NP>(NP) <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[NWV * NP * K * 1024];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long r0 = ((long)blockIdx.x * NWV + w) * R;
  if (r0 >= nrows) return;  // uniform per wave; no barriers below
  const int rn = (int)(r0 + R <= nrows ? R : nrows - r0);
  char* ring = smem + w * NP * K * 1024;
  const uint32_t loff = lane * 16u;
  const long vsb = vs * 16;
  const char* base = reinterpret_cast<const char*>(W) + r0 * 1024;
#define ISSUE(row, sl)                                                                      \
  do {                                                                                      \
    const char* b_ = base + (long)(row) * 1024;                                             \
    char* d_ = ring + (sl) * K * 1024;                                                      \
    _Pragma("unroll") for (int k_ = 0; k_ < K; ++k_) {                                      \
      asm volatile("" : "+s"(b_));                                                          \
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(b_ + loff),                 \
                                       (__attribute__((address_space(3))) void*)(d_ + k_ * 1024), 16, 0, 2); \
      b_ += vsb;                                                                            \
    }                                                                                       \
  } while (0)
#pragma unroll
  for (int g = 0; g < NP - 1; ++g) ISSUE(g < rn ? g : rn - 1, g);
  int sl = 0, sli = NP - 1;
  for (int i = 0; i < rn; ++i) {
    const int nr = i + NP - 1;
    ISSUE(nr < rn ? nr : rn - 1, sli);
    wait_step<K, NW, NP>(i);
    const c2* rv = reinterpret_cast<const c2*>(ring + sl * K * 1024);
    c2 s = {0, 0}, t = {0, 0};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const c2 v = rv[k * 64 + lane];
      s.x += v.x; s.y += v.y;
      t.x += (k + 1) * v.x; t.y -= v.y;
    }
    c2* o = out + (r0 + i) * 64 + lane;
    stnt(o, s);
    if (NW > 1) stnt(o + vs, t);
    sl = sl + 1 == NP ? 0 : sl + 1;
    sli = sli + 1 == NP ? 0 : sli + 1;
  }
#undef ISSUE
  wait_vm<0>();
}

template <class F> float timeit(F f, int reps) {
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  f(); CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a)); for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

static long g_n, g_vs;
static c2 *g_W, *g_out;
static int g_ncu;

template <int K, int NW> void flat_case() {
  for (int g : {g_ncu * 2, g_ncu * 4, g_ncu * 8}) {
    const float ms = timeit([&] { kflat<K, NW><<<g, 256>>>(g_W, g_vs, g_n, g_out); }, 5);
    printf("K=%2d NW=%d flat regs grid %-5d              %7.3f ms %7.1f GB/s\n", K, NW, g, ms,
           (K + NW) * g_n * 16.0 / 1e9 / (ms * 1e-3));
  }
}
template <int K, int NW> void flat1_case() {
  for (int lds : {0, 40 * 1024, 80 * 1024, 160 * 1024}) {
    if (lds > 64 * 1024) CHECK(hipFuncSetAttribute((const void*)kflat1<K, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    const float ms = timeit([&] { kflat1<K, NW><<<(int)((g_n + 255) / 256), 256, lds>>>(g_W, g_vs, g_n, g_out); }, 5);
    printf("K=%2d NW=%d flat one cell/thread, LDS %3d KiB/WG   %7.3f ms %7.1f GB/s\n", K, NW, lds / 1024, ms,
           (K + NW) * g_n * 16.0 / 1e9 / (ms * 1e-3));
  }
}
template <int K, int NW, int NP, int NWV, int OCC> void dma_case() {
  const long nrows = g_n / 64;
  for (int R : {64, 256}) {
    const long waves = (nrows + R - 1) / R;
    const int grid = (int)((waves + NWV - 1) / NWV);
    const float ms = timeit([&] { kdma<K, NW, NP, NWV, OCC><<<grid, 64 * NWV>>>(g_W, g_vs, nrows, R, g_out); }, 5);
    printf("K=%2d NW=%d lds-dma NP=%d waves/WG=%d WG/CU=%d R=%-4d %7.3f ms %7.1f GB/s\n", K, NW, NP, NWV, OCC, R, ms,
           (K + NW) * g_n * 16.0 / 1e9 / (ms * 1e-3));
  }
}

int main(int argc, char** argv) {
  const int n1 = argc > 1 ? atoi(argv[1]) : 512;
  const long pad = argc > 2 ? atol(argv[2]) : 4096;  // stream stride pad in cells (4096: 64 KiB, the library's)
  const int quick = argc > 3 ? atoi(argv[3]) : 0;
  g_n = (long)n1 * n1 * n1;
  g_vs = g_n + pad;
  printf("n = %d^3, stream pad %ld cells\n", n1, pad);
  CHECK(hipMalloc(&g_W, (size_t)15 * g_vs * sizeof(c2)));
  CHECK(hipMalloc(&g_out, (size_t)2 * g_vs * sizeof(c2)));
  CHECK(hipMemset(g_W, 0, (size_t)15 * g_vs * sizeof(c2)));
  CHECK(hipDeviceGetAttribute(&g_ncu, hipDeviceAttributeMultiprocessorCount, 0));
  // the fused tail's pattern
  flat1_case<15, 1>();
  flat_case<15, 1>();
  if (quick) {
    flat1_case<13, 2>();
    flat1_case<1, 1>();
    return 0;
  }
  dma_case<15, 1, 2, 4, 1>();
  dma_case<15, 1, 2, 2, 2>();
  dma_case<15, 1, 3, 1, 3>();
  dma_case<15, 1, 4, 1, 2>();
  dma_case<15, 1, 4, 2, 1>();
  dma_case<15, 1, 3, 2, 1>();
  // the J = 12 pass
  flat_case<13, 2>();
  dma_case<13, 2, 2, 4, 1>();
  dma_case<13, 2, 3, 1, 4>();
  dma_case<13, 2, 4, 1, 3>();
  // the J = 0 pass
  flat_case<1, 2>();
  dma_case<1, 2, 8, 4, 4>();
  dma_case<1, 2, 16, 4, 2>();
  return 0;
}
