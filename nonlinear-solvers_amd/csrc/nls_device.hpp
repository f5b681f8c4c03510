// nls_device.hpp -- device-side types shared by the gfx950 kernels and the
// host code of libnls_amd.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nls {

constexpr int MMAX = 32;      // == NLS_MAX_KRYLOV
constexpr int NTHREADS = 256; // every kernel: 4 wave64s per workgroup

struct __align__(16) cplx {
  double re, im;
};

// ---- scalar helpers: S is double (sine-Gordon, f64) or cplx (NLSE, c128) ----
__host__ __device__ inline cplx operator+(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
__host__ __device__ inline cplx operator-(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }
__host__ __device__ inline cplx operator*(double s, cplx a) { return {s * a.re, s * a.im}; }
__host__ __device__ inline cplx &operator+=(cplx &a, cplx b) { a.re += b.re; a.im += b.im; return a; }
__host__ __device__ inline cplx cmul(cplx a, cplx b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__host__ __device__ inline cplx cconj(cplx a) { return {a.re, -a.im}; }
// product of two scalars of the same type (real or complex)
__host__ __device__ inline double smul(double a, double b) { return a * b; }
__host__ __device__ inline cplx smul(cplx a, cplx b) { return cmul(a, b); }
// acc += a b as fused multiply-adds (two per component for c128: no rounded product)
__host__ __device__ inline void smac(double &acc, double a, double b) { acc = fma(a, b, acc); }
__host__ __device__ inline void smac(cplx &acc, cplx a, cplx b) {
  acc.re = fma(a.re, b.re, acc.re);
  acc.re = fma(-a.im, b.im, acc.re);
  acc.im = fma(a.re, b.im, acc.im);
  acc.im = fma(a.im, b.re, acc.im);
}

// conj(a) * b  -- the Lanczos inner product v^H w
__host__ __device__ inline double cj_mul(double a, double b) { return a * b; }
__host__ __device__ inline cplx cj_mul(cplx a, cplx b) {
  return {a.re * b.re + a.im * b.im, a.re * b.im - a.im * b.re};
}
__host__ __device__ inline double abs2(double a) { return a * a; }
__host__ __device__ inline double abs2(cplx a) { return a.re * a.re + a.im * a.im; }
// coefficient (stored complex, imaginary part 0 on real paths) times element
__host__ __device__ inline double coef_mul(cplx c, double v) { return c.re * v; }
__host__ __device__ inline cplx coef_mul(cplx c, cplx v) { return cmul(c, v); }
__host__ __device__ inline cplx to_c(double v) { return {v, 0.0}; }
__host__ __device__ inline cplx to_c(cplx v) { return v; }
template <class S> __host__ __device__ inline S zero();
template <> __host__ __device__ inline double zero<double>() { return 0.0; }
template <> __host__ __device__ inline cplx zero<cplx>() { return {0.0, 0.0}; }

// ---- geometry of the (local slab of the) grid --------------------------------
// Planes are the slowest dimension: 3D z-planes (P = nx*ny), 2D y-rows (P = nx).
// Every basis vector is stored with one ghost plane below and above its
// nzl local planes; kernels get a pointer to local plane 0, so the ghost
// planes sit at -P and nzl*P (multi-GPU halo; zero and never read on 1 GPU).
struct Geo {
  int64_t nx;     // x extent
  int64_t nyp;    // rows per plane (3D: ny, 2D: 1)
  int64_t P;      // plane size nx*nyp
  int64_t npl;    // global number of planes (3D: nz, 2D: ny)
  int64_t z0;     // first global plane of this slab
  int64_t nzl;    // local planes
  int64_t Ng;     // global cells npl*P
  int64_t nloc;   // local cells nzl*P
  double s;       // off-diagonal value 1/(dx*dy) (2D) or 1/(dx*dx) (3D)
  double sd_in;   // interior diagonal  -4*s / -6*s
  double sd_bd;   // boundary diagonal  -3*s / -5*s
  int32_t kz;     // planes (3D) / rows per wave (2D) per tile of the stencil kernels
  int32_t remap;  // 1: XCD-banded tile order (speed only)
  int32_t qa, qb; // local planes [qa, qb) covered by a stencil launch (default 0, nzl)
  int32_t q2;     // k_p2d only: > 0 adds the range [q2, q2 + qb - qa) to the launch (the two
                  // boundary plane pairs of a split multi-rank pass in one grid); 0: none
  int32_t *tq;       // march only: non-null = dynamic tile queue ([0] next tile, [1] workgroups
                     // done; both back to 0 when the launch ends), else a static tile stride
  const double *cf;  // G2 anisotropic operator: c field at local plane 0 (ghost planes at
                     // -P and nzl*P, like a basis vector); unused by the isotropic operator
};

// Device-resident Lanczos state of one Krylov basis (no host round trip in
// the j-loop; the reference reads every dot back to the host,
// device/lanczos_complex.hpp:413-500).
struct KState {
  double s[MMAX + 1];       // s_k = ||W_k|| (stored vectors are unnormalised)
  cplx H[MMAX][MMAX];       // H[j][k] = v_k^H L v_j  (k <= j), column j of the Hessenberg
  cplx G[MMAX][MMAX];       // G[j][k] = v_k^H v_j   (k <= j), Gram
  double Td[MMAX];          // diag of T (real part of alpha), Td[m-1] = 0
  double To[MMAX];          // sub-diagonal of T: To[j] = T(j+1, j) = s_{j+1}
  cplx coef[MMAX + 2];      // coefficients of the next update kernel
  cplx fin[2][MMAX];        // final combination coefficients, one row per f
  cplx sums[2 * MMAX + 8];  // reduced sums (written by the sum phase)
  double lam[MMAX];         // Ritz values of the last eigensolve
  int32_t breakdown;        // first j with s_j == 0 (+1), 0 if none
  int32_t need_alpha;       // folded alpha ill-conditioned: run the (conditional) alpha pass
  int32_t pad[2];
};

// Epilogues of the fused tail pass k_tail (nls_stencil.hpp) and its arguments.
enum TailMode {
  TAIL_NLSE = 0,        // u = N(y); W_0 <- N(u)       (k_final_nlse; nlse_solver_dev.hpp:94-111)
  TAIL_SG_MID = 1,      // g_0 = m (-sin y_id); up <- 2 y_cos - up   (k_sg_mid; sg_solver.hpp:60-71)
  TAIL_SG_END = 2,      // u <- up + dt^2 y; up <- old u             (k_sg_end; sg_solver.hpp:71-73)
  TAIL_KG_END = 3,      // Gautschi update with the stored sinc^2 basis W2 (k_kg_end; kg_single.cuh:49-86)
  TAIL_COMBINE_W0 = 4,  // W_0 <- y                                  (k_combine_w0; sEWI)
  TAIL_COMBINE = 5,     // out <- y                                  (k_combine; sEWI)
  TAIL_SEWI_END = 6,    // u <- y - 2 tau e; up <- old u             (k_sewi_end; nlse_dev.hpp:52-63)
  TAIL_GG_MID = 7,      // g_0 = -m F(y_id) (F by TailArgs::nonlin, gg_force); up <- 2 y_cos - up
                        //   (G2 Gautschi family, e.g. phi4_single.cuh:33-47)
  TAIL_KG_END1 = 8,     // TAIL_KG_END with the sinc^2 action already combined into W2 (one
                        //   vector: the s-step passes' KG step, whose sinc^2 basis ends in
                        //   its own TAIL_COMBINE_W0 tail)
};
constexpr int TAIL_NMODES = 9;
constexpr int tail_nf(int mode) { return (mode == TAIL_SG_MID || mode == TAIL_GG_MID) ? 2 : 1; }

// Nonlinearity F of the G2 Gautschi family (g = -m F(id u)):
//   0 sin u (sg_single.cuh:18), 1 sin u + sin(u/2) (sg_double.cuh:19),
//   2 sinh u (sg_hyperbolic.cuh:18), 3 u + u^3 (phi4_single.cuh:18)
enum GautschiForce { GG_SIN = 0, GG_SIN_DOUBLE = 1, GG_SINH = 2, GG_PHI4 = 3 };

struct TailArgs {
  void *W;              // the tail basis (local plane 0 of W_0)
  const void *W2;       // KG: the fully stored sinc^2 basis
  int64_t vs;
  const KState *st;     // state of the tail basis (coef of the last update, fin)
  const KState *st2;    // KG: state of W2
  void *u, *up, *v, *out;
  const void *e;
  const double *mf;
  double dt;
  int nonlin;
  cplx s1, s2;
};

}  // namespace nls
