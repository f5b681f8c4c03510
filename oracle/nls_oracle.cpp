// nls_oracle.cpp -- TEST INFRASTRUCTURE ONLY.  See nls_oracle.h for scope.
//
// CPU restatement of the reference G1 Eigen path, written from the reference
// source read as text (never compiled: Eigen3 and the libnpy submodule are
// absent from this image, see DESIGN.md "Oracle").  Every function cites the
// reference lines it follows.  Compiled with -ffp-contract=off so that, like
// the reference's x86-64 Eigen build (no FMA), every product is rounded
// separately.
#include "nls_oracle.h"

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstring>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
// Built a second time with -fopenmp (liboracle_nls_omp.so) for the all-cores
// CPU baseline only: the vector loops run in parallel and the reductions sum
// per-thread partials in thread order.  The checker is the serial build.
#define ORACLE_PFOR _Pragma("omp parallel for schedule(static)")
#else
#define ORACLE_PFOR
#endif

namespace {

using cd = std::complex<double>;

struct Grid {
  int dim;
  uint64_t nx, ny, nz, N;
  double scale;
};

bool make_grid(const oracle_grid *g, Grid &G) {
  if (!g || (g->dim != 2 && g->dim != 3) || g->nx < 1 || g->ny < 1) return false;
  G.dim = g->dim;
  G.nx = g->nx;
  G.ny = g->ny;
  G.nz = g->dim == 3 ? g->nz : 1;
  if (G.nz < 1) return false;
  G.N = G.nx * G.ny * G.nz;
  // laplacians.hpp:49  L *= 1/(dx*dy)   (2D)
  // laplacians.hpp:102 L *= 1/(dx*dx)   (3D; dy, dz only enter the assert)
  G.scale = g->dim == 2 ? 1.0 / (g->dx * g->dy) : 1.0 / (g->dx * g->dx);
  return true;
}

// Matrix-free restatement of build_laplacian_noflux (laplacians.hpp:10-52)
// and build_laplacian_noflux_3d (:55-105) applied like Eigen's column-major
// SpMV: row idx receives its contributions in increasing column order
// (idx-P, idx-nx, idx-1, idx, idx+1, idx+nx, idx+P), each value pre-scaled.
//   diag  -4 / -3 (2D, any coordinate on the boundary, :23-30)
//         -6 / -5 (3D, :69-80)
//   x     idx+-1 unless the row wraps (:32-37, :82-87)
//   "y"   idx+-nx whenever inside [0,N)  -> in 3D this couples (i,ny-1,k) with
//         (i,0,k+1) (:89-92)
//   z     idx+-nx*ny (:94-97)
template <class S>
void lap_apply(const Grid &G, const S *x, S *y) {
  const uint64_t nx = G.nx, ny = G.ny, nz = G.nz, N = G.N, P = nx * ny;
  const double s = G.scale;
  const double d_in = G.dim == 2 ? -4.0 : -6.0;
  const double d_bd = G.dim == 2 ? -3.0 : -5.0;
  const double sd_in = d_in * s, sd_bd = d_bd * s;
  ORACLE_PFOR
  for (uint64_t idx = 0; idx < N; ++idx) {
    const uint64_t i = idx % nx, j = (idx / nx) % ny, k = idx / P;
    bool bnd = (i == 0 || i == nx - 1 || j == 0 || j == ny - 1);
    if (G.dim == 3) bnd = bnd || k == 0 || k == nz - 1;
    S acc = S(0);
    if (G.dim == 3 && idx >= P) acc += s * x[idx - P];
    if (idx >= nx) acc += s * x[idx - nx];
    if (i > 0) acc += s * x[idx - 1];
    acc += (bnd ? sd_bd : sd_in) * x[idx];
    if (i + 1 < nx) acc += s * x[idx + 1];
    if (idx + nx < N) acc += s * x[idx + nx];
    if (G.dim == 3 && idx + P < N) acc += s * x[idx + P];
    y[idx] = acc;
  }
}

struct StencilOp {
  Grid G;
  uint64_t n() const { return G.N; }
  template <class S> void apply(const S *x, S *y) const { lap_apply(G, x, y); }
};

// Matrix-free restatement of the G2 anisotropic builders
// build_anisotropic_laplacian_noflux (nlsolvers/common/include/laplacians.hpp:54-103)
// and build_anisotropic_laplacian_noflux_3d (:158-218), called by the G2
// drivers with nx-2, ny-2(, nz-2) so the operator spans the full grid
// (nlse_cubic_driver_3d.cpp:103-106):
//   x     (i, i+1) unless (i+1) % nx == 0, weight (c_i + c_{i+1}) / 2.0   (:183-191)
//   "y"   (i, i+nx) for every i < N - nx (3D: the same y-wrap as the
//         isotropic builder), weight (c_i + c_{i+nx}) / 2.0             (:193-199)
//   z     (i, i+P) (3D)                                                   (:201-207)
//   diag  -diagonal_sums[i], accumulated in the loop order above          (:209-211)
//   L *= 1/(dx*dy) (2D, :101) or 1/(dx*dx) (3D, :216)
// Row idx is evaluated in Eigen's column order like lap_apply.
template <class S>
void lap_aniso_apply(const Grid &G, const double *c, const S *x, S *y) {
  const uint64_t nx = G.nx, N = G.N, P = G.nx * G.ny;
  const double s = G.scale;
  ORACLE_PFOR
  for (uint64_t idx = 0; idx < N; ++idx) {
    const uint64_t i = idx % nx;
    const bool ezm = G.dim == 3 && idx >= P, ezp = G.dim == 3 && idx + P < N;
    const bool eym = idx >= nx, eyp = idx + nx < N;
    const bool exm = i > 0, exp_ = i + 1 < nx;
    const double wzm = ezm ? (c[idx - P] + c[idx]) / 2.0 : 0.0;
    const double wzp = ezp ? (c[idx] + c[idx + P]) / 2.0 : 0.0;
    const double wym = eym ? (c[idx - nx] + c[idx]) / 2.0 : 0.0;
    const double wyp = eyp ? (c[idx] + c[idx + nx]) / 2.0 : 0.0;
    const double wxm = exm ? (c[idx - 1] + c[idx]) / 2.0 : 0.0;
    const double wxp = exp_ ? (c[idx] + c[idx + 1]) / 2.0 : 0.0;
    double ds = 0.0;  // diagonal_sums[idx] in the builder's accumulation order
    if (exm) ds += wxm;
    if (exp_) ds += wxp;
    if (eym) ds += wym;
    if (eyp) ds += wyp;
    if (ezm) ds += wzm;
    if (ezp) ds += wzp;
    S acc = S(0);
    if (ezm) acc += (wzm * s) * x[idx - P];
    if (eym) acc += (wym * s) * x[idx - nx];
    if (exm) acc += (wxm * s) * x[idx - 1];
    acc += (-ds * s) * x[idx];
    if (exp_) acc += (wxp * s) * x[idx + 1];
    if (eyp) acc += (wyp * s) * x[idx + nx];
    if (ezp) acc += (wzp * s) * x[idx + P];
    y[idx] = acc;
  }
}

struct AnisoOp {
  Grid G;
  const double *c;
  bool negate = false;  // -L as the KG drivers pass it (kg_driver_dev_3d.cpp:110-114)
  uint64_t n() const { return G.N; }
  template <class S> void apply(const S *x, S *y) const {
    lap_aniso_apply(G, c, x, y);
    if (negate)  // negating the assembled values is exact: same bits as -(L x)
      for (uint64_t p = 0; p < G.N; ++p) y[p] = -y[p];
  }
};

struct CsrOp {
  uint64_t N;
  const int64_t *rp, *ci;
  const double *v;
  uint64_t n() const { return N; }
  template <class S> void apply(const S *x, S *y) const {
    for (uint64_t r = 0; r < N; ++r) {
      S acc = S(0);
      for (int64_t q = rp[r]; q < rp[r + 1]; ++q) acc += v[q] * x[ci[q]];
      y[r] = acc;
    }
  }
};

inline double conj_s(double x) { return x; }
inline cd conj_s(cd x) { return std::conj(x); }
inline double abs2_s(double x) { return x * x; }
inline double abs2_s(cd x) { return x.real() * x.real() + x.imag() * x.imag(); }
inline double re_s(double x) { return x; }
inline double re_s(cd x) { return x.real(); }

// serial sum, or (OpenMP build) per-thread partial sums added in thread order
template <class T, class F> T reduce_sum(uint64_t n, F term) {
#ifdef _OPENMP
  const int nt = omp_get_max_threads();
  if (nt > 1 && n > 4096) {
    std::vector<T> part(nt, T(0));
#pragma omp parallel
    {
      T acc = T(0);
#pragma omp for schedule(static)
      for (uint64_t p = 0; p < n; ++p) acc += term(p);
      part[omp_get_thread_num()] = acc;
    }
    T acc = T(0);
    for (int t = 0; t < nt; ++t) acc += part[t];
    return acc;
  }
#endif
  T acc = T(0);
  for (uint64_t p = 0; p < n; ++p) acc += term(p);
  return acc;
}

template <class S> double norm2(const S *x, uint64_t n) {
  return std::sqrt(reduce_sum<double>(n, [&](uint64_t p) { return abs2_s(x[p]); }));
}

// <a, b> = a^H b  (Eigen: V.col(i).adjoint() * w, eigen_krylov_complex.hpp:30;
// for the real path w.dot(V.col(i)) is the same number, eigen_krylov_real.hpp:29)
template <class S> S dot(const S *a, const S *b, uint64_t n) {
  return reduce_sum<S>(n, [&](uint64_t p) { return conj_s(a[p]) * b[p]; });
}

// lanczos_L  (eigen_krylov_complex.hpp:10-53, eigen_krylov_real.hpp:5-51)
// V column-major n x m, T column-major m x m.  Runs m-1 iterations; T(m-1,m-1)
// is never written and stays 0.  Breakdown (T(j+1,j)==0) divides by zero
// exactly like the reference (NaN), see eigen_krylov_complex.hpp:47.
template <class S, class Op>
void lanczos(const Op &op, const S *u, uint32_t m, std::vector<S> &V,
             std::vector<S> &T, double &beta) {
  const uint64_t n = op.n();
  V.assign(n * m, S(0));
  T.assign((size_t)m * m, S(0));
  auto Tm = [&](uint32_t r, uint32_t c) -> S & { return T[(size_t)c * m + r]; };
  beta = norm2(u, n);
  ORACLE_PFOR
  for (uint64_t p = 0; p < n; ++p) V[p] = u[p] / beta;
  std::vector<S> w(n);
  for (uint32_t j = 0; j + 1 < m; ++j) {
    const S *vj = &V[(uint64_t)j * n];
    op.apply(vj, w.data());
    if (j > 0) {
      const S b = Tm(j - 1, j);
      const S *vjm = &V[(uint64_t)(j - 1) * n];
      ORACLE_PFOR
      for (uint64_t p = 0; p < n; ++p) w[p] -= b * vjm[p];
    }
    Tm(j, j) = dot(vj, w.data(), n);
    {
      const S a = Tm(j, j);
      ORACLE_PFOR
      for (uint64_t p = 0; p < n; ++p) w[p] -= a * vj[p];
    }
    // full MGS re-orthogonalisation (eigen_krylov_complex.hpp:29-37)
    for (uint32_t i = 0; i <= j; ++i) {
      const S *vi = &V[(uint64_t)i * n];
      const S c = dot(vi, w.data(), n);
      ORACLE_PFOR
      for (uint64_t p = 0; p < n; ++p) w[p] -= c * vi[p];
    }
    const double nb = norm2(w.data(), n);
    Tm(j + 1, j) = S(nb);
    Tm(j, j + 1) = S(nb);
    S *vn = &V[(uint64_t)(j + 1) * n];
    ORACLE_PFOR
    for (uint64_t p = 0; p < n; ++p) vn[p] = w[p] / nb;
  }
}

// Symmetric eigensolver for the real m x m matrix Eigen's SelfAdjointEigenSolver
// sees: lower triangle of T, real part of the diagonal (Eigen's
// tridiagonalization reads mat.diagonal().real()).  Cyclic Jacobi.  NOTE: the device
// eigensolve (k_reduce_final, nls_kernels.hip) runs this same Jacobi algorithm (same
// rotation and stopping rule, T pre-scaled like Eigen's solver), so a GPU-vs-oracle
// comparison does not check the eigensolve independently; the reference pins do
// (tests/test_oracle.py::test_ref_krylov_action and tests/test_gpu_refpin.py build
// f(T) e_1 with LAPACK eigh on the reference's own T).  A (row-major) is overwritten;
// Q columns = vectors.
void jacobi_eig(std::vector<double> A, int m, std::vector<double> &lam,
                std::vector<double> &Q) {
  Q.assign((size_t)m * m, 0.0);
  for (int i = 0; i < m; ++i) Q[(size_t)i * m + i] = 1.0;
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0, tot = 0.0;
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < m; ++j) {
        const double a = A[(size_t)i * m + j] * A[(size_t)i * m + j];
        tot += a;
        if (i != j) off += a;
      }
    if (off <= 1e-34 * tot || off == 0.0) break;
    for (int p = 0; p < m - 1; ++p)
      for (int q = p + 1; q < m; ++q) {
        const double apq = A[(size_t)p * m + q];
        if (apq == 0.0) continue;
        const double app = A[(size_t)p * m + p], aqq = A[(size_t)q * m + q];
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) /
                         (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < m; ++k) {
          const double akp = A[(size_t)k * m + p], akq = A[(size_t)k * m + q];
          A[(size_t)k * m + p] = c * akp - s * akq;
          A[(size_t)k * m + q] = s * akp + c * akq;
        }
        for (int k = 0; k < m; ++k) {
          const double apk = A[(size_t)p * m + k], aqk = A[(size_t)q * m + k];
          A[(size_t)p * m + k] = c * apk - s * aqk;
          A[(size_t)q * m + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < m; ++k) {
          const double qkp = Q[(size_t)k * m + p], qkq = Q[(size_t)k * m + q];
          Q[(size_t)k * m + p] = c * qkp - s * qkq;
          Q[(size_t)k * m + q] = s * qkp + c * qkq;
        }
      }
  }
  lam.resize(m);
  for (int i = 0; i < m; ++i) lam[i] = A[(size_t)i * m + i];
}

inline double sinc_ref(double x) {  // eigen_krylov_real.hpp:95-97
  return std::fabs(x) < 1e-8 ? 1.0 : std::sin(x) / x;
}

// f(lambda) for every convention the reference uses.
cd eval_f(int func, double lam, cd t) {
  switch (func) {
    case ORACLE_F_EXP_ABS: return std::exp(t * std::fabs(lam));
    case ORACLE_F_EXP: return std::exp(t * lam);
    case ORACLE_F_SINC: {  // nlsolvers/device/include/matfunc_complex.hpp:293-300
      const cd val = t * lam;
      return std::abs(val) < 1e-8 ? cd(1.0, 0.0) : std::sin(val) / val;
    }
    default: break;
  }
  const double x = t.real() * std::sqrt(std::fabs(lam));
  switch (func) {
    case ORACLE_F_COS_SQRT: return std::cos(x);
    case ORACLE_F_SINC_SQRT: return sinc_ref(x);
    case ORACLE_F_SINC2_SQRT: { const double s = sinc_ref(x); return s * s; }
    case ORACLE_F_ID_SQRT: return x;
    case ORACLE_F_SINC2_HALF: {  // eigen_krylov_real.hpp:186-191
      const double xh = t.real() / 2. * std::sqrt(std::fabs(lam));
      if (std::fabs(xh) < 1e-8) return 1.0;
      return (std::sin(xh) / xh) * (std::sin(xh) / xh);
    }
    default: return std::nan("");
  }
}

inline void assign(double &dst, cd v) { dst = v.real(); }
inline void assign(cd &dst, cd v) { dst = v; }

// expm_multiply / *_sqrt_multiply: beta * V * Q f(Lambda) Q^H * e1
// (eigen_krylov_complex.hpp:55-84; eigen_krylov_real.hpp:53-201)
template <class S, class Op>
void krylov_apply(const Op &op, const S *u, cd t, uint32_t m, int func, S *out) {
  const uint64_t n = op.n();
  std::vector<S> V, T;
  double beta = 0.0;
  lanczos(op, u, m, V, T, beta);
  std::vector<double> A((size_t)m * m, 0.0);
  for (uint32_t c = 0; c < m; ++c)
    for (uint32_t r = c; r < m; ++r) {
      const double v = re_s(T[(size_t)c * m + r]);  // lower triangle
      A[(size_t)r * m + c] = v;
      A[(size_t)c * m + r] = v;
    }
  std::vector<double> lam, Q;
  jacobi_eig(A, (int)m, lam, Q);
  std::vector<cd> coef(m, cd(0));  // (Q f Q^H)[:, 0]
  for (uint32_t i = 0; i < m; ++i) {
    cd acc(0);
    for (uint32_t k = 0; k < m; ++k)
      acc += Q[(size_t)i * m + k] * eval_f(func, lam[k], t) * Q[(size_t)0 * m + k];
    coef[i] = acc;
  }
  std::vector<S> c(m);
  for (uint32_t i = 0; i < m; ++i) assign(c[i], coef[i]);
  ORACLE_PFOR
  for (uint64_t p = 0; p < n; ++p) {
    S acc = S(0);
    for (uint32_t k = 0; k < m; ++k) acc += (beta * V[(uint64_t)k * n + p]) * c[k];
    out[p] = acc;
  }
}

const cd *as_c(const double *p) { return reinterpret_cast<const cd *>(p); }
cd *as_c(double *p) { return reinterpret_cast<cd *>(p); }

// nonlinear half step  out = exp(-0.5*tau*rho(u)) * u,  tau = 1j*dt
//   cubic (G1 CPU, nlse_solver.hpp:66-69): rho = re^2 + im^2
//   cubic-quintic (G1 device, device/nlse_cq_solver.hpp:16-39):
//     d = |u|*|u|, rho = s1*d + s2*d^2 (complex), out = exp(-.5*tau*rho) * u
void nonlin_half(cd *u, uint64_t n, double dt, int nonlin, const double *sg) {
  const cd tau(0.0, dt);
  const cd mt = -.5 * tau;
  if (nonlin == 0) {
    ORACLE_PFOR
    for (uint64_t p = 0; p < n; ++p) {
      const double x = u[p].real() * u[p].real() + u[p].imag() * u[p].imag();
      u[p] = std::exp(mt * cd(x)) * u[p];
    }
  } else {
    const cd s1(sg[0], sg[1]), s2(sg[2], sg[3]);
    for (uint64_t p = 0; p < n; ++p) {
      const double a = std::abs(u[p]);
      const double d = a * a;
      const cd rho = s1 * d + s2 * (d * d);
      u[p] = std::exp(mt * rho) * u[p];
    }
  }
}

// G2 nonlinear half step (nlsolvers/device/include/nlse_dev.hpp:20-40):
//   rho = m * (re^2 + im^2);  out = in * exp(0.5*tau * rho),  tau = 1j*dt
void nonlin_half_g2(cd *u, const double *mf, uint64_t n, double dt) {
  const cd ht = 0.5 * cd(0.0, dt);
  for (uint64_t p = 0; p < n; ++p) {
    const double rho = mf[p] * (u[p].real() * u[p].real() + u[p].imag() * u[p].imag());
    u[p] = u[p] * std::exp(ht * cd(rho, 0.0));
  }
}

// neumann_bc_no_velocity_blocking{,_3d} (nlsolvers/device/include/boundaries.cuh:10-19,
// :24-81), the strided copies in the reference's order.  The reference indexes
// u[a*n^2 + b*n + c] (a slowest) on cubic grids; here a = z, b = y, c = x of
// the [nz][ny][nx] layout with per-axis extents (2D: a = y, b = x).
template <class S> void neumann_bc(const Grid &G, S *u) {
  const uint64_t nx = G.nx, ny = G.ny, nz = G.nz;
  auto at3 = [&](uint64_t a, uint64_t b, uint64_t c) -> S & { return u[(a * ny + b) * nx + c]; };
  if (G.dim == 2) {
    auto at2 = [&](uint64_t a, uint64_t b) -> S & { return u[a * nx + b]; };
    for (uint64_t b = 1; b + 1 < nx; ++b) at2(0, b) = at2(1, b);             // :12-13
    for (uint64_t b = 1; b + 1 < nx; ++b) at2(ny - 1, b) = at2(ny - 2, b);   // :14-15
    for (uint64_t a = 0; a < ny; ++a) at2(a, 0) = at2(a, 1);                 // :16-17
    for (uint64_t a = 0; a < ny; ++a) at2(a, nx - 1) = at2(a, nx - 2);       // :18-19
    return;
  }
  for (uint64_t b = 1; b + 1 < ny; ++b)  // x-min / x-max of the reference (:28-45)
    for (uint64_t c = 1; c + 1 < nx; ++c) at3(0, b, c) = at3(1, b, c);
  for (uint64_t b = 1; b + 1 < ny; ++b)
    for (uint64_t c = 1; c + 1 < nx; ++c) at3(nz - 1, b, c) = at3(nz - 2, b, c);
  for (uint64_t a = 0; a < nz; ++a)  // y-min / y-max (:47-63)
    for (uint64_t c = 1; c + 1 < nx; ++c) at3(a, 0, c) = at3(a, 1, c);
  for (uint64_t a = 0; a < nz; ++a)
    for (uint64_t c = 1; c + 1 < nx; ++c) at3(a, ny - 1, c) = at3(a, ny - 2, c);
  for (uint64_t a = 0; a < nz; ++a)  // z-min / z-max (:65-81)
    for (uint64_t b = 0; b < ny; ++b) at3(a, b, 0) = at3(a, b, 1);
  for (uint64_t a = 0; a < nz; ++a)
    for (uint64_t b = 0; b < ny; ++b) at3(a, b, nx - 1) = at3(a, b, nx - 2);
}

}  // namespace

extern "C" {

int oracle_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

int oracle_laplacian_apply_c(const oracle_grid *g, const double *x, double *y) {
  Grid G;
  if (!make_grid(g, G) || !x || !y) return -1;
  lap_apply(G, as_c(x), as_c(y));
  return 0;
}

int oracle_laplacian_apply_r(const oracle_grid *g, const double *x, double *y) {
  Grid G;
  if (!make_grid(g, G) || !x || !y) return -1;
  lap_apply(G, x, y);
  return 0;
}

int oracle_lanczos_c(const oracle_grid *g, const double *u, uint32_t m,
                     double *V, double *T, double *beta) {
  Grid G;
  if (!make_grid(g, G) || m < 1) return -1;
  StencilOp op{G};
  std::vector<cd> Vv, Tv;
  lanczos(op, as_c(u), m, Vv, Tv, *beta);
  std::memcpy(V, Vv.data(), Vv.size() * sizeof(cd));
  std::memcpy(T, Tv.data(), Tv.size() * sizeof(cd));
  return 0;
}

// real lanczos_L (eigen_krylov_real.hpp:5-51): V n*m, T m*m, both column-major f64
int oracle_lanczos_r(const oracle_grid *g, const double *u, uint32_t m,
                     double *V, double *T, double *beta) {
  Grid G;
  if (!make_grid(g, G) || m < 1) return -1;
  StencilOp op{G};
  std::vector<double> Vv, Tv;
  lanczos(op, u, m, Vv, Tv, *beta);
  std::memcpy(V, Vv.data(), Vv.size() * sizeof(double));
  std::memcpy(T, Tv.data(), Tv.size() * sizeof(double));
  return 0;
}

int oracle_krylov_c(const oracle_grid *g, const double *u, double t_re,
                    double t_im, uint32_t m, int func, double *out) {
  Grid G;
  if (!make_grid(g, G) || m < 1) return -1;
  StencilOp op{G};
  krylov_apply(op, as_c(u), cd(t_re, t_im), m, func, as_c(out));
  return 0;
}

int oracle_krylov_r(const oracle_grid *g, const double *u, double t,
                    uint32_t m, int func, double *out) {
  Grid G;
  if (!make_grid(g, G) || m < 1) return -1;
  StencilOp op{G};
  krylov_apply(op, u, cd(t, 0.0), m, func, out);
  return 0;
}

int oracle_krylov_csr_c(uint64_t n, const int64_t *rowptr, const int64_t *col,
                        const double *val, const double *u, double t_re,
                        double t_im, uint32_t m, int func, double *out) {
  if (m < 1) return -1;
  CsrOp op{n, rowptr, col, val};
  krylov_apply(op, as_c(u), cd(t_re, t_im), m, func, as_c(out));
  return 0;
}

int oracle_krylov_csr_r(uint64_t n, const int64_t *rowptr, const int64_t *col,
                        const double *val, const double *u, double t,
                        uint32_t m, int func, double *out) {
  if (m < 1) return -1;
  CsrOp op{n, rowptr, col, val};
  krylov_apply(op, u, cd(t, 0.0), m, func, out);
  return 0;
}

// NLSESolver::step (nlse_solver.hpp:53-77), tau = 1j*dt, called nsteps times.
int oracle_nlse_steps(const oracle_grid *g, double *u_, double dt,
                      uint32_t nsteps, uint32_t m, int nonlin,
                      const double *sigma) {
  Grid G;
  if (!make_grid(g, G) || m < 1 || (nonlin != 0 && nonlin != 1)) return -1;
  if (nonlin == 1 && !sigma) return -1;
  StencilOp op{G};
  const uint64_t n = G.N;
  cd *u = as_c(u_);
  std::vector<cd> rho(u, u + n), buf(n);
  const cd tau(0.0, dt);
  for (uint32_t s = 0; s < nsteps; ++s) {
    std::memcpy(rho.data(), u, n * sizeof(cd));
    nonlin_half(rho.data(), n, dt, nonlin, sigma);
    krylov_apply(op, rho.data(), -tau, m, ORACLE_F_EXP_ABS, buf.data());
    nonlin_half(buf.data(), n, dt, nonlin, sigma);
    std::memcpy(u, buf.data(), n * sizeof(cd));
  }
  return 0;
}

int oracle_laplacian_aniso_apply_c(const oracle_grid *g, const double *c, const double *x,
                                   double *y) {
  Grid G;
  if (!make_grid(g, G) || !c || !x || !y) return -1;
  lap_aniso_apply(G, c, as_c(x), as_c(y));
  return 0;
}

int oracle_krylov_aniso_c(const oracle_grid *g, const double *c, const double *u,
                          double t_re, double t_im, uint32_t m, int func, double *out) {
  Grid G;
  if (!make_grid(g, G) || !c || m < 1) return -1;
  AnisoOp op{G, c};
  krylov_apply(op, as_c(u), cd(t_re, t_im), m, func, as_c(out));
  return 0;
}

int oracle_neumann_bc_c(const oracle_grid *g, double *u) {
  Grid G;
  if (!make_grid(g, G) || !u) return -1;
  if (G.nx < 3 || G.ny < 3 || (G.dim == 3 && G.nz < 3)) return -1;
  neumann_bc(G, as_c(u));
  return 0;
}

// G2 NLSESolverDevice::step (nlsolvers/device/include/nlse_dev.hpp:187-203),
// tau = 1j*dt: u <- N(exp(tau L) N(u)) with N(v) = v exp(tau/2 m|v|^2) and
// the G2 matrix function exp(t*lambda), t = +tau, Q f Q^H
// (nlsolvers/device/include/matfunc_complex.hpp:254-375); the G2 Lanczos is
// the G1 device one (rounding-level equal to this MGS restatement).  With
// bc != 0 the driver's apply_bc() follows every step
// (nlse_cubic_driver_3d.cpp:116-119).
int oracle_nlse_g2_steps(const oracle_grid *g, const double *c, const double *mfield,
                         double *u_, double dt, uint32_t nsteps, uint32_t m, int bc) {
  Grid G;
  if (!make_grid(g, G) || !c || !mfield || m < 1) return -1;
  if (bc && (G.nx < 3 || G.ny < 3 || (G.dim == 3 && G.nz < 3))) return -1;
  AnisoOp op{G, c};
  const uint64_t n = G.N;
  cd *u = as_c(u_);
  std::vector<cd> buf(u, u + n), out(n);
  const cd tau(0.0, dt);
  for (uint32_t s = 0; s < nsteps; ++s) {
    std::memcpy(buf.data(), u, n * sizeof(cd));
    nonlin_half_g2(buf.data(), mfield, n, dt);
    krylov_apply(op, buf.data(), tau, m, ORACLE_F_EXP, out.data());
    nonlin_half_g2(out.data(), mfield, n, dt);
    std::memcpy(u, out.data(), n * sizeof(cd));
    if (bc) neumann_bc(G, u);
  }
  return 0;
}

// G2 cubic-quintic (nlsolvers/device/include/nlse_cubic_quintic.cuh:9-40,
// nlse_cubic_quintic_dev.hpp:79-95): rho = m (s1 |u|^2 + s2 |u|^4) with real s1, s2
// (density_cubic_quintic), u *= exp(-tau/2 rho) (nonlin_part_cubic_quintic with
// -.5*tau), the linear flow matfunc_->apply(u, buf, -tau): exp(t lambda) with
// t = -tau (G2 "exp", matfunc_complex.hpp:281-287), on the isotropic no-flux
// operator (build_laplacian_noflux, nlsolvers/common/include/laplacians.hpp:10-52 --
// the same matrix as G1's 2D operator).  The density is recomputed from the
// post-linear field for the second half-step (_dev.hpp:88-91).
void nonlin_half_cq_g2(cd *u, const double *mf, uint64_t n, double dt, double s1, double s2) {
  const cd ht = -0.5 * cd(0.0, dt);
  for (uint64_t p = 0; p < n; ++p) {
    const double d = u[p].real() * u[p].real() + u[p].imag() * u[p].imag();
    const double rho = mf[p] * (s1 * d + s2 * d * d);
    u[p] = u[p] * std::exp(ht * cd(rho, 0.0));
  }
}

int oracle_nlse_cq_g2_steps(const oracle_grid *g, const double *mfield, double *u_, double dt,
                            uint32_t nsteps, uint32_t m, double s1, double s2, int bc) {
  Grid G;
  if (!make_grid(g, G) || !mfield || m < 1) return -1;
  if (bc && (G.nx < 3 || G.ny < 3 || (G.dim == 3 && G.nz < 3))) return -1;
  StencilOp op{G};
  const uint64_t n = G.N;
  cd *u = as_c(u_);
  std::vector<cd> buf(u, u + n), out(n);
  const cd tau(0.0, dt);
  for (uint32_t s = 0; s < nsteps; ++s) {
    std::memcpy(buf.data(), u, n * sizeof(cd));
    nonlin_half_cq_g2(buf.data(), mfield, n, dt, s1, s2);
    krylov_apply(op, buf.data(), -tau, m, ORACLE_F_EXP, out.data());
    nonlin_half_cq_g2(out.data(), mfield, n, dt, s1, s2);
    std::memcpy(u, out.data(), n * sizeof(cd));
    if (bc) neumann_bc(G, u);
  }
  return 0;
}

int oracle_nlse_sewi_steps(const oracle_grid *g, const double *c, const double *mfield,
                           double *u_, double *up_, double dt, uint32_t first_step,
                           uint32_t nsteps, uint32_t m, int bc) {
  Grid G;
  if (!make_grid(g, G) || !c || !mfield || !u_ || !up_ || m < 1 || first_step < 1) return -1;
  if (bc && (G.nx < 3 || G.ny < 3 || (G.dim == 3 && G.nz < 3))) return -1;
  AnisoOp op{G, c};
  const uint64_t n = G.N;
  cd *u = as_c(u_), *up = as_c(up_);
  std::vector<cd> buf(n), b2(n), b3(n);
  const cd tau(0.0, dt);
  for (uint32_t s = 0; s < nsteps; ++s) {
    const uint32_t step_number = first_step + s;
    if (step_number == 1) {  // nlse_dev.hpp:206-210: u_prev = u; SS2 step
      std::memcpy(up, u, n * sizeof(cd));
      std::memcpy(buf.data(), u, n * sizeof(cd));
      nonlin_half_g2(buf.data(), mfield, n, dt);
      krylov_apply(op, buf.data(), tau, m, ORACLE_F_EXP, b2.data());
      nonlin_half_g2(b2.data(), mfield, n, dt);
      std::memcpy(u, b2.data(), n * sizeof(cd));
    } else {  // nlse_dev.hpp:211-229
      std::memcpy(buf.data(), u, n * sizeof(cd));
      for (uint64_t p = 0; p < n; ++p)  // compute_B, nlse_dev.hpp:42-50
        b2[p] = -mfield[p] * (u[p].real() * u[p].real() + u[p].imag() * u[p].imag()) * u[p];
      krylov_apply(op, b2.data(), cd(dt, 0.0), m, ORACLE_F_SINC, b3.data());
      krylov_apply(op, b3.data(), tau, m, ORACLE_F_EXP, b2.data());
      krylov_apply(op, up, 2.0 * tau, m, ORACLE_F_EXP, b3.data());
      const cd two_tau = 2.0 * tau;
      for (uint64_t p = 0; p < n; ++p) u[p] = b3[p] - two_tau * b2[p];  // apply_sewi :52-63
      std::memcpy(up, buf.data(), n * sizeof(cd));
    }
    if (bc) neumann_bc(G, u);
  }
  return 0;
}

// G2 Klein-Gordon Gautschi step, KGESolver::step
// (nlsolvers/device/include/kg_single.cuh:49-86) on the operator -div(c grad)
// that kg_driver_dev_{2d,3d}.cpp assemble:
//   c2 = 2 cos(t sqrt|L|) u ; g = -m u^3 ; s = sinc^2(t sqrt|L|) g  (t = dt)
//   u_new = (c2 - u_past) + (dt*dt) s ; u_past = u ; v = (u_new - u_past)/dt
// then (bc != 0) the driver's apply_bc() on u only (kg_driver_dev_3d.cpp:150-153).
int oracle_kg_steps(const oracle_grid *g, const double *c, const double *mfield, double *u,
                    double *u_past, double *v, double dt, uint32_t nsteps, uint32_t m, int bc) {
  Grid G;
  if (!make_grid(g, G) || !c || !mfield || !u || !u_past || !v || m < 1) return -1;
  if (bc && (G.nx < 3 || G.ny < 3 || (G.dim == 3 && G.nz < 3))) return -1;
  AnisoOp op{G, c, true};
  const uint64_t n = G.N;
  std::vector<double> c2(n), gb(n), s2(n), old(n);
  const cd t(dt, 0.0);
  for (uint32_t s = 0; s < nsteps; ++s) {
    std::memcpy(old.data(), u, n * sizeof(double));
    krylov_apply(op, u, t, m, ORACLE_F_COS_SQRT, c2.data());
    for (uint64_t p = 0; p < n; ++p) c2[p] = c2[p] * 2.0;
    for (uint64_t p = 0; p < n; ++p) gb[p] = -mfield[p] * u[p] * u[p] * u[p];
    krylov_apply(op, gb.data(), t, m, ORACLE_F_SINC2_SQRT, s2.data());
    const double tt = dt * dt;
    for (uint64_t p = 0; p < n; ++p) u[p] = (c2[p] - u_past[p]) + s2[p] * tt;
    std::memcpy(u_past, old.data(), n * sizeof(double));
    for (uint64_t p = 0; p < n; ++p) v[p] = (u[p] - u_past[p]) / dt;
    if (bc) neumann_bc(G, u);
  }
  return 0;
}

int oracle_neumann_bc_r(const oracle_grid *g, double *u) {
  Grid G;
  if (!make_grid(g, G) || !u) return -1;
  if (G.nx < 3 || G.ny < 3 || (G.dim == 3 && G.nz < 3)) return -1;
  neumann_bc(G, u);
  return 0;
}

// SGESolver::step (sg_solver.hpp:53-74): Gautschi with the id filter.
int oracle_sg_steps(const oracle_grid *g, double *u, double *u_past,
                    const double *mfield, double dt, uint32_t nsteps,
                    uint32_t m) {
  Grid G;
  if (!make_grid(g, G) || m < 1 || !mfield) return -1;
  StencilOp op{G};
  const uint64_t n = G.N;
  std::vector<double> filt(n), gbuf(n), s2(n), cosv(n);
  const cd t(dt, 0.0);
  for (uint32_t s = 0; s < nsteps; ++s) {
    krylov_apply(op, u, t, m, ORACLE_F_ID_SQRT, filt.data());
    for (uint64_t p = 0; p < n; ++p) gbuf[p] = mfield[p] * (-std::sin(filt[p]));
    krylov_apply(op, gbuf.data(), t, m, ORACLE_F_SINC2_HALF, s2.data());
    krylov_apply(op, u, t, m, ORACLE_F_COS_SQRT, cosv.data());
    for (uint64_t p = 0; p < n; ++p) {
      const double uc = u[p];
      u[p] = 2 * cosv[p] - u_past[p] + dt * dt * s2[p];
      u_past[p] = uc;
    }
  }
  return 0;
}

// G2 device Gautschi family, Phi4Solver / SGESolver / SGEDoubleSolver /
// SGEHyperbolicSolver ::step (nlsolvers/device/include/phi4_single.cuh:33-47,
// sg_single.cuh:33-47, sg_double.cuh:34-48, sg_hyperbolic.cuh:33-47) on the
// isotropic no-flux operator the drivers build (phi4_driver_dev.cpp:84-85):
//   buf = u ; buf2 = id_sqrt(u) ; buf2 = -m F(buf2) ; buf3 = sinc2_sqrt(buf2) ;
//   buf2 = cos_sqrt(u) ; u = 2 buf2 - u_past + tau^2 buf3 ; u_past = buf
// (t = tau = dt; matfunc_real.hpp:212-238: f(t sqrt|lambda|)), then (bc != 0)
// the drivers' apply_bc() on u only (phi4_driver_dev.cpp:108-111, phi4_dev.hpp:92).
// kind: 0 sin u (sg_single.cuh:18), 1 sin u + sin(u/2) (sg_double.cuh:19),
//       2 sinh u (sg_hyperbolic.cuh:18), 3 u + u^3 (phi4_single.cuh:18).
int oracle_gautschi_g2_steps(const oracle_grid *g, int kind, double *u, double *u_past,
                             const double *mfield, double dt, uint32_t nsteps, uint32_t m,
                             int bc) {
  Grid G;
  if (!make_grid(g, G) || !u || !u_past || !mfield || m < 1 || kind < 0 || kind > 3) return -1;
  if (bc && (G.nx < 3 || G.ny < 3 || (G.dim == 3 && G.nz < 3))) return -1;
  StencilOp op{G};
  const uint64_t n = G.N;
  std::vector<double> buf(n), buf2(n), buf3(n);
  const cd t(dt, 0.0);
  for (uint32_t s = 0; s < nsteps; ++s) {
    std::memcpy(buf.data(), u, n * sizeof(double));
    krylov_apply(op, u, t, m, ORACLE_F_ID_SQRT, buf2.data());
    for (uint64_t p = 0; p < n; ++p) {
      const double y = buf2[p];
      double f;
      switch (kind) {
        case 0: f = std::sin(y); break;
        case 1: f = std::sin(y) + std::sin(0.5 * y); break;
        case 2: f = std::sinh(y); break;
        default: f = y + y * y * y; break;
      }
      buf2[p] = -(mfield[p] * f);
    }
    krylov_apply(op, buf2.data(), t, m, ORACLE_F_SINC2_SQRT, buf3.data());
    krylov_apply(op, u, t, m, ORACLE_F_COS_SQRT, buf2.data());
    for (uint64_t p = 0; p < n; ++p) u[p] = 2.0 * buf2[p] - u_past[p] + dt * dt * buf3[p];
    std::memcpy(u_past, buf.data(), n * sizeof(double));
    if (bc) neumann_bc(G, u);
  }
  return 0;
}

}  // extern "C"
