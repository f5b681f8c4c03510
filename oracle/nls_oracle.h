/*
 * nls_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain C++17 restatement (no Eigen, no GPU) of the reference's G1 CPU path:
 *   laplacians.hpp:10-105            (no-flux 2D/3D operators, incl. 3D y-wrap)
 *   eigen_krylov_complex.hpp:10-84   (MGS Lanczos, T[m-1,m-1]=0, exp(t*|lambda|))
 *   eigen_krylov_real.hpp:5-201      (real Lanczos, cos/sinc/sinc^2/id of t*sqrt|lambda|)
 *   nlse_solver.hpp:53-77            (Strang SS2 cubic NLSE step)
 *   device/nlse_cq_solver.hpp:16-39  (cubic-quintic density, G1 device semantics)
 *   sg_solver.hpp:53-74              (sine-Gordon Gautschi step)
 * and of the G2 3D/2D device stepper behind nlse_cubic_driver_{2d,3d}.cpp:
 *   nlsolvers/common/include/laplacians.hpp:54-103,158-218 (anisotropic div(c grad))
 *   nlsolvers/device/include/nlse_dev.hpp:20-40,187-203     (m|u|^2, +tau/2, exp(tau L))
 *   nlsolvers/device/include/matfunc_complex.hpp:254-375     (exp(t*lambda), Q f Q^H)
 *   nlsolvers/device/include/boundaries.cuh:10-81            (Neumann copy BC)
 *   nlsolvers/device/include/nlse_dev.hpp:205-238            (sEWI)
 *   nlsolvers/device/include/kg_single.cuh:49-86             (Klein-Gordon Gautschi)
 *   nlsolvers/device/include/{sg_single,sg_double,sg_hyperbolic,phi4_single}.cuh
 *                                                            (G2 Gautschi family)
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product path (libnls_amd.so) never links it.
 *
 * Layout: complex arrays are interleaved doubles (re, im); flat index
 *   2D: idx = j*nx + i ;  3D: idx = (k*ny + j)*nx + i   (reference: nlse_call.cpp,
 *   nlse_driver_3d.cpp:12-18).
 */
#ifndef NLS_ORACLE_H
#define NLS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int dim;             /* 2 or 3 */
  uint32_t nx, ny, nz; /* full grid incl. boundary layer; nz ignored for dim 2 */
  double dx, dy;       /* 2D scale 1/(dx*dy), 3D scale 1/(dx*dx) (laplacians.hpp:49,102) */
} oracle_grid;

/* Krylov matrix functions (eigen_krylov_real.hpp / eigen_krylov_complex.hpp) */
enum {
  ORACLE_F_EXP_ABS = 0,   /* exp(t*|lambda|)           eigen_krylov_complex.hpp:71-77 */
  ORACLE_F_EXP = 1,       /* exp(t*lambda)  (G2)       nlsolvers/host/include/eigen_krylov_complex.hpp:67-72 */
  ORACLE_F_COS_SQRT = 2,  /* cos(t*sqrt|lambda|)       eigen_krylov_real.hpp:53-85 */
  ORACLE_F_SINC_SQRT = 3, /* sinc(t*sqrt|lambda|)      eigen_krylov_real.hpp:87-105 */
  ORACLE_F_SINC2_SQRT = 4,/* sinc^2(t*sqrt|lambda|)    eigen_krylov_real.hpp:107-141 */
  ORACLE_F_ID_SQRT = 5,   /* t*sqrt|lambda|            eigen_krylov_real.hpp:143-170 */
  ORACLE_F_SINC2_HALF = 6,/* sinc^2(t/2*sqrt|lambda|)  eigen_krylov_real.hpp:172-201 */
  ORACLE_F_SINC = 7       /* sinc(t*lambda) (G2 "sinc") nlsolvers/device/include/matfunc_complex.hpp:290-300 */
};

/* threads the loops use: 1 for the serial checker build, OpenMP's count for
 * liboracle_nls_omp.so (all-cores CPU baseline) */
int oracle_threads(void);

int oracle_laplacian_apply_c(const oracle_grid *g, const double *x, double *y);
int oracle_laplacian_apply_r(const oracle_grid *g, const double *x, double *y);

/* V: n*m complex, column-major (V[k*n + p]); T: m*m complex column-major */
int oracle_lanczos_c(const oracle_grid *g, const double *u, uint32_t m,
                     double *V, double *T, double *beta);

/* real lanczos_L (eigen_krylov_real.hpp:5-51): V n*m f64, T m*m f64, column-major */
int oracle_lanczos_r(const oracle_grid *g, const double *u, uint32_t m,
                     double *V, double *T, double *beta);

/* out = f(L) u via m-dim Krylov; t complex for the complex path */
int oracle_krylov_c(const oracle_grid *g, const double *u, double t_re,
                    double t_im, uint32_t m, int func, double *out);
int oracle_krylov_r(const oracle_grid *g, const double *u, double t,
                    uint32_t m, int func, double *out);

/* Same, for an explicit CSR operator (real values), used by the scipy KAT
 * (nlsolvers/host/drivers/test_scipy_matfunc.cpp:41-95). */
int oracle_krylov_csr_c(uint64_t n, const int64_t *rowptr, const int64_t *col,
                        const double *val, const double *u, double t_re,
                        double t_im, uint32_t m, int func, double *out);
int oracle_krylov_csr_r(uint64_t n, const int64_t *rowptr, const int64_t *col,
                        const double *val, const double *u, double t,
                        uint32_t m, int func, double *out);

/* NLSE: nsteps Strang SS2 steps with tau = 1j*dt (nlse_solver.hpp:53-77).
 * nonlin 0 = cubic (G1 CPU), 1 = cubic-quintic (G1 device semantics,
 * device/nlse_cq_solver.hpp:16-39) with sigma = {s1re, s1im, s2re, s2im}. */
int oracle_nlse_steps(const oracle_grid *g, double *u, double dt,
                      uint32_t nsteps, uint32_t m, int nonlin,
                      const double *sigma);

/* G2: anisotropic operator with coefficient field c (real, N cells) */
int oracle_laplacian_aniso_apply_c(const oracle_grid *g, const double *c,
                                   const double *x, double *y);
int oracle_krylov_aniso_c(const oracle_grid *g, const double *c, const double *u,
                          double t_re, double t_im, uint32_t m, int func,
                          double *out);
/* G2 Neumann copy boundary condition, in place (needs >= 3 cells per axis) */
int oracle_neumann_bc_c(const oracle_grid *g, double *u);
/* G2 SS2 steps (tau = 1j*dt) with focusing field m and anisotropy c; bc != 0
 * applies the Neumann copy BC after every step. */
int oracle_nlse_g2_steps(const oracle_grid *g, const double *c,
                         const double *mfield, double *u, double dt,
                         uint32_t nsteps, uint32_t m, int bc);
/* G2 cubic-quintic SS2 steps (tau = 1j*dt): rho = m (s1|u|^2 + s2|u|^4), real
 * s1, s2, N = exp(-tau/2 rho), linear flow exp(-tau lambda) on the isotropic
 * operator; bc != 0: Neumann copy BC after every step (the driver's apply_bc). */
int oracle_nlse_cq_g2_steps(const oracle_grid *g, const double *mfield, double *u,
                            double dt, uint32_t nsteps, uint32_t m, double s1,
                            double s2, int bc);

/* G2 sEWI stepper (NLSESolverDevice::step_sewi, nlsolvers/device/include/nlse_dev.hpp:205-238)
 * for step numbers first_step .. first_step+nsteps-1: step 1 is an SS2 step that
 * saves u_prev = u; later steps u <- exp(2 tau L) u_prev - 2 tau exp(tau L)
 * sinc(dt L) B(u), B(u) = -m|u|^2 u, u_prev <- old u.  bc != 0: Neumann copy BC
 * after every step (nlse_cubic_sewi_driver_3d.cpp).  u, u_prev in/out. */
int oracle_nlse_sewi_steps(const oracle_grid *g, const double *c,
                           const double *mfield, double *u, double *u_prev,
                           double dt, uint32_t first_step, uint32_t nsteps,
                           uint32_t m, int bc);

/* G2 Klein-Gordon Gautschi (nlsolvers/device/include/kg_single.cuh:49-86,
 * kg_driver_dev_{2d,3d}.cpp: operator -div(c grad), m(x), Neumann BC on u after
 * every step when bc != 0); u, u_past, v updated in place. */
int oracle_kg_steps(const oracle_grid *g, const double *c, const double *mfield,
                    double *u, double *u_past, double *v, double dt,
                    uint32_t nsteps, uint32_t m, int bc);
int oracle_neumann_bc_r(const oracle_grid *g, double *u);

/* G2 device Gautschi family (nlsolvers/device/include/{sg_single,sg_double,
 * sg_hyperbolic,phi4_single}.cuh): kind 0 sin, 1 sin + sin(u/2), 2 sinh,
 * 3 u + u^3; g = -m F(id(u)), sinc^2 / cos / id of t sqrt|lambda| (t = dt) on the
 * isotropic operator; bc != 0: Neumann copy BC on u after every step.  u, u_past
 * updated in place. */
int oracle_gautschi_g2_steps(const oracle_grid *g, int kind, double *u, double *u_past,
                             const double *mfield, double dt, uint32_t nsteps, uint32_t m,
                             int bc);

/* sine-Gordon Gautschi (sg_solver.hpp:53-74); u, u_past updated in place. */
int oracle_sg_steps(const oracle_grid *g, double *u, double *u_past,
                    const double *mfield, double dt, uint32_t nsteps,
                    uint32_t m);

#ifdef __cplusplus
}
#endif
#endif
