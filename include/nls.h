/*
 * nls.h -- C-ABI of libnls_amd.so, the MI355X-native (gfx950) Krylov/Lanczos
 * exponential time-stepper for the 2D/3D NLSE and the 2D sine-Gordon
 * Gautschi integrator of konradha/nonlinear-solvers.
 *
 * Plain C types only: no HIP, torch or Eigen types cross this boundary.
 * Every entry point returns an int status (NLS_OK == 0, negative on error)
 * and never throws; nls_last_error() gives the message.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   nls_create       <- NLSESolverDevice(L, host_u0, Parameters)          device/nlse_solver_dev.hpp:53-84
 *                       NLSECubicQuinticSolver(L, host_u0, Parameters)    device/nlse_cq_solver.hpp:55-86
 *                       SGESolverDevice(row_ptr, col_ind, values, c, m, n, nnz, u0, v0, u_past, params)
 *                                                                          device/sg_solver_dev.hpp:104-149
 *                       build_laplacian_noflux{,_3d}(nx-2, ...)            laplacians.hpp:10-105
 *                       (the operator is described by grid parameters, not by a CSR matrix)
 *   nls_set_field    <- cudaMemcpy H2D of host_u0 in the ctors above       device/nlse_solver_dev.hpp:63-64
 *   nls_set_sg_state <- SGESolverDevice ctor u0/u_past/m uploads           device/sg_solver_dev.hpp:118-135
 *                       KGESolverDevice ctor (G2)                          nlsolvers/device/include/kg_dev.hpp
 *   nls_set_coefficients <- NLSESolverDevice(L, u0, m, ...) (G2) m upload  nlsolvers/device/include/nlse_dev.hpp:66-130
 *                       build_anisotropic_laplacian_noflux{,_3d}(.., c)   nlsolvers/common/include/laplacians.hpp:54-103,158-218
 *   nls_apply_bc     <- NLSESolverDevice::apply_bc() (G2)                  nlsolvers/device/include/nlse_dev.hpp:178-185,
 *                       neumann_bc_no_velocity_blocking{,_3d}             nlsolvers/device/include/boundaries.cuh:10-81
 *   nls_step         <- NLSESolverDevice::step(tau=1j*dt, i)               device/nlse_solver_dev.hpp:94-111
 *                       SGESolverDevice::step(tau=dt, i)                   device/sg_solver_dev.hpp:168-193
 *                       G2 NLSESolverDevice::step(tau=1j*dt, i)            nlsolvers/device/include/nlse_dev.hpp:187-203
 *   nls_step_sewi    <- G2 NLSESolverDevice::step_sewi(tau=1j*dt, i)       nlsolvers/device/include/nlse_dev.hpp:205-238
 *   nls_get_field    <- transfer_snapshots(dst) / store_snapshot D2D+D2H   device/nlse_solver_dev.hpp:113-124
 *   nls_get_field_async / nls_wait_field
 *                    <- store_snapshot_online(host_dst) (G2)               nlsolvers/device/include/nlse_dev.hpp:323-334
 *   nls_get_sg_velocity <- transfer_snapshots(dst, 'v')                    device/sg_solver_dev.hpp:195-222
 *   nls_krylov_apply <- MatrixFunctionApplicator{Complex,Real}::apply(out, in, t[, type])
 *                                                                          device/matfunc_complex.hpp:155-177
 *                                                                          device/matfunc_real.hpp:171-233
 *   nls_laplacian_apply <- DeviceSpMV<T>::multiply(x, y)                   device/spmv.hpp:65-73
 *   nls_destroy      <- ~NLSESolverDevice / ~SGESolverDevice (cudaFree)
 *
 * Threading: handles are independent (no globals besides the create-error
 * string); one handle must not be used from two threads at once -- the same
 * contract as one NLSESolverDevice per OpenMP thread in
 * device/nlse_driver_omp.cpp:103-121.  Each handle owns its HIP stream(s),
 * device buffers and (multi-GPU) RCCL communicator.
 *
 * Data layout (host side): complex fields are interleaved (re, im) doubles in
 * C order, 2D [ny][nx], 3D [nz][ny][nx] -- the .npy layout of the reference
 * drivers.  With nranks > 1 each rank passes/receives its slab of planes
 * (3D: z-planes, 2D: y-rows), see nls_local_planes().
 */
#ifndef NLS_AMD_H
#define NLS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NLS_ABI_VERSION 6
#define NLS_MAX_KRYLOV 32

enum nls_status {
  NLS_OK = 0,
  NLS_ERR_ARG = -1,     /* invalid argument / config */
  NLS_ERR_SHAPE = -2,   /* buffer length does not match the grid */
  NLS_ERR_OOM = -3,     /* device allocation failed */
  NLS_ERR_HIP = -4,     /* HIP runtime error (launch or async fault) */
  NLS_ERR_RCCL = -5,    /* RCCL error */
  NLS_ERR_STATE = -6    /* call not valid in this state (e.g. no field set) */
};

enum nls_equation {
  NLS_NLSE_CUBIC = 0,   /* i u_t + Lap u + |u|^2 u = 0, SS2 (nlse_solver.hpp:53-77) */
  NLS_NLSE_CQ = 1,      /* rho = s1|u|^2 + s2|u|^4 (device/nlse_cq_solver.hpp:16-39) */
  NLS_SG_GAUTSCHI = 2,  /* u_tt = Lap u + m sin u, Gautschi (sg_solver.hpp:53-74) */
  NLS_NLSE_G2 = 3,      /* G2 cubic NLSE with focusing field m(x) and anisotropic operator
                           div(c grad): SS2 with exp(+tau/2 m|u|^2) and exp(tau*lambda)
                           (nlsolvers/device/include/nlse_dev.hpp:187-203,
                           nlsolvers/device/drivers/nlse_cubic_driver_{2d,3d}.cpp) */
  NLS_KG_GAUTSCHI = 4,  /* G2 Klein-Gordon u_tt = div(c grad u) - m u^3, Gautschi with
                           cos / sinc^2 of t sqrt|lambda| (nlsolvers/device/include/kg_single.cuh:49-86,
                           kg_driver_dev_{2d,3d}.cpp); real field; m, c via
                           nls_set_coefficients, u / u_past via nls_set_sg_state */
  /* G2 device Gautschi family (nlsolvers/device/include/{sg_single,sg_double,
     sg_hyperbolic,phi4_single}.cuh, drivers {sg_single,sg_double,sg_hyperbolic,
     phi4}_driver_dev.cpp): u_tt = Lap u - m F(u) on the isotropic operator
     (laplacians.hpp:10-52 / :55-105), step
       y = id(u), g = -m F(y), s = sinc^2(t sqrt|L|) g, c = cos(t sqrt|L|) u,
       u+ = 2c - u- + tau^2 s      (id, cos, sinc^2 of t sqrt|lambda|, t = tau = dt)
     with F per equation below; real field; u, u_past, m via nls_set_sg_state;
     Neumann copy BC on u after each step via nls_apply_bc (the drivers' apply_bc). */
  NLS_SG_G2 = 5,           /* F = sin u                sg_single.cuh:14-20 */
  NLS_SG_DOUBLE = 6,       /* F = sin u + sin(u/2)     sg_double.cuh:14-21 */
  NLS_SG_HYPERBOLIC = 7,   /* F = sinh u               sg_hyperbolic.cuh:14-20 */
  NLS_PHI4 = 8,            /* F = u + u^3              phi4_single.cuh:14-20 */
  NLS_NLSE_CQ_G2 = 9       /* G2 cubic-quintic NLSE (nlsolvers/device/include/nlse_cubic_quintic.cuh:9-40,
                              nlse_cubic_quintic_dev.hpp:79-95, driver nlse_cubic_quintic_driver_dev.cpp):
                              rho = m (s1|u|^2 + s2|u|^4) with REAL s1 = sigma1[0], s2 = sigma2[0]
                              (the imaginary parts are ignored), N = exp(-tau/2 rho), linear flow
                              exp(t*lambda) with t = -tau on the isotropic operator; m(x) via
                              nls_set_coefficients (cfield NULL; required before the first step,
                              as for G2); Neumann copy BC
                              via nls_apply_bc (the driver's apply_bc) */
};

/* Krylov matrix functions f, applied as f(L) u (nls_krylov_apply) */
enum nls_func {
  NLS_F_EXP_ABS = 0,    /* exp(t*|lambda|)          eigen_krylov_complex.hpp:71-77 */
  NLS_F_EXP = 1,        /* exp(t*lambda)  (G2)      nlsolvers/host/include/eigen_krylov_complex.hpp:67-72 */
  NLS_F_COS_SQRT = 2,   /* cos(t*sqrt|lambda|)      eigen_krylov_real.hpp:53-85 */
  NLS_F_SINC_SQRT = 3,  /* sinc(t*sqrt|lambda|)     eigen_krylov_real.hpp:87-105 */
  NLS_F_SINC2_SQRT = 4, /* sinc^2(t*sqrt|lambda|)   eigen_krylov_real.hpp:107-141 */
  NLS_F_ID_SQRT = 5,    /* t*sqrt|lambda|           eigen_krylov_real.hpp:143-170 */
  NLS_F_SINC2_HALF = 6, /* sinc^2(t/2*sqrt|lambda|) eigen_krylov_real.hpp:172-201 */
  NLS_F_SINC = 7        /* sinc(t*lambda), G2 "sinc" nlsolvers/device/include/matfunc_complex.hpp:290-300 */
};

typedef struct nls_config {
  int32_t dim;          /* 2 or 3 */
  int32_t equation;     /* enum nls_equation */
  uint32_t nx, ny, nz;  /* full grid incl. boundary layer (nz ignored for dim 2) */
  double dx, dy;        /* operator scale: 2D 1/(dx*dy), 3D 1/(dx*dx) (laplacians.hpp:49,102) */
  uint32_t krylov_m;    /* Krylov dimension, 1..NLS_MAX_KRYLOV (reference default 10) */
  double sigma1[2];     /* CQ only: complex sigma_1 (reference default 0 + 0.5i) */
  double sigma2[2];     /* CQ only: complex sigma_2 (reference default -0.5 + 0i) */
  int32_t device;       /* HIP device ordinal, -1 = current device */
  int32_t nranks;       /* slab decomposition over ranks (1 = single GPU) */
  int32_t rank;         /* this rank, 0..nranks-1 */
  const void *rccl_id;  /* 128-byte RCCL unique id (nls_rccl_unique_id on rank 0), NULL if nranks == 1 */
  void *local_group;    /* in-process rank group (nls_group_create); replaces RCCL when non-NULL */
} nls_config;

typedef struct nls_handle nls_handle;

/* Fill cfg with the reference defaults (m=10, CQ sigmas 0.5i / -0.5, 1 rank). */
void nls_config_default(nls_config *cfg);
int nls_abi_version(void);
/* Build provenance: "src_sha256=<sha256 of the library sources> arch=gfx950 compiler=...
 * built=..." -- the sources are every nonlinear-solvers_amd/csrc/{*.hip,*.hpp,*.cpp} in
 * sorted path order, then include/nls.h (nls_amd.sources_sha256() recomputes it), so a
 * prebuilt library can be checked against the tree it ships in.  No reference counterpart. */
const char *nls_build_info(void);

int nls_create(const nls_config *cfg, nls_handle **out);
int nls_destroy(nls_handle *h);
const char *nls_last_error(const nls_handle *h); /* h == NULL: last nls_create error */

/* Slab owned by this rank: planes [*z0, *z0 + *nzl) of the slowest dimension
 * (3D: z, 2D: y); n_local = nzl * plane size. */
int nls_local_planes(const nls_handle *h, uint32_t *z0, uint32_t *nzl, uint64_t *n_local);

/* Ranks the handle exchanges with, as the transport itself reports them: the RCCL
 * communicator's ncclCommCount (transport 1), the in-process group's size
 * (transport 2), or 1 for a single-rank handle without a communicator
 * (transport 0).  The multi-GPU counterpart of the reference's
 * device/nlse_driver_omp.cpp:103-121 rank loop; bench.py reports it. */
int nls_comm_size(const nls_handle *h, int32_t *nranks, int32_t *transport);

/* The slab decomposition itself (pure function, no device needed): planes
 * [*z0, *z0 + *nzl) of npl planes owned by `rank` of `nranks` -- contiguous,
 * the first npl % nranks ranks one plane larger.  nls_local_planes() of a
 * handle returns the same. */
int nls_slab_planes(uint32_t npl, int32_t nranks, int32_t rank, uint32_t *z0, uint32_t *nzl);

/* NLSE: u (complex interleaved, 2*n_local doubles).  SG: u (n_local doubles).
 * (The G2 drivers do not normalise u0, nlse_cubic_driver_3d.cpp:54-65; the G1
 * drivers do, nlse_call.cpp:41-49 -- the caller decides.) */
int nls_set_field(nls_handle *h, const double *u, uint64_t n_local);
/* SG / KG: u, u_past = u0 - dt*v0 (sg_driver_dev.cpp:64,106) and the m(x) field
 * (KG: mfield may be NULL when nls_set_coefficients supplies it). */
int nls_set_sg_state(nls_handle *h, const double *u, const double *u_past,
                     const double *mfield, uint64_t n_local);

/* G2 only (NLS_NLSE_G2): the focusing field m(x) and the anisotropy c(x) of the
 * operator div(c grad u) (face weights (c_a + c_b)/2, diagonal -sum of weights,
 * scale 1/(dx*dy) in 2D and 1/(dx*dx) in 3D), both real, local slab.  Must be
 * called before the first nls_step.  NLS_NLSE_CQ_G2: m(x) only (cfield NULL,
 * isotropic operator); likewise required before the first nls_step /
 * nls_krylov_apply / nls_laplacian_apply (NLS_ERR_STATE otherwise). */
int nls_set_coefficients(nls_handle *h, const double *mfield, const double *cfield,
                         uint64_t n_local);
/* Neumann "copy" boundary condition of the G2 drivers, applied after every step
 * (boundaries.cuh:10-81): every boundary cell takes the value of the cell with
 * all coordinates clamped into [1, n-2].  Complex (NLSE) handles; needs >= 3
 * cells per dimension.  Like nls_step it is enqueued asynchronously. */
int nls_apply_bc(nls_handle *h);

/* G2 only: one step of the symmetric exponential wave integrator,
 * NLSESolverDevice::step_sewi(tau = 1j*dt, step_number)
 * (nlsolvers/device/include/nlse_dev.hpp:205-238): step_number 1 saves
 * u_prev = u and takes an SS2 step; later steps compute
 *   u <- exp(2 tau L) u_prev - 2 tau exp(tau L) sinc(dt L) B(u),  B(u) = -m|u|^2 u,
 * and u_prev <- the old u (three Krylov actions per step). */
int nls_step_sewi(nls_handle *h, double dt, uint32_t step_number);

/* Enqueue nsteps time steps (NLSE: tau = 1j*dt; SG: tau = dt) on the handle's
 * stream and return.  Errors of asynchronous execution surface at nls_sync /
 * nls_get_field. */
int nls_step(nls_handle *h, double dt, uint32_t nsteps);
int nls_sync(nls_handle *h);

int nls_get_field(nls_handle *h, double *u, uint64_t n_local);

/* Asynchronous snapshot (the online snapshot of
 * nlsolvers/device/include/nlse_dev.hpp:323-334 without stalling the time
 * loop): enqueue, after all work enqueued so far, a device-side copy of the
 * field into a staging buffer and its D2H transfer into dst on a copy stream,
 * then return.  dst must stay valid and must not be read until
 * nls_wait_field(h) returns; pinned memory from nls_host_alloc makes the
 * transfer fully asynchronous.  At most one snapshot is in flight per handle
 * (a new call orders its staging copy after the previous transfer on the
 * device, without blocking the host).  nls_wait_field may be called from
 * another host thread than the one driving the handle. */
int nls_get_field_async(nls_handle *h, double *dst, uint64_t n_local);
int nls_wait_field(nls_handle *h);
/* Page-locked host memory for nls_get_field_async (hipHostMalloc). */
int nls_host_alloc(uint64_t bytes, void **out);
int nls_host_free(void *p);
int nls_get_sg_velocity(nls_handle *h, double dt, double *v, uint64_t n_local);

/* One Krylov matrix-function action out = f(L) in (no time stepping), t complex
 * (real paths use t_re).  Complex for NLSE handles, real for SG handles. */
int nls_krylov_apply(nls_handle *h, const double *in, double t_re, double t_im,
                     int32_t func, double *out, uint64_t n_local);
/* y = L x (stencil only; complex for NLSE handles, real for SG handles). */
int nls_laplacian_apply(nls_handle *h, const double *x, double *y, uint64_t n_local);

/* Multi-GPU: 128-byte RCCL unique id, created on rank 0 and broadcast by the caller. */
int nls_rccl_unique_id(void *out128);

/* In-process rank group: the ranks of one slab decomposition are handles of
 * ONE process, each driven by its own host thread (the reference's
 * one-solver-per-OpenMP-thread model, device/nlse_driver_omp.cpp:103-121).
 * Halo planes move by device-to-device copies and the Lanczos sums are
 * reduced in fixed rank order on the device -- the same kernels and slab
 * layout as the RCCL path, usable on a single GPU.  Pass the group as
 * nls_config.local_group (rccl_id is then ignored). */
typedef struct nls_group nls_group;
int nls_group_create(int32_t nranks, nls_group **out);
int nls_group_destroy(nls_group *g);

/* Instrumentation: HIP-event timing around every launch on the handle's
 * stream.  Classes: 0 alpha (stencil + dot), 1 update (stencil + CGS +
 * write), 2 reduce/eigen, 3 nonlinear/pointwise, 4 halo exchange, 5 fused
 * final pass (last Lanczos vector + combination + nonlinear steps).  For the
 * update class the per-j times are also kept (index = j). */
typedef struct nls_timing {
  double class_ms[6];
  uint64_t class_count[6];
  double update_ms[NLS_MAX_KRYLOV];
  uint64_t update_count[NLS_MAX_KRYLOV];
  uint64_t steps;
  uint64_t graph_steps; /* steps replayed from a captured hipGraph (NLS_GRAPH) */
} nls_timing;
int nls_set_timing(nls_handle *h, int32_t enable);
int nls_get_timing(nls_handle *h, nls_timing *out); /* synchronises */
int nls_reset_timing(nls_handle *h);

/* Debug: the transport operations of a collective handle in issue order, with
 * the cross-stream dependencies between them.  Recorded only when the
 * environment has NLS_OPLOG=1 at nls_create.  Entries are 4 int32 each:
 * {kind, stream (0 compute, 1 halo), count (doubles), peer rank (-1: none)}.
 * Sets *n to the number recorded; with out != NULL also copies the oldest
 * min(*n, cap) entries into out and removes exactly those from the log (out ==
 * NULL: size query only).  The log keeps at most NLS_OPLOG_MAX entries (the newest); once
 * it has dropped any, its first entry is NLS_OP_DROPPED with the number dropped.  The invariant the tests check: an operation
 * on one stream is ordered after every earlier operation on the other stream
 * by a NLS_OP_WAIT_* entry in between (RCCL never sees one communicator's
 * operations in flight on two streams at once). */
enum nls_op_kind {
  NLS_OP_ALLREDUCE = 1,      /* ncclAllReduce / local fixed-order sum of the Lanczos sums */
  NLS_OP_SEND = 2,           /* halo planes to peer */
  NLS_OP_RECV = 3,           /* halo planes from peer */
  NLS_OP_WAIT_HALO = 4,      /* compute stream waits for the halo stream */
  NLS_OP_WAIT_COMPUTE = 5,   /* halo stream waits for the compute stream */
  NLS_OP_ALLGATHER = 6,      /* ncclAllGather of the peer-store IPC handles (NLS_PEER=1, once) */
  NLS_OP_DROPPED = 7         /* first entry of a truncated log: count = entries dropped before it */
};
#define NLS_OPLOG_MAX 65536
int nls_debug_oplog(nls_handle *h, int32_t *out, uint64_t cap, uint64_t *n);

/* Launch-shape knobs of a live handle, for same-allocation A/B measurements
 * (tools/knob_ab.py; the environment variables of the same names set them at
 * nls_create).  Results are unchanged up to the order of partial sums (the
 * k_p2d tile order); not with NLS_GRAPH.  No reference counterpart. */
enum nls_knob {
  NLS_KNOB_TAIL_DYN = 1,  /* fused tail through the dynamic tile queue (NLS_TAIL_DYN) */
  NLS_KNOB_KZ_FUSED = 2,  /* fused tail tile depth (NLS_KZ_FUSED; 0 = the stencil depth) */
  NLS_KNOB_P2_ORDER = 3   /* k_p2d tile order bits */
};
int nls_debug_knob(nls_handle *h, int32_t knob, int32_t value);

/* Basis placement chosen at nls_create.  The streams of one pass run 2-4 % faster or
 * slower depending on which HBM pages back the Krylov basis (DESIGN.md section 4,
 * "Placement"), which no allocation call controls: large single-rank handles allocate
 * up to NLS_PLACE candidate bases (default 8, where free memory allows), time the
 * same probe step sequence on each, keep the fastest and free the rest; the chosen
 * basis is then zeroed, so results do not depend on the choice.  *n = candidates
 * probed (0: no probe on this handle), *chosen = index kept, ms[0..min(n,cap)) =
 * each candidate's probe time (ms).  No reference counterpart (the reference has one
 * cudaMalloc per buffer, device/nlse_solver_dev.hpp:58-93). */
/* The boundary-plane transport of a collective handle.  NLS_PEER=1 at
 * nls_create asks for peer stores (k_p2d writes the neighbours' ghost planes through
 * IPC-mapped allocations) instead of the RCCL send/recv exchange; the mappings are made
 * at the first step, and if any rank cannot open one, every rank falls back to the
 * exchange (agreed by an all-reduce, so the ranks' transport sequences stay identical).
 * No reference counterpart (the reference runs independent single-GPU solvers,
 * device/nlse_driver_omp.cpp:103-121). */
enum nls_peer_state_e {
  NLS_PEER_OFF = 0,        /* exchange path (not asked for, or not available on this handle) */
  NLS_PEER_ACTIVE = 1,     /* peer stores in use */
  NLS_PEER_FELL_BACK = 2,  /* asked for; an IPC open failed on some rank: exchange path */
  NLS_PEER_PENDING = 3     /* asked for; set up at the first step */
};
int nls_peer_state(const nls_handle *h, int32_t *state);

#define NLS_PLACE_MAX 8
int nls_placement(const nls_handle *h, int32_t *n, int32_t *chosen, float *ms, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* NLS_AMD_H */
