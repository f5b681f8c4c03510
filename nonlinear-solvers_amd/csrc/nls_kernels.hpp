// nls_kernels.hpp -- host-visible handles of the kernels in nls_kernels.hip.
// Launched with hipLaunchKernel(fn, grid, block, args, 0, stream).
#pragma once
#include "nls_device.hpp"

namespace nls {

// stencil kernels (tiled march), argument lists:
//   update : (const S* W, S* out, int64_t vs, Geo g, const KState* st, cplx* part,
//             int part_stride, int part_off, S* E)   -- partials at part[k*stride + off + block];
//             E: x-seam edge buffer of the QA variant (unused otherwise)
//   alpha  : (const S* V, Geo g, cplx* part)
//   lap    : (const S* V, Geo g, S* out)
// ani = true: the G2 anisotropic operator (complex only; Geo::cf = c field)
const void *kernel_update(bool complex_, int dim, int J, bool ani, bool qa = false);
const void *kernel_alpha(bool complex_, int dim, bool ani);
const void *kernel_lap(bool complex_, int dim, bool ani);
int64_t stencil_tiles(const Geo &g, int dim, int rows_per_thread);
int update_rows_per_thread(int J, bool ani, bool qa = false);
int alpha_rows_per_thread();
int fused_rows_per_thread();
int alpha_l2_rows_per_thread();
int tq_words();  // int32 words of the tail's tile queue (Geo::tq): heads + done counter

// per-variant tables (nls_stencil.hip, one object per operator x dimension)
enum { NLS_KIND_UPDATE = 0, NLS_KIND_ALPHA = 1, NLS_KIND_LAP = 2, NLS_KIND_ALPHA_L2 = 3,
       NLS_KIND_FINAL = 4, NLS_KIND_REDUCE_QA = 5, NLS_KIND_XPAIRS = 6 };
//   xpairs : (const S* E, Geo g, int ntx, int tw, cplx* part) -- x-tile seam pairs of the
//            folded alpha (one partial column, grid = the QA update pass's grid)
const void *kernel_xpairs(bool complex_, int dim, bool ani);
// tiles of a QA update pass along x (3D: 64 wide; 2D: 64 * rows-per-thread wide)
int64_t xtiles(const Geo &g, int dim, int rows_per_thread);
//   alpha_l2 : (const S* V, Geo g, cplx* part)  -- 3 partial columns: a, ||V||^2, ||L V||^2
//   tail(mode, M): (TailArgs a, Geo g)   -- nls_stencil.hpp TailMode, 3 <= M <= 32;
//                  nullptr where the variant has no such tail (then the unfused path runs)
const void *kernel_alpha_l2(bool complex_, int dim, bool ani, bool pipe = false);
//   reduce_qa  : (KState*, const cplx* partU, int nbU, int j, int do_sum, const cplx* partX,
//                 int nbX, const S* W_j, Geo ga) -- single workgroup: the reduction after a
//                 folded-alpha pass, with the direct alpha of W_j as fallback (need_alpha)
const void *kernel_reduce_qa(bool complex_, int dim, bool ani);
const void *kernel_tail(bool complex_, int dim, int mode, int M, bool ani);
const void *stencil_table_iso2(int kind, bool complex_, int J);
const void *stencil_table_iso3(int kind, bool complex_, int J);
const void *stencil_table_ani2(int kind, bool complex_, int J);
const void *stencil_table_ani3(int kind, bool complex_, int J);

// single workgroup:
//   reduce_iter  : (KState*, const cplx* partA, int nbA, const cplx* partU, int nbU, int j,
//                   int do_sum, int do_coef, int ncA, int qa, const cplx* partX, int nbX)
//                                                       -- ncA = 3 after k_alpha_l2;
//                   qa = 1 (ncA = 0): alpha from the q column of the previous update pass
//   reduce_final : (KState*, const cplx* partU, int nbU, int m, int do_sum, int do_coef,
//                   int nf, int f0, int f1, double t_re, double t_im, int tail)
const void *kernel_reduce_iter();

//   sum_ranks    : (cplx* dst, const cplx* pub, int nranks, int parity, int n, int stride)
const void *kernel_sum_ranks();
const void *kernel_reduce_final();
//   colsum       : (const cplx* partA, int nbA, int ncA, const cplx* partU, int nbU, cplx* dst)
//                  grid = ncA + ncU columns; dst = KState::sums (the do_sum phase, parallel)
const void *kernel_colsum();
// two-vectors-per-pass Lanczos (nls_pass2.hpp, nls_pass2d.hpp; 3D isotropic complex, single rank)
//   pass2 : (cplx* W, int64_t vs, Geo g, const P2State*, cplx* part, int nb, const cplx* zbuf, int poff)
const void *kernel_pass2(int J, bool hz, bool d2 = false, bool pr = false, bool peer = false);  // hz: also Z (k_p2d)
const void *kernel_pass2_peer(int J, bool hz);  // 3D isotropic k_p2d with the peer-store epilogue (nls_pass2p.hip)
bool pass2_jreg(int J, int akind = 0);  // k_p2d<J> reads its J rows into registers (p2d_jreg; akind: 1 G2, 2 G2 pairs)
constexpr int P2D_WAVE_XO = 64, P2D_ROWS = 4, P2D_MAXJ = 14, P2D_MAXJ_A = 22, P2D_MAXJ_A2 = 14;  // == P2D_XO, P2D_TR, P2D_JMAX, P2D_JMAX_A, P2D_JMAX_A2
//   p2m    : (cplx* W, int64_t vs, Geo g, const P2State*, cplx* part, int nb, const cplx* lbuf, int poff)
//            -- the register two-vector pass (nls_pass2g.hpp; lbuf = y = L S_J at local planes
//            [-1, nzl], local plane 0 at lbuf + P, from k_lap); J even <= 28
const void *kernel_p2m(int dim, int J, bool hz, bool ani);
const void *kernel_pass2a(int J, bool hz, bool pr = false);  // k_p2d of the G2 operator div(c grad) (3D; pr: real cell pairs)
int p2m_rows_per_thread(int J);
//   p2tail: (P2State*, KState*, const cplx* sums, int m);  p2tfin: (const P2State*, KState*, int m, int nf)
const void *kernel_p2tail();
const void *kernel_p2tfin();
const void *kernel_colsum_p2coef();  // (partU, nbU, dst, cnt, then k_p2coef's arguments)
const void *kernel_tail_chain();  // (partA, nbA, dst, cnt, ps, st, m, nf, f0, f1, t_re, t_im)
const void *kernel_p2coef();
const void *kernel_pass4(int64_t ny);  // k_p4r / k_p4d0 (nls_pass4.hip): (W, vs, Geo, P2State*, part, nb)
int pass4_tiles(int64_t nx, int64_t ny, int64_t planes, int kz);
int pass4_threads(int64_t ny);  // (P2State*, KState*, int J, int mode, int ns, int nsn)
size_t p2state_bytes();
size_t p2state_sums_offset();
size_t p2state_peer_offset();  // P2State::pdn, then pup (2 x p2state_peer_slots() pointers)
int p2state_peer_slots();

// pointwise (grid-stride):
//   nl_init   : (const cplx* u, cplx* w0, const double* mf, int64_t n, double dt, int nonlin,
//                cplx s1, cplx s2)
//   final_nlse: (cplx* W, int64_t vs, int64_t n, const KState*, cplx* u, const double* mf,
//                double dt, int nonlin, cplx s1, cplx s2)
//   neumann_bc: (cplx* u, cplx* w0, const double* mf, Geo g, int w0_ready, double dt, int nonlin,
//                cplx s1, cplx s2)   -- boundary cells only (grid over neumann_bc_cells())
//   combine   : (const S* W, int64_t vs, int64_t n, const KState*, S* out)
//   sg_mid    : (const double* W, int64_t vs, int64_t n, const KState*, const double* mf,
//                double* up, double* g0, int gfun)   (gfun < 0: G1 m(-sin y); else -m F(y), GautschiForce)
//   sg_end    : (const double* W2, int64_t vs, int64_t n, const KState*, double* u, double* up,
//                double dt)
//   sg_velocity: (const double* u, const double* up, double* v, int64_t n, double dt)
const void *kernel_nl_init();
const void *kernel_final_nlse(int M);
const void *kernel_combine(bool complex_, int M);
const void *kernel_sg_mid(int M);
const void *kernel_sg_end(int M);
const void *kernel_sg_velocity();
const void *kernel_neumann_bc();
//   sewi_b    : (const cplx* u, const double* mf, cplx* w0, int64_t n)
//   combine_w0: (cplx* W, int64_t vs, int64_t n, const KState*)          -- W_0 <- sum fin_k W_k
//   sewi_end  : (const cplx* W, int64_t vs, int64_t n, const KState*, cplx* u, cplx* up,
//                const cplx* e, double dt)
const void *kernel_sewi_b();
//   kg_g      : (const double* u, const double* mf, double* g0, int64_t n)
//   kg_end    : (double* W, const double* W2, int64_t vs, int64_t n, const KState* st,
//                const KState* st2, double* up, double* v, double dt)
//   neumann_bc_r: (double* u, Geo g)
const void *kernel_kg_g();
const void *kernel_kg_end(int M);
const void *kernel_neumann_bc_r();
const void *kernel_combine_w0(int M);
const void *kernel_sewi_end(int M);
int64_t neumann_bc_cells(const Geo &g);

}  // namespace nls
