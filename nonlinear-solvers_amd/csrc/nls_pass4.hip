// nls_pass4.hip -- the first basis pass with FOUR new vectors (k_p4d0): from the start
// vector S_0 alone it writes V_1..V_4 (V_1 = (L - sigma) W_0, V_{i+1} = (L - sigma) V_i as
// combinations of S_0, L S_0, .., L^4 S_0; coefficients from k_p2coef, P2State aX, aZ, aY,
// aW and bX1, bZ1..2, bY1..3, bW1..4) and reduces S_0^H V_i, the Gram V_a^H V_b (a <= b)
// and ||S_0||^2 (the blind start) -- the columns k_p2coef takes for ns = 4 at J = 0.
// Replaces the J = 0 and J = 2 two-vector passes: the schedule continues with two-vector
// passes from J = 4, so a step moves 60 instead of 63 vector transfers at m = 16
// (tests/sstep_model.py sched, tests/test_sstep_model.py: the same Krylov action within
// 1e-12 at the headline stiffness).  The Lanczos recurrence is the reference's
// (eigen_krylov_complex.hpp:21-38, device/lanczos_complex.hpp:413-500) in s-step form.
//
// 3D isotropic operator (laplacians.hpp:55-105), single-rank handles, nx % 64 == 0,
// ny % 4 == 0, ny >= 8 (the host checks).  Workgroup = 4 waves = a tile of 64 x-cells x 4
// rows, marched over the tile's planes.  Per march step the tile takes S_0 plane p (rows
// y0-4..y0+7, cells x0-4..x0+67: the radius-4 neighbourhood, rows outside [0, ny) wrapped
// into the adjacent planes exactly as the flat-index y-neighbour of the reference does,
// cells outside the grid zero) and computes one plane of each stencil level on a shrinking
// region: L S_0 at plane p-1 (rows/cells of radius 3), L^2 S_0 at p-2 (radius 2), L^3 S_0
// at p-3 (radius 1), L^4 S_0 at p-4 on the tile; every level lives in a 3-plane LDS ring
// (120 KiB), level values outside the grid are zero, so each stencil is the plain
// 7-point form with the reference's diagonal.  S_0 is loaded LA planes ahead into registers
// (compiler-tracked loads; no hand-counted vmcnt), the outputs of plane p-4 are stored
// non-temporally.  Barriers: one after each of the four phases per step.
// k_p4r (below, NLS_P4_KIND = 2, the default) computes the same vectors and sums with 64 x 8
// tiles, register z-queues and one barrier per step.
#include "nls_reduce.hpp"
#include "nls_kernels.hpp"
#define NLS_NO_P2_KERNELS
#include "nls_pass2.hpp"

namespace nls {

#ifndef NLS_P4_NT
#define NLS_P4_NT 512  // threads per workgroup: 4 output waves (+ 4 waves that take halo positions)
#endif
#ifndef NLS_P4_LA
#define NLS_P4_LA 2  // planes of S_0 loaded ahead (registers)
#endif

namespace p4 {
constexpr int R = 4;          // stencil radius of the pass (four levels)
constexpr int TR = 4;         // output rows per tile (one per wave)
constexpr int XW = 64;        // output cells per row (one per lane)
constexpr int EH = TR + 2 * R;  // 12 staged rows
constexpr int EW = XW + 2 * R;  // 72 staged cells per row
// level l (0 = S_0) covers rows [l, EH - l) and cells [l, EW - l) of the staged grid
__host__ __device__ constexpr int lw(int l) { return EW - 2 * l; }
__host__ __device__ constexpr int lh(int l) { return EH - 2 * l; }
__host__ __device__ constexpr int lsz(int l) { return lw(l) * lh(l); }
constexpr int OFF1 = 3 * lsz(0), OFF2 = OFF1 + 3 * lsz(1), OFF3 = OFF2 + 3 * lsz(2);
constexpr int LDS_CPLX = OFF3 + 3 * lsz(3);  // 7512 cplx = 120,192 B
constexpr int NC = 4 + 10 + 1;                 // S-dots, Gram (a <= b), ||S_0||^2
// halo positions of level l (its region minus the tile's own 4 x 64 block)
__host__ __device__ constexpr int nhalo(int l) { return (R - l) * (2 * lw(l) + 2 * TR); }
static_assert(nhalo(1) == 444 && nhalo(2) == 288 && nhalo(3) == 140, "halo counts");
}  // namespace p4

// (free functions with value arguments: lambdas capturing the kernel's locals by reference
// kept the closure on the stack -- scratch accesses in the march loop)
struct P4C {
  int nx, ny, nz, x0, y0;
  double s, sdi, sdb;
};
struct P4Cell {
  int row, pl, x;
};
// the grid cell of staged (er, ec) at march plane q: row and plane after the flat-index
// y-wrap (rows outside [0, ny) belong to the adjacent planes), x
__device__ __forceinline__ P4Cell p4_cell(const P4C c, int er, int ec, int q) {
  const int yy = c.y0 - p4::R + er;
  P4Cell r;
  r.pl = q + (yy < 0 ? -1 : (yy >= c.ny ? 1 : 0));
  r.row = yy < 0 ? yy + c.ny : (yy >= c.ny ? yy - c.ny : yy);
  r.x = c.x0 - p4::R + ec;
  return r;
}
// a stencil position of level l, resolved once per tile (the plane-independent parts):
// source index in level l-1's buffer, destination index in level l's, the plane shift of
// the y-wrap, x inside the grid, x or row on the grid boundary
struct P4Pt {
  int src, dst, dpl;
  bool xin, bfix;
};
__device__ __forceinline__ P4Pt p4_pt(const P4C c, int l, int er, int ec) {
  P4Pt r;
  r.src = (er - (l - 1)) * p4::lw(l - 1) + (ec - (l - 1));
  r.dst = (er - l) * p4::lw(l) + (ec - l);
  const P4Cell e = p4_cell(c, er, ec, 0);
  r.dpl = e.pl;
  r.xin = e.x >= 0 && e.x < c.nx;
  r.bfix = e.x == 0 || e.x == c.nx - 1 || e.row == 0 || e.row == c.ny - 1;
  return r;
}
// the stencil at a resolved position, plane q: the reference's 7-point row
// (laplacians.hpp:69-102) from level l-1's ring slots (planes q-1, q, q+1), zero outside the grid
template <int WS>
__device__ __forceinline__ cplx p4_lapt(const P4C c, const cplx *sm, const cplx *sc, const cplx *sp, const P4Pt e,
                                        int q) {
  const int i = e.src;
  const cplx v0 = sc[i], xm = sc[i - 1], xp = sc[i + 1], ym = sc[i - WS], yp = sc[i + WS];
  const cplx zm = sm[i], zp = sp[i];
  const int pl = q + e.dpl;
  const bool in = e.xin && pl >= 0 && pl < c.nz;
  const bool bnd = e.bfix || pl == 0 || pl == c.nz - 1;
  const cplx v = (bnd ? c.sdb : c.sdi) * v0 + c.s * (((zm + zp) + (xm + xp)) + (ym + yp));
  return in ? v : cplx{0.0, 0.0};
}
struct P4Pos {
  int er, ec;
};
// the staged (er, ec) of halo position h of level l: rows above the tile, rows below, then
// the side cells of the tile's own rows
__device__ __forceinline__ P4Pos p4_halo(int l, int h) {
  using namespace p4;
  const int d = R - l, wl = lw(l);
  P4Pos r;
  if (h < d * wl) {
    r.er = l + h / wl;
    r.ec = l + h % wl;
  } else if (h < 2 * d * wl) {
    const int h2 = h - d * wl;
    r.er = R + TR + h2 / wl;
    r.ec = l + h2 % wl;
  } else {
    const int h2 = h - 2 * d * wl;
    r.er = R + h2 / (2 * d);
    const int cc = h2 % (2 * d);
    r.ec = cc < d ? l + cc : R + XW + (cc - d);
  }
  return r;
}
struct P4Ld {
  cplx m[3], h;
};
// S_0 loads of plane p: staged rows w, w+4, w+8 at cells x0..x0+63 (one aligned 1 KiB row
// per wave-load; row w+4 is the thread's own cell; output waves only), on halo-load
// threads ht < 96 the x-halo cell (hr, hec) of row hr = ht/8
__device__ __forceinline__ P4Ld p4_load(const P4C c, const cplx *__restrict__ S0, int64_t P, bool mains, int w,
                                        int lane, int ht, int hr, int hec, int p) {
  P4Ld r;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const P4Cell e = p4_cell(c, w + 4 * j, p4::R + lane, p);
    const bool ok = mains && e.pl >= 0 && e.pl < c.nz;
    r.m[j] = ok ? ld_nt(S0 + (int64_t)e.pl * P + (int64_t)e.row * c.nx + e.x) : cplx{0.0, 0.0};
  }
  r.h = {0.0, 0.0};
  if (ht < p4::EH * 2 * p4::R) {
    const P4Cell e = p4_cell(c, hr, hec, p);
    if (e.pl >= 0 && e.pl < c.nz && e.x >= 0 && e.x < c.nx) r.h = S0[(int64_t)e.pl * P + (int64_t)e.row * c.nx + e.x];
  }
  return r;
}

// NT = 256: the four output waves do every position; NT = 512: four more waves take the halo
// positions of each level (at most two stencils per thread and level)
template <int NT>
__global__ __launch_bounds__(NT, 1) void k_p4d0(cplx *__restrict__ W, int64_t vs, Geo g,
                                                      const P2State *__restrict__ ps,
                                                      cplx *__restrict__ part, int nb) {
  using namespace p4;
  __shared__ __attribute__((aligned(16))) cplx smem[LDS_CPLX];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const bool outw = t < NTHREADS;         // the tile's output waves (uniform per wave)
  const int h0 = (t + NTHREADS) % NT;    // first halo position of this thread
  const int nx = (int)g.nx, ny = (int)g.nyp, nz = (int)g.npl;
  const int64_t P = g.P;
  const int ntx = nx / XW, nty = ny / TR;
  const int b = blockIdx.x;
  const int xt = b % ntx, yt = (b / ntx) % nty, zc = b / (ntx * nty);
  const int x0 = xt * XW, y0 = yt * TR;
  const int k0 = g.qa + zc * g.kz, k1 = min(k0 + g.kz, g.qb);
  const double s = g.s, sdi = g.sd_in, sdb = g.sd_bd;
  // coefficients: V_i = a_i S_0 + sum_{q <= i} b_i[q] L^q S_0
  const cplx a1 = ps->aX[0], a2 = ps->aZ[0], a3 = ps->aY[0], a4 = ps->aW[0];
  const cplx b11 = ps->bX1, b21 = ps->bZ1, b22 = ps->bZ2, b31 = ps->bY1, b32 = ps->bY2, b33 = ps->bY3;
  const cplx b41 = ps->bW[0], b42 = ps->bW[1], b43 = ps->bW[2], b44 = ps->bW[3];

  const P4C cx{nx, ny, nz, x0, y0, s, sdi, sdb};
  const cplx *__restrict__ S0 = W;
  const int ht = h0;  // halo-load index: the helper waves' threads first when NT = 512
  const int hr = ht >> 3, hcn = ht & 7, hec = hcn < R ? hcn : XW + hcn;
  cplx acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = {0.0, 0.0};
  constexpr int LA = NLS_P4_LA;
  P4Ld la[LA];
#pragma unroll
  for (int d = 0; d < LA; ++d) la[d] = p4_load(cx, S0, P, outw, w & 3, lane, ht, hr, hec, k0 - R + d);
  // own-cell queues: S_0 at planes p-4..p, L S_0 at p-4..p-1
  cplx sown[5], l1own[4];
#pragma unroll
  for (int d = 0; d < 5; ++d) sown[d] = {0.0, 0.0};
#pragma unroll
  for (int d = 0; d < 4; ++d) l1own[d] = {0.0, 0.0};
  // ring slot of plane q is (q - base) mod 3 with base = k0 - 8 (the lowest plane any phase
  // names: the first step's L^3 source plane)
  const int base = k0 - 2 * R;
  cplx *const rS = smem, *const r1 = smem + OFF1, *const r2 = smem + OFF2, *const r3 = smem + OFF3;
#define P4_SLOT(q) (((q) - base) % 3)
  const int orow = R + w, ocol = R + lane;  // the own cell in the staged grid
  const int ox = x0 + lane, oy = y0 + w;
  // resolved positions: the own cell at each level, this thread's halo position of levels
  // 1..3 (NT = 512: at most one per level)
  static_assert(NT == 512 || NT == 256, "workgroup size");
  constexpr int NH1 = (nhalo(1) + NT - 1) / NT, NH2 = (nhalo(2) + NT - 1) / NT, NH3 = (nhalo(3) + NT - 1) / NT;
  P4Pt po[4], ph1[NH1], ph2[NH2], ph3[NH3];
#pragma unroll
  for (int l = 1; l <= 4; ++l) po[l - 1] = p4_pt(cx, l, orow, ocol);
#pragma unroll
  for (int u = 0; u < NH1; ++u) {
    const int h = h0 + u * NT;
    const P4Pos e = p4_halo(1, h < nhalo(1) ? h : 0);
    ph1[u] = p4_pt(cx, 1, e.er, e.ec);
  }
#pragma unroll
  for (int u = 0; u < NH2; ++u) {
    const int h = h0 + u * NT;
    const P4Pos e = p4_halo(2, h < nhalo(2) ? h : 0);
    ph2[u] = p4_pt(cx, 2, e.er, e.ec);
  }
#pragma unroll
  for (int u = 0; u < NH3; ++u) {
    const int h = h0 + u * NT;
    const P4Pos e = p4_halo(3, h < nhalo(3) ? h : 0);
    ph3[u] = p4_pt(cx, 3, e.er, e.ec);
  }

  for (int p = k0 - R; p < k1 + R; ++p) {
    // 1. S_0 plane p into its ring slot; the load of plane p + LA
    const P4Ld cur = la[0];
#pragma unroll
    for (int d = 0; d + 1 < LA; ++d) la[d] = la[d + 1];
    if (p + LA < k1 + R) la[LA - 1] = p4_load(cx, S0, P, outw, w & 3, lane, ht, hr, hec, p + LA);  // (uniform)
    {
      cplx *dS = rS + P4_SLOT(p) * lsz(0);
      if (outw) {
#pragma unroll
        for (int j = 0; j < 3; ++j) dS[(w + 4 * j) * EW + R + lane] = cur.m[j];
      }
      if (ht < EH * 2 * R) dS[hr * EW + hec] = cur.h;
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) sown[d] = sown[d + 1];
    sown[4] = cur.m[1];
    __syncthreads();
    // 2. L S_0 at plane p-1
    {
      const int q = p - 1;
      const cplx *sm = rS + P4_SLOT(q - 1) * lsz(0), *sc = rS + P4_SLOT(q) * lsz(0), *sp = rS + P4_SLOT(q + 1) * lsz(0);
      cplx *d1 = r1 + P4_SLOT(q) * lsz(1);
      if (outw) {
        const cplx own = p4_lapt<lw(0)>(cx, sm, sc, sp, po[0], q);
        d1[po[0].dst] = own;
#pragma unroll
        for (int d = 0; d < 3; ++d) l1own[d] = l1own[d + 1];
        l1own[3] = own;
      }
#pragma unroll
      for (int u = 0; u < NH1; ++u)
        if (h0 + u * NT < nhalo(1)) d1[ph1[u].dst] = p4_lapt<lw(0)>(cx, sm, sc, sp, ph1[u], q);
    }
    __syncthreads();
    // 3. L^2 S_0 at plane p-2
    {
      const int q = p - 2;
      const cplx *sm = r1 + P4_SLOT(q - 1) * lsz(1), *sc = r1 + P4_SLOT(q) * lsz(1), *sp = r1 + P4_SLOT(q + 1) * lsz(1);
      cplx *d2 = r2 + P4_SLOT(q) * lsz(2);
      if (outw) d2[po[1].dst] = p4_lapt<lw(1)>(cx, sm, sc, sp, po[1], q);
#pragma unroll
      for (int u = 0; u < NH2; ++u)
        if (h0 + u * NT < nhalo(2)) d2[ph2[u].dst] = p4_lapt<lw(1)>(cx, sm, sc, sp, ph2[u], q);
    }
    __syncthreads();
    // 4. L^3 S_0 at plane p-3
    {
      const int q = p - 3;
      const cplx *sm = r2 + P4_SLOT(q - 1) * lsz(2), *sc = r2 + P4_SLOT(q) * lsz(2), *sp = r2 + P4_SLOT(q + 1) * lsz(2);
      cplx *d3 = r3 + P4_SLOT(q) * lsz(3);
      if (outw) d3[po[2].dst] = p4_lapt<lw(2)>(cx, sm, sc, sp, po[2], q);
#pragma unroll
      for (int u = 0; u < NH3; ++u)
        if (h0 + u * NT < nhalo(3)) d3[ph3[u].dst] = p4_lapt<lw(2)>(cx, sm, sc, sp, ph3[u], q);
    }
    __syncthreads();
    // 5. the outputs of plane k = p-4: L^4 S_0 on the tile, V_1..V_4, their sums
    const int k = p - R;
    if (k >= k0 && outw) {  // uniform
      const cplx *sm = r3 + P4_SLOT(k - 1) * lsz(3), *sc = r3 + P4_SLOT(k) * lsz(3), *sp = r3 + P4_SLOT(k + 1) * lsz(3);
      const cplx L4 = p4_lapt<lw(3)>(cx, sm, sc, sp, po[3], k);
      const cplx L3 = sc[po[2].dst];
      const cplx L2 = r2[P4_SLOT(k) * lsz(2) + po[1].dst];
      const cplx L1 = l1own[0], S = sown[0];
      const cplx V1 = cmul(a1, S) + cmul(b11, L1);
      const cplx V2 = (cmul(a2, S) + cmul(b21, L1)) + cmul(b22, L2);
      const cplx V3 = (cmul(a3, S) + cmul(b31, L1)) + (cmul(b32, L2) + cmul(b33, L3));
      const cplx V4 = ((cmul(a4, S) + cmul(b41, L1)) + (cmul(b42, L2) + cmul(b43, L3))) + cmul(b44, L4);
      const int64_t o = (int64_t)k * P + (int64_t)oy * nx + ox;
      st_nt(W + vs + o, V1);
      st_nt(W + 2 * vs + o, V2);
      st_nt(W + 3 * vs + o, V3);
      st_nt(W + 4 * vs + o, V4);
      const cplx V[4] = {V1, V2, V3, V4};
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] += cj_mul(S, V[i]);
      int c = 4;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        acc[c].re += abs2(V[a]);
        ++c;
#pragma unroll
        for (int bb = a + 1; bb < 4; ++bb) acc[c++] += cj_mul(V[a], V[bb]);
      }
      acc[NC - 1].re += abs2(S);
    }
  }
  // partial sums per workgroup (the staged rings are free after this barrier)
  __syncthreads();
  cplx *red = smem;  // [4][NC]
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const double a = wave_sum(acc[c].re), bb = wave_sum(acc[c].im);
    if (lane == 0 && outw) red[w * NC + c] = {a, bb};
  }
  __syncthreads();
  for (int c = t; c < NC; c += NT) {
    cplx v = red[c];
#pragma unroll
    for (int q = 1; q < TR; ++q) v += red[q * NC + c];
    part[(int64_t)c * nb + blockIdx.x] = v;
  }
}

// ---- k_p4r: the same pass with each staged column's z-neighbours in registers ----------
// Workgroup = 8 waves = a tile of 64 x-cells x 8 rows; staged grid 16 rows x 72 cells (the
// radius-4 neighbourhood).  Wave w OWNS staged rows w and w + 8 at cells x0..x0+63 (lane =
// x) for every level, and waves 0 and 7 own the 128 x-halo cells (4 each side of every
// staged row).  The owner of a staged column computes all its levels, so the stencil's z
// neighbours (the column's previous-level values at planes q-1, q, q+1) are register queues
// and only the x / y neighbours come from LDS.  Level l is computed at plane p - l in march
// step p from level l-1's plane p - l, which step p - 1 wrote into the other half of a
// ping-pong LDS pair: every read of a step names the previous step's half, every write the
// current one, so ONE barrier per step orders both (k_p4d0: four).  Each wave owns exactly
// one output row (rows 4..11), whose queues keep S_0 .. L^3 S_0 of plane p - 4 for the
// combination.  5.8 stencil evaluations per output cell (k_p4d0: 7.4), 4 LDS reads each
// (k_p4d0: 7); LDS 2 x 4 levels x 16 x 72 cplx = 144 KiB (one workgroup per CU).
namespace p4r {
constexpr int R = 4, TR = 8, XW = 64;
constexpr int EH = TR + 2 * R, EW = XW + 2 * R, LV = EH * EW;  // 16 x 72 staged cells
constexpr int NT = 512, NW = NT / 64;
constexpr int NC = 15;
static_assert(2 * NW == EH, "two staged rows per wave");
static_assert(2 * 4 * LV * 16 <= 160 * 1024, "LDS");
__host__ __device__ constexpr bool mem(int l, int r) { return l <= r && r < EH - l; }
}  // namespace p4r

// an owned staged cell: LDS index, plane shift of the y-wrap, offset of plane 0's cell,
// x inside the grid, on the x / row boundary (the reference's -5 diagonal)
struct P4RPos {
  int i, dpl;
  int64_t off;
  bool xin, bfix;
};
__device__ __forceinline__ P4RPos p4r_pos(const P4C c, int er, int ec) {
  const P4Cell e = p4_cell(c, er, ec, 0);
  P4RPos r;
  r.i = er * p4r::EW + ec;
  r.dpl = e.pl;
  r.off = (int64_t)e.row * c.nx + e.x;
  r.xin = e.x >= 0 && e.x < c.nx;
  r.bfix = e.x == 0 || e.x == c.nx - 1 || e.row == 0 || e.row == c.ny - 1;
  return r;
}
__device__ __forceinline__ cplx p4r_load(const P4C c, const cplx *__restrict__ S0, int64_t P, const P4RPos e, int p) {
  const int pl = p + e.dpl;
  return e.xin && pl >= 0 && pl < c.nz ? S0[(int64_t)pl * P + e.off] : cplx{0.0, 0.0};
}
// the 7-point row (laplacians.hpp:69-102) at an owned cell, plane q: z neighbours and centre
// from the owner's queue, x / y neighbours from level l-1's LDS plane q; zero outside the grid.
// MODE 0: any plane; 1: a plane neither outside the grid nor on its z boundary and a cell
// inside the grid in x (the owned rows' cells: x0..x0+63) -- the same value without the
// checks; 2: such a plane with the x check (the x-halo cells)
template <int MODE>
__device__ __forceinline__ cplx p4r_lap(const P4C c, const cplx *prv, const P4RPos e, cplx zp, cplx cc, cplx zm,
                                        int q) {
  const int i = e.i;
  const cplx xm = prv[i - 1], xp = prv[i + 1], ym = prv[i - p4r::EW], yp = prv[i + p4r::EW];
  if constexpr (MODE == 0) {
    const int pl = q + e.dpl;
    const bool in = e.xin && pl >= 0 && pl < c.nz;
    const bool bnd = e.bfix || pl == 0 || pl == c.nz - 1;
    const cplx v = (bnd ? c.sdb : c.sdi) * cc + c.s * (((zm + zp) + (xm + xp)) + (ym + yp));
    return in ? v : cplx{0.0, 0.0};
  } else {
    const cplx v = (e.bfix ? c.sdb : c.sdi) * cc + c.s * (((zm + zp) + (xm + xp)) + (ym + yp));
    if constexpr (MODE == 2) return e.xin ? v : cplx{0.0, 0.0};
    return v;
  }
}
template <int D>
__device__ __forceinline__ void p4r_push(cplx (&q)[D], cplx v) {
#pragma unroll
  for (int d = D - 1; d > 0; --d) q[d] = q[d - 1];
  q[0] = v;
}

#ifndef NLS_P4R_HFAST
#define NLS_P4R_HFAST 1  // 0: the x-halo cells take the checked stencil on every step (A/B only)
#endif
#ifndef NLS_P4R_FAST
#define NLS_P4R_FAST 1  // 0: every step takes the checked stencil (A/B only)
#endif
// one march step; FM / FH: p4r_lap's MODE for the owned rows / the x-halo cells
#define P4R_BODY(FM, FH)                                                                                  \
  do {                                                                                                    \
    const int par = (p - k0) & 1;                                                                         \
    cplx *const cur = lds + par * 4 * LV;                                                                 \
    const cplx *const prv = lds + (par ^ 1) * 4 * LV;                                                     \
    const cplx sO = laO, sN = laN, sH = laH;                                                              \
    if (p + 1 < k1 + R) {  /* uniform */                                                                  \
      laO = p4r_load(cx, S0, P, eO, p + 1);                                                               \
      laN = p4r_load(cx, S0, P, eN, p + 1);                                                               \
      if (hon) laH = p4r_load(cx, S0, P, eH, p + 1);                                                      \
    }                                                                                                     \
    /* level 0: S_0 at plane p */                                                                         \
    p4r_push(o0, sO);                                                                                     \
    cur[eO.i] = sO;                                                                                       \
    p4r_push(n0, sN);                                                                                     \
    cur[eN.i] = sN;                                                                                       \
    if (hon) {                                                                                            \
      p4r_push(h0, sH);                                                                                   \
      cur[eH.i] = sH;                                                                                     \
    }                                                                                                     \
    /* level 1 at plane p - 1 */                                                                          \
    {                                                                                                     \
      const int q = p - 1;                                                                                \
      const cplx *pv = prv;                                                                               \
      cplx *cv = cur + LV;                                                                                \
      const cplx v = p4r_lap<FM>(cx, pv, eO, o0[0], o0[1], o0[2], q);                                     \
      p4r_push(o1, v);                                                                                    \
      cv[eO.i] = v;                                                                                       \
      cplx vn = z;                                                                                        \
      if (mem(1, rN)) {                                                                                   \
        vn = p4r_lap<FM>(cx, pv, eN, n0[0], n0[1], n0[2], q);                                             \
        cv[eN.i] = vn;                                                                                    \
      }                                                                                                   \
      p4r_push(n1, vn);                                                                                   \
      if (hon) {                                                                                          \
        cplx vh = z;                                                                                      \
        if (hm[1]) {                                                                                      \
          vh = p4r_lap<FH>(cx, pv, eH, h0[0], h0[1], h0[2], q);                                           \
          cv[eH.i] = vh;                                                                                  \
        }                                                                                                 \
        p4r_push(h1, vh);                                                                                 \
      }                                                                                                   \
    }                                                                                                     \
    /* level 2 at plane p - 2 */                                                                          \
    {                                                                                                     \
      const int q = p - 2;                                                                                \
      const cplx *pv = prv + LV;                                                                          \
      cplx *cv = cur + 2 * LV;                                                                            \
      const cplx v = p4r_lap<FM>(cx, pv, eO, o1[0], o1[1], o1[2], q);                                     \
      p4r_push(o2, v);                                                                                    \
      cv[eO.i] = v;                                                                                       \
      cplx vn = z;                                                                                        \
      if (mem(2, rN)) {                                                                                   \
        vn = p4r_lap<FM>(cx, pv, eN, n1[0], n1[1], n1[2], q);                                             \
        cv[eN.i] = vn;                                                                                    \
      }                                                                                                   \
      p4r_push(n2, vn);                                                                                   \
      if (hon) {                                                                                          \
        cplx vh = z;                                                                                      \
        if (hm[2]) {                                                                                      \
          vh = p4r_lap<FH>(cx, pv, eH, h1[0], h1[1], h1[2], q);                                           \
          cv[eH.i] = vh;                                                                                  \
        }                                                                                                 \
        p4r_push(h2, vh);                                                                                 \
      }                                                                                                   \
    }                                                                                                     \
    /* level 3 at plane p - 3 (only the output row keeps it: its level 4 needs the z pair) */             \
    {                                                                                                     \
      const int q = p - 3;                                                                                \
      const cplx *pv = prv + 2 * LV;                                                                      \
      cplx *cv = cur + 3 * LV;                                                                            \
      const cplx v = p4r_lap<FM>(cx, pv, eO, o2[0], o2[1], o2[2], q);                                     \
      p4r_push(o3, v);                                                                                    \
      cv[eO.i] = v;                                                                                       \
      if (mem(3, rN)) cv[eN.i] = p4r_lap<FM>(cx, pv, eN, n2[0], n2[1], n2[2], q);                         \
      if (hm[3]) cv[eH.i] = p4r_lap<FH>(cx, pv, eH, h2[0], h2[1], h2[2], q);                              \
    }                                                                                                     \
    /* level 4 and the outputs at plane k = p - 4 */                                                      \
    const int k = p - R;                                                                                  \
    if (k >= k0) {  /* uniform */                                                                         \
      const cplx L4 = p4r_lap<FM>(cx, prv + 3 * LV, eO, o3[0], o3[1], o3[2], k);                          \
      const cplx S = o0[4], L1 = o1[3], L2 = o2[2], L3 = o3[1];                                           \
      const cplx V1 = cmul(a1, S) + cmul(b11, L1);                                                        \
      const cplx V2 = (cmul(a2, S) + cmul(b21, L1)) + cmul(b22, L2);                                      \
      const cplx V3 = (cmul(a3, S) + cmul(b31, L1)) + (cmul(b32, L2) + cmul(b33, L3));                    \
      const cplx V4 = ((cmul(a4, S) + cmul(b41, L1)) + (cmul(b42, L2) + cmul(b43, L3))) + cmul(b44, L4);  \
      const int64_t o = (int64_t)k * P + eO.off;                                                          \
      st_nt(W + vs + o, V1);                                                                              \
      st_nt(W + 2 * vs + o, V2);                                                                          \
      st_nt(W + 3 * vs + o, V3);                                                                          \
      st_nt(W + 4 * vs + o, V4);                                                                          \
      const cplx V[4] = {V1, V2, V3, V4};                                                                 \
_Pragma("unroll")                                                                                         \
      for (int i = 0; i < 4; ++i) acc[i] += cj_mul(S, V[i]);                                              \
      int c = 4;                                                                                          \
_Pragma("unroll")                                                                                         \
      for (int a = 0; a < 4; ++a) {                                                                       \
        acc[c].re += abs2(V[a]);                                                                          \
        ++c;                                                                                              \
_Pragma("unroll")                                                                                         \
        for (int bb = a + 1; bb < 4; ++bb) acc[c++] += cj_mul(V[a], V[bb]);                               \
      }                                                                                                   \
      acc[NC - 1].re += abs2(S);                                                                          \
    }                                                                                                     \
    __syncthreads();                                                                                      \
  } while (0)

// OUTB: the wave's output row is its second row (waves 0..3) or its first (4..7)
template <bool OUTB>
__device__ __forceinline__ void p4r_march(cplx *lds, cplx *__restrict__ W, int64_t vs, const P4C cx, int64_t P,
                                          int k0, int k1, const P2State *__restrict__ ps, cplx (&acc)[p4r::NC],
                                          int w, int lane) {
  using namespace p4r;
  const int rO = OUTB ? w + NW : w, rN = OUTB ? w : w + NW;  // output row, the other row
  const P4RPos eO = p4r_pos(cx, rO, R + lane), eN = p4r_pos(cx, rN, R + lane);
  const bool hon = w == 0 || w == NW - 1;  // x-halo owners (uniform)
  const int hidx = (w == 0 ? 0 : 64) + lane, rH = hidx >> 3, cH = hidx & 7, ecH = cH < R ? cH : XW + cH;
  const P4RPos eH = p4r_pos(cx, rH, ecH);
  bool hm[4];
  hm[0] = hon;
#pragma unroll
  for (int l = 1; l < 4; ++l) hm[l] = hon && mem(l, rH) && l <= ecH && ecH < EW - l;
  const cplx *__restrict__ S0 = W;
  const cplx a1 = ps->aX[0], a2 = ps->aZ[0], a3 = ps->aY[0], a4 = ps->aW[0];
  const cplx b11 = ps->bX1, b21 = ps->bZ1, b22 = ps->bZ2, b31 = ps->bY1, b32 = ps->bY2, b33 = ps->bY3;
  const cplx b41 = ps->bW[0], b42 = ps->bW[1], b43 = ps->bW[2], b44 = ps->bW[3];
  const cplx z{0.0, 0.0};
  // queues, index 0 = newest: output row S_0 at p..p-4, L at p-1..p-4, L^2 at p-2..p-4,
  // L^3 at p-3..p-5; the other row and the x-halo cells the three planes their next level needs
  cplx o0[5], o1[4], o2[3], o3[3], n0[3], n1[3], n2[3], h0[3], h1[3], h2[3];
#pragma unroll
  for (int d = 0; d < 5; ++d) o0[d] = z;
#pragma unroll
  for (int d = 0; d < 4; ++d) o1[d] = z;
#pragma unroll
  for (int d = 0; d < 3; ++d) o2[d] = o3[d] = n0[d] = n1[d] = n2[d] = h0[d] = h1[d] = h2[d] = z;
  cplx laO = p4r_load(cx, S0, P, eO, k0 - R), laN = p4r_load(cx, S0, P, eN, k0 - R);
  cplx laH = hon ? p4r_load(cx, S0, P, eH, k0 - R) : z;
  // the steps whose planes (p - 5 .. p) all lie inside the grid and off its z boundary form
  // one contiguous range [pf0, pf1): their own loop takes the check-free stencil
  const int pe = k1 + R, pf0 = min(max(k0 - R, 6), pe), pf1 = NLS_P4R_FAST ? max(min(pe, cx.nz - 1), pf0) : pf0;
  int p = k0 - R;
  for (; p < pf0; ++p) P4R_BODY(0, 0);
  for (; p < pf1; ++p) P4R_BODY(1, NLS_P4R_HFAST ? 2 : 0);
  for (; p < pe; ++p) P4R_BODY(0, 0);
}
#undef P4R_BODY


__global__ __launch_bounds__(p4r::NT, 1) void k_p4r(cplx *__restrict__ W, int64_t vs, Geo g,
                                                     const P2State *__restrict__ ps, cplx *__restrict__ part,
                                                     int nb) {
  using namespace p4r;
  __shared__ __attribute__((aligned(16))) cplx lds[2 * 4 * LV];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nx = (int)g.nx, ny = (int)g.nyp, nz = (int)g.npl;
  const int ntx = nx / XW, nty = ny / TR;
  const int b = blockIdx.x;
  const int xt = b % ntx, yt = (b / ntx) % nty, zc = b / (ntx * nty);
  const int k0 = g.qa + zc * g.kz, k1 = min(k0 + g.kz, g.qb);
  const P4C cx{nx, ny, nz, xt * XW, yt * TR, g.s, g.sd_in, g.sd_bd};
  cplx acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = {0.0, 0.0};
  if (w < NW / 2)  // uniform
    p4r_march<true>(lds, W, vs, cx, g.P, k0, k1, ps, acc, w, lane);
  else
    p4r_march<false>(lds, W, vs, cx, g.P, k0, k1, ps, acc, w, lane);
  // partial sums per workgroup (the march ended on a barrier: the LDS is free)
  cplx *red = lds;  // [NW][NC]
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const double a = wave_sum(acc[c].re), bb = wave_sum(acc[c].im);
    if (lane == 0) red[w * NC + c] = {a, bb};
  }
  __syncthreads();
  for (int c = t; c < NC; c += NT) {
    cplx v = red[c];
#pragma unroll
    for (int q = 1; q < NW; ++q) v += red[q * NC + c];
    part[(int64_t)c * nb + blockIdx.x] = v;
  }
}

#ifndef NLS_P4_KIND
#define NLS_P4_KIND 2  // 2: k_p4r (register z-queues, one barrier per step) where ny % 8 == 0; 1: k_p4d0
#endif
// k_p4r takes grids with ny % 8 == 0, k_p4d0 the others (ny % 4 == 0)
static bool pass4_r(int64_t ny) { return NLS_P4_KIND == 2 && ny % p4r::TR == 0; }
const void *kernel_pass4(int64_t ny) {
  return pass4_r(ny) ? reinterpret_cast<const void *>(&k_p4r) : reinterpret_cast<const void *>(&k_p4d0<NLS_P4_NT>);
}
int pass4_threads(int64_t ny) { return pass4_r(ny) ? p4r::NT : NLS_P4_NT; }
int pass4_tiles(int64_t nx, int64_t ny, int64_t planes, int kz) {
  return (int)((nx / p4::XW) * (ny / (pass4_r(ny) ? p4r::TR : p4::TR)) * ((planes + kz - 1) / kz));
}

}  // namespace nls
