// nls_pass2d.hpp -- the two-vector basis pass with LDS-DMA staging (k_p2d), the
// form the two-vectors-per-pass Lanczos runs by default.  Scheme, coefficients
// and the per-cell formulas: nls_pass2.hpp (P2State, k_p2coef) and DESIGN.md §3.
//
// Why a new form: the pass holds 2(J+1)+3 complex accumulators per lane, so
// with the streamed S_l in VGPRs it runs at one wave per SIMD with too few
// bytes in flight (a register-march form streamed at ~55 % of the pattern's
// rate; measured in round 2 and removed).  Here every byte the pass reads moves HBM -> LDS by
// global_load_lds_dwordx4 (1 KiB per wave-instruction, no VGPR destination),
// issued ahead of its use, so the in-flight bytes no longer compete
// with the accumulators for registers:
//
//   workgroup = 4 waves = one tile of 64 x-cells x 4 rows (one row per wave),
//               marched over kz planes; one or two workgroups per CU (p2d_occ).
//   S ring:     S_J rows y0-2 .. y0+5 of DS+3 planes (shared by the 4 waves;
//               each wave DMAs 2 rows of each plane).  L S_J of the next plane
//               is computed from it for the wave's rows -1, 0, +1 and kept in a
//               register queue (3 planes), L^2 S_J of the current plane from
//               that queue (x neighbours by lane shuffles).
//   J ring:     the J other stored vectors S_0..S_{J-1} of the wave's row,
//               RS rows of 1 KiB per wave (private to the wave): RS/J planes,
//               as deep as the LDS left by the S ring allows (2.2 planes at
//               J = 14, up to 5).
//   lanes:      x = x0 + lane, x0 a multiple of 64: every streamed row is one
//               aligned 1 KiB (a 60-wide tile read 20 % more than it used:
//               9 lines per 1 KiB and the x halo, PMC-measured).  The S_J rows
//               add their 4 x-halo cells by a 4-byte DMA on 16 lanes; the two
//               L S_J values just outside the tile come from one extra pass.
//
// Completion is counted by hand (hipcc does not track LDS-DMA writes): every
// wave issues, per step, exactly one group of J + 2 DMAs (its 2 S rows of
// plane k+DS+2, the next J rows of its J ring) followed by STW (1 or 2)
// stores, so the ops issued after the last one a step needs are a known count
// N_i and s_waitcnt vmcnt(N_i) retires exactly that much; groups beyond the
// tile's planes DMA a zero row (zbuf, nx cells) instead, and
// stores from non-output lanes duplicate an output lane's store (same value,
// same address), so no instruction is ever skipped by an all-false branch.
// A raw s_barrier after the wait publishes the other waves' S rows.
#pragma once
#include "nls_pass2.hpp"

namespace nls {

constexpr int P2D_XO = 64;            // output x per wave (128-B aligned rows)
constexpr int P2D_TR = 4;             // rows per tile (one per wave)
constexpr int P2D_SR = P2D_TR + 4;    // S_J rows staged per plane (y0-2 .. y0+5)
constexpr int P2D_SRB = 1024 + 64;    // bytes per staged S_J row: x0..x0+63, then x0-2, x0-1, x0+64, x0+65
constexpr int P2D_LR = P2D_TR + 2;    // L S_J rows shared per plane (y0-1 .. y0+4)
constexpr int P2D_JMAX = 14;          // largest J of the isotropic passes (m <= 18)
constexpr int P2D_JMAX_A = 22;        // largest J of the anisotropic passes (G2: m = 25 -> J <= 22)
constexpr int P2D_JMAX_A2 = 14;       // largest J of the anisotropic cell-pair passes (Klein-Gordon, m <= 18)
constexpr int P2D_GHOST = 2;          // ghost planes per side of a stored vector (radius-2 march)
constexpr int P2D_LDS = 160 * 1024;   // LDS per CU
// A (the G2 operator div(c grad)): the c field staged beside S_J, same rows and
// planes: 8 rows of x0..x0+63 (512 B of f64 each), then the 8 rows' 4 halo cells
// (x0-2, x0-1, x0+64, x0+65; 32 B each)
constexpr int P2D_CRB = 512;
constexpr int P2D_CSB = P2D_SR * P2D_CRB + P2D_SR * 32;
// Anisotropic kinds (the A argument of the ring functions): 0 isotropic, 1 the G2
// operator on a complex field, 2 the G2 operator on a real field as pairs of cells
// (Klein-Gordon): c is then one f64 per cell, so a row of 64 pairs is 128 c values =
// the same 1 KiB + 4 halo pairs as an S_J row, and its c ring is staged exactly like
// the S ring (P2D_SRB per row; c of cell 2P + h at double index 2P + h of the row,
// halo pairs P = 64..67 as in S); 3 the isotropic 2D passes (planes of 4 rows, D2), which
// are kind 0 except where their register rows start (p2d_jreg).  p2d_kind maps 3 to 0 for
// every other rule.
__host__ __device__ constexpr int p2d_kind(int A) { return A == 3 ? 0 : A; }
__host__ __device__ constexpr int p2d_csb(int A) {
  return p2d_kind(A) == 2 ? P2D_SR * P2D_SRB : (p2d_kind(A) ? P2D_CSB : 0);
}
// Timing diagnostic only (wrong results; never a product build): the S ring takes its halo
// from the zero row instead of the grid -- bit 1 the x-halo cells, bit 2 the rows above and
// below the tile -- so a variant library shows what the stencil vector's halo costs a pass
// (profiles/r06/p2_halo_diag.txt)
#ifndef NLS_DIAG_P2HALO
#define NLS_DIAG_P2HALO 0
#endif
#ifndef NLS_P2D_OCC2_MAXJ
#define NLS_P2D_OCC2_MAXJ 6   // two workgroups per CU up to this J (J = 6: late J ring, 512^3 4.08 -> 3.64 ms; J = 8 no gain)
#endif
#ifndef NLS_P2A_OCC2_MAXJ
#define NLS_P2A_OCC2_MAXJ 4   // anisotropic passes: two workgroups per CU up to this J (J = 4: late J ring, 0.655 -> 0.416 ms at G2 256^3)
#endif
#ifndef NLS_P2A_EARLY
#define NLS_P2A_EARLY 1       // anisotropic passes at one workgroup per CU: early issue (J < 22)
#endif
#ifndef NLS_P2A_DS1
#define NLS_P2A_DS1 1         // anisotropic passes at one workgroup per CU, J > NLS_P2D_DS3_MAXJ: S look-ahead
#endif
#ifndef NLS_P2D_EARLY
#define NLS_P2D_EARLY 1  // one workgroup per CU: issue a step's DMAs before its wait (needs an extra S slot)
#endif
#ifndef NLS_P2D_NP_MAX
#define NLS_P2D_NP_MAX 5      // J-ring depth cap in planes
#endif
#ifndef NLS_P2D_PRE_LA
#define NLS_P2D_PRE_LA 1      // issue the look-ahead before the prologue's wait (p2d_dspre)
#endif
#ifndef NLS_P2D_EXT1
#define NLS_P2D_EXT1 1        // the tile's 8 x-halo L values computed by one wave (P2D_LROWS)
#endif
#ifndef NLS_P2D_WCACHE
#define NLS_P2D_WCACHE 1      // anisotropic passes: L^2's face weights from the L S_J of the step before
#endif
#ifndef NLS_P2D_VCOEF_MAXJ
#define NLS_P2D_VCOEF_MAXJ 8  // the march's uniform f64 operands in VGPRs up to this J
#endif
#ifndef NLS_P2D_JREG
#define NLS_P2D_JREG 1        // isotropic passes from J = NLS_P2D_JREG_MINJ: J rows in registers (p2d_jreg)
#endif
#ifndef NLS_P2D_JREG_MINJ
#define NLS_P2D_JREG_MINJ 2    // 3D
#endif
#ifndef NLS_P2D_JREG2D_MINJ
#define NLS_P2D_JREG2D_MINJ 8  // 2D (kind 3)
#endif
#ifndef NLS_P2D_JREG_MAXJ
#define NLS_P2D_JREG_MAXJ 10
#endif
// The isotropic passes at J = 2 .. 10 in 3D, J = 8, 10 in 2D read their J stored rows straight into registers
// (one non-temporal load per row at the top of each step, awaited by the compiler's own
// counted vmcnt before the first use) instead of through an LDS ring: without the J
// ring the rings take ~47 KiB, so two workgroups fit per CU and the second covers the
// first's barriers and waits, and short tiles (no J-ring prologue) stream from a
// compact address window (512^3, same box: J = 10 5.17 ms at kz 32 vs 5.36 at 256 and
// 5.22 through the ring).  From J = 2 (round 5, same box): 3D 512^3 J = 2 2.00 -> 1.93 ms,
// J = 4 2.78 -> 2.71, the step -0.1 ms; but SG 8192^2 +0.2 ms (2.7 %) and 2D 4096^2 and G2
// (A = 1) unchanged, so 2D keeps the ring below J = 8 (profiles/r05/p2ab_jreg24.txt,
// ab_jreg24.txt).  J = 12 with Z does not fit: all rows live across the step
// took 256 VGPRs and scratch; half of them loaded after the S issue (SGPR-walked
// addresses) fit but ran slower than the ring (6.16 vs 6.06 ms; round 4,
// profiles/r04/p2ab_512.txt).
#ifndef NLS_P2A_JREG_MINJ
#define NLS_P2A_JREG_MINJ 6  // the complex anisotropic passes (G2): register rows, two workgroups per CU
#endif
#ifndef NLS_P2A_JREG_MAXJ
#define NLS_P2A_JREG_MAXJ 8  // J = 10 with Z: 255 VGPRs and scratch
#endif
// The real cell-pair passes of the G2 operator (Klein-Gordon, A = 2) at two workgroups per
// CU up to J = NLS_P2A2_OCC2_MAXJ: their S and c rings (4 slots each) and the L ring fill
// exactly 80 KiB once the tile's x-halo L values stay in registers (no EXT1) and the
// coefficients of X and Z in registers (p2d_rcoef); the J rows then come straight into
// registers (no J ring: p2d_jreg).  At one workgroup per CU these passes were latency-
// bound (KG 256^3: J = 0 at 1.7 TB/s, 742 instructions per step at one wave per SIMD)
#ifndef NLS_P2A2_OCC2_MAXJ
#define NLS_P2A2_OCC2_MAXJ 6  // KG 256^3: 5190 -> 5712 Mcells*steps/s (profiles/r05/ab_kg_occ2.txt)
#endif
__host__ __device__ constexpr bool p2d_jreg(int J, int A = 0) {
  return NLS_P2D_JREG && (A == 0   ? J >= NLS_P2D_JREG_MINJ && J <= NLS_P2D_JREG_MAXJ
                          : A == 3 ? J >= NLS_P2D_JREG2D_MINJ && J <= NLS_P2D_JREG_MAXJ
                          : A == 1 ? J >= NLS_P2A_JREG_MINJ && J <= NLS_P2A_JREG_MAXJ
                                   : J > 0 && J <= NLS_P2A2_OCC2_MAXJ);
}
// JPF: a register-row pass loads plane k+1's J rows at the top of step k (one step of
// look-ahead, J more registers: J = 8 fits two workgroups per CU, J = 10 would not);
// the prologue loads plane k0's, the last step reloads its own plane (every step issues
// the same loads, which the vmcnt replay counts).  Off (NLS_P2D_JPF_MAXJ 0): no gain
// measured (round 5, with RF: passes +0.35 ms per step, profiles/r05/ab_r5d.txt)
#ifndef NLS_P2D_JPF_MAXJ
#define NLS_P2D_JPF_MAXJ 0
#endif
__host__ __device__ constexpr bool p2d_jpf(int J, int A = 0) {
  return p2d_jreg(J, A) && p2d_kind(A) == 0 && J <= NLS_P2D_JPF_MAXJ;
}
// Workgroups per CU: two where the registers (<= 256 per lane) and the rings
// (<= 80 KiB) allow, so the second workgroup's waves cover the first's barriers
// and LDS latencies; one for the long passes.
#ifndef NLS_P2D_DS2_MAXJ
#define NLS_P2D_DS2_MAXJ 0  // two workgroups per CU: two planes of S look-ahead up to this J, then one (J = 2: NP 4, 2.10 vs 2.14 ms)
#endif
#ifndef NLS_P2D_DS3_MAXJ
#define NLS_P2D_DS3_MAXJ 4  // one workgroup per CU: three planes of S look-ahead up to this J, then one (J = 6: 3.78 vs 3.90 ms, NP 4 vs 3)
#endif
#ifndef NLS_P2D_DS2O_MAXJ
#define NLS_P2D_DS2O_MAXJ 4  // one WG per CU: two planes of S look-ahead up to this J (above DS3_MAXJ; 12: J = 12 no gain, r05)
#endif
#ifndef NLS_P2D_OCC0
#define NLS_P2D_OCC0 3  // workgroups per CU of the J = 0 pass (S look-ahead 1; 512^3: 1.40 vs 1.61 ms at 2)
#endif
__host__ __device__ constexpr int p2d_occ(int J, int A = 0) {
  return A == 1   ? (J <= NLS_P2A_OCC2_MAXJ || p2d_jreg(J, A) ? 2 : 1)
         : A == 2 ? (J <= NLS_P2A2_OCC2_MAXJ ? 2 : 1)  // pairs: the c ring as large as S's
                  : (J == 0 ? NLS_P2D_OCC0 : (J <= NLS_P2D_OCC2_MAXJ || p2d_jreg(J, A) ? 2 : 1));
}
// the x-halo L values of the tile computed by one wave into LDS (EXT1), and the X / Z
// coefficients in LDS -- except on the cell-pair passes at two workgroups per CU (above)
__host__ __device__ constexpr bool p2d_ext1(int J, int A = 0) { return NLS_P2D_EXT1 && !(A == 2 && p2d_occ(J, A) == 2); }
__host__ __device__ constexpr bool p2d_rcoef(int J, int A = 0) { return A == 2 && p2d_occ(J, A) == 2; }
// (these two test A == 2 only, which kind 3 never is)
// S ring: the planes k .. k+2 being read, DS planes of look-ahead and the slot of
// plane k-2 (free since the previous step's barrier), into which a step issues
// before its own wait and barrier
__host__ __device__ constexpr int p2d_ds(int J, int A = 0) {
  return p2d_kind(A) ? (p2d_occ(J, A) == 2 ? (J == 0 && A == 1 ? 2 : 1) : (J <= NLS_P2D_DS3_MAXJ ? 3 : (J >= 22 ? 1 : NLS_P2A_DS1)))
           : (p2d_occ(J, A) >= 3 ? 1
                                : (p2d_occ(J, A) == 2
                                       ? (J == 0 ? 3 : (J <= NLS_P2D_DS2_MAXJ ? 2 : 1))
                                       : (J == 0 ? 6
                                                 : (J <= NLS_P2D_DS3_MAXJ
                                                        ? 3
                                                        : (J <= NLS_P2D_DS2O_MAXJ
                                                               ? 2
                                                               : (J <= 12 || !NLS_P2D_EARLY ? 1 : 0))))));
}
// early issue only at one workgroup per CU (two: the other workgroup covers the wait,
// and the LDS is short); not where the anisotropic rings leave no slot for it
__host__ __device__ constexpr bool p2d_early(int J, int A = 0) {
  return p2d_kind(A) ? NLS_P2A_EARLY && p2d_occ(J, A) == 1 && J < 22 : NLS_P2D_EARLY && p2d_occ(J, A) == 1;
}
__host__ __device__ constexpr int p2d_nsl(int J, int A = 0) { return p2d_ds(J, A) + 3 + (p2d_early(J, A) ? 1 : 0); }
__host__ __device__ constexpr int p2d_off_c_ring(int J, int A = 0) { return p2d_nsl(J, A) * P2D_SR * P2D_SRB; }
__host__ __device__ constexpr int p2d_off_l(int J, int A = 0) {
  return p2d_off_c_ring(J, A) + p2d_nsl(J, A) * p2d_csb(A);
}
// the L ring: [2][P2D_LR] rows of 64, then [2][P2D_TR][2] x-halo values (x0-1, x0+64)
constexpr int P2D_LXB = 2 * P2D_TR * 2 * 16;
__host__ __device__ constexpr int p2d_off_j(int J, int A = 0) {
  return p2d_off_l(J, A) + 2 * P2D_LR * 1024 + (p2d_ext1(J, A) ? P2D_LXB : 0);
}
__host__ __device__ constexpr int p2d_coef_bytes(int J, int A = 0) { return p2d_rcoef(J, A) ? 0 : 2 * (J + 1) * 16; }
__host__ __device__ constexpr int p2d_avail(int J, int A = 0) {
  return P2D_LDS / p2d_occ(J, A) - p2d_off_j(J, A) - p2d_coef_bytes(J, A);
}
// J ring: NP whole planes of the J stored vectors of the wave's row (1 KiB each),
// the plane being read + NP-1 planes of look-ahead.  NP = 1 ("late" J ring, the long
// anisotropic passes): the wave reads its J rows of plane k into registers and then
// DMAs plane k+1 into the same slot, so the look-ahead is one step
__host__ __device__ constexpr int p2d_np(int J, int A = 0) {
  return J == 0 || p2d_jreg(J, A) ? 0
                : (p2d_avail(J, A) / (P2D_TR * 1024 * J) < NLS_P2D_NP_MAX ? p2d_avail(J, A) / (P2D_TR * 1024 * J)
                                                                          : NLS_P2D_NP_MAX);
}
__host__ __device__ constexpr bool p2d_late(int J, int A = 0) { return J > 0 && p2d_np(J, A) == 1; }
// RF ("refill"): a J ring of NP >= 2 planes whose slot is refilled with plane k + NP as soon
// as the wave has read plane k's rows into registers (every step reads all J rows into
// sv[] anyway), instead of issuing plane k + NP - 1 into the slot plane k - 1 freed: NP
// planes of look-ahead instead of NP - 1 from the same LDS (J = 12: two instead of one).
// Off: no pass got faster (J = 2, 4 unchanged, J = 12 5.93-6.00 vs 5.82-5.88 ms, same box,
// profiles/r05/p2ab_rf_ds2.txt) -- the ring passes are not waiting on the J look-ahead
#ifndef NLS_P2D_RF
#define NLS_P2D_RF 0
#endif
__host__ __device__ constexpr bool p2d_rf(int J, int A = 0) {
  return NLS_P2D_RF && p2d_kind(A) == 0 && J > 0 && !p2d_jreg(J, A) && p2d_np(J, A) >= 2;
}
__host__ __device__ constexpr int p2d_off_c(int J, int A = 0) {
  return p2d_off_j(J, A) + p2d_np(J, A) * J * P2D_TR * 1024;
}
__host__ __device__ constexpr int p2d_lds_bytes(int J, int A = 0) { return p2d_off_c(J, A) + p2d_coef_bytes(J, A); }
__host__ __device__ constexpr bool p2d_rings_ok(int J, int A = 0) {
  return J == 0 ? p2d_lds_bytes(J, A) * p2d_occ(J, A) <= P2D_LDS
                : (J <= (A == 2 ? P2D_JMAX_A2 : (p2d_kind(A) ? P2D_JMAX_A : P2D_JMAX)) &&
                   (p2d_np(J, A) >= 1 || p2d_jreg(J, A)) &&
                   p2d_lds_bytes(J, A) * p2d_occ(J, A) <= P2D_LDS);
}
static_assert(p2d_rings_ok(2) && p2d_rings_ok(4) && p2d_rings_ok(6) && p2d_rings_ok(8) && p2d_rings_ok(10) &&
              p2d_rings_ok(12) && p2d_rings_ok(14), "rings do not fit the LDS");
static_assert(p2d_rings_ok(0, true) && p2d_rings_ok(2, true) && p2d_rings_ok(4, true) && p2d_rings_ok(6, true) &&
              p2d_rings_ok(8, true) && p2d_rings_ok(10, true) && p2d_rings_ok(12, true) &&
              p2d_rings_ok(14, true) && p2d_rings_ok(16, true) && p2d_rings_ok(18, true) &&
              p2d_rings_ok(20, true) && p2d_rings_ok(22, true),
              "anisotropic rings do not fit the LDS");
static_assert(p2d_rings_ok(0, 2) && p2d_rings_ok(2, 2) && p2d_rings_ok(4, 2) && p2d_rings_ok(6, 2) &&
              p2d_rings_ok(8, 2) && p2d_rings_ok(10, 2) && p2d_rings_ok(12, 2) && p2d_rings_ok(14, 2),
              "anisotropic cell-pair rings do not fit the LDS");

// (occupancy experiment: LDS padding that caps the 3D isotropic passes 0 < J <= NLS_P2D_CAP2_MAXJ
// at two workgroups per CU; 0: off)
#ifndef NLS_P2D_CAP2_MAXJ
#define NLS_P2D_CAP2_MAXJ 0
#endif
__host__ __device__ constexpr int p2d_cap_pad(int J, int A = 0) {
  return (A == 0 && J > 0 && J <= NLS_P2D_CAP2_MAXJ && p2d_lds_bytes(J, A) < 56 * 1024) ? 56 * 1024 - p2d_lds_bytes(J, A)
                                                                                         : 0;
}

// VMEM ops issued after the last one step i needs, up to its wait (see k_p2d): a
// replay of the wave's issue order.  After the prologue's full wait the wave issues
// the S groups of planes k0+2 .. k0+1+DS (NSD DMAs each: 2 S rows, main + halo, and
// with A the 2 c rows, main + halo) and the J groups of planes k0 .. k0+NP-2 (late:
// plane k0); then per step: [S group k+DS+2 and J group k+NP-1] before the wait
// (early) or after it, the late J group k+1 after the J rows are read, then the STW
// stores.  Step i needs S(k+2) and J plane k.
__host__ __device__ constexpr int p2d_nsd(int A) { return A == 2 ? 8 : (p2d_kind(A) ? 6 : 4); }
// look-ahead S groups issued, with the J groups, before the prologue's wait (their slots
// (4 + d) % NSL are clear of the prologue's slots 0..3: the one-workgroup-per-CU passes
// with early issue); 0: every look-ahead group after the wait, S before J (the round-3
// order; also the order with NLS_P2D_PRE_LA = 0)
__host__ __device__ constexpr int p2d_dspre(int J, int A = 0) {
  return NLS_P2D_PRE_LA ? (p2d_ds(J, A) < p2d_nsl(J, A) - 4 ? p2d_ds(J, A) : p2d_nsl(J, A) - 4) : 0;
}
__host__ __device__ constexpr int p2d_after(int J, int STW, int i, int A = 0) {
  const int DS = p2d_ds(J, A), NP = p2d_np(J, A), NSD = p2d_nsd(A);
  const bool early = p2d_early(J, A), late = p2d_late(J, A), jreg = p2d_jreg(J, A), rf = p2d_rf(J, A);
  // the issue order ahead of the loop: [S groups d < DSPRE][J groups][S groups d >= DSPRE]
  // (DSPRE = 0: every S group first, as the round-3 kernel issued them)
  const int dspre = p2d_dspre(J, A) > 0 ? p2d_dspre(J, A) : DS;
  int n = 0, lastS = 0, lastJ = 0;
  for (int d = 0; d < dspre; ++d) {
    n += NSD;
    if (d == i) lastS = n;
  }
  if (J > 0 && !jreg) {
    const int pj = late ? 1 : (rf ? NP : NP - 1);
    for (int d = 0; d < pj; ++d) {
      n += J;
      if (d == i) lastJ = n;
    }
  }
  for (int d = dspre; d < DS; ++d) {
    n += NSD;
    if (d == i) lastS = n;
  }
  if (p2d_jpf(J, A)) n += J;  // plane k0's J rows, the last prologue loads
  for (int s = 0;; ++s) {
    if (jreg) n += J;  // the step's J row loads at its top (the compiler awaits them)
    if (early) {
      n += NSD;
      if (s + DS == i) lastS = n;
      if (J > 0 && !late && !jreg && !rf) {
        n += J;
        if (s + NP - 1 == i) lastJ = n;
      }
    }
    if (s == i) break;  // the wait of step i
    if (!early) {
      n += NSD;
      if (s + DS == i) lastS = n;
      if (J > 0 && !late && !jreg && !rf) {
        n += J;
        if (s + NP - 1 == i) lastJ = n;
      }
    }
    if (late || rf) {  // the slot just read takes plane s + 1 (late) / s + NP (rf)
      n += J;
      if (s + (late ? 1 : NP) == i) lastJ = n;
    }
    n += STW;
  }
  const int aS = n - lastS, aJ = J > 0 && !jreg ? n - lastJ : 1 << 20;
  return aS < aJ ? aS : aJ;
}
// from this step on every wait is the same (a safe bound of the replay's warm-up)
__host__ __device__ constexpr int p2d_i0(int J, int A = 0) { return p2d_ds(J, A) + p2d_np(J, A) + 1; }
// the first step from which the replay's wait equals the steady one (every warm-up
// step of the current schedules but step 0 already waits the steady count)
__host__ __device__ constexpr int p2d_isteady(int J, int STW, int A = 0) {
  int s = p2d_i0(J, A);
  while (s > 0 && p2d_after(J, STW, s - 1, A) == p2d_after(J, STW, p2d_i0(J, A), A)) --s;
  return s;
}
template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 0 ? 0 : (N > 63 ? 63 : N)) : "memory");
}
// one compare per distinct warm-up step (a chain over every step < p2d_i0 cost ~20
// SALU per march step at J = 12)
template <int J, int STW, int A, int I = 0> __device__ __forceinline__ void wait_step(int i) {
  if constexpr (I >= p2d_isteady(J, STW, A)) {
    wait_vm<p2d_after(J, STW, p2d_i0(J, A), A)>();
  } else {
    if (i == I) {
      wait_vm<p2d_after(J, STW, I, A)>();
      return;
    }
    wait_step<J, STW, A, I + 1>(i);
  }
}

// 16 lanes x 4 B (one 64-B piece: the four halo cells of a staged row) into lds
__device__ __forceinline__ void dma4(const void *base, uint32_t voff, char *lds) {
  const void *g = static_cast<const char *>(base) + voff;
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 4, 0, 0);
}
// one wave-instruction: 64 lanes x 16 B from base + voff (base wave-uniform, so the
// SGPR-base + 32-bit VGPR-offset form is selected) into lds .. lds + 1 KiB
__device__ __forceinline__ void dma16(const void *base, uint32_t voff, char *lds, unsigned aux) {
  const void *g = static_cast<const char *>(base) + voff;
  if (aux) __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 16, 0, 2);
  else __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}
// face weight of the G2 operator (nls_stencil.hpp face_w): (c_a + c_b)/2 where the face exists
__device__ __forceinline__ double p2d_face(bool e, double ca, double cb) { return e ? 0.5 * (ca + cb) : 0.0; }
// the same with a per-lane source address (the c rows: two rows per instruction)
__device__ __forceinline__ void glds16(const char *g, char *lds) {
  __builtin_amdgcn_global_load_lds(static_cast<const void *>(g), (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const char *g, char *lds) {
  __builtin_amdgcn_global_load_lds(static_cast<const void *>(g), (__attribute__((address_space(3))) void *)lds, 4, 0, 0);
}
// lane i <- lane i-1 / i+1 by DPP wave shifts (GFX9 wave_shr:1 / wave_shl:1; the
// lane shifted in from outside the wave reads 0)
__device__ __forceinline__ double dpp_d(double v, int ctrl_shr) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  int a, b;
  if (ctrl_shr) {
    a = __builtin_amdgcn_update_dpp(0, lo, 0x138, 0xf, 0xf, true);
    b = __builtin_amdgcn_update_dpp(0, hi, 0x138, 0xf, 0xf, true);
  } else {
    a = __builtin_amdgcn_update_dpp(0, lo, 0x130, 0xf, 0xf, true);
    b = __builtin_amdgcn_update_dpp(0, hi, 0x130, 0xf, 0xf, true);
  }
  return __hiloint2double(b, a);
}
// acc += a b and acc += conj(a) b as four FMAs (no rounded product temporaries)
__device__ __forceinline__ void cmac(cplx &acc, cplx a, cplx b) {
  acc.re = fma(a.re, b.re, acc.re);
  acc.re = fma(-a.im, b.im, acc.re);
  acc.im = fma(a.re, b.im, acc.im);
  acc.im = fma(a.im, b.re, acc.im);
}
__device__ __forceinline__ void cjmac(cplx &acc, cplx a, cplx b) {
  acc.re = fma(a.re, b.re, acc.re);
  acc.re = fma(a.im, b.im, acc.re);
  acc.im = fma(a.re, b.im, acc.im);
  acc.im = fma(-a.im, b.re, acc.im);
}
__device__ __forceinline__ cplx lane_prev(cplx v) { return {dpp_d(v.re, 1), dpp_d(v.im, 1)}; }
__device__ __forceinline__ cplx lane_next(cplx v) { return {dpp_d(v.re, 0), dpp_d(v.im, 0)}; }
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Output planes [g.qa, g.qb) of the slab, plus [g.q2, g.q2 + qb - qa) when g.q2 > 0
// (multi-rank handles launch the two boundary plane pairs as one grid apart from
// the interior, so the halo exchange overlaps);
// partial sums at part[c * nb + poff + blockIdx.x].
// D2: a 2D [ny][nx] grid seen as planes of 4 rows (g: nyp = 4, npl = ny/4, P = 4 nx):
// the row-wrap of the 3D march is then exactly the 2D y neighbour, the plane
// neighbours (2D rows +-4) are dropped, and the boundary rows are 2D rows 0, ny-1.
// PR: a real field seen as pairs of cells (nx = pairs, one cplx = cells 2x, 2x+1;
// real coefficients, so every linear combination acts per component and the real
// part of each complex dot is the real dot): only the x neighbours differ (cell
// 2x-1 is pair x-1's second, cell 2x+2 pair x+1's first) and the x boundary
// diagonal applies per cell.
__device__ __forceinline__ cplx pr_lap(cplx c, cplx xm, cplx xp, cplx yz, double dga, double dgb, double s) {
  return {dga * c.re + s * (yz.re + (xm.im + c.im)), dgb * c.im + s * (yz.im + (c.re + xp.re))};
}

// PEER: the multi-rank peer-store variant (3D isotropic; NLS_PEER=1): after the march the
// pass's last output's boundary planes also go to the neighbours' ghost planes
template <int J, bool HZ, bool D2 = false, bool PR = false, bool A = false, bool PEER = false>
__global__ __launch_bounds__(NTHREADS, p2d_occ(J, A ? (PR ? 2 : 1) : (D2 ? 3 : 0))) void k_p2d(cplx *__restrict__ W, int64_t vs, Geo g,
                                                              const P2State *__restrict__ ps,
                                                              cplx *__restrict__ part, int nb,
                                                              const cplx *__restrict__ zbuf, int poff) {
  // the anisotropic kind of the ring functions (p2d_csb): 1 complex, 2 real cell pairs
  constexpr int AK = A ? (PR ? 2 : 1) : 0;
  constexpr int KA = !A && D2 ? 3 : AK;  // the kind the ring and wait rules take (3: isotropic 2D)
  static_assert(p2d_rings_ok(J, KA), "rings exceed LDS");
  static_assert(!(A && D2), "the anisotropic pass is 3D");
  constexpr int DS = p2d_ds(J, KA), NSL = p2d_nsl(J, KA), NP = p2d_np(J, KA);
  constexpr bool LATE = p2d_late(J, KA), JREG = p2d_jreg(J, KA), RF = p2d_rf(J, KA), JPF = p2d_jpf(J, KA);
  constexpr bool EXT1 = p2d_ext1(J, KA), RCOEF = p2d_rcoef(J, KA);
  // WC: the own row's face weights div(c grad) needs at plane k were computed with its
  // L S_J one step earlier (same c, same conditions, so the same bits): kept in
  // registers (nwc -> cwc) instead of recomputed from the c ring by L^2 S_J
  constexpr bool WC = NLS_P2D_WCACHE && A && HZ && (p2d_occ(J, KA) == 1 || J <= 6);  // (J = 8 at two per CU: scratch)
  constexpr int NWC = AK == 2 ? 13 : 7;
  double nwc[NWC], cwc[NWC];
  constexpr int STW = HZ ? 2 : 1;            // stores per step
  // columns: gX[0..J], (HZ: gZ[0..J], xx, xz, zz | xx); J = 0 also ||S_0||^2 (the
  // blind start, k_p2coef mode 2)
  constexpr int NC = (HZ ? 2 * (J + 1) + 3 : J + 2) + (J == 0 ? 1 : 0);
  constexpr int NPD = NP > 0 ? NP : 1;
  constexpr int RW = P2D_SRB / 16;           // cplx per staged S row (68)
  __shared__ __attribute__((aligned(16))) char smem[p2d_lds_bytes(J, KA) + p2d_cap_pad(J, KA)];
  const cplx *Sr = reinterpret_cast<const cplx *>(smem);             // [NSL][P2D_SR][RW]
  const double *Cr = reinterpret_cast<const double *>(smem + p2d_off_c_ring(J, KA));  // A: [NSL][p2d_csb/8]
  cplx *Lr = reinterpret_cast<cplx *>(smem + p2d_off_l(J, KA));       // [2][P2D_LR][64]
  cplx *Lx = Lr + 2 * P2D_LR * 64;                                     // [2][P2D_TR][2]
  cplx *cX = reinterpret_cast<cplx *>(smem + p2d_off_c(J, KA));       // [J+1] (not with RCOEF)
  cplx *cZ = cX + (J + 1);                                           // [J+1]
  cplx rcX[RCOEF ? J + 1 : 1], rcZ[RCOEF ? J + 1 : 1];               // RCOEF: in registers
  // w through readfirstlane: wave-uniform for the compiler too, so row and plane
  // logic stays scalar
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  // planes: local k (slab of nzl planes, ghost planes -2, -1, nzl, nzl+1 filled by the
  // halo exchange on multi-rank handles), global z0 + k for the reference's couplings
  const int nx = (int)g.nx, ny = (int)g.nyp, P = (int)g.P, nz = (int)g.npl;
  const int nzl = (int)g.nzl, z0 = (int)g.z0;
  const int ntx = (nx + P2D_XO - 1) / P2D_XO, nty = ny / P2D_TR;
  const int qa = g.qa, qb = g.qb;
  // z chunks of [qa, qb), and with g.q2 > 0 as many again of [q2, q2 + qb - qa)
  const int nz1 = (qb - qa + g.kz - 1) / g.kz;
  const int nzc = g.q2 > 0 ? 2 * nz1 : nz1;
  const int ntiles = ntx * nty * nzc;
  // XCD-banded order: the 8 XCDs take contiguous tile ranges, so the y-adjacent
  // tiles sharing S_J halo rows run on one XCD (its L2) at the same time (g.remap
  // bit 4: plain order).  y-fastest inside a band, or (bit 2) x-fastest: the tiles
  // of one 4-row group are then consecutive and read its rows whole together
  const int b = blockIdx.x;
  const int T8 = ntiles / 8;
  const int tile = (g.remap & 4) || b >= 8 * T8 ? b : (b % 8) * T8 + b / 8;
  int yt, xt, zc;
  if (g.remap & 2) {
    xt = tile % ntx;
    const int r_ = tile / ntx;
    yt = r_ % nty;
    zc = r_ / nty;
  } else {
    yt = tile % nty;
    const int r_ = tile / nty;
    xt = r_ % ntx;
    zc = r_ / ntx;
  }
  const int x0 = xt * P2D_XO, y0 = yt * P2D_TR;
  const bool hi = g.q2 > 0 && zc >= nz1;  // uniform
  const int za = hi ? g.q2 : qa, zb = hi ? g.q2 + (qb - qa) : qb;
  const int k0 = za + (hi ? zc - nz1 : zc) * g.kz, k1 = min(k0 + g.kz, zb);
  const int x = x0 + lane;
  const bool xin = x < nx;
  const bool full = x0 + P2D_XO <= nx;                    // uniform
  const int src_lane = xin ? lane : nx - 1 - x0;          // last valid lane of a ragged tile
  const int y = y0 + w;  // this wave's row (ny % 4 == 0: always a real row)
  if constexpr (RCOEF) {
#pragma unroll
    for (int l = 0; l <= J; ++l) {
      rcX[l] = ps->aX[l];
      rcZ[l] = ps->aZ[l];
    }
  } else {
    for (int l = t; l <= J; l += NTHREADS) {
      cX[l] = ps->aX[l];
      cZ[l] = ps->aZ[l];
    }
  }
  cplx bX1 = ps->bX1, bZ1 = ps->bZ1, bZ2 = ps->bZ2;
  double s = g.s, sdi = g.sd_in, sdb = g.sd_bd;
  // the anisotropic passes up to J = NLS_P2D_VCOEF_MAXJ keep the uniform f64 operands
  // of the march in VGPRs: as SGPRs (18 of them) they were among the values spilled to
  // VGPR lanes, a v_readlane / v_writelane per use (KG 256^3 passes 2.38 -> 2.26 ms per
  // step, G2 neutral; above J = 8 the VGPRs are the scarcer).  The isotropic passes
  // lost with it (512^3: 24.3 -> 25.3 ms of passes, fewer instructions notwithstanding;
  // profiles/r04/ab_vcoef.txt)
  if constexpr (AK > 0 && J <= NLS_P2D_VCOEF_MAXJ) {
    asm volatile("" : "+v"(bX1.re), "+v"(bX1.im), "+v"(bZ1.re), "+v"(bZ1.im), "+v"(bZ2.re), "+v"(bZ2.im));
    asm volatile("" : "+v"(s), "+v"(sdi), "+v"(sdb));
  }
  const int64_t P16 = (int64_t)P * 16;
  const char *__restrict__ SJb = reinterpret_cast<const char *>(W + (int64_t)J * vs);
  cplx *__restrict__ Xo = W + (int64_t)(J + 1) * vs;
  cplx *__restrict__ Zo = W + (int64_t)(J + 2) * vs;
  __syncthreads();  // coefficients in LDS (no DMA in flight yet)

  // per lane: the cell byte offset (clamped into the row; unused when outside),
  // the halo piece (lanes 0..15: dword lane&3 of cell x0-2, x0-1, x0+64, x0+65)
  auto clampx = [nx](int v) { return v < 0 ? 0 : (v >= nx ? nx - 1 : v); };
  const uint32_t xoff = (uint32_t)clampx(x) * 16u;
  const int hc = (lane >> 2) & 3;
  const uint32_t hoff = (uint32_t)clampx(hc < 2 ? x0 - 2 + hc : x0 + 62 + hc) * 16u + (uint32_t)(lane & 3) * 4u;
  // A: the c field (f64, nx even so that every pair of cells is one aligned 16 B):
  // lane -> cells x0 + 2 (lane & 31) + {0, 1} (clamped into the row), halo lane
  // (0..15) -> dword lane & 1 of cell x0-2, x0-1, x0+64, x0+65
  const char *__restrict__ Cg = reinterpret_cast<const char *>(g.cf);
  const int64_t coff = (int64_t)min(x0 + 2 * (lane & 31), nx - 2) * 8;
  const int hcc = (lane >> 1) & 3;
  const int64_t choff = (int64_t)clampx(hcc < 2 ? x0 - 2 + hcc : x0 + 62 + hcc) * 8 + (lane & 1) * 4;
  // L S_J positions: main lane i -> x0 + i (row index i, x neighbours i-1 / i+1,
  // the halo cells 65 / 66 at the tile edges); extra pass lane 0 -> x0-1, lane 1
  // -> x0+64 (row indices 65 / 66, neighbours 64,0 / 63,67)
  const int mi = lane > 0 ? lane - 1 : 65, pi = lane < 63 ? lane + 1 : 66;
  // (EXT1: lane 2r + h -> tile row r, h as above)
  const int xe = (lane & 1) ? x0 + 64 : x0 - 1;
  const int eci = (lane & 1) ? 66 : 65, emi = (lane & 1) ? 63 : 64, epi = (lane & 1) ? 67 : 0;
  const int xr = 2 + ((lane >> 1) & (P2D_TR - 1));
  // (macros, not lambdas capturing by reference: hipcc kept such captures on the
  // stack, and every scratch access is a VMEM op that breaks the vmcnt counting)
#define P2D_PLANE(p, yy) (z0 + ((yy) < 0 ? (p) - 1 : ((yy) >= ny ? (p) + 1 : (p))))  // global
#define P2D_ROW(yy) ((yy) < 0 ? (yy) + ny : ((yy) >= ny ? (yy) - ny : (yy)))
// boundary cell in y / z (D2: 2D rows 0 and ny - 1 of the 4-row planes)
#define P2D_BYZ(j, kk)                                                                     \
  (D2 ? ((((kk) == 0) & ((j) == 0)) | (((kk) == nz - 1) & ((j) == ny - 1)))                \
      : (((j) == 0) | ((j) == ny - 1) | ((kk) == 0) | ((kk) == nz - 1)))
#define P2D_DIAG(xx, j, kk) ((((xx) == 0) | ((xx) == nx - 1) | P2D_BYZ(j, kk)) ? sdb : sdi)
// PR: the diagonals of the pair's first / second cell
#define P2D_DIAGA(xx, j, kk) ((((xx) == 0) | P2D_BYZ(j, kk)) ? sdb : sdi)
#define P2D_DIAGB(xx, j, kk) ((((xx) == nx - 1) | P2D_BYZ(j, kk)) ? sdb : sdi)
  // this wave's two staged S rows yy = y0 - 2 + 2w + r (r = 0, 1): the plane shift of
  // the y-wrap (rows -2, -1 are the previous plane's last, ny, ny+1 the next plane's
  // first), the issue planes p for which the row's global plane lies in the grid, its
  // local plane in the allocation (ghosts) and p <= k1 + 1 (not past the tile's last
  // needed plane), and the row's byte offset: computed once per tile, not per DMA
  const int s_yy0 = y0 - 2 + 2 * w, s_yy1 = s_yy0 + 1;
  const int s_dr0 = s_yy0 < 0 ? -1 : (s_yy0 >= ny ? 1 : 0), s_dr1 = s_yy1 < 0 ? -1 : (s_yy1 >= ny ? 1 : 0);
  const int s_lo0 = max(-z0 - s_dr0, -P2D_GHOST - s_dr0), s_lo1 = max(-z0 - s_dr1, -P2D_GHOST - s_dr1);
  const int s_hi0 = min(min(nz - z0 - s_dr0, nzl + P2D_GHOST - s_dr0) - 1, k1 + 1);
  const int s_hi1 = min(min(nz - z0 - s_dr1, nzl + P2D_GHOST - s_dr1) - 1, k1 + 1);
  const int64_t s_yo0 = (int64_t)s_yy0 * nx * 16, s_yo1 = s_yo0 + (int64_t)nx * 16;
  // DMA this wave's two S_J rows of plane p into ring slot sl: the 64 aligned
  // cells and the 4 halo cells (the zero row outside the grid and past the
  // tile's last needed plane)
// (P2D_ISSUE_SO: with the plane's byte offset pb = p * P16 kept by the caller -- the
// march steps it by an add instead of a 64-bit multiply per step)
#define P2D_ISSUE_S(p, sl) P2D_ISSUE_SO(p, (int64_t)(p) * P16, sl)
#define P2D_ISSUE_SO(p, pb, sl)                                                         \
  do {                                                                                  \
    const int p_ = (p);                                                                 \
    const int64_t pb_ = (pb);                                                           \
    char *dst_ = smem + ((sl) * P2D_SR + 2 * w) * P2D_SRB;                              \
    _Pragma("unroll") for (int r_ = 0; r_ < 2; ++r_) {                                  \
      /* the row inside the grid and the allocation and needed (s_lo / s_hi) */       \
      const bool ok_ = p_ >= (r_ ? s_lo1 : s_lo0) && p_ <= (r_ ? s_hi1 : s_hi0) &&       \
                       !((NLS_DIAG_P2HALO & 2) && (w == 0 || w == 3));                  \
      const int64_t o_ = pb_ + (r_ ? s_yo1 : s_yo0);                                    \
      const char *b_ = ok_ ? SJb + o_ : reinterpret_cast<const char *>(zbuf);           \
      asm volatile("" : "+s"(b_)); /* one select, not a DMA per branch */               \
      dma16(b_, xoff, dst_ + r_ * P2D_SRB, 0);                                          \
      if (lane < 16)                                                                    \
        dma4((NLS_DIAG_P2HALO & 1) ? reinterpret_cast<const char *>(zbuf) : b_,         \
             (NLS_DIAG_P2HALO & 1) ? (uint32_t)(lane & 3) * 4u : hoff, dst_ + r_ * P2D_SRB + 1024); \
      if constexpr (AK == 2) {                                                          \
        /* cell pairs: the c row of the same S row, staged as S rows are */           \
        char *cd_ = smem + p2d_off_c_ring(J, KA) + ((sl) * P2D_SR + 2 * w + r_) * P2D_SRB; \
        const char *c_ = ok_ ? Cg + o_ : reinterpret_cast<const char *>(zbuf);          \
        asm volatile("" : "+s"(c_));                                                    \
        dma16(c_, xoff, cd_, 0);                                                        \
        if (lane < 16) dma4(c_, hoff, cd_ + 1024);                                      \
      }                                                                                 \
    }                                                                                   \
    if constexpr (AK == 1) {                                                           \
      /* the c rows of the same two S rows: lanes 0..31 / 32..63 two cells each of   \
         row 2w / 2w+1, then their halo cells on lanes 0..15 (8 lanes x 4 B a row) */ \
      char *cd_ = smem + p2d_off_c_ring(J, KA) + (sl) * P2D_CSB;                        \
      const int yc_ = y0 - 2 + 2 * w + (lane >> 5), kc_ = P2D_PLANE(p_, yc_), lc_ = kc_ - z0; \
      const bool okc_ = kc_ >= 0 && kc_ < nz && lc_ >= -P2D_GHOST && lc_ < nzl + P2D_GHOST && \
                        p_ <= k1 + 1;                                                   \
      const char *cb_ = okc_ ? Cg + ((pb_ >> 1) + (int64_t)yc_ * nx * 8)                \
                             : reinterpret_cast<const char *>(zbuf);                    \
      glds16(cb_ + coff, cd_ + 2 * w * P2D_CRB);                                        \
      const int yh_ = y0 - 2 + 2 * w + ((lane >> 3) & 1), kh_ = P2D_PLANE(p_, yh_), lh_ = kh_ - z0; \
      const bool okh_ = kh_ >= 0 && kh_ < nz && lh_ >= -P2D_GHOST && lh_ < nzl + P2D_GHOST && \
                        p_ <= k1 + 1;                                                   \
      const char *hb_ = okh_ ? Cg + ((pb_ >> 1) + (int64_t)yh_ * nx * 8)                \
                             : reinterpret_cast<const char *>(zbuf);                    \
      if (lane < 16) glds4(hb_ + choff, cd_ + P2D_SR * P2D_CRB + 2 * w * 32);           \
    }                                                                                   \
  } while (0)
  // DMA the J stored vectors of this wave's row of plane p into J-ring slot sl.  One
  // scalar pointer walks the vectors (vector stride vsb): J per-vector pointers were
  // 2J SGPRs (spilled to VGPR lanes from J ~ 10) and 3J SALU per step.  A plane past
  // the tile re-reads the tile's last plane: those rows are never used, the DMA only
  // keeps every step's issue count the same.
  const char *const jb0 = reinterpret_cast<const char *>(W) + (int64_t)y * nx * 16;
  const int64_t vsb = vs * 16;
#define P2D_ISSUE_J(p, sl) P2D_ISSUE_JO((int64_t)min((p), k1 - 1) * P16, sl)
#define P2D_ISSUE_JO(jo, sl)                                                            \
  do {                                                                                  \
    const char *b_ = jb0 + (jo);                                                        \
    char *dst_ = smem + p2d_off_j(J, KA) + (((sl) * J) * P2D_TR + w) * 1024;             \
    _Pragma("unroll") for (int l_ = 0; l_ < J; ++l_) {                                  \
      asm volatile("" : "+s"(b_));  /* keep the walk: no J loop-invariant pointers */   \
      dma16(b_, xoff, dst_ + l_ * P2D_TR * 1024, 1);                                    \
      b_ += vsb;                                                                        \
    }                                                                                   \
  } while (0)
  // A: c of ring slot sl, tile row tr, row index i (0..63: x0 + i; 64..67: the halo
  // cells x0-2, x0-1, x0+64, x0+65)
#define P2D_CV(sl, tr, i)                                                                \
  Cr[(sl) * (P2D_CSB / 8) + ((i) < 64 ? (tr) * 64 + (i) : P2D_SR * 64 + (tr) * 4 + (i) - 64)]
  // cell pairs: c of cell h (0: 2P, 1: 2P + 1) of pair row index P (0..67, as S_J's)
#define P2D_CV2(sl, tr, P, h) Cr[((sl) * P2D_SR + (tr)) * (P2D_SRB / 8) + 2 * (P) + (h)]
  // L S_J at plane p, S tile row tr (yy = y0 - 2 + tr), x position xx with row
  // indices ci (centre), mi_ / pi_ (x - 1 / x + 1), from ring slots sm, sc, sp
  // (planes p-1, p, p+1)
#define P2D_LAP(dst, p, tr, sm, sc, sp, xx, ci, mi_, pi_, ws)                           \
  do {                                                                                  \
    const int p_ = (p), tr_ = (tr), xx_ = (xx);                                         \
    const cplx *Sm_ = Sr + ((sm) * P2D_SR + tr_) * RW;                                  \
    const cplx *Sc_ = Sr + ((sc) * P2D_SR + tr_) * RW;                                  \
    const cplx *Sp_ = Sr + ((sp) * P2D_SR + tr_) * RW;                                  \
    const int yy_ = y0 - 2 + tr_, kk_ = P2D_PLANE(p_, yy_);                             \
    const cplx c_ = Sc_[(ci)];                                                          \
    const cplx xm_ = xx_ > 0 ? Sc_[(mi_)] : cplx{0.0, 0.0};                             \
    const cplx xp_ = xx_ + 1 < nx ? Sc_[(pi_)] : cplx{0.0, 0.0};                        \
    const cplx ym_ = Sc_[(ci) - RW], yp_ = Sc_[(ci) + RW];                              \
    const cplx zm_ = D2 ? cplx{0.0, 0.0} : Sm_[(ci)], zp_ = D2 ? cplx{0.0, 0.0} : Sp_[(ci)]; \
    const bool ok_ = xx_ >= 0 && xx_ < nx && kk_ >= 0 && kk_ < nz;                      \
    cplx v_;                                                                            \
    if constexpr (AK == 2) {                                                            \
      /* div(c grad) per cell of the pair (a = 2 xx, b = 2 xx + 1): the a|b face     \
         always exists, a's x - 1 is the previous pair's b, b's x + 1 the next      \
         pair's a; y, z faces per cell as in the complex form */                     \
      const int jj_ = P2D_ROW(yy_);                                                     \
      const double ca_ = P2D_CV2(sc, tr_, ci, 0), cb_ = P2D_CV2(sc, tr_, ci, 1);        \
      const double wab_ = 0.5 * (ca_ + cb_);                                            \
      const double wam_ = p2d_face(xx_ > 0, ca_, P2D_CV2(sc, tr_, mi_, 1));             \
      const double wbp_ = p2d_face(xx_ + 1 < nx, cb_, P2D_CV2(sc, tr_, pi_, 0));        \
      const bool ym_ok_ = kk_ > 0 || jj_ > 0, yp_ok_ = kk_ < nz - 1 || jj_ < ny - 1;    \
      const double wyam_ = p2d_face(ym_ok_, ca_, P2D_CV2(sc, tr_ - 1, ci, 0));          \
      const double wyap_ = p2d_face(yp_ok_, ca_, P2D_CV2(sc, tr_ + 1, ci, 0));          \
      const double wybm_ = p2d_face(ym_ok_, cb_, P2D_CV2(sc, tr_ - 1, ci, 1));          \
      const double wybp_ = p2d_face(yp_ok_, cb_, P2D_CV2(sc, tr_ + 1, ci, 1));          \
      const double wzam_ = p2d_face(kk_ > 0, ca_, P2D_CV2(sm, tr_, ci, 0));             \
      const double wzap_ = p2d_face(kk_ < nz - 1, ca_, P2D_CV2(sp, tr_, ci, 0));        \
      const double wzbm_ = p2d_face(kk_ > 0, cb_, P2D_CV2(sm, tr_, ci, 1));             \
      const double wzbp_ = p2d_face(kk_ < nz - 1, cb_, P2D_CV2(sp, tr_, ci, 1));        \
      v_.re = s * ((((wzam_ * zm_.re + wzap_ * zp_.re) + (wam_ * xm_.im + wab_ * c_.im)) + \
                    (wyam_ * ym_.re + wyap_ * yp_.re)) -                                \
                   (((wzam_ + wzap_) + (wam_ + wab_)) + (wyam_ + wyap_)) * c_.re);      \
      v_.im = s * ((((wzbm_ * zm_.im + wzbp_ * zp_.im) + (wab_ * c_.re + wbp_ * xp_.re)) + \
                    (wybm_ * ym_.im + wybp_ * yp_.im)) -                                \
                   (((wzbm_ + wzbp_) + (wab_ + wbp_)) + (wybm_ + wybp_)) * c_.im);      \
      if constexpr (ws && WC) {                                                         \
        nwc[0] = wab_; nwc[1] = wam_; nwc[2] = wbp_; nwc[3] = wyam_; nwc[4] = wyap_;    \
        nwc[5] = wybm_; nwc[6] = wybp_; nwc[7] = wzam_; nwc[8] = wzap_; nwc[9] = wzbm_; \
        nwc[10] = wzbp_;                                                                \
        nwc[11] = ((wzam_ + wzap_) + (wam_ + wab_)) + (wyam_ + wyap_);                  \
        nwc[12] = ((wzbm_ + wzbp_) + (wab_ + wbp_)) + (wybm_ + wybp_);                  \
      }                                                                                 \
    } else if constexpr (A) {                                                           \
      /* div(c grad) (laplacians.hpp:158-218): face weights (c_a + c_b)/2 where the  \
         reference's flat-index neighbour exists, diagonal -sum of the weights */     \
      const int jj_ = P2D_ROW(yy_);                                                     \
      const double cc_ = P2D_CV(sc, tr_, ci);                                           \
      const double wxm_ = p2d_face(xx_ > 0, cc_, P2D_CV(sc, tr_, mi_));                   \
      const double wxp_ = p2d_face(xx_ + 1 < nx, cc_, P2D_CV(sc, tr_, pi_));              \
      const double wym_ = p2d_face(kk_ > 0 || jj_ > 0, cc_, P2D_CV(sc, tr_ - 1, ci));     \
      const double wyp_ = p2d_face(kk_ < nz - 1 || jj_ < ny - 1, cc_, P2D_CV(sc, tr_ + 1, ci)); \
      const double wzm_ = p2d_face(kk_ > 0, cc_, P2D_CV(sm, tr_, ci));                    \
      const double wzp_ = p2d_face(kk_ < nz - 1, cc_, P2D_CV(sp, tr_, ci));               \
      if constexpr (ws && WC) {                                                         \
        nwc[0] = wxm_; nwc[1] = wxp_; nwc[2] = wym_; nwc[3] = wyp_; nwc[4] = wzm_;      \
        nwc[5] = wzp_; nwc[6] = ((wzm_ + wzp_) + (wxm_ + wxp_)) + (wym_ + wyp_);         \
      }                                                                                 \
      v_ = s * ((((wzm_ * zm_ + wzp_ * zp_) + (wxm_ * xm_ + wxp_ * xp_)) + (wym_ * ym_ + wyp_ * yp_)) - \
                (((wzm_ + wzp_) + (wxm_ + wxp_)) + (wym_ + wyp_)) * c_);                 \
    } else if constexpr (PR) {                                                          \
      const int jj_ = P2D_ROW(yy_);                                                     \
      v_ = pr_lap(c_, xm_, xp_, (zm_ + zp_) + (ym_ + yp_), P2D_DIAGA(xx_, jj_, kk_),    \
                  P2D_DIAGB(xx_, jj_, kk_), s);                                         \
    } else {                                                                            \
      const double dg_ = P2D_DIAG(xx_, P2D_ROW(yy_), kk_);                              \
      v_ = dg_ * c_ + s * (((zm_ + zp_) + (xm_ + xp_)) + (ym_ + yp_));                  \
    }                                                                                   \
    dst = ok_ ? v_ : cplx{0.0, 0.0};                                                    \
  } while (0)
  // per plane a wave computes L S_J of its own row (main lanes, kept in a
  // register); the tile's halo rows (L rows 0 and P2D_LR-1) and its 8 x-halo values
  // (x0-1, x0+64 of each row) are spread over the waves, one extra stencil each
  // (EXT1: wave 0 the x-halo values on lanes 0..7 into Lx, waves 1 / 2 the halo
  // rows, wave 3 none: at most two stencils per wave and step instead of three;
  // NLS_P2D_EXT1 = 0: every wave its own two x-halo values in a register, the halo
  // rows on waves 0 / 3); the main rows go to the L ring for the y neighbours of
  // the other waves' L^2 S_J
#define P2D_LROWS(p, sm, sc, sp, slot, own, ext)                                        \
  do {                                                                                  \
    P2D_LAP(own, p, w + 2, sm, sc, sp, x, lane, mi, pi, 1);                             \
    if constexpr (!EXT1) P2D_LAP(ext, p, w + 2, sm, sc, sp, xe, eci, emi, epi, 0);     \
    Lr[((slot) * P2D_LR + w + 1) * 64 + lane] = own;                                    \
    if (EXT1 && w == 0) {                                                               \
      cplx e_;                                                                          \
      P2D_LAP(e_, p, xr, sm, sc, sp, xe, eci, emi, epi, 0);                             \
      if (lane < 2 * P2D_TR) Lx[(slot) * 2 * P2D_TR + lane] = e_;                       \
    }                                                                                   \
    if (EXT1 ? (w == 1 || w == 2) : (w == 0 || w == P2D_TR - 1)) {                      \
      const int er_ = (EXT1 ? w == 1 : w == 0) ? 0 : P2D_LR - 1;                        \
      cplx e_;                                                                          \
      P2D_LAP(e_, p, er_ + 1, sm, sc, sp, x, lane, mi, pi, 0);                          \
      Lr[((slot) * P2D_LR + er_) * 64 + lane] = e_;                                     \
    }                                                                                   \
  } while (0)

  cplx acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = {0.0, 0.0};

  // prologue: S planes k0-2 .. k0+1 (slots 0..3), L S_J of planes k0-1 (own row,
  // register) and k0 (own row + halo values; L ring slot 0); then the look-ahead
  // S planes and J planes
  for (int p = k0 - 2; p <= k0 + 1; ++p) P2D_ISSUE_S(p, p - k0 + 2);
  // the look-ahead S planes whose ring slots are clear of the prologue's, and the J
  // planes, go out before the prologue's wait (p2d_dspre): a tile then starts after
  // one memory latency, not two
  // (the J groups the prologue issues: none for J = 0 and the register-row passes, which
  // have no J ring -- as p2d_after's replay skips them)
  constexpr int DSPRE = p2d_dspre(J, KA), PJ = (J == 0 || JREG) ? 0 : (LATE ? 1 : (RF ? NP : NP - 1));
#pragma unroll
  for (int d = 0; d < DSPRE; ++d) P2D_ISSUE_S(k0 + 2 + d, (4 + d) % NSL);
  if constexpr (DSPRE > 0) {
    if constexpr (LATE) {
      P2D_ISSUE_J(k0, 0);
    } else if constexpr (J > 0) {
#pragma unroll
      for (int d = 0; d < PJ; ++d) P2D_ISSUE_J(k0 + d, d);
    }
  }
  wait_vm<DSPRE * p2d_nsd(KA) + (DSPRE > 0 ? PJ * J : 0)>();
  raw_barrier();
  cplx lq0, lq1, le1 = {0.0, 0.0};  // L S_J of planes k-1 and k (own row), (!EXT1) halo values of plane k
  P2D_LAP(lq0, k0 - 1, w + 2, 0, 1, 2, x, lane, mi, pi, 0);
  // A: c of the own cell at plane k-1 (its slot is reused before L^2 S_J of plane k needs it)
  double cq0 = 0.0, cq0b = 0.0;  // (pairs: cells a, b)
  if constexpr (AK == 1 && HZ) cq0 = P2D_CV(1, w + 2, lane);
  if constexpr (AK == 2 && HZ) {
    cq0 = P2D_CV2(1, w + 2, lane, 0);
    cq0b = P2D_CV2(1, w + 2, lane, 1);
  }
  P2D_LROWS(k0, 1, 2, 3, 0, lq1, le1);
  if constexpr (WC) {
#pragma unroll
    for (int q = 0; q < NWC; ++q) cwc[q] = nwc[q];
  }
  raw_barrier();  // L ring slot 0 published; every wave is done with S slot 0 (plane k0-2)
#pragma unroll
  for (int d = DSPRE; d < DS; ++d) P2D_ISSUE_S(k0 + 2 + d, (4 + d) % NSL);
  if constexpr (DSPRE == 0) {
    if constexpr (LATE) {
      P2D_ISSUE_J(k0, 0);
    } else if constexpr (J > 0) {
#pragma unroll
      for (int d = 0; d < PJ; ++d) P2D_ISSUE_J(k0 + d, d);
    }
  }
  // ring slots as running counters (no divisions in the loop)
  int sk = 2;                  // S slot of plane k (k+1, k+2 follow cyclically)
  int sis = (DS + 4) % NSL;    // S slot of the next issued plane k+DS+2
  int jr = 0;                  // J slot of plane k
  int jis = NP > 0 ? NP - 1 : 0;  // J slot of the next issued plane k+NP-1
  int lsl = 0;                 // L ring slot of plane k

  // JREG: this lane's cell of plane k in the stored vectors (a ragged tile's extra lanes
  // read the row's last cell)
  const cplx *__restrict__ jrow = W + ((int64_t)y * nx + x0 + src_lane);
  cplx svn[JPF ? J : 1];  // JPF: plane k+1's J rows, loaded one step ahead
  // byte offsets of the planes the step issues: S plane k+DS+2, J plane min(k+NP-1, k1-1)
  int64_t sob = (int64_t)(k0 + DS + 2) * P16;
  int64_t job = (int64_t)min(k0 + NP - 1, k1 - 1) * P16;
  if constexpr (JPF) {
    const cplx *__restrict__ src = jrow + (int64_t)k0 * P;
#pragma unroll
    for (int l = 0; l < J; ++l) svn[l] = ld_nt(src + (int64_t)l * vs);
  }
  for (int k = k0; k < k1; ++k) {
    const int i = k - k0;
    cplx sv[J + 1];
    if constexpr (JPF) {
#pragma unroll
      for (int l = 0; l < J; ++l) sv[l] = svn[l];
      const cplx *__restrict__ src = jrow + (int64_t)min(k + 1, k1 - 1) * P;
#pragma unroll
      for (int l = 0; l < J; ++l) svn[l] = ld_nt(src + (int64_t)l * vs);
    } else if constexpr (JREG) {
      const cplx *__restrict__ src = jrow + (int64_t)k * P;
#pragma unroll
      for (int l = 0; l < J; ++l) sv[l] = ld_nt(src + (int64_t)l * vs);
    }
    // NLS_P2D_EARLY: issue first (the slots are free: S plane k-2 since the last
    // barrier, the wave's own J plane k-1 since its last step), then wait
    if constexpr (p2d_early(J, KA)) {
      P2D_ISSUE_SO(k + DS + 2, sob, sis);
      if constexpr (J > 0 && !LATE && !JREG && !RF) P2D_ISSUE_JO(job, jis);
    }
    wait_step<J, STW, KA>(i);
    raw_barrier();
    if constexpr (!p2d_early(J, KA)) {
      P2D_ISSUE_SO(k + DS + 2, sob, sis);
      if constexpr (J > 0 && !LATE && !JREG && !RF) P2D_ISSUE_JO(job, jis);
    }
    const int s1 = sk + 1 == NSL ? 0 : sk + 1, s2 = s1 + 1 == NSL ? 0 : s1 + 1;
    // L S_J of plane k+1: own row (register) + halo values, shared rows into L slot lsl^1
    cplx ln, lne = {0.0, 0.0};
    P2D_LROWS(k + 1, sk, s1, s2, lsl ^ 1, ln, lne);
    // the J stored vectors of this cell and S_J itself
    if constexpr (J > 0 && !JREG) {
      const cplx *jv = reinterpret_cast<const cplx *>(smem + p2d_off_j(J, KA) + ((jr * J) * P2D_TR + w) * 1024);
#pragma unroll
      for (int l = 0; l < J; ++l) sv[l] = jv[l * P2D_TR * 64 + lane];
      if constexpr (LATE) {
        // the rows are in registers: the slot takes plane k+1 (one step of look-ahead)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        P2D_ISSUE_J(k + 1, 0);
      }
    }
    sv[J] = Sr[(sk * P2D_SR + w + 2) * RW + lane];
    const cplx l1 = lq1;
    // X (and Z) as two partial sums: shorter dependent FMA chains
    cplx Xa = cmul(bX1, l1), Xb = {0.0, 0.0};
#pragma unroll
    for (int l = 0; l <= J; ++l) cmac((l & 1) ? Xb : Xa, RCOEF ? rcX[l] : cX[l], sv[l]);
    const cplx X = Xa + Xb;
    cplx Z = {0.0, 0.0};
    if constexpr (HZ) {
      // x neighbours: lanes i-1 / i+1 by DPP, the tile-edge ones from the halo values
      // (EXT1: Lx of the wave's row; else x0-1 on lane 0 of le1, x0+64 on its lane 1)
      cplx xm = lane_prev(l1), xp = lane_next(l1);
      if constexpr (EXT1) {
        const cplx hm = Lx[lsl * 2 * P2D_TR + 2 * w], hp = Lx[lsl * 2 * P2D_TR + 2 * w + 1];
        if (lane == 0) xm = hm;
        if (lane == 63) xp = hp;
      } else {
        const cplx er = {__hiloint2double(__builtin_amdgcn_readlane(__double2hiint(le1.re), 1),
                                          __builtin_amdgcn_readlane(__double2loint(le1.re), 1)),
                         __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(le1.im), 1),
                                          __builtin_amdgcn_readlane(__double2loint(le1.im), 1))};
        if (lane == 0) xm = le1;
        if (lane == 63) xp = er;
      }
      const cplx ym = Lr[(lsl * P2D_LR + w) * 64 + lane], yp = Lr[(lsl * P2D_LR + w + 2) * 64 + lane];
      const cplx zz = D2 ? cplx{0.0, 0.0} : lq0 + ln;
      cplx l2;
      if constexpr (AK == 2 && WC) {
        l2.re = s * ((((cwc[7] * lq0.re + cwc[8] * ln.re) + (cwc[1] * xm.im + cwc[0] * l1.im)) +
                      (cwc[3] * ym.re + cwc[4] * yp.re)) - cwc[11] * l1.re);
        l2.im = s * ((((cwc[9] * lq0.im + cwc[10] * ln.im) + (cwc[0] * l1.re + cwc[2] * xp.re)) +
                      (cwc[5] * ym.im + cwc[6] * yp.im)) - cwc[12] * l1.im);
      } else if constexpr (A && WC) {
        l2 = s * ((((cwc[4] * lq0 + cwc[5] * ln) + (cwc[0] * xm + cwc[1] * xp)) + (cwc[2] * ym + cwc[3] * yp)) -
                  cwc[6] * l1);
      } else if constexpr (AK == 2) {
        // cell pairs: per cell as in LROWS (a's x - 1 is xm's b, b's x + 1 is xp's a),
        // z faces from c of planes k-1 (registers) and k+1
        const int gk = z0 + k;
        const double ca = P2D_CV2(sk, w + 2, lane, 0), cb = P2D_CV2(sk, w + 2, lane, 1);
        const double wab = 0.5 * (ca + cb);
        const double wam = p2d_face(x > 0, ca, P2D_CV2(sk, w + 2, mi, 1));
        const double wbp = p2d_face(x + 1 < nx, cb, P2D_CV2(sk, w + 2, pi, 0));
        const bool ymk = gk > 0 || y > 0, ypk = gk < nz - 1 || y < ny - 1;
        const double wyam = p2d_face(ymk, ca, P2D_CV2(sk, w + 1, lane, 0));
        const double wyap = p2d_face(ypk, ca, P2D_CV2(sk, w + 3, lane, 0));
        const double wybm = p2d_face(ymk, cb, P2D_CV2(sk, w + 1, lane, 1));
        const double wybp = p2d_face(ypk, cb, P2D_CV2(sk, w + 3, lane, 1));
        const double wzam = p2d_face(gk > 0, ca, cq0), wzbm = p2d_face(gk > 0, cb, cq0b);
        const double wzap = p2d_face(gk < nz - 1, ca, P2D_CV2(s1, w + 2, lane, 0));
        const double wzbp = p2d_face(gk < nz - 1, cb, P2D_CV2(s1, w + 2, lane, 1));
        l2.re = s * ((((wzam * lq0.re + wzap * ln.re) + (wam * xm.im + wab * l1.im)) + (wyam * ym.re + wyap * yp.re)) -
                     (((wzam + wzap) + (wam + wab)) + (wyam + wyap)) * l1.re);
        l2.im = s * ((((wzbm * lq0.im + wzbp * ln.im) + (wab * l1.re + wbp * xp.re)) + (wybm * ym.im + wybp * yp.im)) -
                     (((wzbm + wzbp) + (wab + wbp)) + (wybm + wybp)) * l1.im);
        cq0 = ca;
        cq0b = cb;
      } else if constexpr (A) {
        // the same operator at the same cell: c of the own row at planes k-1 (register),
        // k (x, y neighbours from the ring) and k+1
        const int gk = z0 + k;
        const double cc = P2D_CV(sk, w + 2, lane);
        const double wxm = p2d_face(x > 0, cc, P2D_CV(sk, w + 2, mi));
        const double wxp = p2d_face(x + 1 < nx, cc, P2D_CV(sk, w + 2, pi));
        const double wym = p2d_face(gk > 0 || y > 0, cc, P2D_CV(sk, w + 1, lane));
        const double wyp = p2d_face(gk < nz - 1 || y < ny - 1, cc, P2D_CV(sk, w + 3, lane));
        const double wzm = p2d_face(gk > 0, cc, cq0);
        const double wzp = p2d_face(gk < nz - 1, cc, P2D_CV(s1, w + 2, lane));
        l2 = s * ((((wzm * lq0 + wzp * ln) + (wxm * xm + wxp * xp)) + (wym * ym + wyp * yp)) -
                  (((wzm + wzp) + (wxm + wxp)) + (wym + wyp)) * l1);
        cq0 = cc;
      } else if constexpr (PR)
        l2 = pr_lap(l1, xm, xp, zz + (ym + yp), P2D_DIAGA(x, y, z0 + k), P2D_DIAGB(x, y, z0 + k), s);
      else
        l2 = P2D_DIAG(x, y, z0 + k) * l1 + s * ((zz + (xm + xp)) + (ym + yp));
      cplx Za = cmul(bZ2, l2) + cmul(bZ1, l1), Zb = {0.0, 0.0};
#pragma unroll
      for (int l = 0; l <= J; ++l) cmac((l & 1) ? Zb : Za, RCOEF ? rcZ[l] : cZ[l], sv[l]);
      Z = Za + Zb;
    }
    if constexpr (RF) {
      // plane k's J rows are consumed (X, Z): the slot takes plane k + NP
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      P2D_ISSUE_J(k + NP, jr);
    }
    // stores from every lane (a ragged last tile repeats its last valid lane's store)
    const int flat = k * P + y * nx + x0 + src_lane;
    if (full) {
      st_nt(Xo + flat, X);
      if constexpr (HZ) st_nt(Zo + flat, Z);
    } else {
      st_nt(Xo + flat, cplx{__shfl(X.re, src_lane, 64), __shfl(X.im, src_lane, 64)});
      if constexpr (HZ) st_nt(Zo + flat, cplx{__shfl(Z.re, src_lane, 64), __shfl(Z.im, src_lane, 64)});
    }
    if (xin) {
#pragma unroll
      for (int l = 0; l <= J; ++l) cjmac(acc[l], sv[l], X);
      if constexpr (HZ) {
#pragma unroll
        for (int l = 0; l <= J; ++l) cjmac(acc[J + 1 + l], sv[l], Z);
        acc[2 * J + 2].re = fma(X.re, X.re, fma(X.im, X.im, acc[2 * J + 2].re));
        cjmac(acc[2 * J + 3], X, Z);
        acc[2 * J + 4].re = fma(Z.re, Z.re, fma(Z.im, Z.im, acc[2 * J + 4].re));
      } else {
        acc[J + 1].re = fma(X.re, X.re, fma(X.im, X.im, acc[J + 1].re));
      }
      if constexpr (J == 0) acc[NC - 1].re = fma(sv[0].re, sv[0].re, fma(sv[0].im, sv[0].im, acc[NC - 1].re));
    }
    lq0 = lq1;
    lq1 = ln;
    if constexpr (WC) {
#pragma unroll
      for (int q = 0; q < NWC; ++q) cwc[q] = nwc[q];
    }
    le1 = lne;
    sk = s1;
    sis = sis + 1 == NSL ? 0 : sis + 1;
    sob += P16;
    if (k + NP < k1) job += P16;
    if constexpr (J > 0) {
      jr = jr + 1 == NPD ? 0 : jr + 1;
      jis = jis + 1 == NPD ? 0 : jis + 1;
    }
    lsl ^= 1;
  }
#undef P2D_PLANE
#undef P2D_ROW
#undef P2D_DIAG
#undef P2D_DIAGA
#undef P2D_DIAGB
#undef P2D_BYZ
#undef P2D_ISSUE_S
#undef P2D_ISSUE_J
#undef P2D_ISSUE_SO
#undef P2D_ISSUE_JO
#undef P2D_LAP
#undef P2D_CV
#undef P2D_CV2
#undef P2D_LROWS
  wait_vm<0>();  // the look-ahead DMAs land before the LDS is reused (and this wave's stores)
  raw_barrier();
  // Peer stores (multi-rank handles, NLS_PEER=1): the pass's last output -- the next
  // stencil vector -- of local planes 0, 1 straight into the neighbour below's upper
  // ghost planes (ps->pdn), of planes nzl-2, nzl-1 into the neighbour above's lower
  // ones (ps->pup): no exchange step and no boundary/interior split.  Read back from
  // this wave's own stores (complete after the wait above), after the march loop, so
  // the loop and its hand-counted vmcnt are untouched.  Ordering: inside a
  // step, the pass's all-reduce, which every rank joins after its pass, orders the stores
  // before the neighbour's next pass reads them.  The blind J = 0 pass that opens a step
  // has no all-reduce before it in that step: its stores into the neighbour's ghost planes
  // (with m = 3, 4 those of S_{m-2}, which the neighbour's previous tail reads) are ordered
  // after that tail by the per-step W_0 halo exchange (ss2_step's halo(h, 0, 0) after the
  // tail: the neighbour's send follows its tail, our J = 0 pass follows our receive).
  // tests/test_gpu_multirank.py checks m = 3, 4 over several steps bit for bit against
  // the exchange path.
  // (a separate instantiation: the epilogue's live values cost the plain pass's march
  // loop ~20 instructions per step at J = 12)
  if (PEER && (k0 < 2 || k1 > nzl - 2)) {  // uniform: a tile holding a boundary plane
    constexpr int OUT = J + (HZ ? 2 : 1);
    cplx *const tdn = static_cast<cplx *>(ps->pdn[OUT]), *const tup = static_cast<cplx *>(ps->pup[OUT]);
    const cplx *__restrict__ ov = HZ ? Zo : Xo;
    const int64_t ro = (int64_t)y * nx + x0 + src_lane;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kk = e < 2 ? e : nzl - 4 + e;
      cplx *dst = e < 2 ? tdn : tup;
      if (dst && kk >= k0 && kk < k1) {
        // a global (not flat) store: the table's pointers are generic
        typedef double __attribute__((ext_vector_type(2))) d2v;
        const cplx v = ld_nt(ov + (int64_t)kk * P + ro);
        __attribute__((address_space(1))) d2v *gp =
            (__attribute__((address_space(1))) d2v *)(dst + (int64_t)(e & 1) * P + ro);
        __builtin_nontemporal_store(d2v{v.re, v.im}, gp);
      }
    }
  }
  cplx *red = reinterpret_cast<cplx *>(smem);  // [4][NC]
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const double a = wave_sum(acc[c].re), bb = wave_sum(acc[c].im);
    if (lane == 0) red[w * NC + c] = {a, bb};
  }
  __syncthreads();
  for (int c = t; c < NC; c += NTHREADS) {
    cplx v = red[c];
#pragma unroll
    for (int q = 1; q < P2D_TR; ++q) v += red[q * NC + c];
    part[(int64_t)c * nb + poff + blockIdx.x] = v;
  }
}

#ifndef NLS_NO_P2_KERNELS
// ---- fused tail of the two-vector scheme ----------------------------------
// After the last basis pass the stored vectors are S_0..S_j (j = m-2) with
// W = S C orthonormal and the H columns < j known.  One k_alpha_l2 pass over
// S_j reduces a = S_j^H L S_j and l2 = ||L S_j||^2 (sums[0], sums[2]); with
// y = L S_j and D = C^-1 (ps->D):
//   t_k = W_k^H y = sum_i conj(H[i][k]) D[i][j]        (k < j)
//   t_j = conj(C_jj) (a - sum_{i<j} conj(D[i][j]) t_i)
//   lw  = -C_jj H[:, :j] D[:j, j]        (L W_j = C_jj y + sum_k lw_k W_k)
//   alpha_j = C_jj t_j + lw_j,  beta_{j+1} = |C_jj| sqrt(l2 - sum_k |t_k|^2)
//   W_{j+1} = C_jj (y - sum_k t_k W_k) / beta_{j+1}
// (tests/sstep_model.py tail_coefficients; 20-step trajectories at the
// headline stiffness within 1e-14 of the MGS oracle).  k_p2tail completes T
// (s[] = 1: k_reduce_final's fin is then f(T) e_1 in the W basis) and keeps
// t, beta in the P2State; k_p2tfin maps fin to the coefficients k_tail reads:
// fin'[k] over the stored S_k (k <= j), fin'[j+1] for y, coef = e_{j+1}.
__device__ __forceinline__ void p2tail_body(P2State *__restrict__ ps, KState *__restrict__ st,
                                            const cplx *__restrict__ sums, int m) {
  __shared__ cplx tk[P2M];
  const int j = m - 2, t = threadIdx.x;
  for (int k = t; k < j; k += NTHREADS) {
    cplx v = {0.0, 0.0};
    for (int i = 0; i <= k + 1 && i <= j; ++i) v += cj_mul(ps->H[i][k], ps->D[i][j]);
    tk[k] = v;
  }
  __syncthreads();
  if (t == 0) {
    const cplx cjj = ps->C[j][j];
    cplx r = sums[0];
    for (int i = 0; i < j; ++i) r = r - cj_mul(ps->D[i][j], tk[i]);
    const cplx tj = cj_mul(cjj, r);
    tk[j] = tj;
    cplx lwj = {0.0, 0.0};
    for (int i = (j > 0 ? j - 1 : 0); i < j; ++i) lwj += cmul(ps->H[j][i], ps->D[i][j]);
    lwj = cmul(cjj, lwj);
    const double alpha = cmul(cjj, tj).re - lwj.re;
    double n2 = sums[2].re;
    for (int k = 0; k <= j; ++k) n2 -= abs2(tk[k]);
    const double b = sqrt(abs2(cjj)) * (n2 > 0.0 ? sqrt(n2) : 0.0);
    ps->beta_t = b;
    st->Td[j] = alpha;
    st->To[j] = b;
    if (!(b > 0.0) && st->breakdown == 0) st->breakdown = m;
  }
  __syncthreads();
  for (int k = t; k <= j; k += NTHREADS) ps->tk[k] = tk[k];
  if (t < MMAX) {
    if (t < j) {
      st->Td[t] = ps->H[t][t].re;
      st->To[t] = ps->H[t + 1][t].re;
    }
    st->s[t] = 1.0;
  }
}
__global__ __launch_bounds__(NTHREADS) void k_p2tail(P2State *__restrict__ ps, KState *__restrict__ st,
                                                     const cplx *__restrict__ sums, int m) {
  p2tail_body(ps, st, sums, m);
}

__device__ __forceinline__ void p2tfin_body(const P2State *__restrict__ ps, KState *__restrict__ st, int m, int nf) {
  __shared__ cplx fw[2][MMAX];
  const int j = m - 2, t = threadIdx.x;
  for (int e = t; e < nf * m; e += NTHREADS) fw[e / m][e % m] = st->fin[e / m][e % m];
  __syncthreads();
  const cplx cjj = ps->C[j][j];
  const double b = ps->beta_t, ib = b > 0.0 ? 1.0 / b : 0.0;
  for (int e = t; e < nf * (j + 2); e += NTHREADS) {
    const int f = e / (j + 2), l = e % (j + 2);
    const cplx cl = fw[f][j + 1];  // coefficient of W_{j+1}
    const cplx g = ib * cmul(cl, cjj);
    cplx v = {0.0, 0.0};
    if (l <= j) {
      // sum_{k >= l} C[l][k] (fin_k - g t_k)
      for (int k = l; k <= j; ++k) v += cmul(ps->C[l][k], fw[f][k] - cmul(g, ps->tk[k]));
    } else {
      v = g;
    }
    st->fin[f][l] = ps->beta * v;
  }
  for (int l = t; l <= j + 1; l += NTHREADS) st->coef[l] = {l == j + 1 ? 1.0 : 0.0, 0.0};
}
__global__ __launch_bounds__(NTHREADS) void k_p2tfin(const P2State *__restrict__ ps,
                                                     KState *__restrict__ st, int m, int nf) {
  p2tfin_body(ps, st, m, nf);
}

#endif  // NLS_NO_P2_KERNELS

}  // namespace nls
