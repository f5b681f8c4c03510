// nls_api.cpp -- host side of libnls_amd.so: the C-ABI of include/nls.h.
//
// A handle owns one HIP stream, the Krylov bases in HBM, the device-resident
// Lanczos state and (nranks > 1) an RCCL communicator.  A time step is a
// fixed sequence of launches on that stream with no host synchronisation
// (the reference synchronises on every dot product: host-pointer-mode cuBLAS
// in device/lanczos_complex.hpp:413-500 and a D2H of T per dot in
// device/lanczos.hpp:126-194).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <deque>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "nls.h"
#include "nls_device.hpp"
#include "nls_kernels.hpp"

#ifndef NLS_VPAD
#define NLS_VPAD 8192  // stride pad of a stored vector, elements (see the default's note in nls_create)
#endif
#ifndef NLS_KZ_L2
#define NLS_KZ_L2 32  // tile depth of k_alpha_l2 (with NLS_RB_L2 rows per thread, nls_stencil.hpp)
#endif

using namespace nls;

namespace {

thread_local std::string g_create_error;

struct Basis {
  void *W = nullptr;      // m vectors x vs elements (ghost plane, nzl planes, ghost plane)
  KState *st = nullptr;   // device-resident Lanczos state
};

struct TimingRec {
  int cls, j;
  hipEvent_t a, b;
};

struct Fail {
  int code;
};

// Launches of one update pass: a single full-slab launch, or (collective
// handles) the two boundary planes first and the interior after, so the halo
// exchange of the new vector overlaps the interior launch.  All launches write
// one column-major partial array (stride = total blocks).
struct UpdPlan {
  int n = 0;
  int qa[3] = {}, qb[3] = {}, grid[3] = {}, off[3] = {};
  int total = 0;
  int nbnd = 0;  // the first nbnd launches cover the boundary planes
};

constexpr int NSUM = 2 * MMAX + 8;  // cplx words of KState::sums
#ifndef NLS_KG_CONCURRENT
#define NLS_KG_CONCURRENT 1  // the two Klein-Gordon bases / sEWI's third action on two streams (one rank, s-step passes)
#endif
constexpr int EVRING = 8;            // events per handle for the local transport

}  // namespace

// In-process rank group (local transport): a host-side rendezvous per exchange
// plus device buffers for the fixed-order all-reduce.
struct nls_group {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  int arrived = 0;
  bool aborted = false;
  std::vector<std::vector<uint64_t>> slots, done;
  cplx *pub = nullptr;  // [rank][parity][NSUM]
  int dev = -1;
};

struct nls_handle {
  nls_config cfg{};
  int dev = 0;
  hipStream_t stream = nullptr;
  bool cplx_ = true;
  size_t esize = 16;
  Geo geo{};
  int ghost = 1;   // ghost planes per side of a stored vector: 2 on two-vector handles
  int64_t vpad = 4096;  // stride pad of a stored vector (elements)
  int64_t vs = 0;  // elements per stored vector (incl. 2 x ghost planes and the pad)
  int m = 10;
  int nbasis = 1;
  Basis B[2];
  void *u = nullptr;        // NLSE state u (nloc complex)
  double *up = nullptr;     // SG u_past
  double *mf = nullptr;     // SG m(x), G2 NLSE focusing field m(x)
  double *cfb = nullptr;    // G2 anisotropy c(x): nzl + 2 ghost planes, local plane 0 at +ghost P
  bool ani = false;         // G2 operator div(c grad) (laplacians.hpp:54-218)
  bool kg = false;          // G2 Klein-Gordon Gautschi (real, ani)
  int gfun = -1;            // G2 Gautschi family (NLS_SG_G2 .. NLS_PHI4): GautschiForce; -1 G1 sine-Gordon
  double *vel = nullptr;    // KG velocity v = (u - u_past)/dt of the last step
  bool vel_valid = false;   //   (set by every KG step, before the driver's BC)
  int nvec[2] = {0, 0};     // vectors stored per basis (m, or m - 1 with a fused tail)
  void *uprev = nullptr;    // G2 sEWI: u of the previous step (nlse_dev.hpp:206-229)
  bool uprev_set = false;
  bool coef_set = false;
  void *scratch = nullptr;  // nloc elements
  cplx *partA = nullptr, *partU = nullptr;
  int grid_alpha = 1, grid_lap = 1, grid_pw = 1;
  int kz_alpha = 4;
  // fused tail (m >= 3): the last update pass of a basis and the combination
  // that ends the step are one pass, k_tail (NLS_FUSED_TAIL=0 disables)
  bool fused_tail = false;
  // two new Lanczos vectors per basis pass (nls_pass2.hpp, nls_pass2d.hpp; 3D isotropic
  // NLSE, one rank), ending in the fused tail k_tail over the stored S vectors
  bool pass2 = false;
  void *p2 = nullptr;          // P2State
  cplx *partP2 = nullptr;      // per-workgroup partials of the pass
  int p2grid = 0, p2kz = 32;
  int p2kzj = 32;              // tile depth of the register-row passes (pass2_jreg)
  int p2kz0 = 64;              // tile depth cap of the 3D J = 0 pass (NLS_P2_KZ0)
  bool p2_d2 = false;          // 2D grid seen as planes of 4 rows by k_p2d (p2_geo)
  bool p2_split_on = true;     // collective handles: boundary/interior split (NLS_P2_SPLIT=0: off)
  cplx *zbuf = nullptr;        // one zero row (nx cells): the DMA source of out-of-grid rows
  // register form of the two-vector pass (k_lap + k_p2m, nls_pass2g.hpp): the G2
  // anisotropic NLSE and the isotropic shapes k_p2d does not take
  bool p2reg = false;
  cplx *p2gbuf = nullptr;      // L S_J at local planes [-1, nzl] (nzl + 2 planes)
  int p2mgrid[MMAX] = {};      // k_p2m grid per J
  int p2lapgrid = 0;           // k_lap grid over planes [-1, nzl]
  int p2mkz = 16;              // tile depth of k_lap / k_p2m (G2 256^3 m=25: 13.36 ms/step vs 13.76 at 32)
  bool p2_blind = true;        // J = 0 pass without an alpha pass once warm
  bool large = false;          // large-slab launch shapes (setup_geometry)
  // Klein-Gordon s-step passes on one rank: the sinc^2 basis of g runs on stream2,
  // concurrently with the cos basis of u on stream (their own partial buffers), joined
  // before the Gautschi tail (kg_concurrent)
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  cplx *partP2b = nullptr, *partAb = nullptr;
  void *prepad = nullptr;  // NLS_DEBUG_PREPAD_KB: a dummy allocation ahead of the bases (placement probe)
  // basis placement (place_basis, DESIGN.md section 4 "Placement"): candidate allocations
  // probed at nls_create, the fastest kept; place_ms[i] = probe time of candidate i
  int place_n = 0, place_pick = -1;
  float place_ms[NLS_PLACE_MAX] = {};
  bool sewi_serial = false;  // the second sEWI basis could not be allocated
  int p2order = 0;             // k_p2d tile order (Geo::remap bits: 2 x-fastest, 4 no XCD bands; debug knob 3)
  bool p2_warm[2] = {false, false};  // the basis' P2State holds a previous alpha_0
  // a new state was set (nls_set_*): the next step starts its bases cold, so it is
  // issued eagerly, never replayed from a graph captured warm (run-to-run bitwise
  // reproducibility of "set state; step" sequences)
  bool p2_fresh = true;
  bool p2_pr = false;          // real field marched as cell pairs by k_p2d (p2_geo)
  bool p2_ani = false;         // k_p2d with the G2 operator (nls_pass2a.hip)
  int grid_alpha2 = 1, kz_alpha2 = NLS_KZ_L2, kz_fused = 0;  // kz_fused 0: geo.kz
  bool l2pipe = false;  // 3D k_alpha_l2 through the pipelined march (small slabs; NLS_L2_PIPE=0/1 forces)
  int tail_grid[TAIL_NMODES] = {};  // per TailMode; 0: no such kernel (unfused path)
  int tail_dyn_grid[TAIL_NMODES] = {};  // resident workgroups of each tail kernel (dynamic tile queue)
  bool tail_dyn = false;      // fused tail through the dynamic tile queue (debug knob 1)
  bool tail_one_tile = false; // one tile per workgroup for the static tail grids
  int32_t *tailq = nullptr;   // its counters (Geo::tq)
  // folded alpha (single-rank handles): update pass j also reduces q = y^H L y and
  // the alpha pass j+1 is skipped (march_q; NLS_FUSED_ALPHA=0 disables)
  bool fused_alpha = false;
  int qgrid[MMAX] = {};  // grid of k_update<j, QA>
  void *xedge = nullptr;    // x-tile seam values of L W_j (folded alpha, k_xpairs)
  cplx *partX = nullptr;    // k_xpairs partials (xgrid of them)
  int xgrid = 1024;  // 4 per CU: the seam pairs (~60 MB at 512^3) at full bandwidth, few partials
  UpdPlan plan[MMAX];
  bool field_set = false, w0_ready = false;
  double w0_dt = 0.0;  // dt the live start vector W_0 = N(u) was built with
  int nonlin = 0;
  cplx s1{0.0, 0.5}, s2{-0.5, 0.0};
  std::string err;
  // timing
  bool timing = false;
  std::vector<TimingRec> recs;
  std::vector<hipEvent_t> evpool;
  nls_timing tacc{};
  // multi-rank
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  nls_group *group = nullptr;  // local transport when non-NULL
  bool collective = false;     // split reductions + exchanges (nranks > 1, or NLS_FORCE_RCCL=1)
  hipEvent_t evring[EVRING] = {};
  uint64_t evnext = 0, ar_count = 0;
  // halo/compute overlap (collective handles): exchange on cstream
  hipStream_t cstream = nullptr;
  hipEvent_t ev_bnd = nullptr, ev_halo = nullptr, ev_bdone = nullptr;
  bool halo_pending = false;
  bool bnd_side = true;  // boundary-plane launches on cstream
  // peer stores (NLS_PEER=1): k_p2d writes each pass's next stencil
  // vector's boundary planes straight into the neighbours' ghost planes -- no exchange
  // step, no split.  peer_W[side][b]: allocation base of basis b of the neighbour below
  // (side 0) / above (side 1), nullptr where there is none; a 1-rank handle points both
  // at itself (its out-of-grid ghost planes: a cost probe that changes no result)
  bool peer = false, peer_ready = false, peer_ipc = false;
  bool peer_fallback = false;  // NLS_PEER=1 asked, an IPC open failed on some rank: exchange path
  char *peer_W[2][2] = {};
  int64_t peer_vs[2] = {}, peer_nzl[2] = {};
  // debug (NLS_OPLOG=1 at nls_create): the transport operations in issue order, with
  // the cross-stream waits between them (nls_debug_oplog; tests/test_gpu_oplog.py)
  bool oplog_on = false;
  std::deque<std::array<int32_t, 4>> oplog;  // {kind, stream, count, peer} per entry (nls.h NLS_OP_*)
  // debug switches read once at nls_create (never on the per-reduction path)
  bool dbg_sums = false, dbg_alpha = false;
  // asynchronous snapshots: staging copy on the compute stream, D2H on xstream
  hipStream_t xstream = nullptr;
  hipEvent_t ev_snap = nullptr, ev_snap_done = nullptr;
  void *snap = nullptr;
  bool snap_issued = false;
  // hipGraph replay of steady-state steps (single-rank handles): one graph
  // launch per step instead of ~3m kernel launches; keyed by dt
  bool use_graph = false;
  bool skip_u = false;         // the next NLSE tail may skip its u store (another step follows)
  hipGraphExec_t gexec = nullptr;
  double gdt = 0.0;
};

namespace {

void hip_check(nls_handle *h, hipError_t e, const char *what) {
  if (e != hipSuccess) {
    h->err = std::string(what) + ": " + hipGetErrorString(e);
    throw Fail{e == hipErrorOutOfMemory ? NLS_ERR_OOM : NLS_ERR_HIP};
  }
}

void rccl_check(nls_handle *h, ncclResult_t e, const char *what) {
  if (e != ncclSuccess) {
    h->err = std::string(what) + ": " + ncclGetErrorString(e);
    throw Fail{NLS_ERR_RCCL};
  }
}

template <class F> int guarded(nls_handle *h, F &&f) {
  if (!h) return NLS_ERR_ARG;
  try {
    hip_check(h, hipSetDevice(h->dev), "hipSetDevice");
    f();
    return NLS_OK;
  } catch (const Fail &e) {
    return e.code;
  } catch (const std::bad_alloc &) {
    h->err = "host allocation failed";
    return NLS_ERR_OOM;
  } catch (...) {
    h->err = "unknown error";
    return NLS_ERR_HIP;
  }
}

void fail(nls_handle *h, int code, const std::string &msg) {
  h->err = msg;
  throw Fail{code};
}

// Basis vectors carry h->ghost ghost planes below and above the slab: one for the
// radius-1 stencils of the one-vector passes, two (P2D_GHOST) for the radius-2
// march of the two-vector passes (k_p2d).  The 32-bit index check at nls_create
// assumes the larger (GHOST_MAX).
constexpr int GHOST_MAX = 2;  // == P2D_GHOST (nls_pass2d.hpp)
char *vec_ptr(nls_handle *h, int b, int k) {  // local plane 0 of vector k of basis b
  return static_cast<char *>(h->B[b].W) + ((int64_t)k * h->vs + h->ghost * h->geo.P) * (int64_t)h->esize;
}

// debug op log (NLS_OPLOG=1): transport operations and cross-stream waits in issue order
void oplog(nls_handle *h, int kind, int stream, int64_t count, int peer) {
  // bounded (NLS_OPLOG_MAX entries): a long run with the log on keeps the newest ones,
  // and a leading NLS_OP_DROPPED entry counts the entries that went (a truncated log is
  // never mistaken for a complete one by the ordering checks)
  if (!h->oplog_on) return;
  if (h->oplog.size() >= (size_t)NLS_OPLOG_MAX) {
    int64_t dropped = 0;
    if (h->oplog.front()[0] == NLS_OP_DROPPED) {
      dropped = h->oplog.front()[2];
      h->oplog.pop_front();
    }
    for (; h->oplog.size() + 2 > (size_t)NLS_OPLOG_MAX; ++dropped) h->oplog.pop_front();  // room: marker + new
    h->oplog.push_front({NLS_OP_DROPPED, 0, (int32_t)std::min<int64_t>(dropped, INT32_MAX), -1});
  }
  h->oplog.push_back({(int32_t)kind, (int32_t)stream, (int32_t)count, (int32_t)peer});
}
int stream_id(const nls_handle *h, hipStream_t st) { return st && st == h->cstream ? 1 : 0; }
// the halo stream (cstream) waits for the work enqueued so far on the compute stream
void halo_after_compute(nls_handle *h) {
  hip_check(h, hipEventRecord(h->ev_bnd, h->stream), "hipEventRecord");
  hip_check(h, hipStreamWaitEvent(h->cstream, h->ev_bnd, 0), "hipStreamWaitEvent");
  oplog(h, NLS_OP_WAIT_COMPUTE, 1, 0, -1);
}

hipEvent_t get_event(nls_handle *h) {
  if (!h->evpool.empty()) {
    hipEvent_t e = h->evpool.back();
    h->evpool.pop_back();
    return e;
  }
  hipEvent_t e;
  hip_check(h, hipEventCreate(&e), "hipEventCreate");
  return e;
}

void harvest_timing(nls_handle *h) {
  if (h->recs.empty()) return;
  hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  if (h->stream2) hip_check(h, hipStreamSynchronize(h->stream2), "hipStreamSynchronize");  // (KG's second basis)
  for (auto &r : h->recs) {
    float ms = 0.f;
    hip_check(h, hipEventElapsedTime(&ms, r.a, r.b), "hipEventElapsedTime");
    h->tacc.class_ms[r.cls] += ms;
    h->tacc.class_count[r.cls] += 1;
    if (r.cls == 1 && r.j >= 0 && r.j < NLS_MAX_KRYLOV) {
      h->tacc.update_ms[r.j] += ms;
      h->tacc.update_count[r.j] += 1;
    }
    h->evpool.push_back(r.a);
    h->evpool.push_back(r.b);
  }
  h->recs.clear();
}

void launch(nls_handle *h, int cls, int j, const void *fn, int grid, void **args,
            hipStream_t stream = nullptr, int block = NTHREADS) {
  if (!fn) fail(h, NLS_ERR_ARG, "kernel variant not instantiated");
  if (!stream) stream = h->stream;
  TimingRec rec{cls, j, nullptr, nullptr};
  if (h->timing) {
    if (h->recs.size() >= 4096) harvest_timing(h);
    rec.a = get_event(h);
    rec.b = get_event(h);
    hip_check(h, hipEventRecord(rec.a, stream), "hipEventRecord");
  }
  hip_check(h, hipLaunchKernel(fn, dim3(grid), dim3(block), args, 0, stream),
            "hipLaunchKernel");
  if (h->timing) {
    hip_check(h, hipEventRecord(rec.b, stream), "hipEventRecord");
    h->recs.push_back(rec);
  }
}

// ---- multi-rank plumbing ---------------------------------------------------

// Host rendezvous of the local transport: every rank deposits a payload, the
// last arrival publishes the round; bounded wait (a failed rank aborts all).
std::vector<std::vector<uint64_t>> rendezvous(nls_handle *h, std::vector<uint64_t> payload) {
  nls_group *g = h->group;
  std::unique_lock<std::mutex> lk(g->mu);
  if (g->aborted) fail(h, NLS_ERR_RCCL, "local group aborted by another rank");
  const uint64_t my_gen = g->gen;
  g->slots[h->rank] = std::move(payload);
  if (++g->arrived == g->n) {
    g->done = g->slots;
    g->arrived = 0;
    ++g->gen;
    g->cv.notify_all();
  } else if (!g->cv.wait_for(lk, std::chrono::seconds(300),
                             [&] { return g->gen != my_gen || g->aborted; })) {
    g->aborted = true;
    g->cv.notify_all();
    fail(h, NLS_ERR_RCCL, "local group rendezvous timed out");
  }
  if (g->aborted) fail(h, NLS_ERR_RCCL, "local group aborted by another rank");
  return g->done;
}

hipEvent_t next_event(nls_handle *h) { return h->evring[h->evnext++ % EVRING]; }

void halo_local(nls_handle *h, hipStream_t st, char *first, char *last, char *gbelow, char *gabove,
                size_t bytes) {
  hipEvent_t ev = next_event(h);
  hip_check(h, hipEventRecord(ev, st), "hipEventRecord");
  auto all = rendezvous(h, {(uint64_t)(uintptr_t)first, (uint64_t)(uintptr_t)last,
                            (uint64_t)(uintptr_t)ev});
  if (h->rank > 0) {
    const auto &nb = all[h->rank - 1];
    hip_check(h, hipStreamWaitEvent(st, (hipEvent_t)(uintptr_t)nb[2], 0), "hipStreamWaitEvent");
    hip_check(h, hipMemcpyAsync(gbelow, (const void *)(uintptr_t)nb[1], bytes, hipMemcpyDeviceToDevice,
                                st), "hipMemcpyAsync(halo)");
  }
  if (h->rank < h->nranks - 1) {
    const auto &nb = all[h->rank + 1];
    hip_check(h, hipStreamWaitEvent(st, (hipEvent_t)(uintptr_t)nb[2], 0), "hipStreamWaitEvent");
    hip_check(h, hipMemcpyAsync(gabove, (const void *)(uintptr_t)nb[0], bytes, hipMemcpyDeviceToDevice,
                                st), "hipMemcpyAsync(halo)");
  }
}

// Exchange the np boundary planes of a slab-stored array (local plane 0 at v,
// ghost planes at -np*P .. -P and nzl*P ..) into the neighbours' ghost planes
// (z-slab decomposition; one plane covers the 3D y-wrap of a radius-1 stencil,
// the two-vector passes' radius-2 march needs two).
void halo_planes(nls_handle *h, char *v, int64_t es, hipStream_t st = nullptr, int np = 1) {
  if (!h->collective) return;
  if (!st) st = h->stream;
  const int64_t P = h->geo.P;
  const size_t cnt = (size_t)P * (size_t)(es / 8) * (size_t)np;
  char *first = v, *last = v + (h->geo.nzl - np) * P * es;
  char *gbelow = v - np * P * es, *gabove = v + h->geo.nzl * P * es;
  TimingRec rec{4, -1, nullptr, nullptr};
  if (h->timing) {
    rec.a = get_event(h);
    rec.b = get_event(h);
    hip_check(h, hipEventRecord(rec.a, st), "hipEventRecord");
  }
  const int sid = stream_id(h, st);
  if (h->rank > 0) {
    oplog(h, NLS_OP_SEND, sid, (int64_t)cnt, h->rank - 1);
    oplog(h, NLS_OP_RECV, sid, (int64_t)cnt, h->rank - 1);
  }
  if (h->rank < h->nranks - 1) {
    oplog(h, NLS_OP_SEND, sid, (int64_t)cnt, h->rank + 1);
    oplog(h, NLS_OP_RECV, sid, (int64_t)cnt, h->rank + 1);
  }
  if (h->group) {
    halo_local(h, st, first, last, gbelow, gabove, (size_t)P * es * np);
    if (h->timing) {
      hip_check(h, hipEventRecord(rec.b, st), "hipEventRecord");
      h->recs.push_back(rec);
    }
    return;
  }
  rccl_check(h, ncclGroupStart(), "ncclGroupStart");
  if (h->rank > 0) {
    rccl_check(h, ncclSend(first, cnt, ncclDouble, h->rank - 1, h->comm, st), "ncclSend");
    rccl_check(h, ncclRecv(gbelow, cnt, ncclDouble, h->rank - 1, h->comm, st), "ncclRecv");
  }
  if (h->rank < h->nranks - 1) {
    rccl_check(h, ncclSend(last, cnt, ncclDouble, h->rank + 1, h->comm, st), "ncclSend");
    rccl_check(h, ncclRecv(gabove, cnt, ncclDouble, h->rank + 1, h->comm, st), "ncclRecv");
  }
  rccl_check(h, ncclGroupEnd(), "ncclGroupEnd");
  if (h->timing) {
    hip_check(h, hipEventRecord(rec.b, st), "hipEventRecord");
    h->recs.push_back(rec);
  }
}

// ---- peer stores (NLS_PEER=1) ------------------------------------------------

// The neighbours' basis allocations, once per handle (they never move): over the local
// group's rendezvous (plain device pointers: the ranks share the device), or for RCCL
// ranks by an all-gather of IPC handles (hipIpcOpenMemHandle maps the neighbour's HBM
// over xGMI); a 1-rank handle points at itself.
struct PeerMsg {
  hipIpcMemHandle_t hd[2];
  int64_t vs, nzl;
};
void peer_close(nls_handle *h);
void peer_setup(nls_handle *h) {
  if (h->peer_ready) return;
  if (h->nranks == 1) {
    for (int side = 0; side < 2; ++side) {
      for (int b = 0; b < h->nbasis; ++b) h->peer_W[side][b] = static_cast<char *>(h->B[b].W);
      h->peer_vs[side] = h->vs;
      h->peer_nzl[side] = h->geo.nzl;
    }
  } else if (h->group) {
    auto all = rendezvous(h, {(uint64_t)(uintptr_t)h->B[0].W, (uint64_t)(uintptr_t)h->B[1].W, (uint64_t)h->vs,
                              (uint64_t)h->geo.nzl});
    for (int side = 0; side < 2; ++side) {
      const int nb = h->rank + (side ? 1 : -1);
      if (nb < 0 || nb >= h->nranks) continue;
      for (int b = 0; b < h->nbasis; ++b) h->peer_W[side][b] = reinterpret_cast<char *>((uintptr_t)all[nb][b]);
      h->peer_vs[side] = (int64_t)all[nb][2];
      h->peer_nzl[side] = (int64_t)all[nb][3];
    }
  } else {
    PeerMsg mine{};
    for (int b = 0; b < h->nbasis; ++b) hip_check(h, hipIpcGetMemHandle(&mine.hd[b], h->B[b].W), "hipIpcGetMemHandle");
    mine.vs = h->vs;
    mine.nzl = h->geo.nzl;
    const size_t sz = sizeof(PeerMsg);
    char *d = nullptr;
    hip_check(h, hipMalloc(&d, sz * (h->nranks + 1)), "hipMalloc(peer msg)");
    std::vector<PeerMsg> all(h->nranks);
    try {
      hip_check(h, hipMemcpyAsync(d + sz * h->nranks, &mine, sz, hipMemcpyHostToDevice, h->stream), "H2D");
      oplog(h, NLS_OP_ALLGATHER, 0, (int64_t)(sz / 8), -1);
      rccl_check(h, ncclAllGather(d + sz * h->nranks, d, sz, ncclChar, h->comm, h->stream), "ncclAllGather");
      hip_check(h, hipMemcpyAsync(all.data(), d, sz * h->nranks, hipMemcpyDeviceToHost, h->stream), "D2H");
      hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    } catch (...) {
      (void)hipFree(d);
      throw;
    }
    h->peer_ipc = true;
    // An open can fail (a neighbour in the same process: HIP refuses a handle exported by
    // the importing process; no peer path between the devices).  Every rank must then
    // leave the peer path together -- the ranks' transport sequences must stay identical
    // -- so the outcome is agreed by an all-reduce (min) of the ranks' success flags
    // before any pass uses a mapping.
    int32_t ok = 1;
    for (int side = 0; side < 2 && ok; ++side) {
      const int nb = h->rank + (side ? 1 : -1);
      if (nb < 0 || nb >= h->nranks) continue;
      for (int b = 0; b < h->nbasis && ok; ++b) {
        void *p = nullptr;
        if (hipIpcOpenMemHandle(&p, all[nb].hd[b], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
          (void)hipGetLastError();
          ok = 0;
          break;
        }
        h->peer_W[side][b] = static_cast<char *>(p);
      }
      h->peer_vs[side] = all[nb].vs;
      h->peer_nzl[side] = all[nb].nzl;
    }
    int32_t *dok = reinterpret_cast<int32_t *>(d);
    try {
      hip_check(h, hipMemcpyAsync(dok, &ok, sizeof(ok), hipMemcpyHostToDevice, h->stream), "H2D");
      oplog(h, NLS_OP_ALLREDUCE, 0, 0, -1);
      rccl_check(h, ncclAllReduce(dok, dok, 1, ncclInt32, ncclMin, h->comm, h->stream), "ncclAllReduce(peer ok)");
      hip_check(h, hipMemcpyAsync(&ok, dok, sizeof(ok), hipMemcpyDeviceToHost, h->stream), "D2H");
      hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    } catch (...) {
      (void)hipFree(d);
      throw;
    }
    (void)hipFree(d);
    if (!ok) {
      // back to the exchange path on every rank (partP2 is sized for both launch plans)
      peer_close(h);
      h->peer = false;
      h->peer_fallback = true;
      return;
    }
  }
  h->peer_ready = true;
}
void peer_close(nls_handle *h) {
  if (h->peer_ipc)
    for (auto &side : h->peer_W)
      for (char *&p : side)
        if (p) (void)hipIpcCloseMemHandle(p);
  h->peer_ipc = h->peer_ready = false;
  for (auto &side : h->peer_W)
    for (char *&p : side) p = nullptr;
}
// k_p2d's peer targets of every stored vector k of each basis (P2State pdn / pup,
// once): the neighbour below's upper ghost planes (its local planes nzl, nzl + 1) and
// the neighbour above's lower ones (-2, -1)
void peer_tables(nls_handle *h) {
  if (h->peer_ready) return;
  peer_setup(h);
  if (!h->peer) return;  // the ranks fell back to the exchange path (peer_setup)
  const int64_t P = h->geo.P, es = (int64_t)h->esize;
  const int NK = p2state_peer_slots();
  for (int b = 0; b < h->nbasis; ++b) {
    std::vector<void *> t(2 * NK, nullptr);
    for (int k = 0; k < NK && k < h->nvec[b]; ++k) {
      if (char *w = h->peer_W[0][b]) t[k] = w + (k * h->peer_vs[0] + (GHOST_MAX + h->peer_nzl[0]) * P) * es;
      if (char *w = h->peer_W[1][b]) t[NK + k] = w + k * h->peer_vs[1] * es;
    }
    char *ps = static_cast<char *>(h->p2) + (size_t)b * p2state_bytes() + p2state_peer_offset();
    hip_check(h, hipMemcpyAsync(ps, t.data(), t.size() * sizeof(void *), hipMemcpyHostToDevice, h->stream),
              "hipMemcpy(peer tables)");
  }
  hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
}

// vector k of basis b (two planes on two-vector handles: every halo'd basis vector
// of theirs is, or may become, the radius-2 stencil vector of a pass)
void halo(nls_handle *h, int b, int k) {
  halo_planes(h, vec_ptr(h, b, k), (int64_t)h->esize, nullptr, h->pass2 ? 2 : 1);
}

// Overlapped form: called once the boundary planes of vector k are enqueued on
// the compute stream; the exchange runs on cstream while the interior planes
// are computed.  halo_wait() orders the compute stream after it.
void halo_begin(nls_handle *h, int b, int k) {
  halo_after_compute(h);
  halo_planes(h, vec_ptr(h, b, k), (int64_t)h->esize, h->cstream, h->pass2 ? 2 : 1);
  hip_check(h, hipEventRecord(h->ev_halo, h->cstream), "hipEventRecord");
  h->halo_pending = true;
}
void halo_wait(nls_handle *h) {
  if (!h->halo_pending) return;
  hip_check(h, hipStreamWaitEvent(h->stream, h->ev_halo, 0), "hipStreamWaitEvent");
  oplog(h, NLS_OP_WAIT_HALO, 0, 0, -1);
  h->halo_pending = false;
}

// On the compute stream, after any halo exchange still in flight on the halo
// stream (halo_wait): the communicator never has operations of two streams in
// flight at once, so nothing relies on RCCL ordering one communicator's work
// across streams.  The exchange has overlapped the pass's interior
// launch by then, which is all the overlap there is to gain.
void allreduce_sums(nls_handle *h, int b, int ncplx, void *where = nullptr) {
  void *p = where ? where : static_cast<void *>(&h->B[b].st->sums[0]);
  halo_wait(h);
  oplog(h, NLS_OP_ALLREDUCE, 0, 2 * (int64_t)ncplx, -1);
  if (h->group) {
    // publish my partial sums, rendezvous, then every rank sums all ranks'
    // publications in rank order (identical result on every rank)
    nls_group *g = h->group;
    const int parity = (int)(h->ar_count++ & 1);
    cplx *mine = g->pub + ((int64_t)h->rank * 2 + parity) * NSUM;
    hip_check(h, hipMemcpyAsync(mine, p, (size_t)ncplx * sizeof(cplx), hipMemcpyDeviceToDevice,
                                h->stream), "hipMemcpyAsync(pub)");
    hipEvent_t ev = next_event(h);
    hip_check(h, hipEventRecord(ev, h->stream), "hipEventRecord");
    auto all = rendezvous(h, {(uint64_t)(uintptr_t)ev});
    for (int r = 0; r < h->nranks; ++r)
      if (r != h->rank)
        hip_check(h, hipStreamWaitEvent(h->stream, (hipEvent_t)(uintptr_t)all[r][0], 0),
                  "hipStreamWaitEvent");
    cplx *dst = static_cast<cplx *>(p);
    int nr = h->nranks, par = parity, cnt = ncplx, stride = NSUM;
    void *args[] = {&dst, &g->pub, &nr, &par, &cnt, &stride};
    launch(h, 2, -1, kernel_sum_ranks(), 1, args);
    if (h->dbg_sums) {
      std::vector<cplx> hv(ncplx), hp(ncplx);
      hip_check(h, hipStreamSynchronize(h->stream), "sync");
      hip_check(h, hipMemcpy(hv.data(), p, ncplx * sizeof(cplx), hipMemcpyDeviceToHost), "d2h");
      hip_check(h, hipMemcpy(hp.data(), mine, ncplx * sizeof(cplx), hipMemcpyDeviceToHost), "d2h");
      std::fprintf(stderr, "[rank %d ar %llu n %d] pub0 %.6e sum0 %.6e | pub1 %.6e sum1 %.6e\n", h->rank,
                   (unsigned long long)h->ar_count, ncplx, hp[0].re, hv[0].re, ncplx > 1 ? hp[1].re : 0.0,
                   ncplx > 1 ? hv[1].re : 0.0);
    }
    return;
  }
  rccl_check(h, ncclAllReduce(p, p, (size_t)ncplx * 2, ncclDouble, ncclSum, h->comm, h->stream),
             "ncclAllReduce");
}

// ---- one Krylov basis: Lanczos + eigensolve + final coefficients ----------

// Partial arrays longer than this are summed by the parallel k_colsum
// (one workgroup per column) instead of inside the single-workgroup reduction.
constexpr int COLSUM_MIN = 2048;

void colsum(nls_handle *h, int b, int j, const cplx *pA, int nbA, int ncA, int nbU, int ncU) {
  cplx *dst = &h->B[b].st->sums[0];
  void *args[] = {(void *)&pA, &nbA, &ncA, &h->partU, &nbU, &dst};
  launch(h, 2, j, kernel_colsum(), ncA + ncU, args);
}

// Last alpha pass of a fused-tail basis: k_alpha_l2 (also ||L W_j||^2)
void alpha_l2_pass(nls_handle *h, int b, int j) {
  void *vj = vec_ptr(h, b, j);
  Geo gg = h->geo;
  gg.kz = h->kz_alpha2;
  void *args[] = {&vj, &gg, &h->partA};
  launch(h, 0, j, kernel_alpha_l2(h->cplx_, (int)h->cfg.dim, h->ani, h->l2pipe), h->grid_alpha2, args);
}

// Launch k_alpha<j> on vector j of basis b
void alpha_pass(nls_handle *h, int b, int j, const Geo &ga) {
  void *vj = vec_ptr(h, b, j);
  Geo gg = ga;
  void *args[] = {&vj, &gg, &h->partA};
  launch(h, 0, j, kernel_alpha(h->cplx_, (int)h->cfg.dim, h->ani), h->grid_alpha, args);
}

// After a folded-alpha pass (single-rank handles): one k_reduce_qa launch (after
// k_colsum for large grids), which also holds the near-breakdown fallback.
void reduce_qa(nls_handle *h, int b, int j, const Geo &ga) {
  KState *st = h->B[b].st;
  int nbU = h->qgrid[j - 1], ncU = j + 3;
  int ds = 1;
  if (nbU > COLSUM_MIN) {
    colsum(h, b, j, h->partA, 0, 0, nbU, ncU);
    ds = 0;
  }
  const void *vj = vec_ptr(h, b, j);
  Geo gg = ga;
  int jj = j, nbX = h->xgrid;
  void *args[] = {&st, &h->partU, &nbU, &jj, &ds, &h->partX, &nbX, (void *)&vj, &gg};
  launch(h, 2, j, kernel_reduce_qa(h->cplx_, (int)h->cfg.dim, h->ani), 1, args);
}

// ncA = 2 after k_alpha, 3 after k_alpha_l2 (fused tail); qa = 1: no alpha pass,
// alpha_j from the q column of k_update<j-1, QA> (ncA = 0)
void reduce_iter(nls_handle *h, int b, int j, int ncA = 2, int qa = 0) {
  KState *st = h->B[b].st;
  int nbA = qa ? 0 : (ncA == 3 ? h->grid_alpha2 : h->grid_alpha);
  int nbU = j >= 1 ? (qa ? h->qgrid[j - 1] : h->plan[j - 1].total) : 0;
  const void *fn = kernel_reduce_iter();
  const int ncU = j >= 1 ? j + 1 + 2 * qa : 0;
  cplx *px = h->partX;
  int nbX = h->xgrid;
  const int ncols = ncA + ncU;
  if (nbA > COLSUM_MIN || nbU > COLSUM_MIN) {
    colsum(h, b, j, h->partA, nbA, ncA, nbU, ncU);
    if (h->collective) allreduce_sums(h, b, ncols);
    int ds = 0, dc = 1;
    void *args[] = {&st, &h->partA, &nbA, &h->partU, &nbU, &j, &ds, &dc, &ncA, &qa, &px, &nbX};
    launch(h, 2, j, fn, 1, args);
    return;
  }
  if (!h->collective) {
    int ds = 1, dc = 1;
    void *args[] = {&st, &h->partA, &nbA, &h->partU, &nbU, &j, &ds, &dc, &ncA, &qa, &px, &nbX};
    launch(h, 2, j, fn, 1, args);
  } else {
    int ds = 1, dc = 0;
    void *a1[] = {&st, &h->partA, &nbA, &h->partU, &nbU, &j, &ds, &dc, &ncA, &qa, &px, &nbX};
    launch(h, 2, j, fn, 1, a1);
    allreduce_sums(h, b, ncols);
    ds = 0;
    dc = 1;
    void *a2[] = {&st, &h->partA, &nbA, &h->partU, &nbU, &j, &ds, &dc, &ncA, &qa, &px, &nbX};
    launch(h, 2, j, fn, 1, a2);
  }
}

void reduce_final(nls_handle *h, int b, int nf, int f0, int f1, double tr, double ti, int tail = 0) {
  KState *st = h->B[b].st;
  int m = h->m, nbU = m >= 2 ? h->plan[m - 2].total : 0;
  const void *fn = kernel_reduce_final();
  if (tail) {  // s_{m-1} already set by the last reduce_iter; no sums
    int ds = 0, dc = 1;
    void *args[] = {&st, &h->partU, &nbU, &m, &ds, &dc, &nf, &f0, &f1, &tr, &ti, &tail};
    launch(h, 2, m, fn, 1, args);
    return;
  }
  if (nbU > COLSUM_MIN) {
    colsum(h, b, m, nullptr, 0, 0, nbU, m);
    if (h->collective) allreduce_sums(h, b, m);
    int ds = 0, dc = 1;
    void *args[] = {&st, &h->partU, &nbU, &m, &ds, &dc, &nf, &f0, &f1, &tr, &ti, &tail};
    launch(h, 2, m, fn, 1, args);
    return;
  }
  if (!h->collective) {
    int ds = 1, dc = 1;
    void *args[] = {&st, &h->partU, &nbU, &m, &ds, &dc, &nf, &f0, &f1, &tr, &ti, &tail};
    launch(h, 2, m, fn, 1, args);
  } else {
    int ds = 1, dc = 0;
    void *a1[] = {&st, &h->partU, &nbU, &m, &ds, &dc, &nf, &f0, &f1, &tr, &ti, &tail};
    launch(h, 2, m, fn, 1, a1);
    if (m >= 2) allreduce_sums(h, b, m);
    ds = 0;
    dc = 1;
    void *a2[] = {&st, &h->partU, &nbU, &m, &ds, &dc, &nf, &f0, &f1, &tr, &ti, &tail};
    launch(h, 2, m, fn, 1, a2);
  }
}

// Precondition: vector 0 of basis b holds the start vector and its halo.
// tail = true (m >= 3): stop after the alpha pass of W_{m-2} (k_alpha_l2); the
// last vector W_{m-1} is recomputed inside the caller's k_final_fused.
void run_lanczos(nls_handle *h, int b, int nf, int f0, int f1, double tr, double ti,
                 bool tail = false) {
  const int m = h->m;
  Geo g = h->geo;
  Geo ga = g;  // the alpha pass has its own tile depth
  ga.kz = h->kz_alpha;
  alpha_pass(h, b, 0, ga);
  reduce_iter(h, b, 0);
  void *W = vec_ptr(h, b, 0);
  int64_t vs = h->vs;
  KState *st = h->B[b].st;
  bool prev_qa = false;
  for (int j = 0; j + 1 < m; ++j) {
    void *out = vec_ptr(h, b, j + 1);
    if (j >= 1) {
      halo_wait(h);
      if (tail && j + 2 == m) {
        alpha_l2_pass(h, b, j);
        reduce_iter(h, b, j, 3);
        reduce_final(h, b, nf, f0, f1, tr, ti, 1);
        return;
      }
      if (prev_qa) {
        reduce_qa(h, b, j, ga);
        if (h->dbg_alpha) {  // debug: folded vs directly reduced alpha_j
          KState hs;
          hip_check(h, hipStreamSynchronize(h->stream), "sync");
          hip_check(h, hipMemcpy(&hs, st, sizeof(KState), hipMemcpyDeviceToHost), "d2h");
          alpha_pass(h, b, j, ga);
          hip_check(h, hipStreamSynchronize(h->stream), "sync");
          std::vector<cplx> pa(2 * (size_t)h->grid_alpha);
          hip_check(h, hipMemcpy(pa.data(), h->partA, pa.size() * sizeof(cplx), hipMemcpyDeviceToHost), "d2h");
          double a = 0.0;
          for (int q = 0; q < h->grid_alpha; ++q) a += pa[q].re;
          std::fprintf(stderr, "[alpha j=%d] folded %.17e direct %.17e rel %.3e\n", j, hs.Td[j],
                       a / (hs.s[j] * hs.s[j]), std::fabs(hs.Td[j] - a / (hs.s[j] * hs.s[j])) / std::fabs(hs.Td[j]));
        }
      } else {
        alpha_pass(h, b, j, ga);
        reduce_iter(h, b, j);
      }
    }
    // fold the next alpha into this pass unless the next iteration has none or
    // is the fused tail's k_alpha_l2
    const bool qa = h->fused_alpha && j + 2 < m && !(tail && j + 3 == m);
    prev_qa = qa;
    if (qa) {
      const int dim = (int)h->cfg.dim;
      const void *fq = kernel_update(h->cplx_, dim, j, h->ani, true);
      int ps = h->qgrid[j], po = 0;
      void *args[] = {&W, &out, &vs, &g, &st, &h->partU, &ps, &po, &h->xedge};
      launch(h, 1, j, fq, h->qgrid[j], args);
      // x-tile seam pairs of q: xgrid partials in partX (summed by the next reduction)
      const int rb = update_rows_per_thread(j, h->ani, true);
      int ntx = (int)xtiles(g, dim, rb), tw = dim == 3 ? 64 : 64 * rb;
      void *ax[] = {&h->xedge, &g, &ntx, &tw, &h->partX};
      launch(h, 2, j, kernel_xpairs(h->cplx_, dim, h->ani), h->xgrid, ax);
      continue;
    }
    const void *fu = kernel_update(h->cplx_, (int)h->cfg.dim, j, h->ani);
    const UpdPlan &pl = h->plan[j];
    const bool need_halo = j + 1 <= m - 2 && h->collective;
    // With a halo to send, the boundary-plane launches run on the halo stream,
    // followed there by the exchange, concurrently with the interior launch on
    // the compute stream (disjoint output planes and partial columns); the next
    // pass waits on the halo event.
    const bool side = need_halo && pl.nbnd > 0 && h->bnd_side;
    if (side) halo_after_compute(h);
    for (int i = 0; i < pl.n; ++i) {
      Geo gi = g;
      gi.qa = pl.qa[i];
      gi.qb = pl.qb[i];
      int ps = pl.total, po = pl.off[i];
      void *nul = nullptr;
      void *args[] = {&W, &out, &vs, &gi, &st, &h->partU, &ps, &po, &nul};
      const bool bnd = i < pl.nbnd;
      launch(h, 1, j, fu, pl.grid[i], args, side && bnd ? h->cstream : nullptr);
      if (need_halo && i + 1 == pl.nbnd) {
        if (side) {
          halo_planes(h, vec_ptr(h, b, j + 1), (int64_t)h->esize, h->cstream);
          hip_check(h, hipEventRecord(h->ev_halo, h->cstream), "hipEventRecord");
          h->halo_pending = true;
        } else {
          halo_begin(h, b, j + 1);
        }
      }
    }
    if (need_halo && pl.nbnd == 0) halo(h, b, j + 1);
  }
  halo_wait(h);
  reduce_final(h, b, nf, f0, f1, tr, ti);
}

Geo p2m_lap_geo(const nls_handle *h);
// y = L S_J of the register two-vector pass into lbuf (k_lap)
void p2m_lap(nls_handle *h, int b, int J, hipStream_t st) {
  void *SJ = vec_ptr(h, b, J);
  Geo gl = p2m_lap_geo(h);
  void *lb0 = h->p2gbuf + h->geo.P;  // local plane 0 of y
  void *la[] = {&SJ, &gl, &lb0};
  launch(h, 1, J, kernel_lap(true, (int)h->cfg.dim, h->ani), h->p2lapgrid, la, st);
}

// y = L S_J of the register two-vector pass: the slab's planes and, where they exist
// in the grid, the neighbouring slabs' first plane on each side (ghost planes)
Geo p2m_lap_geo(const nls_handle *h) {
  Geo g = h->geo;
  g.kz = h->p2mkz;
  g.qa = g.z0 > 0 ? -1 : 0;
  g.qb = (int32_t)(g.nzl + (g.z0 + g.nzl < g.npl ? 1 : 0));
  return g;
}

constexpr int64_t P2D_MIN_TILES = 1024;

// The smallest slab of the decomposition (nls_slab_planes: npl / nranks planes).
// Every choice that changes a step's sequence of transport operations is made from
// it, never from this rank's own slab, so that all ranks issue the same sequence.
int64_t min_slab_planes(const nls_handle *h) { return h->geo.npl / std::max(1, h->nranks); }

// The geometry k_p2d marches: the handle's, or for a 2D grid planes of 4 rows
// (nyp = 4, npl = ny/4, P = 4 nx; single rank), whose row wrap is the 2D y neighbour
Geo p2_geo(const nls_handle *h) {
  Geo g = h->geo;
  if (h->p2reg) return g;  // k_lap + k_p2m work on the handle's own planes
  if (h->p2_pr) {  // pairs of cells along x
    g.nx = h->geo.nx / 2;
    g.P = h->geo.P / 2;
  }
  if (h->p2_d2) {
    g.nyp = P2D_ROWS;
    g.npl = h->geo.npl / P2D_ROWS;
    g.P = P2D_ROWS * g.nx;
    g.nzl = g.npl;
    g.z0 = 0;
    g.qa = 0;
    g.qb = (int32_t)g.npl;
  }
  return g;
}
// tiles of one k_p2d launch over local planes [qa, qb) with tile depth kz: one
// workgroup per 64 x 4-row tile column chunk
int p2_tiles(const nls_handle *h, int64_t qa, int64_t qb, int64_t kz) {
  const Geo g = p2_geo(h);
  const int64_t nzc = (qb - qa + kz - 1) / kz;
  return (int)(((g.nx + P2D_WAVE_XO - 1) / P2D_WAVE_XO) * (g.nyp / P2D_ROWS) * nzc);
}
// Multi-rank handles (3D slabs of >= 8 planes) compute each pass's first two and
// last two planes first (k_p2d tiles of depth 2, one launch for both ends), then
// exchange the new stencil vector's two boundary planes on the halo stream while
// the interior planes run as k_p2d on the compute stream (run_lanczos2).
bool p2_split(const nls_handle *h) {
  return h->collective && min_slab_planes(h) >= 8 && h->p2_split_on && !h->peer && !h->p2_d2 && !h->p2_pr &&
         !h->p2reg && !h->p2_ani;
}
int p2_bnd_tiles(const nls_handle *h) { return 2 * p2_tiles(h, 0, 2, 2); }
// tile depth of pass J: the register-row passes (J rows loaded straight into
// registers, no J-ring prologue) stream faster from shorter tiles (512^3 J = 10: 4.77 ms
// at kz 32 vs 4.89 at 256; the J-ring passes lose: J = 12 6.45 vs 5.80; round 4,
// profiles/r04/p2ab_512.txt)
int p2_kz(const nls_handle *h, int J) {
  // (the G2 register-row pass at J = 6 keeps the general depth: 256^3 0.473 ms at kz 128
  // vs 0.491 at 32, profiles/r04/g2_probe_jreg.txt)
  if (h->cfg.dim != 3 || h->p2_ani) return h->p2kz;
  if (pass2_jreg(J, 0)) return std::min(h->p2kz, h->p2kzj);
  // the J = 0 pass (one read, two writes, three workgroups per CU) also streams faster
  // from 64-plane tiles: 512^3 1.29-1.30 vs 1.33-1.34 ms on two boxes; the ring passes at
  // J = 2..6, 12 lose at 64 (profiles/r04/p2ab_512.txt, calls r4g and r4w)
  if (J == 0) return std::min(h->p2kz, h->p2kz0);
  return h->p2kz;
}
int p2_grid(const nls_handle *h, int J = 0) {
  if (h->p2reg) return h->p2mgrid[J];
  const int64_t nzl = p2_geo(h).nzl;
  if (!p2_split(h)) return p2_tiles(h, 0, nzl, p2_kz(h, J));
  return p2_bnd_tiles(h) + p2_tiles(h, 2, nzl - 2, p2_kz(h, J));
}

// Two new vectors per pass (nls_pass2.hpp): the alpha pass + reduction of W_0
// give beta and alpha_0 (the first shift); then passes at J = 0, 2, 4, ... each
// followed by its column sums and k_p2coef, until S_0..S_{m-2} are stored; the
// last alpha pass (k_alpha_l2 over S_{m-2}) and k_p2tail complete T; the
// eigensolve; k_p2tfin maps fin to the coefficients of the caller's k_tail
// (S_0..S_{m-2} and L S_{m-2}: the last Lanczos vector is never stored).
// The s-step schedule (tests/sstep_model.py sstep_schedule): [(J, ns)] of the
// passes storing S_0..S_{nstore-1}, two new vectors per pass at even J, the last
// pass one or two.  (Three-vector passes at J = 2, 5 move 6 % fewer bytes at
// m = 16 but were issue-bound on MI355X, 29.5 vs 26.4 ms of passes at 512^3;
// measured in round 2 and removed)
std::vector<std::pair<int, int>> p2_schedule(const nls_handle *, int nstore) {
  std::vector<std::pair<int, int>> out;
  for (int J = 0; J + 1 < nstore;) {
    const int ns = std::min(2, nstore - 1 - J);
    out.emplace_back(J, ns);
    J += ns;
  }
  return out;
}

void run_lanczos2(nls_handle *h, int b, int nf, int f0, int f1, double tr, double ti) {
  if (h->peer) peer_tables(h);
  const int m = h->m, nstore = m - 1;
  KState *st = h->B[b].st;
  void *ps = static_cast<char *>(h->p2) + (size_t)b * p2state_bytes();
  int real = h->p2_pr ? 1 : 0;
  const std::vector<std::pair<int, int>> sched = p2_schedule(h, nstore);
  // blind start once a previous basis left its alpha_0 (the shift of the J = 0
  // pass): no alpha pass over W_0, beta from the pass's own ||S_0||^2
  const bool blind = h->p2_warm[b] && h->p2_blind;  // k_p2d<0> reduces ||S_0||^2
  if (!blind) {
    Geo ga = h->geo;
    ga.kz = h->kz_alpha;
    alpha_pass(h, b, 0, ga);
    reduce_iter(h, b, 0);
  }
  {
    int J = 0, mode = blind ? 2 : 0, ns = 0, nsn = sched[0].second;
    void *args[] = {&ps, &st, &J, &mode, &ns, &nsn, &real};
    launch(h, 2, 0, kernel_p2coef(), 1, args);
  }
  h->p2_warm[b] = true;
  void *W = vec_ptr(h, b, 0);
  int64_t vs = h->p2_pr ? h->vs / 2 : h->vs;  // in the kernel's 16-B cells
  Geo g = p2_geo(h);
  g.kz = h->p2kz;
  g.remap = h->p2order;
  cplx *sums = reinterpret_cast<cplx *>(static_cast<char *>(ps) + p2state_sums_offset());
  const bool split = p2_split(h);
  for (size_t si = 0; si < sched.size(); ++si) {
    int J = sched[si].first, ns = sched[si].second;
    const int out = J + ns;  // the pass's last vector: the next stencil vector
    int nb = p2_grid(h, J);
    g.kz = p2_kz(h, J);
    const void *fn = h->p2reg ? nullptr
                     : h->p2_ani ? kernel_pass2a(J, ns == 2, h->p2_pr)
                                 : kernel_pass2(J, ns == 2, h->p2_d2, h->p2_pr, h->peer);
    halo_wait(h);  // the stencil vector S_J's ghost planes (previous pass's exchange)
    if (h->p2reg) {
      // y = L S_J over the slab and its neighbour planes, then the pass over y.  (Issuing
      // the next pass's y on a second stream, to overlap the column sums and k_p2coef,
      // measured no gain at G2 256^3: 13.76 vs 13.75 ms/step.)
      const int dim = (int)h->cfg.dim;
      p2m_lap(h, b, J, nullptr);
      int poff = 0;
      Geo gp = h->geo;
      gp.kz = h->p2mkz;
      void *args[] = {&W, &vs, &gp, &ps, &h->partP2, &nb, &h->p2gbuf, &poff};
      launch(h, 1, J, kernel_p2m(dim, J, ns == 2, h->ani), nb, args);
      if (h->collective) halo_begin(h, b, out);
    } else if (!split) {
      int poff = 0;
      void *args[] = {&W, &vs, &g, &ps, &h->partP2, &nb, &h->zbuf, &poff};
      launch(h, 1, J, fn, nb, args);
      // peer stores: the exchange is the pass's own stores (P2State peer tables)
      if (h->collective && !h->peer) halo_begin(h, b, out);
    } else {
      // the boundary planes [0, 2) and [nzl-2, nzl) first, as k_p2d tiles of depth 2 in
      // one grid (Geo::q2), on the compute stream; the exchange of the new stencil
      // vector's two boundary planes then runs on the halo stream while the interior
      // planes are computed.  The all-reduce waits for the exchange (halo_wait), which
      // the interior has covered by then: one communicator, one stream at a time.
      const int64_t nzl = h->geo.nzl;
      const int tb = p2_bnd_tiles(h);
      Geo gb = g;
      gb.kz = 2;
      gb.qa = 0;
      gb.qb = 2;
      gb.q2 = (int32_t)(nzl - 2);
      int poff = 0;
      void *args[] = {&W, &vs, &gb, &ps, &h->partP2, &nb, &h->zbuf, &poff};
      launch(h, 1, J, fn, tb, args);
      halo_begin(h, b, out);
      Geo gi = g;
      gi.qa = 2;
      gi.qb = (int32_t)(nzl - 2);
      int poffi = tb;
      void *argsi[] = {&W, &vs, &gi, &ps, &h->partP2, &nb, &h->zbuf, &poffi};
      launch(h, 1, J, fn, nb - tb, argsi);
    }
    // columns: S-dots per new vector, the Gram's upper triangle, J = 0: ||S_0||^2
    const cplx *pA = nullptr;
    int nbA = 0, ncA = 0, ncU = ns * (J + 1) + ns * (ns + 1) / 2 + (J == 0 ? 1 : 0);
    void *cargs[] = {(void *)&pA, &nbA, &ncA, &h->partP2, &nb, &sums};
    launch(h, 2, J, kernel_colsum(), ncU, cargs);
    if (h->collective) allreduce_sums(h, b, ncU, sums);
    int mode = 1, nsn = si + 1 < sched.size() ? sched[si + 1].second : 0;
    void *a2[] = {&ps, &st, &J, &mode, &ns, &nsn, &real};
    launch(h, 2, J, kernel_p2coef(), 1, a2);
  }
  halo_wait(h);
  // the tail's alpha pass over S_{m-2}: a = S^H L S, ||S||^2, ||L S||^2
  alpha_l2_pass(h, b, m - 2);
  {
    const cplx *pU = nullptr;
    int nbA = h->grid_alpha2, ncA = 3, nbU = 0;
    void *cargs[] = {(void *)&h->partA, &nbA, &ncA, (void *)&pU, &nbU, &sums};
    launch(h, 2, m - 2, kernel_colsum(), ncA, cargs);
    if (h->collective) allreduce_sums(h, b, ncA, sums);
    int mm = m;
    void *a2[] = {&ps, &st, &sums, &mm};
    launch(h, 2, m - 2, kernel_p2tail(), 1, a2);
  }
  reduce_final(h, b, nf, f0, f1, tr, ti, 1);
  int mm = m, nff = nf;
  void *fa[] = {&ps, &st, &mm, &nff};
  launch(h, 2, m, kernel_p2tfin(), 1, fa);
}

int occupancy_grid(nls_handle *h, const void *fn, int64_t work_items) {
  int per_cu = 0;
  hip_check(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NTHREADS, 0),
            "hipOccupancyMaxActiveBlocksPerMultiprocessor");
  int ncu = 0;
  hip_check(h, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->dev),
            "hipDeviceGetAttribute");
  // Large slabs: 16 x the resident workgroups, in practice one tile per
  // workgroup, so the hardware dispatcher balances the tail (measured -2.7 %
  // update time at 512^3, -1 % at 8192^2 SG); the partials of such grids are
  // summed by k_colsum.  Small slabs (<= 32 M cells): a persistent grid, where
  // the extra reduction launch costs more than the balance gains (4096^2, 256^3).
  int mult = h->large ? 16 : 1;
  if (const char *e = std::getenv("NLS_GRID_MULT")) mult = std::max(1, std::atoi(e));
  int64_t grid = (int64_t)std::max(per_cu, 1) * std::max(ncu, 1) * mult;
  grid = std::min<int64_t>(grid, std::max<int64_t>(work_items, 1));
  return (int)grid;
}

void setup_geometry(nls_handle *h) {
  const nls_config &c = h->cfg;
  Geo &g = h->geo;
  if (c.dim == 3) {
    g.nx = c.nx;
    g.nyp = c.ny;
    g.npl = c.nz;
  } else {
    g.nx = c.nx;
    g.nyp = 1;
    g.npl = c.ny;
  }
  g.P = g.nx * g.nyp;
  g.Ng = g.P * g.npl;
  uint32_t z0 = 0, nzl = 0;
  nls_slab_planes((uint32_t)g.npl, h->nranks, h->rank, &z0, &nzl);
  g.nzl = nzl;
  g.z0 = z0;
  g.qa = 0;
  g.qb = (int32_t)g.nzl;
  g.nloc = g.nzl * g.P;
  // Large slabs (> 32 M cells) take their own launch shapes: 16x grids of one tile per
  // workgroup, 4-plane alpha tiles, the one-tile / tile-queue fused tail.
  // NLS_LARGE_SLAB=1 forces them on any grid, so the tests run the bench's code path on
  // grids the oracle and the reference fixtures cover (tests/test_gpu_refpin.py).
  h->large = g.nloc > (int64_t(1) << 25);
  if (const char *e = std::getenv("NLS_LARGE_SLAB")) h->large = std::atoi(e) != 0;
  // laplacians.hpp:49 (2D 1/(dx*dy)) and :102 (3D 1/(dx*dx)); values -4/-3, -6/-5 times scale
  g.s = c.dim == 2 ? 1.0 / (c.dx * c.dy) : 1.0 / (c.dx * c.dx);
  g.sd_in = (c.dim == 2 ? -4.0 : -6.0) * g.s;
  g.sd_bd = (c.dim == 2 ? -3.0 : -5.0) * g.s;
  // tile depth: 3D planes per tile, 2D rows per wave (tile = 4 waves)
  g.kz = c.dim == 3 ? 32 : 16;
  if (const char *e = std::getenv("NLS_KZ")) g.kz = std::max(1, std::atoi(e));
  // alpha pass on large 3D slabs (one-tile-per-workgroup grids, see
  // occupancy_grid): shallower tiles, -9 % alpha time at 512^3 with kz 4 vs
  // 16-32; on small slabs (persistent grids) it is slower (tools/exp_kz.sh)
  h->kz_alpha = (c.dim == 3 && h->large) ? 4 : g.kz;
  if (const char *e = std::getenv("NLS_KZ_ALPHA")) h->kz_alpha = std::max(1, std::atoi(e));
  g.remap = 0;  // (march's XCD-banded order, Geo::remap, measured no gain for these kernels)
  // Pad the vector stride so the m streams of one update pass do not start on
  // the same HBM channel (strides of 2^k * plane bytes camp on one channel).
  // 4096 elements (64 KiB of complex<double>): same-box A/B sweeps (tools/exp_pad3.sh,
  // exp_pad4.sh) gave 512^3 update passes -5 % (two boxes), 4096^2 +6 % vs the former
  // 4 KiB pad, within 1 % elsewhere; no pad at all is ~15 % slower (tools/bw_probe.hip).
  // Round 4, with the s-step passes and the tail: 8192 elements, 512^3 passes 24.39-24.57
  // -> 24.15-24.27 ms per step on two boxes (2048: +0.1; 4160: +0.3; 16384: +0.0), 4096^2
  // and G2 256^3 within 1 % (profiles/r04/ab_vpad.txt)
  h->vpad = NLS_VPAD;
  if (const char *e = std::getenv("NLS_DEBUG_VPAD")) h->vpad = std::max<int64_t>(0, std::atoll(e));  // (A/B sweeps)
  // (the vector stride h->vs follows in alloc_all, once the ghost depth is known)
}

// scalar type of a tail kernel on this handle: the NLSE and sEWI epilogues are
// complex, the Gautschi ones real, the plain combinations follow the handle
bool tail_is_cplx(const nls_handle *h, int mode) {
  if (mode == TAIL_COMBINE || mode == TAIL_COMBINE_W0) return h->cplx_;
  return mode == TAIL_NLSE || mode == TAIL_SEWI_END;
}

// the scratch vector (sEWI's e, API outputs) is allocated on first use only
void ensure_scratch(nls_handle *h) {
  if (!h->scratch)
    hip_check(h, hipMalloc(&h->scratch, (size_t)h->geo.nloc * h->esize), "hipMalloc(scratch)");
}

// grids of the fused tail kernels for the handle's tail depth: one tile per workgroup
// (large slabs) or the occupancy grid, and the resident grid of the dynamic tile queue
void tail_grids(nls_handle *h, bool one_tile) {
  const int dim = h->cfg.dim;
  Geo gf = h->geo;
  if (h->kz_fused) gf.kz = h->kz_fused;
  const int64_t tt = stencil_tiles(gf, dim, fused_rows_per_thread());
  int ncu = 0;
  hip_check(h, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->dev), "hipDeviceGetAttribute");
  for (int mode = 0; mode < TAIL_NMODES; ++mode) {
    const void *ft = kernel_tail(tail_is_cplx(h, mode), dim, mode, h->m, h->ani);
    h->tail_grid[mode] = h->tail_dyn_grid[mode] = 0;
    if (!ft) continue;
    h->tail_grid[mode] = one_tile ? (int)tt : occupancy_grid(h, ft, tt);
    int per_cu = 0;
    hip_check(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ft, NTHREADS, 0),
              "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    h->tail_dyn_grid[mode] = (int)std::min<int64_t>(tt, (int64_t)std::max(per_cu, 1) * std::max(ncu, 1));
  }
}

void alloc_all(nls_handle *h) {
  const Geo &g = h->geo;
  const bool c = h->cplx_;
  const int dim = h->cfg.dim;
  const bool ani = h->ani;
  // two-vectors-per-pass Lanczos: stores S_0..S_{m-2}, ends in the fused tail.
  // Default on for the isotropic NLSE: 3D (k_p2d: 4-row tiles, m <= 18; also on
  // slabs) and 2D on one rank (ny % 4 == 0, planes of 4 rows);
  // NLS_PASS2=0/1 forces it off / on where a pass form exists.
  h->pass2 = false;
  if (const char *e = std::getenv("NLS_P2_SPLIT")) h->p2_split_on = std::atoi(e) != 0;
  {
    const char *e = std::getenv("NLS_PASS2");
    const bool want = e ? std::atoi(e) != 0 : true;
    // 2D (one rank): k_p2d on planes of 4 rows (p2_geo), ny % 4 == 0
    const bool d2 = dim == 2 && !h->collective && g.npl % P2D_ROWS == 0 && g.npl >= 2 * P2D_ROWS;
    // real 2D Gautschi (sine-Gordon, G1 and the G2 family; not KG's anisotropic
    // operator): the field as pairs of cells, nx even
    const bool pr = !c && !h->kg && !ani && d2 && g.nx % 2 == 0 && g.nx >= 4;
    // multi-rank: slabs of >= 4 planes (two-plane halos)
    const bool base = (c || pr) && !ani && (dim == 3 || d2) && (!h->collective || min_slab_planes(h) >= 4) &&
                      (h->nbasis == 1 || pr) && h->m >= 3 &&
                      g.nloc + 2 * g.P < (int64_t(1) << 31);  // 32-bit cell indices
    // k_p2d: whole 4-row tiles, rings for J <= m-4 within LDS
    const bool dma = (dim == 3 ? g.nyp % P2D_ROWS == 0 && g.nyp >= 4 : d2) && h->m - 4 <= P2D_MAXJ;
    // the register form k_lap + k_p2m (complex fields): the G2 anisotropic NLSE (div(c grad); not
    // the real Klein-Gordon) and the isotropic grids k_p2d does not take (ny % 4 != 0,
    // 2D slabs, m > 18); J <= 28
    const bool reg = c && !h->kg && h->nbasis == 1 && h->m >= 3 && h->m <= MMAX - 2 &&
                     (!h->collective || min_slab_planes(h) >= 4) && g.nloc + 2 * g.P < (int64_t(1) << 31);
    // k_p2d with the G2 operator div(c grad) (the c field staged beside S_J): 3D
    // complex, whole 4-row tiles, nx even (16-B pairs of c), J <= P2D_MAXJ_A (m <= 26);
    // NLS_P2_REG=1 keeps the register form
    const int maxj = ((h->m - 3) / 2) * 2;  // the schedule's last J
    const bool adma = c && ani && !h->kg && dim == 3 && h->nbasis == 1 && h->m >= 3 && g.nyp % P2D_ROWS == 0 &&
                      g.nyp >= P2D_ROWS && g.nx % 2 == 0 && g.nx >= 4 && maxj <= P2D_MAXJ_A &&
                      (!h->collective || min_slab_planes(h) >= 4) && g.nloc + 2 * g.P < (int64_t(1) << 31) &&
                      !(std::getenv("NLS_P2_REG") && std::atoi(std::getenv("NLS_P2_REG")));
    // the Klein-Gordon Gautschi step (3D, real, div(c grad)): k_p2d with the G2 operator
    // on pairs of cells (nx even), J <= P2D_MAXJ_A2; both bases end in fused tails
    const bool kdma = h->kg && dim == 3 && h->m >= 3 && g.nyp % P2D_ROWS == 0 && g.nyp >= P2D_ROWS &&
                      g.nx % 2 == 0 && g.nx >= 4 && maxj <= P2D_MAXJ_A2 &&
                      (!h->collective || min_slab_planes(h) >= 4) && g.nloc + 2 * g.P < (int64_t(1) << 31);
    h->pass2 = want && ((base && dma) || adma || reg || kdma);
    h->p2reg = h->pass2 && !(base && dma) && !adma && !kdma;
    h->p2_ani = h->pass2 && !h->p2reg && ani;
    h->p2_d2 = h->pass2 && !h->p2reg && dim == 2;
    h->p2_pr = h->pass2 && !h->p2reg && !c;
  }
  // peer stores (NLS_PEER=1): the 3D isotropic k_p2d passes of
  // collective handles write their next stencil vector's boundary planes into the
  // neighbours' ghost planes; a 1-rank handle into its own out-of-grid ghost planes (a
  // cost probe).  (The anisotropic and cell-pair passes keep the RCCL exchange.)
  if (const char *e = std::getenv("NLS_PEER"))
    h->peer = std::atoi(e) != 0 && h->pass2 && !h->p2reg && !h->p2_d2 && !h->p2_ani && !h->p2_pr && dim == 3 &&
              (h->collective || h->nranks == 1);
  // stored vectors: slab + ghost planes (two for the two-vector passes' radius-2
  // march) + the stride pad
  h->ghost = h->pass2 ? GHOST_MAX : 1;
  h->vs = (g.nzl + 2 * h->ghost) * g.P + h->vpad;
  if (h->pass2) {
    // z depth of a k_p2d tile: deep (each tile's prologue is a latency chain), but at
    // least ~P2D_MIN_TILES tiles, from the planes this launch covers: the slab's (ADVICE
    // r02: not the global count), its interior on split multi-rank handles.  512^3:
    // 256 (2048 tiles, capped); the 8-rank slab 512^2 x 64: 64 / 60 (one tile per
    // column) measured 4.40 / 4.77 ms/step against 4.57 / 4.98 at 32 / 30
    // (tools/slab_probe.py, profiles/r03/slab_probe.txt)
    const Geo gm = p2_geo(h);
    const int64_t cols = ((gm.nx + P2D_WAVE_XO - 1) / P2D_WAVE_XO) * std::max<int64_t>(1, gm.nyp / P2D_ROWS);
    // 3D: at least ~two tiles per CU (G2 256^3 m = 25: kz 128, 512 tiles: passes 10.42 ->
    // 10.15 ms per step against kz 64 / 1024 tiles, 10.59 at kz 256 / 256 tiles; round 3,
    // tools/wl_ab.sh); 2D planes of 4 rows keep P2D_MIN_TILES
    const int64_t min_tiles = dim == 3 ? P2D_MIN_TILES / 2 : P2D_MIN_TILES;
    const int64_t nzc = std::max<int64_t>(1, (min_tiles + cols - 1) / cols);
    if (h->p2reg) {
      const size_t lb = (size_t)(g.nzl + 2) * g.P * sizeof(cplx);
      hip_check(h, hipMalloc(&h->p2gbuf, lb), "hipMalloc(p2gbuf)");
      hip_check(h, hipMemsetAsync(h->p2gbuf, 0, lb, h->stream), "hipMemset");
      const Geo gl = p2m_lap_geo(h);
      h->p2lapgrid = occupancy_grid(h, kernel_lap(true, dim, ani), stencil_tiles(gl, dim, alpha_rows_per_thread()));
      Geo gm = g;
      gm.kz = h->p2mkz;
      for (int J = 0; J + 1 < h->m - 1; J += 2) {
        const void *fm = kernel_p2m(dim, J, true, ani);
        h->p2mgrid[J] = fm ? occupancy_grid(h, fm, stencil_tiles(gm, dim, p2m_rows_per_thread(J))) : 0;
      }
    }
    const int64_t span = p2_split(h) ? gm.nzl - 4 : gm.nzl;
    h->p2kz = (int)std::max<int64_t>(std::min<int64_t>(16, span), std::min<int64_t>(256, (span + nzc - 1) / nzc));
    if (const char *e = std::getenv("NLS_P2_KZ")) h->p2kz = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("NLS_P2_KZJ")) h->p2kzj = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("NLS_P2_KZ0")) h->p2kz0 = std::max(1, std::atoi(e));
    // tile order (round 3, tools/order_sweep.py, tools/wl_ab.sh): 3D x-fastest without XCD
    // bands (512^3 passes 25.6 -> 25.1 ms per step; 256^3 -0.5 %); 2D keeps the bands
    // (4096^2 passes 3.14 -> 3.34 ms without them)
    h->p2order = dim == 3 ? 6 : 0;
    h->p2grid = 0;
    for (int J = 0; J < MMAX; J += 2) h->p2grid = std::max(h->p2grid, p2_grid(h, J));
    if (h->peer) {  // room for the exchange path's launch plan too (peer_setup's fallback)
      h->peer = false;
      for (int J = 0; J < MMAX; J += 2) h->p2grid = std::max(h->p2grid, p2_grid(h, J));
      h->peer = true;
    }
    if (h->p2reg)
      for (int J = 0; J < MMAX; J += 2) h->p2grid = std::max(h->p2grid, h->p2mgrid[J]);
    hip_check(h, hipMalloc(&h->p2, p2state_bytes() * h->nbasis), "hipMalloc(p2)");  // one per basis
    hip_check(h, hipMemsetAsync(h->p2, 0, p2state_bytes() * h->nbasis, h->stream), "hipMemset");
    hip_check(h, hipMalloc(&h->partP2, (size_t)h->p2grid * (3 * MMAX + 8) * sizeof(cplx)),
              "hipMalloc(partP2)");
    const size_t zb = (size_t)std::max<int64_t>(g.nx, 64) * sizeof(cplx);
    hip_check(h, hipMalloc(&h->zbuf, zb), "hipMalloc(zbuf)");
    hip_check(h, hipMemsetAsync(h->zbuf, 0, zb, h->stream), "hipMemset");
  }
  // fused tails first: a basis that always ends in one never stores W_{m-1}
  h->fused_tail = h->m >= 3;
  if (const char *e = std::getenv("NLS_FUSED_TAIL")) h->fused_tail = h->fused_tail && (std::atoi(e) != 0 || h->pass2);
  if (h->fused_tail) {
    // the pipelined march where the alpha pass is latency-bound: slabs below the large
    // class, whose one-tile-per-workgroup grids leave each wave a whole z column of
    // exposed plane-by-plane latencies (KG / G2 256^3); the 512^3 slab is bandwidth-bound
    // and runs the plain march faster (profiles/r06/ab_alpha_l2_pipe.txt)
    h->l2pipe = dim == 3 && !h->large;
    if (const char *e = std::getenv("NLS_L2_PIPE")) h->l2pipe = dim == 3 && std::atoi(e) != 0;
    Geo g2 = g;
    g2.kz = h->kz_alpha2;
    h->grid_alpha2 = occupancy_grid(h, kernel_alpha_l2(c, dim, ani, h->l2pipe),
                                    stencil_tiles(g2, dim, alpha_l2_rows_per_thread()));
    // large slabs: one tile per workgroup (the tail reduces nothing, so the grid
    // size only sets the dispatch balance): 512^3 m=16 tail 6.64 -> 6.38 ms against
    // two tiles per workgroup (tools/tail_sweep.sh, same box, two rounds)
    const bool one_tile = h->large && !std::getenv("NLS_GRID_MULT");
    // shallow tail tiles there and in 2D (4 planes / rows per wave; round 3,
    // tools/order_sweep.py, tools/wl_ab.sh, same box): 512^3 6.25 -> 6.00 ms, 4096^2
    // 0.775 -> 0.74, SG 8192^2 2.62 -> 2.51; the persistent grids of small 3D slabs keep
    // the stencil depth (256^3: no gain)
    h->kz_fused = (one_tile || dim == 2) ? 4 : 0;
    // the dynamic tile queue on a resident grid: large 3D slabs with 16-plane tiles (512^3,
    // same handle, tools/knob_ab.py: tail 6.03 -> 5.93 and 6.19 -> 6.13 ms on two boxes
    // against one 4-plane tile per workgroup; profiles/r03/knob_ab_*.txt) and the complex
    // 2D fields with 4 rows per wave (4096^2: 0.744 -> 0.684-0.69 ms, tools/wl_ab.sh, two
    // rounds); not the real 2D Gautschi tails (SG 8192^2: 2.53 -> 2.55) nor small 3D slabs
    // (G2 256^3: 1.23-1.31 -> 1.26-1.36)
    h->tail_dyn = (one_tile && dim == 3) || (dim == 2 && c);
    // 8-plane queue tiles in 3D (512^3 m = 16, one handle, three interleaved rounds:
    // 5.77 ms against 5.86 with 16 planes and 5.95 with 4, profiles/r04/knob_ab_512.txt)
    if (h->tail_dyn && dim == 3) h->kz_fused = 8;
    // the dynamic tile queue of the tail (nls_common.hpp tq_next_xcd: eight band heads and
    // a done counter), zero between launches (the last workgroup of each launch resets them)
    hip_check(h, hipMalloc(&h->tailq, tq_words() * sizeof(int32_t)), "hipMalloc(tailq)");
    hip_check(h, hipMemsetAsync(h->tailq, 0, tq_words() * sizeof(int32_t), h->stream), "hipMemset");
    h->tail_one_tile = one_tile;
    tail_grids(h, one_tile);
  }
  // vectors stored per basis: m - 1 where every Lanczos run on it ends in a fused
  // tail (its k_tail exists for each use), else m.  1024^3 m=16 NLSE: 15 x 17.2 GB.
  h->nvec[0] = h->nvec[1] = h->m;
  if (h->fused_tail) {
    auto has = [&](int mode) { return h->tail_grid[mode] > 0; };
    if (c) {
      bool ok = has(TAIL_NLSE) && has(TAIL_COMBINE);
      if (ani) ok = ok && has(TAIL_COMBINE_W0) && has(TAIL_SEWI_END);
      if (ok) h->nvec[0] = h->m - 1;
    } else if (h->kg && h->pass2) {
      // the s-step passes store m-1 vectors of each basis: the sinc^2 basis ends in a
      // combining tail into its own W_0, the cos basis in the Gautschi update
      if (!has(TAIL_COMBINE_W0) || !has(TAIL_KG_END1)) fail(h, NLS_ERR_STATE, "KG s-step tails missing");
      h->nvec[0] = h->nvec[1] = h->m - 1;
    } else if (h->kg) {
      if (has(TAIL_KG_END)) h->nvec[0] = h->m - 1;  // the sinc^2 basis is stored in full
    } else if (has(h->gfun >= 0 ? TAIL_GG_MID : TAIL_SG_MID) && has(TAIL_SG_END) && has(TAIL_COMBINE)) {
      h->nvec[0] = h->nvec[1] = h->m - 1;
    }
  }

  // (u in an extra slot after the basis vectors measured no systematic effect against
  // its own allocation, tools/exp_uslot.sh in round 1; removed in round 4.  Physically
  // contiguous allocations (hipDeviceMallocContiguous) were slower: 512^3 update 24.8-24.9
  // vs 24.3 ms per step, profiles/r05/envab_contig.txt; round 5, not kept)
  // (placement probe: shifts every later allocation by the given size; the same code then
  // runs on other physical pages -- tools/gpu.sh envab with NLS_DEBUG_PREPAD_KB=...)
  if (const char *e = std::getenv("NLS_DEBUG_PREPAD_KB"))
    if (const size_t kb = std::strtoull(e, nullptr, 10))
      hip_check(h, hipMalloc(&h->prepad, kb * 1024), "hipMalloc(prepad)");
  // (NLS_DEBUG_CONTIG=1: physically contiguous bases, for the placement A/B)
  const bool contig = std::getenv("NLS_DEBUG_CONTIG") && std::atoi(std::getenv("NLS_DEBUG_CONTIG"));
  for (int b = 0; b < h->nbasis; ++b) {
    const size_t bytes = (size_t)h->nvec[b] * h->vs * h->esize;
    if (contig)
      hip_check(h, hipExtMallocWithFlags(&h->B[b].W, bytes, hipDeviceMallocContiguous), "hipExtMallocWithFlags(basis)");
    else
      hip_check(h, hipMalloc(&h->B[b].W, bytes), "hipMalloc(basis)");
    hip_check(h, hipMemsetAsync(h->B[b].W, 0, bytes, h->stream), "hipMemset");
    hip_check(h, hipMalloc(&h->B[b].st, sizeof(KState)), "hipMalloc(state)");
    hip_check(h, hipMemsetAsync(h->B[b].st, 0, sizeof(KState), h->stream), "hipMemset");
  }
  const size_t nbytes = (size_t)g.nloc * h->esize;
  if (h->cplx_) {
    hip_check(h, hipMalloc(&h->u, nbytes), "hipMalloc(u)");
    if (h->ani || h->nonlin == 3) hip_check(h, hipMalloc(&h->mf, (size_t)g.nloc * sizeof(double)), "hipMalloc(m)");
  } else {
    hip_check(h, hipMalloc(&h->up, nbytes), "hipMalloc(u_past)");
    hip_check(h, hipMalloc(&h->mf, nbytes), "hipMalloc(m)");
    if (h->kg) hip_check(h, hipMalloc(&h->vel, nbytes), "hipMalloc(v)");
  }
  if (h->ani) {
    // the same ghost depth as a stored vector (two for the two-vector passes' radius-2
    // stencil of div(c grad))
    const size_t cbytes = (size_t)(g.nzl + 2 * h->ghost) * g.P * sizeof(double);
    hip_check(h, hipMalloc(&h->cfb, cbytes), "hipMalloc(c)");
    hip_check(h, hipMemsetAsync(h->cfb, 0, cbytes, h->stream), "hipMemset");
    h->geo.cf = h->cfb + h->ghost * g.P;
  }
  // grid sizes from measured occupancy; partial buffers sized for the largest
  Geo ga = g;
  ga.kz = h->kz_alpha;
  h->grid_alpha = occupancy_grid(h, kernel_alpha(c, dim, ani), stencil_tiles(ga, dim, alpha_rows_per_thread()));
  h->grid_lap = occupancy_grid(h, kernel_lap(c, dim, ani), stencil_tiles(g, dim, alpha_rows_per_thread()));
  int64_t cap = 2 * (int64_t)h->grid_alpha;
  // On by default where it was measured to pay: each folded pass costs more than the
  // plain update (3D: halo row + peek plane, 4-14 %) plus the seam-pair launch, against
  // the alpha pass it removes.  Same-box A/B (tools/exp_qa2.sh): 512^3 +4.5 %, 384^3
  // +6 %, 2D 4096^2 +2.4 %, SG 8192^2 +1 %, but 3D 256^3 -3 % -> 3D slabs above 32 M
  // cells, 2D slabs from 16 M.  NLS_FUSED_ALPHA=1/0 forces it on/off (single rank).
  h->fused_alpha = !h->collective &&
                   (g.nloc > (int64_t(1) << 25) || (dim == 2 && g.nloc >= (int64_t(1) << 24)));
  if (const char *e = std::getenv("NLS_FUSED_ALPHA")) h->fused_alpha = !h->collective && std::atoi(e) != 0;
  if (h->pass2) h->fused_alpha = false;
  if (h->fused_alpha) {  // seam buffer for the narrowest x tiles (64 wide)
    const size_t xe = 2 * (size_t)g.nzl * (size_t)g.nyp * (size_t)xtiles(g, dim, 1) * h->esize;
    hip_check(h, hipMalloc(&h->xedge, xe), "hipMalloc(xedge)");
    hip_check(h, hipMalloc(&h->partX, (size_t)h->xgrid * sizeof(cplx)), "hipMalloc(partX)");
  }
  for (int j = 0; j + 1 < h->m; ++j) {
    const void *fu = kernel_update(c, dim, j, ani);
    UpdPlan &pl = h->plan[j];
    pl = UpdPlan{};
    auto add = [&](int qa, int qb, bool bnd) {
      Geo gi = g;
      gi.qa = qa;
      gi.qb = qb;
      const int i = pl.n++;
      pl.qa[i] = qa;
      pl.qb[i] = qb;
      pl.grid[i] = occupancy_grid(h, fu, stencil_tiles(gi, dim, update_rows_per_thread(j, ani)));
      pl.off[i] = pl.total;
      pl.total += pl.grid[i];
      if (bnd) pl.nbnd = pl.n;
    };
    const int nzl = (int)g.nzl;
    if (h->collective && nzl >= 3) {
      add(0, 1, true);
      add(nzl - 1, nzl, true);
      add(1, nzl - 1, false);
    } else {
      add(0, nzl, false);
    }
    cap = std::max<int64_t>(cap, (int64_t)pl.total * (j + 2));
    if (h->fused_alpha) {
      const void *fq = kernel_update(c, dim, j, ani, true);
      h->qgrid[j] = fq ? occupancy_grid(h, fq, stencil_tiles(g, dim, update_rows_per_thread(j, ani, true))) : 0;
      if (!fq) h->fused_alpha = false;
      cap = std::max<int64_t>(cap, (int64_t)h->qgrid[j] * (j + 4));
    }
  }
  const size_t na = std::max<size_t>(2 * (size_t)h->grid_alpha, h->fused_tail ? 3 * (size_t)h->grid_alpha2 : 0);
  hip_check(h, hipMalloc(&h->partA, na * sizeof(cplx)), "hipMalloc(partA)");
  hip_check(h, hipMalloc(&h->partU, (size_t)cap * sizeof(cplx)), "hipMalloc(partU)");
  // (NLS_KG_CONCURRENT=0 in the environment: the serial order, for the bitwise check)
  const char *kgc = std::getenv("NLS_KG_CONCURRENT");
  if (NLS_KG_CONCURRENT && !(kgc && std::atoi(kgc) == 0) && h->kg && h->pass2 && !h->collective) {
    // the second basis' own partials and stream
    hip_check(h, hipMalloc(&h->partAb, na * sizeof(cplx)), "hipMalloc(partA)");
    hip_check(h, hipMalloc(&h->partP2b, (size_t)h->p2grid * (3 * MMAX + 8) * sizeof(cplx)), "hipMalloc(partP2)");
    hip_check(h, hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking), "hipStreamCreate");
    hip_check(h, hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming), "hipEventCreate");
    hip_check(h, hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming), "hipEventCreate");
  }
  h->grid_pw = (int)std::max<int64_t>(1, std::min<int64_t>((g.nloc + NTHREADS - 1) / NTHREADS, 8192));
}

void free_all(nls_handle *h) {
  for (int b = 0; b < 2; ++b) {
    if (h->B[b].W) (void)hipFree(h->B[b].W);
    if (h->B[b].st) (void)hipFree(h->B[b].st);
    h->B[b] = Basis{};
  }
  for (void *p : {h->u, (void *)h->up, (void *)h->mf, (void *)h->cfb, h->scratch, h->snap, h->uprev,
                  (void *)h->vel, h->xedge, (void *)h->partX, h->p2, (void *)h->partP2,
                  (void *)h->zbuf, (void *)h->p2gbuf, (void *)h->partA, (void *)h->partU,
                  (void *)h->tailq, (void *)h->partAb, (void *)h->partP2b, h->prepad})
    if (p) (void)hipFree(p);
  h->partAb = h->partP2b = nullptr;
  h->prepad = nullptr;
  h->p2 = nullptr;
  h->tailq = nullptr;
  h->partP2 = h->zbuf = h->p2gbuf = nullptr;
  h->u = h->scratch = h->snap = h->uprev = nullptr;
  h->up = h->mf = h->cfb = h->vel = nullptr;
  h->xedge = nullptr;
  h->partX = nullptr;
  h->partA = h->partU = nullptr;
}

void copy_in_vector(nls_handle *h, int b, int k, const double *src) {
  hip_check(h, hipMemcpyAsync(vec_ptr(h, b, k), src, (size_t)h->geo.nloc * h->esize,
                              hipMemcpyHostToDevice, h->stream),
            "hipMemcpy H2D");
}

void check_len(nls_handle *h, uint64_t n) {
  if (n != (uint64_t)h->geo.nloc)
    fail(h, NLS_ERR_SHAPE,
         "length " + std::to_string(n) + " != local cells " + std::to_string(h->geo.nloc));
}

void pw_launch(nls_handle *h, int cls, const void *fn, void **args) {
  launch(h, cls, -1, fn, h->grid_pw, args);
}

// The stencil kernels index a stored vector with 32-bit ints (nls_stencil.hpp
// march: p = q * P + off over the ghost planes -P .. (nzl + 1) * P, tile counts);
// the largest slab (rank 0, nls_slab_planes) must stay below 2^31 elements incl.
// the ghost planes and the stride pad.  Checked before any allocation.
bool slab_index_limit_exceeded(const nls_config &c) {
  const uint64_t npl = c.dim == 3 ? c.nz : c.ny;
  const uint64_t P = c.dim == 3 ? (uint64_t)c.nx * c.ny : (uint64_t)c.nx;
  uint32_t z0 = 0, nzl = 0;
  if (nls_slab_planes((uint32_t)npl, c.nranks, 0, &z0, &nzl) != NLS_OK) return true;
  return ((uint64_t)nzl + 2 * GHOST_MAX) * P + 4096 >= (uint64_t(1) << 31);
}

}  // namespace

// ============================================================================
extern "C" {

int nls_abi_version(void) { return NLS_ABI_VERSION; }

void nls_config_default(nls_config *c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->dim = 2;
  c->equation = NLS_NLSE_CUBIC;
  c->krylov_m = 10;                // device/nlse_solver_dev.hpp:48
  c->sigma1[0] = 0.0;              // device/nlse_cq_solver.hpp:19
  c->sigma1[1] = 0.5;
  c->sigma2[0] = -0.5;
  c->sigma2[1] = 0.0;
  c->device = -1;
  c->nranks = 1;
  c->rank = 0;
  c->rccl_id = nullptr;
}

void place_basis(nls_handle *h);

int nls_create(const nls_config *cfg, nls_handle **out) {
  if (!out) return NLS_ERR_ARG;
  *out = nullptr;
  if (!cfg) {
    g_create_error = "cfg is NULL";
    return NLS_ERR_ARG;
  }
  const nls_config &c = *cfg;
  std::string why;
  if (c.dim != 2 && c.dim != 3) why = "dim must be 2 or 3";
  else if (c.equation < 0 || c.equation > NLS_NLSE_CQ_G2) why = "unknown equation";
  else if (c.equation == NLS_SG_GAUTSCHI && c.dim != 2 && c.dim != 3) why = "bad dim";
  else if (c.nx < 2 || c.ny < 2 || (c.dim == 3 && c.nz < 2)) why = "grid too small (need >= 2 per dimension)";
  else if (!(c.dx > 0.0) || !(c.dy > 0.0)) why = "dx, dy must be > 0";
  else if (c.krylov_m < 1 || c.krylov_m > NLS_MAX_KRYLOV) why = "krylov_m must be in 1..32";
  else if (c.nranks < 1 || c.rank < 0 || c.rank >= c.nranks) why = "bad rank/nranks";
  else if (c.nranks > 1 && !c.rccl_id && !c.local_group) why = "nranks > 1 needs rccl_id or local_group";
  else if (c.local_group && static_cast<nls_group *>(c.local_group)->n != c.nranks)
    why = "local_group size != nranks";
  else if ((uint32_t)c.nranks > (c.dim == 3 ? c.nz : c.ny)) why = "more ranks than planes";
  else if ((c.equation == NLS_NLSE_G2 || c.equation == NLS_KG_GAUTSCHI) &&
           (c.nx < 3 || c.ny < 3 || (c.dim == 3 && c.nz < 3)))
    why = "G2 NLSE / KG need >= 3 cells per dimension (Neumann copy boundary)";
  else if ((c.equation == NLS_NLSE_G2 || c.equation == NLS_KG_GAUTSCHI) &&
           (uint32_t)(2 * c.nranks) > (c.dim == 3 ? c.nz : c.ny))
    why = "G2 NLSE / KG need >= 2 planes per rank";
  else if (slab_index_limit_exceeded(c))
    why = "slab too large for 32-bit cell indices: (planes per rank + 4) * plane size + 4096 must be "
          "< 2^31 (two ghost planes per side; use more ranks)";
  if (!why.empty()) {
    g_create_error = why;
    return NLS_ERR_ARG;
  }
  nls_handle *h = new (std::nothrow) nls_handle();
  if (!h) {
    g_create_error = "host allocation failed";
    return NLS_ERR_OOM;
  }
  h->cfg = c;
  h->gfun = (c.equation >= NLS_SG_G2 && c.equation <= NLS_PHI4) ? c.equation - NLS_SG_G2 : -1;
  h->cplx_ = c.equation != NLS_SG_GAUTSCHI && c.equation != NLS_KG_GAUTSCHI && h->gfun < 0;
  h->esize = h->cplx_ ? 16 : 8;
  h->m = (int)c.krylov_m;
  h->nbasis = h->cplx_ ? 1 : 2;
  h->nonlin = c.equation == NLS_NLSE_CQ ? 1 : (c.equation == NLS_NLSE_G2 ? 2 : (c.equation == NLS_NLSE_CQ_G2 ? 3 : 0));
  h->kg = c.equation == NLS_KG_GAUTSCHI;
  h->ani = c.equation == NLS_NLSE_G2 || h->kg;
  h->s1 = {c.sigma1[0], c.sigma1[1]};
  h->s2 = {c.sigma2[0], c.sigma2[1]};
  h->rank = c.rank;
  h->nranks = c.nranks;
  if (const char *e = std::getenv("NLS_GRAPH")) h->use_graph = std::atoi(e) != 0;
  if (const char *e = std::getenv("NLS_OPLOG")) h->oplog_on = std::atoi(e) != 0;
  h->dbg_sums = std::getenv("NLS_DEBUG_SUMS") != nullptr;
  h->dbg_alpha = std::getenv("NLS_DEBUG_ALPHA") != nullptr;
  if (c.device >= 0) {
    h->dev = c.device;
  } else if (hipGetDevice(&h->dev) != hipSuccess) {
    g_create_error = "no HIP device";
    delete h;
    return NLS_ERR_HIP;
  }
  int rc = guarded(h, [&] {
    hip_check(h, hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking), "hipStreamCreate");
    setup_geometry(h);
    if (h->nranks > 1 && c.local_group) {
      h->group = static_cast<nls_group *>(c.local_group);
      for (auto &e : h->evring)
        hip_check(h, hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
      std::lock_guard<std::mutex> lk(h->group->mu);
      if (!h->group->pub) {
        hip_check(h, hipMalloc(&h->group->pub, (size_t)h->nranks * 2 * NSUM * sizeof(cplx)),
                  "hipMalloc(group)");
        hip_check(h, hipMemset(h->group->pub, 0, (size_t)h->nranks * 2 * NSUM * sizeof(cplx)),
                  "hipMemset(group)");
        h->group->dev = h->dev;
      }
    } else if (h->nranks > 1) {
      ncclUniqueId id;
      std::memcpy(&id, c.rccl_id, sizeof(id));
      rccl_check(h, ncclCommInitRank(&h->comm, h->nranks, id, h->rank), "ncclCommInitRank");
    } else if (const char *e = std::getenv("NLS_FORCE_RCCL"); e && std::atoi(e)) {
      // debug: run the collective code path through a 1-rank RCCL communicator
      ncclUniqueId id;
      rccl_check(h, ncclGetUniqueId(&id), "ncclGetUniqueId");
      rccl_check(h, ncclCommInitRank(&h->comm, 1, id, 0), "ncclCommInitRank");
    }
    h->collective = h->nranks > 1 || h->comm != nullptr;
    if (h->collective) {
      // (a high-priority stream here measured every kernel of the process 2x slower)
      hip_check(h, hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking), "hipStreamCreate");
      hip_check(h, hipEventCreateWithFlags(&h->ev_bnd, hipEventDisableTiming), "hipEventCreate");
      hip_check(h, hipEventCreateWithFlags(&h->ev_halo, hipEventDisableTiming), "hipEventCreate");
      hip_check(h, hipEventCreateWithFlags(&h->ev_bdone, hipEventDisableTiming), "hipEventCreate");
    }
    alloc_all(h);  // the update launch plan depends on h->collective
    hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    place_basis(h);
  });
  if (rc != NLS_OK) {
    g_create_error = h->err;
    free_all(h);
    if (h->comm) ncclCommDestroy(h->comm);
    for (hipEvent_t e : {h->ev_bnd, h->ev_halo, h->ev_bdone})
      if (e) (void)hipEventDestroy(e);
    for (auto e : h->evring)
      if (e) (void)hipEventDestroy(e);
    if (h->cstream) (void)hipStreamDestroy(h->cstream);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return rc;
  }
  *out = h;
  return NLS_OK;
}

int nls_destroy(nls_handle *h) {
  if (!h) return NLS_ERR_ARG;
  (void)hipSetDevice(h->dev);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->cstream) (void)hipStreamSynchronize(h->cstream);
  if (h->xstream) (void)hipStreamSynchronize(h->xstream);
  if (h->stream2) (void)hipStreamSynchronize(h->stream2);
  peer_close(h);  // the neighbours' IPC mappings before our own allocations go
  if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
  for (hipEvent_t e : {h->ev_bnd, h->ev_halo, h->ev_bdone, h->ev_snap, h->ev_snap_done, h->ev_fork, h->ev_join})
    if (e) (void)hipEventDestroy(e);
  if (h->cstream) (void)hipStreamDestroy(h->cstream);
  if (h->xstream) (void)hipStreamDestroy(h->xstream);
  if (h->stream2) (void)hipStreamDestroy(h->stream2);
  for (auto &r : h->recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : h->evpool) (void)hipEventDestroy(e);
  for (auto e : h->evring)
    if (e) (void)hipEventDestroy(e);
  free_all(h);
  if (h->comm) ncclCommDestroy(h->comm);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return NLS_OK;
}

const char *nls_last_error(const nls_handle *h) {
  return h ? h->err.c_str() : g_create_error.c_str();
}

int nls_slab_planes(uint32_t npl, int32_t nranks, int32_t rank, uint32_t *z0, uint32_t *nzl) {
  if (nranks < 1 || rank < 0 || rank >= nranks || (uint32_t)nranks > npl) return NLS_ERR_ARG;
  const uint32_t base = npl / (uint32_t)nranks, rem = npl % (uint32_t)nranks;
  if (nzl) *nzl = base + ((uint32_t)rank < rem ? 1u : 0u);
  if (z0) *z0 = (uint32_t)rank * base + std::min<uint32_t>((uint32_t)rank, rem);
  return NLS_OK;
}

int nls_comm_size(const nls_handle *h, int32_t *nranks, int32_t *transport) {
  if (!h || !nranks) return NLS_ERR_ARG;
  int n = 1, tr = 0;
  if (h->comm) {
    if (ncclCommCount(h->comm, &n) != ncclSuccess) return NLS_ERR_RCCL;
    tr = 1;
  } else if (h->group) {
    n = h->group->n;
    tr = 2;
  }
  *nranks = n;
  if (transport) *transport = tr;
  return NLS_OK;
}

int nls_local_planes(const nls_handle *h, uint32_t *z0, uint32_t *nzl, uint64_t *n_local) {
  if (!h) return NLS_ERR_ARG;
  if (z0) *z0 = (uint32_t)h->geo.z0;
  if (nzl) *nzl = (uint32_t)h->geo.nzl;
  if (n_local) *n_local = (uint64_t)h->geo.nloc;
  return NLS_OK;
}

// A new solver state: the s-step bases forget the previous alpha_0 (the blind
// start's shift), so "set state; step" is bitwise reproducible run to run.
void p2_cold(nls_handle *h) {
  h->p2_warm[0] = h->p2_warm[1] = false;
  h->p2_fresh = true;
  // the tail's tile-queue counters return to 0 at the end of every launch; a launch
  // that did not complete would leave them set, and every later tail on this handle
  // would skip tiles -- every new state starts from zeroed counters
  if (h->tailq) hip_check(h, hipMemsetAsync(h->tailq, 0, tq_words() * sizeof(int32_t), h->stream), "hipMemset");
}

int nls_set_field(nls_handle *h, const double *u, uint64_t n) {
  return guarded(h, [&] {
    if (!u) fail(h, NLS_ERR_ARG, "u is NULL");
    check_len(h, n);
    if (h->cplx_) {
      hip_check(h, hipMemcpyAsync(h->u, u, (size_t)n * h->esize, hipMemcpyHostToDevice, h->stream),
                "hipMemcpy H2D");
      h->w0_ready = false;
    } else {
      copy_in_vector(h, 0, 0, u);
      halo(h, 0, 0);
    }
    p2_cold(h);  // a new field: the next bases measure alpha_0 again
    h->field_set = true;
    hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int nls_set_sg_state(nls_handle *h, const double *u, const double *u_past, const double *mfield,
                     uint64_t n) {
  return guarded(h, [&] {
    if (h->cplx_) fail(h, NLS_ERR_STATE, "nls_set_sg_state on an NLSE handle");
    // KG: m(x) may instead come with nls_set_coefficients (NULL keeps it)
    if (!u || !u_past || (!mfield && !h->kg)) fail(h, NLS_ERR_ARG, "NULL input");
    check_len(h, n);
    copy_in_vector(h, 0, 0, u);
    const size_t bytes = (size_t)n * sizeof(double);
    hip_check(h, hipMemcpyAsync(h->up, u_past, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    if (mfield)
      hip_check(h, hipMemcpyAsync(h->mf, mfield, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    halo(h, 0, 0);
    p2_cold(h);
    h->field_set = true;
    h->vel_valid = false;
    hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int nls_set_coefficients(nls_handle *h, const double *mfield, const double *cfield, uint64_t n) {
  return guarded(h, [&] {
    const bool cq_g2 = h->nonlin == 3;  // m(x) only: isotropic operator, cfield ignored
    if (!h->ani && !cq_g2) fail(h, NLS_ERR_STATE, "nls_set_coefficients on a non-G2 handle");
    if (!mfield || (!cfield && !cq_g2)) fail(h, NLS_ERR_ARG, "NULL input");
    check_len(h, n);
    const size_t bytes = (size_t)n * sizeof(double);
    hip_check(h, hipMemcpyAsync(h->mf, mfield, bytes, hipMemcpyHostToDevice, h->stream), "H2D");
    if (!cq_g2) {
      hip_check(h, hipMemcpyAsync(h->cfb + h->ghost * h->geo.P, cfield, bytes, hipMemcpyHostToDevice, h->stream),
                "H2D");
      halo_planes(h, reinterpret_cast<char *>(h->cfb + h->ghost * h->geo.P), (int64_t)sizeof(double), nullptr,
                  h->ghost);
    }
    h->coef_set = true;
    h->w0_ready = false;  // the start vector depends on m
    p2_cold(h);
    hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int nls_apply_bc(nls_handle *h) {
  return guarded(h, [&] {
    if (!h->cplx_ && !h->kg && h->gfun < 0) fail(h, NLS_ERR_STATE, "nls_apply_bc on a G1 sine-Gordon handle");
    if (!h->field_set) fail(h, NLS_ERR_STATE, "no field set");
    const Geo &g = h->geo;
    if (g.nx < 3 || g.npl < 3 || (h->cfg.dim == 3 && g.nyp < 3))
      fail(h, NLS_ERR_ARG, "Neumann copy boundary needs >= 3 cells per dimension");
    if ((g.z0 == 0 || g.z0 + g.nzl == g.npl) && g.nzl < 2)
      fail(h, NLS_ERR_ARG, "Neumann copy boundary needs >= 2 planes on the boundary slabs");
    // KGESolverDevice::apply_bc (nlsolvers/device/include/kg_dev.hpp) and the G2
    // Gautschi family's apply_bc (e.g. phi4_dev.hpp:92): u only
    if (!h->cplx_) {
      void *u = vec_ptr(h, 0, 0);
      Geo gg = g;
      const int64_t cells = neumann_bc_cells(g);
      const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((cells + NTHREADS - 1) / NTHREADS, 4096));
      void *args[] = {&u, &gg};
      launch(h, 3, -1, kernel_neumann_bc_r(), grid, args);
      halo(h, 0, 0);
      hip_check(h, hipGetLastError(), "kernel launch");
      return;
    }
    // the start vector of the next step (N(u) with the last step's dt, kept
    // from the final pass) is refreshed on the same boundary cells
    const bool refresh = h->w0_ready;
    double dt = h->w0_dt;
    void *w0 = vec_ptr(h, 0, 0);
    Geo gg = g;
    int wr = refresh ? 1 : 0, nl = h->nonlin;
    const int64_t cells = neumann_bc_cells(g);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((cells + NTHREADS - 1) / NTHREADS, 4096));
    void *args[] = {&h->u, &w0, &h->mf, &gg, &wr, &dt, &nl, &h->s1, &h->s2};
    launch(h, 3, -1, kernel_neumann_bc(), grid, args);
    if (refresh) halo(h, 0, 0);
    hip_check(h, hipGetLastError(), "kernel launch");
  });
}

// One Strang SS2 step of an NLSE handle.
// NLSESolverDevice::step (device/nlse_solver_dev.hpp:94-111), tau = 1j*dt:
//   N(1/2) -> exp(L*dt) via exp(t|lambda|), t = -tau -> N(1/2)
// G2 (nlsolvers/device/include/nlse_dev.hpp:187-203): N uses +tau/2 m|u|^2
// and the linear flow is exp(t*lambda) with t = +tau
// (nlsolvers/device/include/matfunc_complex.hpp:281-287).
// Does the step end this basis with the fused tail k_tail<mode>?
bool use_tail(const nls_handle *h, int mode) { return h->fused_tail && h->tail_grid[mode] > 0; }

void tail_launch(nls_handle *h, int mode, TailArgs ta) {
  Geo g = h->geo;
  if (h->kz_fused) g.kz = h->kz_fused;
  if (h->tail_dyn) g.tq = h->tailq;
  void *args[] = {&ta, &g};
  launch(h, 5, h->m, kernel_tail(tail_is_cplx(h, mode), (int)h->cfg.dim, mode, h->m, h->ani),
         h->tail_dyn ? h->tail_dyn_grid[mode] : h->tail_grid[mode], args);
}

TailArgs tail_args(nls_handle *h, int b) {
  TailArgs ta{};
  ta.W = vec_ptr(h, b, 0);
  ta.vs = h->vs;
  ta.st = h->B[b].st;
  ta.mf = h->mf;
  ta.nonlin = h->nonlin;
  ta.s1 = h->s1;
  ta.s2 = h->s2;
  return ta;
}

void ss2_step(nls_handle *h, double dt) {
  const int m = h->m;
  const int64_t n = h->geo.nloc;
  int64_t vs = h->vs;
  if (!h->w0_ready || h->w0_dt != dt) {
    void *w0 = vec_ptr(h, 0, 0);
    int nl = h->nonlin;
    void *args[] = {&h->u, &w0, &h->mf, (void *)&n, &dt, &nl, &h->s1, &h->s2};
    pw_launch(h, 3, kernel_nl_init(), args);
    halo(h, 0, 0);
  }
  const bool tail = use_tail(h, TAIL_NLSE);
  // the linear flow: G1 exp(t|lambda|), t = -tau (eigen_krylov_complex.hpp:71-77); G2
  // cubic exp(t lambda), t = +tau (nlse_dev.hpp:196); G2 cubic-quintic exp(t lambda),
  // t = -tau (nlse_cubic_quintic_dev.hpp:86)
  const int lf = (h->ani || h->nonlin == 3) ? NLS_F_EXP : NLS_F_EXP_ABS;
  const double ltr = h->ani ? 0.0 : -0.0, lti = h->ani ? dt : -dt;
  if (h->pass2) run_lanczos2(h, 0, 1, lf, 0, ltr, lti);
  else run_lanczos(h, 0, 1, lf, 0, ltr, lti, tail);
  void *W = vec_ptr(h, 0, 0);
  KState *st = h->B[0].st;
  int nl = h->nonlin;
  if (tail) {
    TailArgs ta = tail_args(h, 0);
    // u = N(y) only where a caller can see it: a step followed by another step of
    // the same nls_step call needs just the next start vector N(N(y)) (W_0)
    ta.u = h->skip_u ? nullptr : h->u;
    ta.dt = dt;
    tail_launch(h, TAIL_NLSE, ta);
  } else {
    void *args[] = {&W, &vs, (void *)&n, &st, &h->u, &h->mf, &dt, &nl, &h->s1, &h->s2};
    pw_launch(h, 3, kernel_final_nlse(m), args);
  }
  halo(h, 0, 0);
  h->w0_ready = true;
  h->w0_dt = dt;
}

// Basis placement (nls_placement; DESIGN.md section 4 "Placement").  The same kernels on
// the same handle run 2-4 % faster or slower in different processes according to which
// HBM pages back the basis (profiles/r05/envab_prepad.txt: a 4 GB dummy allocation ahead
// of the basis selected the fast passes in every process); no allocation call chooses
// pages.  So the handle chooses among allocations: up to NLS_PLACE candidate bases
// (default 8; those that fit in free memory beside an 8 GB reserve) are allocated while
// the earlier ones are held, each runs the same probe -- one cold SS2 step, then
// PLACE_STEPS timed steps of the real launch sequence on a constant field -- and the
// fastest is kept.  512^3 m = 16 (profiles/r06/envab_place.txt): 30.40-31.52 ms per step
// with one allocation, 29.98-30.44 with the probe.
// Everything the probe wrote is reset to the state alloc_all left (bases, Lanczos state,
// tile-queue counters zero; no live start vector), so no result depends on the choice.
// Large single-rank complex handles with the s-step passes (the 512^3 class); others
// keep their one allocation.
constexpr int PLACE_STEPS = 3;  // timed probe steps per candidate
void place_basis(nls_handle *h) {
  int K = 8;
  if (const char *e = std::getenv("NLS_PLACE")) K = std::atoi(e);
  K = std::min(K, NLS_PLACE_MAX);
  const bool contig = std::getenv("NLS_DEBUG_CONTIG") && std::atoi(std::getenv("NLS_DEBUG_CONTIG"));
  if (K <= 1 || contig || h->collective || !h->cplx_ || !h->pass2 || h->p2reg || h->ani || !h->large ||
      h->nbasis != 1 || h->cfg.dim != 3 || h->prepad)
    return;
  const size_t bytes = (size_t)h->nvec[0] * h->vs * h->esize;
  size_t fr = 0, tot = 0;
  hip_check(h, hipMemGetInfo(&fr, &tot), "hipMemGetInfo");
  const size_t reserve = size_t(8) << 30;
  const int fit = fr > reserve ? (int)((fr - reserve) / bytes) : 0;
  K = std::min(K, 1 + fit);
  if (K <= 1) return;
  std::vector<void *> cand{h->B[0].W};
  hipEvent_t e0 = nullptr, e1 = nullptr;
  auto reset = [&] {
    // the state alloc_all leaves: zero basis (out-of-grid ghost planes included), zero
    // Lanczos state, zero tile-queue counters, no live start vector
    hip_check(h, hipMemsetAsync(h->B[0].W, 0, bytes, h->stream), "hipMemset");
    hip_check(h, hipMemsetAsync(h->B[0].st, 0, sizeof(KState), h->stream), "hipMemset");
    hip_check(h, hipMemsetAsync(h->p2, 0, p2state_bytes() * h->nbasis, h->stream), "hipMemset");
    p2_cold(h);
    h->w0_ready = false;
  };
  try {
    hip_check(h, hipEventCreate(&e0), "hipEventCreate");
    hip_check(h, hipEventCreate(&e1), "hipEventCreate");
    const size_t nb = (size_t)h->geo.nloc * h->esize;
    const double dt = 1e-3;
    for (int c = 0; c < K; ++c) {
      if (c > 0) {
        void *w = nullptr;
        if (hipMalloc(&w, bytes) != hipSuccess) {
          (void)hipGetLastError();
          break;
        }
        cand.push_back(w);
      }
      h->B[0].W = cand[c];
      reset();
      // a constant field (0x3FF00000 words: each value ~ 1 + 2^-20 in both parts); its
      // Krylov space grows from the boundary layer, no breakdown within m vectors
      hip_check(h, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(h->u), 0x3FF00000, nb / 4, h->stream),
                "hipMemsetD32");
      ss2_step(h, dt);  // cold: the alpha_0 pass; later steps start blind, as a run does
      hip_check(h, hipEventRecord(e0, h->stream), "hipEventRecord");
      for (int s = 0; s < PLACE_STEPS; ++s) ss2_step(h, dt);
      hip_check(h, hipEventRecord(e1, h->stream), "hipEventRecord");
      hip_check(h, hipEventSynchronize(e1), "hipEventSynchronize");
      float ms = 0.f;
      hip_check(h, hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
      h->place_ms[c] = ms;
    }
  } catch (...) {
    h->B[0].W = cand[0];
    for (size_t c = 1; c < cand.size(); ++c) (void)hipFree(cand[c]);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    throw;
  }
  h->place_n = (int)cand.size();
  int best = 0;
  for (int c = 1; c < h->place_n; ++c)
    if (h->place_ms[c] < h->place_ms[best]) best = c;
  h->place_pick = best;
  hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  for (int c = 0; c < h->place_n; ++c)
    if (c != best) (void)hipFree(cand[c]);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  h->B[0].W = cand[best];
  reset();
  hip_check(h, hipMemsetAsync(h->u, 0, (size_t)h->geo.nloc * h->esize, h->stream), "hipMemset");
  hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  if (std::getenv("NLS_PLACE_LOG")) {
    std::fprintf(stderr, "[nls] placement: %d candidates, kept %d; probe ms", h->place_n, best);
    for (int c = 0; c < h->place_n; ++c) std::fprintf(stderr, " %.3f", h->place_ms[c]);
    std::fprintf(stderr, "\n");
  }
}

// Work issued inside the scope goes to the handle's second stream with the second set
// of partial buffers (KG's sinc^2 basis, sEWI's exp(2 tau L) action): everything in
// the issue path takes h->stream / h->partP2 / h->partA.
struct OnStream2 {
  nls_handle *h;
  explicit OnStream2(nls_handle *hh) : h(hh) { flip(); }
  ~OnStream2() { flip(); }
  void flip() {
    std::swap(h->stream, h->stream2);
    std::swap(h->partP2, h->partP2b);
    std::swap(h->partA, h->partAb);
  }
};

// sEWI on one rank with the s-step passes: the third Krylov action (exp(2 tau L) u_prev)
// does not depend on the first two, so it runs on a second basis and stream while they
// run (its Lanczos and theirs overlap each other's chains of small reduction kernels).
// The second basis is allocated on the first sEWI step; if the memory is not there the
// step stays serial.
bool sewi_concurrent(nls_handle *h) {
  // (not the register form: its y = L S_J buffer is one per handle)
  if (!NLS_KG_CONCURRENT || h->collective || !h->pass2 || h->p2reg || !use_tail(h, TAIL_SEWI_END)) return false;
  if (h->timing) return false;  // per-kernel timing: the serial order (bit-identical; see issue_step's KG)
  if (h->B[1].W) return true;
  if (h->sewi_serial) return false;
  if (const char *e = std::getenv("NLS_SEWI_CONCURRENT"))  // 0: the serial order (A/B)
    if (std::atoi(e) == 0) return false;
  const size_t bytes = (size_t)h->nvec[0] * h->vs * h->esize;
  const size_t psb = p2state_bytes();
  const size_t na = std::max<size_t>(2 * (size_t)h->grid_alpha, 3 * (size_t)h->grid_alpha2);
  // The second basis doubles the handle's basis memory (knob table): take
  // it only with a quarter of the device's memory (at least 4 GB) still free beside it, so
  // buffers this handle or the application allocate later do not fail where they would
  // not have; otherwise the step stays serial
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < bytes + std::max(tot / 4, size_t(4) << 30)) {
    (void)hipGetLastError();
    h->sewi_serial = true;
    return false;
  }
  void *W = nullptr, *st = nullptr, *p2 = nullptr, *pa = nullptr, *pp = nullptr;
  bool ok = hipMalloc(&W, bytes) == hipSuccess && hipMalloc(&st, sizeof(KState)) == hipSuccess &&
            hipMalloc(&p2, 2 * psb) == hipSuccess && hipMalloc(&pa, na * sizeof(cplx)) == hipSuccess &&
            hipMalloc(&pp, (size_t)h->p2grid * (3 * MMAX + 8) * sizeof(cplx)) == hipSuccess;
  if (ok && !h->stream2) {
    ok = hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking) == hipSuccess &&
         hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) == hipSuccess;
  }
  if (!ok) {
    (void)hipGetLastError();
    for (void *q : {W, st, p2, pa, pp})
      if (q) (void)hipFree(q);
    h->sewi_serial = true;
    return false;
  }
  hip_check(h, hipMemsetAsync(W, 0, bytes, h->stream), "hipMemset");
  hip_check(h, hipMemsetAsync(st, 0, sizeof(KState), h->stream), "hipMemset");
  hip_check(h, hipMemsetAsync(static_cast<char *>(p2) + psb, 0, psb, h->stream), "hipMemset");
  hip_check(h, hipMemcpyAsync(p2, h->p2, psb, hipMemcpyDeviceToDevice, h->stream), "hipMemcpy(P2State)");
  hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  // a step graph captured by nls_step holds the old P2State address: re-capture
  if (h->gexec) {
    hip_check(h, hipGraphExecDestroy(h->gexec), "hipGraphExecDestroy");
    h->gexec = nullptr;
  }
  (void)hipFree(h->p2);
  h->p2 = p2;
  h->B[1].W = W;
  h->B[1].st = static_cast<KState *>(st);
  h->nvec[1] = h->nvec[0];
  h->partAb = static_cast<cplx *>(pa);
  h->partP2b = static_cast<cplx *>(pp);
  return true;
}

// One of the three Krylov actions of an sEWI step on basis 0: the two-vector passes
// where the handle has them (always ending in the fused tail; each action starts cold,
// with its own alpha_0 as the first shift -- the three start vectors differ), else the
// one-vector passes.
void sewi_lanczos(nls_handle *h, int f, double tr, double ti, bool &tail) {
  if (h->pass2) {
    if (!tail) fail(h, NLS_ERR_STATE, "two-vector passes without a fused tail kernel");
    h->p2_warm[0] = false;
    run_lanczos2(h, 0, 1, f, 0, tr, ti);
  } else {
    run_lanczos(h, 0, 1, f, 0, tr, ti, tail);
  }
}

int nls_step_sewi(nls_handle *h, double dt, uint32_t step_number) {
  return guarded(h, [&] {
    if (!h->ani || h->kg) fail(h, NLS_ERR_STATE, "nls_step_sewi needs a G2 (NLS_NLSE_G2) handle");
    if (!h->field_set) fail(h, NLS_ERR_STATE, "no field set");
    if (!h->coef_set) fail(h, NLS_ERR_STATE, "G2: nls_set_coefficients not called");
    if (!std::isfinite(dt)) fail(h, NLS_ERR_ARG, "dt not finite");
    if (step_number == 0) fail(h, NLS_ERR_ARG, "step numbers start at 1 (nlse_dev.hpp:206)");
    h->skip_u = false;  // step 1's SS2 step writes u
    const int m = h->m;
    int64_t n = h->geo.nloc, vs = h->vs;
    const size_t bytes = (size_t)n * sizeof(cplx);
    if (!h->uprev) hip_check(h, hipMalloc(&h->uprev, bytes), "hipMalloc(u_prev)");
    if (step_number == 1) {  // nlse_dev.hpp:206-210: u_prev = u, then an SS2 step
      hip_check(h, hipMemcpyAsync(h->uprev, h->u, bytes, hipMemcpyDeviceToDevice, h->stream), "D2D");
      h->uprev_set = true;
      ss2_step(h, dt);
    } else {
      if (!h->uprev_set) fail(h, NLS_ERR_STATE, "sEWI step > 1 before step 1 (no u_prev)");
      ensure_scratch(h);
      void *W = vec_ptr(h, 0, 0);
      KState *st = h->B[0].st;
      // exp(2 tau L) u_prev on the second basis and stream, concurrently with the rest
      const bool conc = sewi_concurrent(h);
      if (conc) {
        hip_check(h, hipEventRecord(h->ev_fork, h->stream), "hipEventRecord");
        hip_check(h, hipStreamWaitEvent(h->stream2, h->ev_fork, 0), "hipStreamWaitEvent");
        OnStream2 sw(h);
        hip_check(h, hipMemcpyAsync(vec_ptr(h, 1, 0), h->uprev, bytes, hipMemcpyDeviceToDevice, h->stream), "D2D");
        halo(h, 1, 0);
        h->p2_warm[1] = false;
        run_lanczos2(h, 1, 1, NLS_F_EXP, 0, 0.0, 2.0 * dt);
        hip_check(h, hipEventRecord(h->ev_join, h->stream), "hipEventRecord");
      }
      // B(u) -> sinc(dt L) B -> exp(tau L) (.) -> e (scratch)
      {
        void *args[] = {&h->u, &h->mf, &W, &n};
        pw_launch(h, 3, kernel_sewi_b(), args);
        halo(h, 0, 0);
      }
      // each of the three actions may end in a fused tail (k_tail)
      bool tail = use_tail(h, TAIL_COMBINE_W0);
      sewi_lanczos(h, NLS_F_SINC, dt, 0.0, tail);
      if (tail) {
        tail_launch(h, TAIL_COMBINE_W0, tail_args(h, 0));
      } else {
        void *args[] = {&W, &vs, &n, &st};
        pw_launch(h, 3, kernel_combine_w0(m), args);
      }
      halo(h, 0, 0);
      tail = use_tail(h, TAIL_COMBINE);
      sewi_lanczos(h, NLS_F_EXP, 0.0, dt, tail);
      if (tail) {
        TailArgs ta = tail_args(h, 0);
        ta.out = h->scratch;
        tail_launch(h, TAIL_COMBINE, ta);
      } else {
        void *args[] = {&W, &vs, &n, &st, &h->scratch};
        pw_launch(h, 3, kernel_combine(true, m), args);
      }
      // exp(2 tau L) u_prev, then u = that - 2 tau e, u_prev <- old u
      const int b3 = conc ? 1 : 0;
      if (conc) {
        hip_check(h, hipStreamWaitEvent(h->stream, h->ev_join, 0), "hipStreamWaitEvent");
        tail = true;
      } else {
        hip_check(h, hipMemcpyAsync(W, h->uprev, bytes, hipMemcpyDeviceToDevice, h->stream), "D2D");
        halo(h, 0, 0);
        tail = use_tail(h, TAIL_SEWI_END);
        sewi_lanczos(h, NLS_F_EXP, 0.0, 2.0 * dt, tail);
      }
      if (tail) {
        TailArgs ta = tail_args(h, b3);
        ta.u = h->u;
        ta.up = h->uprev;
        ta.e = h->scratch;
        ta.dt = dt;
        tail_launch(h, TAIL_SEWI_END, ta);
      } else {
        void *args[] = {&W, &vs, &n, &st, &h->u, &h->uprev, &h->scratch, &dt};
        pw_launch(h, 3, kernel_sewi_end(m), args);
      }
      h->w0_ready = false;
    }
    h->tacc.steps += 1;
    hip_check(h, hipGetLastError(), "kernel launch");
  });
}

// Device work of one nls_step step (every equation but sEWI).
void issue_step(nls_handle *h, double dt) {
  const int m = h->m;
  const int64_t n = h->geo.nloc;
  int64_t vs = h->vs;
  if (h->cplx_) {
    ss2_step(h, dt);
  } else if (h->kg) {
    // KGESolver::step (nlsolvers/device/include/kg_single.cuh:49-86): sinc^2 basis
    // of g = -m u^3, cos basis of u (the operator sign is immaterial: both
    // functions depend on sqrt|lambda| only)
    {
      void *u = vec_ptr(h, 0, 0);
      void *g0 = vec_ptr(h, 1, 0);
      void *args[] = {&u, &h->mf, &g0, (void *)&n};
      pw_launch(h, 3, kernel_kg_g(), args);
      halo(h, 1, 0);
    }
    if (h->pass2) {
      // s-step passes (k_p2d on cell pairs): the sinc^2 action into the g basis's own
      // W_0 (TAIL_COMBINE_W0), then the cos basis ends in the Gautschi update that reads
      // that one vector (TAIL_KG_END1).  On one rank the two bases run concurrently
      // (each basis' chain of small reduction kernels then overlaps the other's passes)
      // (with per-kernel timing on, the serial order -- bit-identical -- so no kernel's
      // events span another stream's work and the class times add up to wall time)
      if (h->stream2 && !h->timing) {
        hip_check(h, hipEventRecord(h->ev_fork, h->stream), "hipEventRecord");
        hip_check(h, hipStreamWaitEvent(h->stream2, h->ev_fork, 0), "hipStreamWaitEvent");
        {
          OnStream2 sw(h);
          run_lanczos2(h, 1, 1, NLS_F_SINC2_SQRT, 0, dt, 0.0);
          tail_launch(h, TAIL_COMBINE_W0, tail_args(h, 1));
          hip_check(h, hipEventRecord(h->ev_join, h->stream), "hipEventRecord");
        }
        run_lanczos2(h, 0, 1, NLS_F_COS_SQRT, 0, dt, 0.0);
        hip_check(h, hipStreamWaitEvent(h->stream, h->ev_join, 0), "hipStreamWaitEvent");
      } else {
        run_lanczos2(h, 1, 1, NLS_F_SINC2_SQRT, 0, dt, 0.0);
        tail_launch(h, TAIL_COMBINE_W0, tail_args(h, 1));
        run_lanczos2(h, 0, 1, NLS_F_COS_SQRT, 0, dt, 0.0);
      }
      TailArgs ta = tail_args(h, 0);
      ta.W2 = vec_ptr(h, 1, 0);
      ta.up = h->up;
      ta.v = h->vel;
      ta.dt = dt;
      tail_launch(h, TAIL_KG_END1, ta);
      halo(h, 0, 0);
      h->vel_valid = true;
      return;
    }
    // the sinc^2 basis is stored in full; the cos basis may end in the fused tail
    const bool tail = use_tail(h, TAIL_KG_END);
    run_lanczos(h, 1, 1, NLS_F_SINC2_SQRT, 0, dt, 0.0);
    run_lanczos(h, 0, 1, NLS_F_COS_SQRT, 0, dt, 0.0, tail);
    if (tail) {
      TailArgs ta = tail_args(h, 0);
      ta.W2 = vec_ptr(h, 1, 0);
      ta.st2 = h->B[1].st;
      ta.up = h->up;
      ta.v = h->vel;
      ta.dt = dt;
      tail_launch(h, TAIL_KG_END, ta);
    } else {
      void *W = vec_ptr(h, 0, 0);
      void *W2 = vec_ptr(h, 1, 0);
      KState *st = h->B[0].st, *st2 = h->B[1].st;
      void *args[] = {&W, &W2, &vs, (void *)&n, &st, &st2, &h->up, &h->vel, &dt};
      pw_launch(h, 3, kernel_kg_end(m), args);
    }
    halo(h, 0, 0);
    h->vel_valid = true;
  } else {
    // SGESolver::step (sg_solver.hpp:53-74): id and cos share the basis of u.
    // G2 Gautschi family (e.g. phi4_single.cuh:33-47): the same sequence with
    // g = -m F(id u) and sinc^2(t sqrt|lambda|) instead of the G1 half argument.
    const int mid = h->gfun >= 0 ? TAIL_GG_MID : TAIL_SG_MID;
    bool tail = use_tail(h, mid) || h->pass2;  // the s-step passes always end in the tail
    if (h->pass2) run_lanczos2(h, 0, 2, NLS_F_ID_SQRT, NLS_F_COS_SQRT, dt, 0.0);
    else run_lanczos(h, 0, 2, NLS_F_ID_SQRT, NLS_F_COS_SQRT, dt, 0.0, tail);
    if (tail) {
      TailArgs ta = tail_args(h, 0);
      ta.out = vec_ptr(h, 1, 0);
      ta.up = h->up;
      ta.nonlin = h->gfun;
      tail_launch(h, mid, ta);
    } else {
      void *W = vec_ptr(h, 0, 0);
      void *g0 = vec_ptr(h, 1, 0);
      KState *st = h->B[0].st;
      int gf = h->gfun;
      void *args[] = {&W, &vs, (void *)&n, &st, &h->mf, &h->up, &g0, &gf};
      pw_launch(h, 3, kernel_sg_mid(m), args);
    }
    halo(h, 1, 0);
    tail = use_tail(h, TAIL_SG_END) || h->pass2;
    if (h->pass2) run_lanczos2(h, 1, 1, h->gfun >= 0 ? NLS_F_SINC2_SQRT : NLS_F_SINC2_HALF, 0, dt, 0.0);
    else run_lanczos(h, 1, 1, h->gfun >= 0 ? NLS_F_SINC2_SQRT : NLS_F_SINC2_HALF, 0, dt, 0.0, tail);
    if (tail) {
      TailArgs ta = tail_args(h, 1);
      ta.u = vec_ptr(h, 0, 0);
      ta.up = h->up;
      ta.dt = dt;
      tail_launch(h, TAIL_SG_END, ta);
    } else {
      void *W2 = vec_ptr(h, 1, 0);
      void *u = vec_ptr(h, 0, 0);
      KState *st = h->B[1].st;
      void *args[] = {&W2, &vs, (void *)&n, &st, &u, &h->up, &dt};
      pw_launch(h, 3, kernel_sg_end(m), args);
    }
    halo(h, 0, 0);
  }
}

// Host-side state a step leaves behind (what issue_step sets besides the launches).
void finish_step_flags(nls_handle *h, double dt) {
  if (h->cplx_) {
    h->w0_ready = true;
    h->w0_dt = dt;
  } else if (h->kg) {
    h->vel_valid = true;
  }
}

// A step whose launch sequence is fixed can replay a captured graph: single
// rank (no RCCL / local-transport exchanges in the step), no per-kernel timing
// events, and for the NLSE a live start vector W_0 built with this dt (otherwise
// the step begins with k_nl_init).  The graph is captured on first use per dt.
bool graph_ready(nls_handle *h, double dt) {
  if (!h->use_graph || h->collective || h->timing) return false;
  if (h->pass2 && h->p2_fresh) return false;  // the first step after nls_set_*: cold bases
  if (h->cplx_ && (!h->w0_ready || h->w0_dt != dt)) return false;
  if (h->gexec && h->gdt == dt) return true;
  if (h->gexec) {
    hip_check(h, hipGraphExecDestroy(h->gexec), "hipGraphExecDestroy");
    h->gexec = nullptr;
  }
  hipGraph_t g = nullptr;
  h->skip_u = false;  // a captured step always writes u
  hip_check(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
  try {
    issue_step(h, dt);
  } catch (...) {
    (void)hipStreamEndCapture(h->stream, &g);
    if (g) (void)hipGraphDestroy(g);
    throw;
  }
  hip_check(h, hipStreamEndCapture(h->stream, &g), "hipStreamEndCapture");
  const hipError_t e = hipGraphInstantiate(&h->gexec, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  hip_check(h, e, "hipGraphInstantiate");
  h->gdt = dt;
  return true;
}

int nls_step(nls_handle *h, double dt, uint32_t nsteps) {
  return guarded(h, [&] {
    if (!h->field_set) fail(h, NLS_ERR_STATE, "no field set");
    if ((h->ani || h->nonlin == 3) && !h->coef_set) fail(h, NLS_ERR_STATE, "G2: nls_set_coefficients not called");
    if (!std::isfinite(dt)) fail(h, NLS_ERR_ARG, "dt not finite");
    if (h->kg && !(dt > 0.0)) fail(h, NLS_ERR_ARG, "KG: dt must be > 0 (v = (u - u_past)/dt)");
    for (uint32_t s = 0; s < nsteps; ++s) {
      if (graph_ready(h, dt)) {
        hip_check(h, hipGraphLaunch(h->gexec, h->stream), "hipGraphLaunch");
        finish_step_flags(h, dt);
        h->tacc.graph_steps += 1;
      } else {
        // u = N(y) is skipped only inside this call (another step follows); the
        // guard clears the flag however issue_step leaves
        struct SkipU {
          nls_handle *h;
          ~SkipU() { h->skip_u = false; }
        } guard{h};
        h->skip_u = s + 1 < nsteps;
        issue_step(h, dt);
        h->p2_fresh = false;  // every basis of the step is warm now
      }
      h->tacc.steps += 1;
    }
    hip_check(h, hipGetLastError(), "kernel launch");
  });
}

int nls_sync(nls_handle *h) {
  return guarded(h, [&] { hip_check(h, hipStreamSynchronize(h->stream), "nls_sync"); });
}

int nls_get_field(nls_handle *h, double *u, uint64_t n) {
  return guarded(h, [&] {
    if (!u) fail(h, NLS_ERR_ARG, "u is NULL");
    check_len(h, n);
    const void *src = h->cplx_ ? h->u : (const void *)vec_ptr(h, 0, 0);
    hip_check(h, hipMemcpyAsync(u, src, (size_t)n * h->esize, hipMemcpyDeviceToHost, h->stream),
              "hipMemcpy D2H");
    hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int nls_get_field_async(nls_handle *h, double *dst, uint64_t n) {
  return guarded(h, [&] {
    if (!dst) fail(h, NLS_ERR_ARG, "dst is NULL");
    check_len(h, n);
    const size_t bytes = (size_t)n * h->esize;
    if (!h->xstream) {
      hip_check(h, hipStreamCreateWithFlags(&h->xstream, hipStreamNonBlocking), "hipStreamCreate");
      hip_check(h, hipEventCreateWithFlags(&h->ev_snap, hipEventDisableTiming), "hipEventCreate");
      hip_check(h, hipEventCreateWithFlags(&h->ev_snap_done, hipEventDisableTiming), "hipEventCreate");
      hip_check(h, hipMalloc(&h->snap, bytes), "hipMalloc(snapshot staging)");
    }
    // the staging buffer is free once the previous transfer has finished
    if (h->snap_issued)
      hip_check(h, hipStreamWaitEvent(h->stream, h->ev_snap_done, 0), "hipStreamWaitEvent");
    const void *src = h->cplx_ ? h->u : (const void *)vec_ptr(h, 0, 0);
    hip_check(h, hipMemcpyAsync(h->snap, src, bytes, hipMemcpyDeviceToDevice, h->stream),
              "hipMemcpyAsync(snapshot D2D)");
    hip_check(h, hipEventRecord(h->ev_snap, h->stream), "hipEventRecord");
    hip_check(h, hipStreamWaitEvent(h->xstream, h->ev_snap, 0), "hipStreamWaitEvent");
    hip_check(h, hipMemcpyAsync(dst, h->snap, bytes, hipMemcpyDeviceToHost, h->xstream),
              "hipMemcpyAsync(snapshot D2H)");
    hip_check(h, hipEventRecord(h->ev_snap_done, h->xstream), "hipEventRecord");
    h->snap_issued = true;
  });
}

int nls_wait_field(nls_handle *h) {
  if (!h) return NLS_ERR_ARG;
  if (!h->snap_issued) return NLS_OK;
  // no handle state is touched: safe from a second host thread
  (void)hipSetDevice(h->dev);
  const hipError_t e = hipEventSynchronize(h->ev_snap_done);
  if (e != hipSuccess) return e == hipErrorOutOfMemory ? NLS_ERR_OOM : NLS_ERR_HIP;
  return NLS_OK;
}

int nls_host_alloc(uint64_t bytes, void **out) {
  if (!out) return NLS_ERR_ARG;
  *out = nullptr;
  if (hipHostMalloc(out, bytes == 0 ? 1 : (size_t)bytes, hipHostMallocDefault) != hipSuccess) {
    g_create_error = "hipHostMalloc failed";
    return NLS_ERR_OOM;
  }
  return NLS_OK;
}

int nls_host_free(void *p) {
  if (p && hipHostFree(p) != hipSuccess) return NLS_ERR_HIP;
  return NLS_OK;
}

int nls_get_sg_velocity(nls_handle *h, double dt, double *v, uint64_t n) {
  return guarded(h, [&] {
    if (h->cplx_) fail(h, NLS_ERR_STATE, "velocity of an NLSE handle");
    if (!v) fail(h, NLS_ERR_ARG, "v is NULL");
    check_len(h, n);
    if (h->kg && h->vel_valid) {  // stored by the last step (kg_single.cuh:80-85)
      hip_check(h, hipMemcpyAsync(v, h->vel, (size_t)n * 8, hipMemcpyDeviceToHost, h->stream),
                "hipMemcpy D2H");
      hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
      return;
    }
    ensure_scratch(h);
    void *u = vec_ptr(h, 0, 0);
    int64_t nn = (int64_t)n;
    void *args[] = {&u, &h->up, &h->scratch, &nn, &dt};
    pw_launch(h, 3, kernel_sg_velocity(), args);
    hip_check(h, hipMemcpyAsync(v, h->scratch, (size_t)n * 8, hipMemcpyDeviceToHost, h->stream),
              "hipMemcpy D2H");
    hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int nls_krylov_apply(nls_handle *h, const double *in, double t_re, double t_im, int32_t func,
                     double *out, uint64_t n) {
  return guarded(h, [&] {
    if (!in || !out) fail(h, NLS_ERR_ARG, "NULL buffer");
    if (func < 0 || func > 7) fail(h, NLS_ERR_ARG, "unknown func");
    if ((h->ani || h->nonlin == 3) && !h->coef_set) fail(h, NLS_ERR_STATE, "G2: nls_set_coefficients not called");
    check_len(h, n);
    const int b = h->cplx_ ? 0 : 1;  // SG: the scratch basis keeps u intact
    ensure_scratch(h);
    copy_in_vector(h, b, 0, in);
    if (h->cplx_) h->w0_ready = false;
    halo(h, b, 0);
    const bool tail = use_tail(h, TAIL_COMBINE);
    run_lanczos(h, b, 1, func, 0, t_re, t_im, tail);
    if (tail) {
      TailArgs ta = tail_args(h, b);
      ta.out = h->scratch;
      tail_launch(h, TAIL_COMBINE, ta);
    } else {
      void *W = vec_ptr(h, b, 0);
      int64_t vs = h->vs, nn = (int64_t)n;
      KState *st = h->B[b].st;
      void *args[] = {&W, &vs, &nn, &st, &h->scratch};
      pw_launch(h, 3, kernel_combine(h->cplx_, h->m), args);
    }
    hip_check(h, hipMemcpyAsync(out, h->scratch, (size_t)n * h->esize, hipMemcpyDeviceToHost,
                                h->stream),
              "hipMemcpy D2H");
    hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int nls_laplacian_apply(nls_handle *h, const double *x, double *y, uint64_t n) {
  return guarded(h, [&] {
    if (!x || !y) fail(h, NLS_ERR_ARG, "NULL buffer");
    if ((h->ani || h->nonlin == 3) && !h->coef_set) fail(h, NLS_ERR_STATE, "G2: nls_set_coefficients not called");
    check_len(h, n);
    const int b = h->cplx_ ? 0 : 1;
    ensure_scratch(h);
    copy_in_vector(h, b, 0, x);
    if (h->cplx_) h->w0_ready = false;
    halo(h, b, 0);
    void *v0 = vec_ptr(h, b, 0);
    Geo g = h->geo;
    void *args[] = {&v0, &g, &h->scratch};
    launch(h, 0, -1, kernel_lap(h->cplx_, (int)h->cfg.dim, h->ani), h->grid_lap, args);
    hip_check(h, hipMemcpyAsync(y, h->scratch, (size_t)n * h->esize, hipMemcpyDeviceToHost,
                                h->stream),
              "hipMemcpy D2H");
    hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int nls_rccl_unique_id(void *out128) {
  if (!out128) return NLS_ERR_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) {
    g_create_error = "ncclGetUniqueId failed";
    return NLS_ERR_RCCL;
  }
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out128, &id, sizeof(id));
  return NLS_OK;
}

int nls_group_create(int32_t nranks, nls_group **out) {
  if (!out || nranks < 1) return NLS_ERR_ARG;
  nls_group *g = new (std::nothrow) nls_group();
  if (!g) return NLS_ERR_OOM;
  g->n = nranks;
  g->slots.resize(nranks);
  g->done.resize(nranks);
  *out = g;
  return NLS_OK;
}

int nls_group_destroy(nls_group *g) {
  if (!g) return NLS_ERR_ARG;
  if (g->pub) {
    (void)hipSetDevice(g->dev);
    (void)hipFree(g->pub);
  }
  delete g;
  return NLS_OK;
}

int nls_set_timing(nls_handle *h, int32_t enable) {
  return guarded(h, [&] {
    if (!enable) harvest_timing(h);
    h->timing = enable != 0;
  });
}

int nls_get_timing(nls_handle *h, nls_timing *out) {
  return guarded(h, [&] {
    if (!out) fail(h, NLS_ERR_ARG, "out is NULL");
    harvest_timing(h);
    *out = h->tacc;
  });
}

int nls_debug_oplog(nls_handle *h, int32_t *out, uint64_t cap, uint64_t *n) {
  if (!h || !n) return NLS_ERR_ARG;
  const uint64_t cnt = h->oplog.size();
  *n = cnt;
  if (!out) return NLS_OK;  // size query: the log is kept
  // copy the oldest min(n, cap) entries and drop only those: a short buffer drains the
  // log over several calls instead of losing the rest
  const uint64_t take = std::min(cnt, cap);
  for (uint64_t i = 0; i < take; ++i) {
    std::memcpy(out + 4 * i, h->oplog.front().data(), 4 * sizeof(int32_t));
    h->oplog.pop_front();
  }
  return NLS_OK;
}

int nls_debug_knob(nls_handle *h, int32_t knob, int32_t value) {
  return guarded(h, [&] {
    if (h->use_graph) fail(h, NLS_ERR_STATE, "nls_debug_knob: not with NLS_GRAPH");
    switch (knob) {
      case NLS_KNOB_TAIL_DYN: h->tail_dyn = value != 0; break;
      case NLS_KNOB_KZ_FUSED:
        h->kz_fused = std::max(0, (int)value);
        if (h->fused_tail) tail_grids(h, h->tail_one_tile);
        break;
      case NLS_KNOB_P2_ORDER: h->p2order = value; break;
      default: fail(h, NLS_ERR_ARG, "nls_debug_knob: unknown knob");
    }
  });
}

int nls_peer_state(const nls_handle *h, int32_t *state) {
  if (!h || !state) return NLS_ERR_ARG;
  *state = h->peer_fallback ? NLS_PEER_FELL_BACK : !h->peer ? NLS_PEER_OFF
           : h->peer_ready  ? NLS_PEER_ACTIVE : NLS_PEER_PENDING;
  return NLS_OK;
}

int nls_placement(const nls_handle *h, int32_t *n, int32_t *chosen, float *ms, uint32_t cap) {
  if (!h || !n) return NLS_ERR_ARG;
  *n = h->place_n;
  if (chosen) *chosen = h->place_pick;
  if (ms)
    for (int c = 0; c < h->place_n && (uint32_t)c < cap; ++c) ms[c] = h->place_ms[c];
  return NLS_OK;
}

int nls_reset_timing(nls_handle *h) {
  return guarded(h, [&] {
    harvest_timing(h);
    h->tacc = nls_timing{};
  });
}

}  // extern "C"
