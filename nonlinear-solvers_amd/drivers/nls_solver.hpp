// nls_solver.hpp -- C++ host-side mirror of the reference solver classes on
// top of the C-ABI (include/nls.h).  Pure host code: compiles with g++ and
// links libnls_amd.so; no HIP, Eigen or torch types.
//
//   nls::NLSESolverDevice   <- device/nlse_solver_dev.hpp:41-138 (+ CQ variant,
//                              device/nlse_cq_solver.hpp:41-140)
//   nls::SGESolverDevice    <- device/sg_solver_dev.hpp:92-294
//   nls::g2::NLSESolverDevice <- nlsolvers/device/include/nlse_dev.hpp:66-361 (G2:
//                              m(x) focusing field, div(c grad) operator, online
//                              snapshots, apply_bc)
//
// Differences from the reference, by design: the Laplacian is described by the
// grid (no CSR argument); snapshots are streamed to a callback/host buffer as
// they are produced instead of living in a device trajectory buffer (which
// would need 215 GB at 512^3); errors are reported as
// std::runtime_error carrying nls_last_error().
#pragma once
#include <chrono>
#include <complex>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "nls.h"

namespace nls {

inline void check(int rc, const nls_handle *h) {
  if (rc != NLS_OK) throw std::runtime_error(std::string("libnls_amd: ") + nls_last_error(h));
}

struct Grid {
  int dim = 2;
  uint32_t nx = 0, ny = 0, nz = 1;
  double dx = 1.0, dy = 1.0;
  uint64_t cells() const { return (uint64_t)nx * ny * (dim == 3 ? nz : 1); }
};

// Double-buffered snapshot pipeline: snapshot k is copied on the device and
// transferred into pinned buffer k % 2 (nls_get_field_async) while the time
// loop continues; a writer thread hands completed buffers to the callback in
// order.  The host blocks only when the writer still holds the buffer it
// needs (blocked_seconds() reports that time).
template <class T> class SnapshotPipe {
 public:
  using Fn = std::function<void(uint32_t index, const T *u, uint64_t n)>;
  SnapshotPipe(nls_handle *h, uint64_t n, Fn cb) : h_(h), n_(n), cb_(std::move(cb)) {
    for (auto &b : buf_) {
      void *p = nullptr;
      check(nls_host_alloc(n * sizeof(T), &p), nullptr);
      b = static_cast<T *>(p);
    }
    writer_ = std::thread([this] { run(); });
  }
  ~SnapshotPipe() {
    try {
      finish();
    } catch (...) {
    }
    for (auto b : buf_) nls_host_free(b);
  }
  SnapshotPipe(const SnapshotPipe &) = delete;
  SnapshotPipe &operator=(const SnapshotPipe &) = delete;

  // enqueue snapshot `index` of the field as of all work enqueued so far
  void push(uint32_t index) {
    rethrow();
    const int b = next_;
    next_ ^= 1;
    {  // the writer must be done with this buffer (from two snapshots ago)
      auto t0 = std::chrono::steady_clock::now();
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return !busy_[b] || err_; });
      blocked_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      busy_[b] = true;
    }
    hand_over_pending();  // the previous transfer is complete by now or soon
    check(nls_get_field_async(h_, reinterpret_cast<double *>(buf_[b]), n_), h_);
    pending_ = true;
    pend_index_ = index;
    pend_buf_ = b;
  }
  // all snapshots written; rethrows a callback error
  void finish() {
    if (done_) return;
    hand_over_pending();
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (writer_.joinable()) writer_.join();
    done_ = true;
    rethrow();
  }
  double blocked_seconds() const { return blocked_; }

 private:
  void hand_over_pending() {
    if (!pending_) return;
    check(nls_wait_field(h_), h_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.push_back({pend_index_, pend_buf_});
    }
    cv_.notify_all();
    pending_ = false;
  }
  void run() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
        if (jobs_.empty()) return;
        j = jobs_.front();
        jobs_.pop_front();
      }
      try {
        if (!err_ && cb_) cb_(j.index, buf_[j.buf], n_);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        if (!err_) err_ = std::current_exception();
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        busy_[j.buf] = false;
      }
      cv_.notify_all();
    }
  }
  void rethrow() {
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> lk(mu_);
      e = err_;
    }
    if (e) std::rethrow_exception(e);
  }
  struct Job {
    uint32_t index = 0;
    int buf = 0;
  };
  nls_handle *h_;
  uint64_t n_;
  Fn cb_;
  T *buf_[2] = {nullptr, nullptr};
  bool busy_[2] = {false, false};
  int next_ = 0;
  bool pending_ = false, done_ = false, stop_ = false;
  uint32_t pend_index_ = 0;
  int pend_buf_ = 0;
  double blocked_ = 0.0;
  std::deque<Job> jobs_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::exception_ptr err_;
  std::thread writer_;
};

class Handle {
 public:
  Handle(const Grid &g, int equation, uint32_t m, int device = -1,
         std::complex<double> s1 = {0.0, 0.5}, std::complex<double> s2 = {-0.5, 0.0}) {
    nls_config c;
    nls_config_default(&c);
    c.dim = g.dim;
    c.equation = equation;
    c.nx = g.nx;
    c.ny = g.ny;
    c.nz = g.dim == 3 ? g.nz : 1;
    c.dx = g.dx;
    c.dy = g.dy;
    c.krylov_m = m;
    c.sigma1[0] = s1.real();
    c.sigma1[1] = s1.imag();
    c.sigma2[0] = s2.real();
    c.sigma2[1] = s2.imag();
    c.device = device;
    check(nls_create(&c, &h_), nullptr);
    uint64_t n = 0;
    check(nls_local_planes(h_, nullptr, nullptr, &n), h_);
    n_ = n;
  }
  ~Handle() {
    if (h_) nls_destroy(h_);
  }
  Handle(const Handle &) = delete;
  Handle &operator=(const Handle &) = delete;
  nls_handle *get() const { return h_; }
  uint64_t n() const { return n_; }

 private:
  nls_handle *h_ = nullptr;
  uint64_t n_ = 0;
};

// NLSE (cubic or cubic-quintic) Strang SS2 stepper.
class NLSESolverDevice {
 public:
  struct Parameters {
    uint32_t num_snapshots, snapshot_freq, krylov_dim;
    Parameters(uint32_t ns = 100, uint32_t freq = 5, uint32_t m = 10)
        : num_snapshots(ns), snapshot_freq(freq), krylov_dim(m) {}
  };
  using SnapshotFn = std::function<void(uint32_t index, const std::complex<double> *u, uint64_t n)>;

  // ctor stores snapshot 0 (the initial field), like device/nlse_solver_dev.hpp:83.
  // Later snapshots go through a SnapshotPipe: the callback runs on its writer
  // thread, in snapshot order; call finish() before using its results.
  NLSESolverDevice(const Grid &g, const std::complex<double> *host_u0, const Parameters &p,
                   SnapshotFn on_snapshot, int equation = NLS_NLSE_CUBIC, int device = -1,
                   std::complex<double> s1 = {0.0, 0.5}, std::complex<double> s2 = {-0.5, 0.0})
      : h_(g, equation, p.krylov_dim, device, s1, s2), p_(p), cb_(std::move(on_snapshot)),
        pipe_(h_.get(), h_.n(), cb_) {
    check(nls_set_field(h_.get(), reinterpret_cast<const double *>(host_u0), h_.n()), h_.get());
    // snapshot 0 = u0, taken from the device copy (bit-identical) so that its
    // file write also runs on the writer thread
    pipe_.push(stored_++);
  }

  // tau = 1j*dt as in the reference (device/nlse_solver_dev.hpp:94); snapshot
  // when step_number % freq == 0, at most num_snapshots in total.
  void step(std::complex<double> tau, uint32_t step_number) {
    check(nls_step(h_.get(), tau.imag(), 1), h_.get());
    if (p_.snapshot_freq && step_number % p_.snapshot_freq == 0 && stored_ < p_.num_snapshots)
      pipe_.push(stored_++);
  }
  void finish() { pipe_.finish(); }
  // all enqueued steps and snapshot transfers complete (file writes may still run)
  void sync() {
    check(nls_sync(h_.get()), h_.get());
    check(nls_wait_field(h_.get()), h_.get());
  }
  double blocked_seconds() const { return pipe_.blocked_seconds(); }
  void get_field(std::complex<double> *dst) {
    check(nls_get_field(h_.get(), reinterpret_cast<double *>(dst), h_.n()), h_.get());
  }
  uint32_t snapshots_stored() const { return stored_; }
  uint64_t n() const { return h_.n(); }

 private:
  Handle h_;
  Parameters p_;
  SnapshotFn cb_;
  SnapshotPipe<std::complex<double>> pipe_;
  uint32_t stored_ = 0;
};

// sine-Gordon Gautschi stepper (u_tt = Lap u + m sin u).
class SGESolverDevice {
 public:
  using SnapshotFn = std::function<void(uint32_t index, const double *u, const double *v, uint64_t n)>;
  SGESolverDevice(const Grid &g, const double *u0, const double *v0, const double *mfield, double dt,
                  uint32_t num_snapshots, uint32_t freq, uint32_t m, SnapshotFn cb, int device = -1)
      : h_(g, NLS_SG_GAUTSCHI, m, device), ns_(num_snapshots), freq_(freq), cb_(std::move(cb)),
        u_(h_.n()), v_(h_.n()) {
    std::vector<double> up(h_.n());
    for (uint64_t i = 0; i < h_.n(); ++i) up[i] = u0[i] - dt * v0[i];  // sg_driver_dev.cpp:106
    check(nls_set_sg_state(h_.get(), u0, up.data(), mfield, h_.n()), h_.get());
    if (cb_) cb_(stored_, u0, v0, h_.n());
    ++stored_;
  }
  void step(double tau, uint32_t step_number) {
    check(nls_step(h_.get(), tau, 1), h_.get());
    if (freq_ && step_number % freq_ == 0 && stored_ < ns_) {
      check(nls_get_field(h_.get(), u_.data(), h_.n()), h_.get());
      check(nls_get_sg_velocity(h_.get(), tau, v_.data(), h_.n()), h_.get());
      if (cb_) cb_(stored_, u_.data(), v_.data(), h_.n());
      ++stored_;
    }
  }
  uint64_t n() const { return h_.n(); }

 private:
  Handle h_;
  uint32_t ns_, freq_;
  SnapshotFn cb_;
  std::vector<double> u_, v_;
  uint32_t stored_ = 0;
};

// G2 Klein-Gordon Gautschi stepper (u_tt = div(c grad u) - m u^3), the
// KGESolverDevice of nlsolvers/device/include/kg_dev.hpp as
// kg_driver_dev_{2d,3d}.cpp drive it: ctor stores snapshot 0 = (u0, v0); per
// step i: step(), apply_bc(), store_snapshot(i / freq) when i % freq == 0.
class KGESolverDevice {
 public:
  using SnapshotFn = std::function<void(uint32_t index, const double *u, const double *v, uint64_t n)>;
  KGESolverDevice(const Grid &g, const double *u0, const double *v0, const double *mfield,
                  const double *cfield, double dt, uint32_t num_snapshots, uint32_t krylov_m,
                  SnapshotFn cb, int device = -1)
      : h_(g, NLS_KG_GAUTSCHI, krylov_m, device), ns_(num_snapshots), dt_(dt), cb_(std::move(cb)),
        u_(h_.n()), v_(h_.n()) {
    std::vector<double> up(h_.n());
    for (uint64_t i = 0; i < h_.n(); ++i) up[i] = u0[i] - dt * v0[i];  // kg_dev.hpp ctor
    check(nls_set_coefficients(h_.get(), mfield, cfield, h_.n()), h_.get());
    check(nls_set_sg_state(h_.get(), u0, up.data(), nullptr, h_.n()), h_.get());
    if (cb_ && ns_ > 0) cb_(0, u0, v0, h_.n());
  }
  void step() { check(nls_step(h_.get(), dt_, 1), h_.get()); }
  void apply_bc() { check(nls_apply_bc(h_.get()), h_.get()); }
  void store_snapshot(uint32_t idx) {
    if (idx >= ns_) return;
    check(nls_get_field(h_.get(), u_.data(), h_.n()), h_.get());
    check(nls_get_sg_velocity(h_.get(), dt_, v_.data(), h_.n()), h_.get());
    if (cb_) cb_(idx, u_.data(), v_.data(), h_.n());
  }
  uint64_t n() const { return h_.n(); }

 private:
  Handle h_;
  uint32_t ns_;
  double dt_;
  SnapshotFn cb_;
  std::vector<double> u_, v_;
};

// G2 device Gautschi family -- SGESolverDevice / SGEDoubleSolverDevice /
// SGEHyperbolicSolverDevice / Phi4SolverDevice of nlsolvers/device/include/
// {sg_single,sg_double,sg_hyperbolic,phi4}_dev.hpp as their drivers use them
// (phi4_driver_dev.cpp:103-118): the ctor stores snapshot 0 = u0 (phi4_dev.hpp:65)
// and sets u_past = u0 - dt v0 (:43-46); per step i = 1 .. nt-1 the driver calls
// step(), apply_bc() (u only, :92) and store_snapshot(i / freq) when i % freq == 0.
// equation: NLS_SG_G2, NLS_SG_DOUBLE, NLS_SG_HYPERBOLIC or NLS_PHI4.
class GautschiSolverDevice {
 public:
  using SnapshotFn = std::function<void(uint32_t index, const double *u, uint64_t n)>;
  GautschiSolverDevice(const Grid &g, int equation, const double *u0, const double *v0,
                       const double *mfield, double dt, uint32_t num_snapshots, uint32_t krylov_m,
                       SnapshotFn cb, int device = -1)
      : h_(g, equation, krylov_m, device), ns_(num_snapshots), dt_(dt), cb_(std::move(cb)), u_(h_.n()) {
    std::vector<double> up(h_.n());
    for (uint64_t i = 0; i < h_.n(); ++i) up[i] = u0[i] - dt * v0[i];
    check(nls_set_sg_state(h_.get(), u0, up.data(), mfield, h_.n()), h_.get());
    if (cb_ && ns_ > 0) cb_(0, u0, h_.n());
  }
  void step() { check(nls_step(h_.get(), dt_, 1), h_.get()); }
  void apply_bc() { check(nls_apply_bc(h_.get()), h_.get()); }
  void store_snapshot(uint32_t idx) {
    if (idx >= ns_) return;
    check(nls_get_field(h_.get(), u_.data(), h_.n()), h_.get());
    if (cb_) cb_(idx, u_.data(), h_.n());
  }
  uint64_t n() const { return h_.n(); }

 private:
  Handle h_;
  uint32_t ns_;
  double dt_;
  SnapshotFn cb_;
  std::vector<double> u_;
};

namespace g2 {

// G2 cubic NLSE stepper (nlsolvers/device/include/nlse_dev.hpp:66-361) as the
// G2 drivers use it (nlse_cubic_driver_{2d,3d}.cpp): the caller stores
// snapshot 0 with store_snapshot_online(), then per step i = 1 .. nt-1 calls
// step(tau, i) -- which stores the (pre-BC) field when i % freq == 0 -- and
// apply_bc().  The operator is div(c grad) built from c(x) (laplacians.hpp:
// 54-103, 158-218); the C-ABI takes c itself instead of an assembled CSR.
class NLSESolverDevice {
 public:
  struct Parameters {
    uint32_t num_snapshots, snapshot_freq, krylov_dim;
    Parameters(uint32_t ns = 100, uint32_t freq = 5, uint32_t m = 10)  // nlse_dev.hpp:66-75
        : num_snapshots(ns), snapshot_freq(freq), krylov_dim(m) {}
  };
  using SnapshotFn = std::function<void(uint32_t index, const std::complex<double> *u, uint64_t n)>;

  NLSESolverDevice(const Grid &g, const std::complex<double> *host_u0, const double *host_m,
                   const double *host_c, const Parameters &p, SnapshotFn on_snapshot, int device = -1)
      : h_(g, NLS_NLSE_G2, p.krylov_dim, device), p_(p), cb_(std::move(on_snapshot)),
        pipe_(h_.get(), h_.n(), cb_) {
    check(nls_set_field(h_.get(), reinterpret_cast<const double *>(host_u0), h_.n()), h_.get());
    check(nls_set_coefficients(h_.get(), host_m, host_c, h_.n()), h_.get());
  }

  // nlse_dev.hpp:187-203 (the snapshot is taken before the driver's apply_bc)
  void step(std::complex<double> tau, uint32_t step_number) {
    check(nls_step(h_.get(), tau.imag(), 1), h_.get());
    if (p_.snapshot_freq && step_number % p_.snapshot_freq == 0) store_snapshot_online();
  }
  void apply_bc() { check(nls_apply_bc(h_.get()), h_.get()); }  // nlse_dev.hpp:178-185

  // nlse_dev.hpp:205-238 (step 1: SS2 + u_prev; snapshots as step())
  void step_sewi(std::complex<double> tau, uint32_t step_number) {
    check(nls_step_sewi(h_.get(), tau.imag(), step_number), h_.get());
    if (p_.snapshot_freq && step_number % p_.snapshot_freq == 0) store_snapshot_online();
  }

  // nlse_dev.hpp:323-334: at most num_snapshots, silently ignored beyond.
  // Asynchronous (SnapshotPipe): the callback runs on the writer thread.
  void store_snapshot_online() {
    if (stored_ >= p_.num_snapshots) return;
    pipe_.push(stored_++);
  }
  void finish() { pipe_.finish(); }
  // all enqueued steps and snapshot transfers complete (file writes may still run)
  void sync() {
    check(nls_sync(h_.get()), h_.get());
    check(nls_wait_field(h_.get()), h_.get());
  }
  double blocked_seconds() const { return pipe_.blocked_seconds(); }
  uint32_t snapshots_stored() const { return stored_; }
  uint64_t n() const { return h_.n(); }

 private:
  Handle h_;
  Parameters p_;
  SnapshotFn cb_;
  SnapshotPipe<std::complex<double>> pipe_;
  uint32_t stored_ = 0;
};

// G2 cubic-quintic stepper (nlsolvers/device/include/nlse_cubic_quintic_dev.hpp:
// 16-95): real sigma1, sigma2 and m(x), no-flux 5-point Laplacian; the
// constructor stores snapshot 0 (:62), step() stores the pre-BC field when
// i % freq == 0 (:87-89).  Snapshots past num_snapshots are dropped (the
// reference writes past the end of its trajectory buffer there).
class NLSECubicQuinticSolverDevice {
 public:
  struct Parameters {
    uint32_t num_snapshots, snapshot_freq, krylov_dim;
    double sigma1, sigma2;
    Parameters(uint32_t ns = 100, uint32_t freq = 5, uint32_t m = 10, double s1 = 1.0,
               double s2 = 1.0)  // nlse_cubic_quintic_dev.hpp:18-29
        : num_snapshots(ns), snapshot_freq(freq), krylov_dim(m), sigma1(s1), sigma2(s2) {}
  };
  using SnapshotFn = std::function<void(uint32_t index, const std::complex<double> *u, uint64_t n)>;

  NLSECubicQuinticSolverDevice(const Grid &g, const std::complex<double> *host_u0, const double *host_m,
                               const Parameters &p, SnapshotFn on_snapshot, int device = -1)
      : h_(g, NLS_NLSE_CQ_G2, p.krylov_dim, device, {p.sigma1, 0.0}, {p.sigma2, 0.0}), p_(p),
        cb_(std::move(on_snapshot)), pipe_(h_.get(), h_.n(), cb_) {
    check(nls_set_field(h_.get(), reinterpret_cast<const double *>(host_u0), h_.n()), h_.get());
    check(nls_set_coefficients(h_.get(), host_m, nullptr, h_.n()), h_.get());
    store_snapshot();
  }

  // nlse_cubic_quintic_dev.hpp:79-95
  void step(std::complex<double> tau, uint32_t step_number) {
    check(nls_step(h_.get(), tau.imag(), 1), h_.get());
    if (p_.snapshot_freq && step_number % p_.snapshot_freq == 0) store_snapshot();
  }
  void apply_bc() { check(nls_apply_bc(h_.get()), h_.get()); }  // :75-77
  void finish() { pipe_.finish(); }
  uint32_t snapshots_stored() const { return stored_; }
  uint64_t n() const { return h_.n(); }

 private:
  void store_snapshot() {
    if (stored_ >= p_.num_snapshots) return;
    pipe_.push(stored_++);
  }
  Handle h_;
  Parameters p_;
  SnapshotFn cb_;
  SnapshotPipe<std::complex<double>> pipe_;
  uint32_t stored_ = 0;
};

}  // namespace g2

}  // namespace nls
