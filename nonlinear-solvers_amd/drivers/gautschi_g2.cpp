// sg_single_dev / sg_double_dev / sg_hyperbolic_dev / phi4_dev -- drop-in
// replacements of the G2 device Gautschi drivers
// nlsolvers/device/drivers/{sg_single,sg_double,sg_hyperbolic,phi4}_driver_dev.cpp
// (CMake targets sg_single_dev, sg_double_dev, sg_hyperbolic_dev, phi4_dev,
// nlsolvers/device/drivers/CMakeLists.txt:13-33), on the MI355X library:
//
//   prog nx ny Lx Ly input_u0.npy input_v0.npy output_traj.npy T nt num_snapshots [input_m.npy]
//        [--m=K] [--device=D]   (optional extension flags)
//
// Semantics kept (phi4_driver_dev.cpp:16-127; the four drivers differ only in
// the solver class): 11 or 12 argv else usage + exit 1; dx = 2 Lx/(nx-1),
// dy = 2 Ly/(ny-1), dt = T/nt, freq = nt/num_snapshots; float64 u0, v0 of shape
// [ny, nx] ("Error: Input array dimensions mismatch" + exit 1); m(x) optional,
// and a missing / misshapen m file falls back to m = 1 everywhere with the
// reference's messages; isotropic no-flux operator (build_laplacian_noflux,
// :84-85); Krylov m = 10 (:103); snapshot 0 = u0, then for i = 1 .. nt-1: step,
// apply_bc (u only), snapshot i / freq when i % freq == 0 and < num_snapshots;
// output [num_snapshots, ny, nx] float64; nothing on stdout.
// Differences: the reference checks the shape of v0 only (the second read
// overwrites the shape vector); both are checked here.  num_snapshots > nt
// exits 1 (the reference takes i % 0).
#include <iostream>
#include <string>
#include <vector>

#include "cli_common.hpp"
#include "nls_solver.hpp"
#include "npy.hpp"

#ifndef GG_EQUATION
#define GG_EQUATION NLS_PHI4
#endif

namespace {

void print_usage(const char *p) {
  std::cerr << "Usage: " << p
            << " nx ny Lx Ly input_u0.npy input_v0.npy output_traj.npy T nt "
               "num_snapshots [input_m.npy]\n";
  std::cerr << "Example: " << p
            << " 256 256 10.0 10.0 initial.npy velocity.npy evolution.npy "
               "1.5 500 100\n";
  std::cerr << "Example with m(x,y): " << p
            << " 256 256 10.0 10.0 initial.npy velocity.npy evolution.npy "
               "1.5 500 100 coupling.npy\n";
}

}  // namespace

int main(int argc, char **argv) {
  const cli::Args a = cli::parse(argc, argv);
  if (a.pos.size() != 10 && a.pos.size() != 11) {
    print_usage(argv[0]);
    return 1;
  }
  uint32_t nx, ny, nt, ns;
  double Lx, Ly, T;
  int m, device;
  try {
    nx = std::stoul(a.pos[0]);
    ny = std::stoul(a.pos[1]);
    Lx = std::stod(a.pos[2]);
    Ly = std::stod(a.pos[3]);
    T = std::stod(a.pos[7]);
    nt = std::stoul(a.pos[8]);
    ns = std::stoul(a.pos[9]);
    m = cli::flag_int(a, "m", 10);  // phi4_driver_dev.cpp:103
    device = cli::flag_int(a, "device", -1);
  } catch (const std::exception &e) {
    std::cerr << "Error: bad argument (" << e.what() << ")\n";
    print_usage(argv[0]);
    return 1;
  }
  if (nx < 3 || ny < 3 || nt < 1 || ns < 1) {
    std::cerr << "Error: need nx, ny >= 3 and nt, num_snapshots >= 1\n";
    return 1;
  }
  const double dx = 2 * Lx / (nx - 1), dy = 2 * Ly / (ny - 1);
  const double dt = T / nt;
  const uint32_t freq = nt / ns;
  if (freq == 0) {
    std::cerr << "Error: num_snapshots (" << ns << ") > nt (" << nt << ")\n";
    return 1;
  }
  std::vector<uint64_t> ushape, vshape;
  std::vector<double> u0, v0;
  try {
    u0 = npy::load<double>(a.pos[4], ushape);
    v0 = npy::load<double>(a.pos[5], vshape);
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  const std::vector<uint64_t> fshape = {ny, nx};
  if (ushape != fshape || vshape != fshape) {
    const std::vector<uint64_t> &got = vshape != fshape ? vshape : ushape;
    std::cerr << "Error: Input array dimensions mismatch\n";
    std::cerr << "Expected: " << ny << "x" << nx << "\n";
    std::cerr << "Got: " << (got.size() > 0 ? got[0] : 0) << "x" << (got.size() > 1 ? got[1] : 0) << "\n";
    return 1;
  }
  std::vector<double> mfield;
  if (a.pos.size() == 11) {  // phi4_driver_dev.cpp:62-79
    try {
      std::vector<uint64_t> mshape;
      mfield = npy::load<double>(a.pos[10], mshape);
      if (mshape != fshape) {
        std::cerr << "Error: Coupling array dimensions mismatch\n";
        std::cerr << "Expected: " << ny << "x" << nx << "\n";
        std::cerr << "Got: " << (mshape.size() > 0 ? mshape[0] : 0) << "x"
                  << (mshape.size() > 1 ? mshape[1] : 0) << "\n";
        std::cerr << "Using default m=1.0 everywhere\n";
        mfield.assign((size_t)nx * ny, 1.0);
      }
    } catch (const std::exception &e) {
      std::cerr << "Error loading m(x,y): " << e.what() << "\n";
      std::cerr << "Using default m=1.0 everywhere\n";
      mfield.assign((size_t)nx * ny, 1.0);
    }
  } else {
    mfield.assign((size_t)nx * ny, 1.0);
  }

  try {
    npy::Writer w = npy::Writer::open<double>(a.pos[6], {ns, ny, nx});
    nls::Grid g;
    g.dim = 2;
    g.nx = nx;
    g.ny = ny;
    g.dx = dx;
    g.dy = dy;
    uint32_t next = 0;
    nls::GautschiSolverDevice solver(
        g, GG_EQUATION, u0.data(), v0.data(), mfield.data(), dt, ns, (uint32_t)m,
        [&](uint32_t idx, const double *u, uint64_t n) {
          if (idx != next) throw std::runtime_error("snapshot order");
          w.append(u, n * sizeof(double));
          ++next;
        },
        device);
    for (uint32_t i = 1; i < nt; ++i) {
      solver.step();
      solver.apply_bc();
      if (i % freq == 0) solver.store_snapshot(i / freq);
    }
    w.close();
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
