// nlse_cubic_quintic_dev -- drop-in replacement of the G2 cubic-quintic device
// driver nlsolvers/device/drivers/nlse_cubic_quintic_driver_dev.cpp (its CMake
// target is commented out, nlsolvers/device/drivers/CMakeLists.txt:43), on the
// MI355X library.
//
//   prog nx ny Lx Ly sigma1 sigma2 input_u0.npy output_traj.npy T nt num_snapshots [input_m.npy]
//        [--m=K] [--device=D]   (optional extension flags)
//
// Semantics kept (:16-104): 11 or 12 positional arguments, else usage + exit 1;
// dx = 2 Lx/(nx-1), dy = 2 Ly/(ny-1); dt = T/nt; freq = nt/num_snapshots; u0 is
// complex128 [ny, nx] and is NOT normalised; the optional m(x, y) falls back to
// m = 1 with the reference's messages when it cannot be read or has the wrong
// shape; real sigma1, sigma2; Krylov m = 15 (:91); snapshot 0 = u0, then for
// i = 1 .. nt-1: step (snapshot when i % freq == 0, before the BC), apply_bc;
// output complex128 [ns, ny, nx]; nothing on stdout.
// Differences: snapshots stream to the output file as they are produced;
// num_snapshots > nt is rejected with exit 1 (the reference takes i % 0);
// snapshots past num_snapshots are dropped (the reference writes past its
// buffer when nt % num_snapshots leaves room for more).
#include <complex>
#include <iostream>
#include <string>
#include <vector>

#include "cli_common.hpp"
#include "nls_solver.hpp"
#include "npy.hpp"

namespace {

void print_usage(const char *p) {
  std::cerr << "Usage: " << p
            << " nx ny Lx Ly sigma1 sigma2 input_u0.npy output_traj.npy T nt "
               "num_snapshots [input_m.npy]\n";
  std::cerr << "Example: " << p
            << " 256 256 10.0 10.0 1.0 0.5 initial.npy evolution.npy "
               "1.5 500 100\n";
  std::cerr << "Example with m(x,y): " << p
            << " 256 256 10.0 10.0 1.0 0.5 initial.npy evolution.npy "
               "1.5 500 100 coupling.npy\n";
}

}  // namespace

int main(int argc, char **argv) {
  const cli::Args a = cli::parse(argc, argv);
  if (a.pos.size() != 11 && a.pos.size() != 12) {
    print_usage(argv[0]);
    return 1;
  }
  uint32_t nx, ny, nt, ns;
  double Lx, Ly, s1, s2, T;
  int m, device;
  try {
    nx = std::stoul(a.pos[0]);
    ny = std::stoul(a.pos[1]);
    Lx = std::stod(a.pos[2]);
    Ly = std::stod(a.pos[3]);
    s1 = std::stod(a.pos[4]);
    s2 = std::stod(a.pos[5]);
    T = std::stod(a.pos[8]);
    nt = std::stoul(a.pos[9]);
    ns = std::stoul(a.pos[10]);
    m = cli::flag_int(a, "m", 15);  // nlse_cubic_quintic_driver_dev.cpp:91
    device = cli::flag_int(a, "device", -1);
  } catch (const std::exception &e) {
    std::cerr << "Error: bad argument (" << e.what() << ")\n";
    print_usage(argv[0]);
    return 1;
  }
  const std::string in_file = a.pos[6], out_file = a.pos[7];
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
  std::vector<uint64_t> shape;
  std::vector<std::complex<double>> u0;
  try {
    u0 = npy::load<std::complex<double>>(in_file, shape);
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  const std::vector<uint64_t> fshape = {ny, nx};
  if (shape != fshape) {  // :58-63
    std::cerr << "Error: Input array dimensions mismatch\n";
    std::cerr << "Expected: " << ny << "x" << nx << "\n";
    std::cerr << "Got: " << (shape.size() > 0 ? shape[0] : 0) << "x" << (shape.size() > 1 ? shape[1] : 0)
              << "\n";
    return 1;
  }
  std::vector<double> mfield;
  if (a.pos.size() == 12) {  // :65-85
    std::vector<uint64_t> mshape;
    try {
      mfield = npy::load<double>(a.pos[11], mshape);
      if (mshape != fshape) {
        std::cerr << "Error: Coupling array dimensions mismatch\n";
        std::cerr << "Expected: " << ny << "x" << nx << "\n";
        std::cerr << "Got: " << (mshape.size() > 0 ? mshape[0] : 0) << "x"
                  << (mshape.size() > 1 ? mshape[1] : 0) << "\n";
        std::cerr << "Using default m=1.0 everywhere\n";
        mfield.clear();
      }
    } catch (const std::exception &e) {
      std::cerr << "Error loading m(x,y): " << e.what() << "\n";
      std::cerr << "Using default m=1.0 everywhere\n";
      mfield.clear();
    }
  }
  if (mfield.empty()) mfield.assign((size_t)nx * ny, 1.0);

  try {
    npy::Writer out = npy::Writer::open<std::complex<double>>(out_file, {ns, ny, nx});
    nls::Grid g;
    g.dim = 2;
    g.nx = nx;
    g.ny = ny;
    g.dx = dx;
    g.dy = dy;
    nls::g2::NLSECubicQuinticSolverDevice::Parameters params(ns, freq, (uint32_t)m, s1, s2);
    nls::g2::NLSECubicQuinticSolverDevice solver(
        g, u0.data(), mfield.data(), params,
        [&](uint32_t, const std::complex<double> *u, uint64_t n) {
          out.append(u, n * sizeof(std::complex<double>));
        },
        device);
    const std::complex<double> dti(0.0, dt);
    for (uint32_t i = 1; i < nt; ++i) {
      solver.step(dti, i);
      solver.apply_bc();
    }
    solver.finish();
    out.close();
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
