// nlse_3d_dev / nlse_2d_dev -- drop-in replacements of the G2 device drivers
// nlsolvers/device/drivers/nlse_cubic_driver_3d.cpp (13 positional args,
// Krylov m = 25) and nlse_cubic_driver_2d.cpp (11 positional args, m = 20),
// CMake targets nlse_3d_dev / nlse_2d_dev (nlsolvers/device/drivers/
// CMakeLists.txt:63-65), on the MI355X library.  Built with -DG2_SEWI=1 the
// same source gives nlse_sewi_3d_dev / nlse_sewi_2d_dev
// (nlse_cubic_sewi_driver_{3d,2d}.cpp, CMakeLists.txt:64,66): step_sewi
// instead of step, Krylov m = 15 (3D) / 25 (2D), otherwise identical.
//
//   3D: prog nx ny nz Lx Ly Lz input_u0.npy output_traj.npy T nt num_snapshots input_m.npy input_c.npy
//   2D: prog nx ny Lx Ly input_u0.npy output_traj.npy T nt num_snapshots input_m.npy input_c.npy
//       [--m=K] [--device=D]   (optional extension flags)
//
// Semantics kept: dx = 2 Lx/(nx-1) (the operator scale, :47 / :39); dt = T/nt;
// freq = nt/num_snapshots; u0 is NOT normalised; the shape checks and their
// messages (3D expects [nz,ny,nx]; 2D expects [nx,ny] as the reference checks
// it); m and c are float64 of the same shape; snapshot 0 = u0, then for
// i = 1 .. nt-1: step (snapshot when i % freq == 0, before the BC), apply_bc;
// output complex128 [ns, nz, ny, nx] (3D) or [ns, ny, nx] (2D); nothing on stdout.
// Differences: snapshots are streamed to the output file as they are produced,
// by a writer thread overlapping the time loop (the reference holds ns*n
// complex values on the host and copies each snapshot synchronously); num_snapshots > nt is
// rejected with exit 1 (the reference takes i % 0); a failed m/c load exits 1
// after the reference's messages (the reference rethrows into std::terminate).
#include <complex>
#include <iostream>
#include <string>
#include <vector>

#include "cli_common.hpp"
#include "nls_solver.hpp"
#include "npy.hpp"

#ifndef G2_DIM
#define G2_DIM 3
#endif
#ifndef G2_SEWI
#define G2_SEWI 0
#endif
// Krylov dimension of each reference driver
#if G2_SEWI
constexpr int G2_M = G2_DIM == 3 ? 15 : 25;  // nlse_cubic_sewi_driver_3d.cpp:113, _2d.cpp:105
#else
constexpr int G2_M = G2_DIM == 3 ? 25 : 20;  // nlse_cubic_driver_3d.cpp:113, _2d.cpp:105
#endif

namespace {

void print_usage(const char *p) {
#if G2_DIM == 3
  std::cerr << "Usage: " << p
            << " nx ny nz Lx Ly Lz input_u0.npy output_traj.npy T nt "
               "num_snapshots input_m.npy input_c.npy\n";
  std::cerr << "Example: " << p
            << " 256 256 256 10.0 10.0 10.0 initial.npy evolution_u.npy "
               "1.5 500 100 coupling.npy anisotropy.npy\n";
#else
  std::cerr << "Usage: " << p
            << " nx ny Lx Ly input_u0.npy output_traj.npy T nt "
               "num_snapshots input_m.npy input_c.npy\n";
  std::cerr << "Example: " << p
            << " 256 256 10.0 10.0 initial.npy evolution_u.npy "
               "1.5 500 100\n";
#endif
}

// The reference's field-shape check for m / c (3D :66-101, 2D :57-90)
bool load_field(const std::string &path, const std::vector<uint64_t> &expect, const char *what,
                std::vector<double> &out) {
  std::vector<uint64_t> shape;
  try {
    out = npy::load<double>(path, shape);
  } catch (const std::exception &e) {
    std::cerr << "Error loading " << what << "(x, y, z): " << e.what() << "\n";
    return false;
  }
  if (shape != expect) {
    std::cerr << "Error: Coupling array dimensions mismatch\n";
    std::cerr << "Expected: ";
    for (size_t i = 0; i < expect.size(); ++i) std::cerr << (i ? "x" : "") << expect[i];
    std::cerr << "\nGot: ";
    for (size_t i = 0; i < shape.size(); ++i) std::cerr << (i ? "x" : "") << shape[i];
    std::cerr << "\n";
    std::cerr << "Error loading " << what << "(x, y, z): Faulty " << what << " (1)\n";
    return false;
  }
  return true;
}

}  // namespace

int main(int argc, char **argv) {
  const cli::Args a = cli::parse(argc, argv);
  constexpr size_t NPOS = G2_DIM == 3 ? 13 : 11;
  if (a.pos.size() != NPOS) {
    print_usage(argv[0]);
    return 1;
  }
  constexpr int o = G2_DIM == 3 ? 1 : 0;  // positional offset after the grid extents
  uint32_t nx, ny, nz = 1, nt, ns;
  double Lx, T;
  int m, device;
  try {
    nx = std::stoul(a.pos[0]);
    ny = std::stoul(a.pos[1]);
    if (G2_DIM == 3) nz = std::stoul(a.pos[2]);
    Lx = std::stod(a.pos[2 + o]);
    (void)std::stod(a.pos[3 + o]);                 // Ly
    if (G2_DIM == 3) (void)std::stod(a.pos[5]);   // Lz (the reference never uses it)
    T = std::stod(a.pos[6 + 2 * o]);
    nt = std::stoul(a.pos[7 + 2 * o]);
    ns = std::stoul(a.pos[8 + 2 * o]);
    m = cli::flag_int(a, "m", G2_M);
    device = cli::flag_int(a, "device", -1);
  } catch (const std::exception &e) {
    std::cerr << "Error: bad argument (" << e.what() << ")\n";
    print_usage(argv[0]);
    return 1;
  }
  const std::string in_file = a.pos[4 + 2 * o], out_file = a.pos[5 + 2 * o];
  const std::string m_file = a.pos[9 + 2 * o], c_file = a.pos[10 + 2 * o];
  if (nx < 3 || ny < 3 || (G2_DIM == 3 && nz < 3) || nt < 1 || ns < 1) {
    std::cerr << "Error: need nx, ny" << (G2_DIM == 3 ? ", nz" : "") << " >= 3 and nt, num_snapshots >= 1\n";
    return 1;
  }
  // Only dx enters the operator: 1/(dx*dx) in 3D; 1/(dx*dy) in 2D with dy the
  // same formula on Ly (laplacians.hpp:101, :216).
  const double dx = 2 * Lx / (nx - 1);
  const double dy = 2 * std::stod(a.pos[3 + o]) / (ny - 1);
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
#if G2_DIM == 3
  const std::vector<uint64_t> fshape = {nz, ny, nx};
  if (shape != fshape) {
    std::cerr << "Error: Input array dimensions mismatch\n";
    std::cerr << "Expected: " << ny << "x" << nx << "\n";
    std::cerr << "Got: " << (shape.size() > 0 ? shape[0] : 0) << "x" << (shape.size() > 1 ? shape[1] : 0)
              << "x" << (shape.size() > 2 ? shape[2] : 0) << "\n";
    return 1;
  }
  const std::vector<uint64_t> out_shape = {ns, nz, ny, nx};
#else
  // the 2D reference checks [nx, ny] (nlse_cubic_driver_2d.cpp:49-56) but
  // builds the operator with the fast axis of length nx; both agree on the
  // square grids its builder asserts (laplacians.hpp:63)
  const std::vector<uint64_t> fshape = {nx, ny};
  if (shape != fshape) {
    std::cerr << "Error: Input array dimensions mismatch\n";
    std::cerr << "Expected: " << ny << "x" << nx << "\n";
    std::cerr << "Got: " << (shape.size() > 0 ? shape[0] : 0) << "x" << (shape.size() > 1 ? shape[1] : 0)
              << "\n";
    return 1;
  }
  const std::vector<uint64_t> out_shape = {ns, ny, nx};
#endif
  std::vector<double> mfield, cfield;
  if (!load_field(m_file, fshape, "m", mfield)) return 1;
  if (!load_field(c_file, fshape, "c", cfield)) return 1;

  try {
    npy::Writer out = npy::Writer::open<std::complex<double>>(out_file, out_shape);
    nls::Grid g;
    g.dim = G2_DIM;
#if G2_DIM == 3
    g.nx = nx;
    g.ny = ny;
    g.nz = nz;
#else
    g.nx = (uint32_t)fshape[1];  // C layout of the array: fast axis last
    g.ny = (uint32_t)fshape[0];
#endif
    g.dx = dx;
    g.dy = G2_DIM == 3 ? dx : dy;
    nls::g2::NLSESolverDevice::Parameters params(ns, freq, (uint32_t)m);
    nls::g2::NLSESolverDevice solver(
        g, u0.data(), mfield.data(), cfield.data(), params,
        [&](uint32_t, const std::complex<double> *u, uint64_t n) {
          out.append(u, n * sizeof(std::complex<double>));
        },
        device);
    solver.store_snapshot_online();
    const std::complex<double> dti(0.0, dt);
    for (uint32_t i = 1; i < nt; ++i) {
#if G2_SEWI
      solver.step_sewi(dti, i);
#else
      solver.step(dti, i);
#endif
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
