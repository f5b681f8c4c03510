// kg_gautschi_3d_dev / kg_gautschi_2d_dev -- drop-in replacements of the G2
// Klein-Gordon Gautschi drivers nlsolvers/device/drivers/kg_driver_dev_3d.cpp
// and kg_driver_dev_2d.cpp (CMake targets kg_gautschi_{3d,2d}_dev,
// nlsolvers/device/drivers/CMakeLists.txt:56,58), on the MI355X library:
//
//   3D: prog nx ny nz Lx Ly Lz u0.npy v0.npy traj_u.npy traj_v.npy T nt num_snapshots m.npy c.npy
//   2D: prog nx ny Lx Ly u0.npy v0.npy traj_u.npy traj_v.npy T nt num_snapshots m.npy c.npy
//       [--m=K] [--device=D] [--true-shape]   (optional extension flags)
//
// Semantics kept: float64 inputs; dx = 2 Lx/(nx-1) (scale 1/dx^2 in 3D,
// 1/(dx*dy) in 2D) on -div(c grad) (the drivers negate the anisotropic
// builder, :110-114); u_past = u0 - dt v0; Krylov m = 10; snapshot 0 =
// (u0, v0), then for i = 1 .. nt-1: step, apply_bc (u only), and snapshot
// i / freq when i % freq == 0 (u after the BC, v as the step computed it);
// the reference's shape checks and messages (2D checks u0 as [nx, ny], m as
// [ny, nx], c as [nx, ny]); the 3D outputs carry the reference's header
// [ns, ny, nx] over ns*nz*ny*nx values (kg_driver_dev_3d.cpp:161-163: numpy
// reads the first ns*ny*nx of them unless the consumer reshapes the raw
// payload); --true-shape writes the header [ns, nz, ny, nx] of the data
// instead.  Differences: num_snapshots > nt
// exits 1 (the reference takes i % 0); failed m / c loads exit 1 after the
// reference's messages (the reference rethrows into std::terminate).
#include <iostream>
#include <string>
#include <vector>

#include "cli_common.hpp"
#include "nls_solver.hpp"
#include "npy.hpp"

#ifndef KG_DIM
#define KG_DIM 3
#endif

namespace {

void print_usage(const char *p) {
#if KG_DIM == 3
  std::cerr << "Usage: " << p
            << " nx ny nz Lx Ly Lz input_u0.npy input_v0.npy output_traj.npy "
               "output_vel.npy T nt num_snapshots input_m.npy input_c.npy\n";
#else
  std::cerr << "Usage: " << p
            << " nx ny Lx Ly input_u0.npy input_v0.npy output_traj.npy "
               "output_vel.npy T nt num_snapshots input_m.npy input_c.npy\n";
#endif
  std::cerr << "Example: " << p
            << " 256 256 256 10.0 10.0 10.0 initial.npy velocity.npy "
               "evolution_u.npy evolution_v.npy 1.5 500 100 coupling.npy anisotropy.npy\n";
}

std::string shape_text(const std::vector<uint64_t> &s) {
  std::string t;
  for (size_t i = 0; i < s.size(); ++i) t += (i ? "x" : "") + std::to_string(s[i]);
  return t;
}

bool load_field(const std::string &path, const std::vector<uint64_t> &expect, const char *what,
                std::vector<double> &out) {
  std::vector<uint64_t> shape;
  try {
    out = npy::load<double>(path, shape);
  } catch (const std::exception &e) {
    std::cerr << "Error loading " << what << (KG_DIM == 3 ? "(x, y, z): " : "(x, y): ") << e.what() << "\n";
    return false;
  }
  if (shape != expect) {
    std::cerr << "Error: Coupling array dimensions mismatch\n";
    std::cerr << "Expected: " << shape_text(expect) << "\n";
    std::cerr << "Got: " << shape_text(shape) << "\n";
    std::cerr << "Error loading " << what << (KG_DIM == 3 ? "(x, y, z): " : "(x, y): ") << "Faulty "
              << what << " (1)\n";
    return false;
  }
  return true;
}

}  // namespace

int main(int argc, char **argv) {
  const cli::Args a = cli::parse(argc, argv);
  constexpr size_t NPOS = KG_DIM == 3 ? 15 : 13;
  if (a.pos.size() != NPOS) {
    print_usage(argv[0]);
    return 1;
  }
  constexpr int o = KG_DIM == 3 ? 1 : 0;  // extra z extent / Lz in 3D
  uint32_t nx, ny, nz = 1, nt, ns;
  double Lx, Ly, T;
  int m, device;
  try {
    nx = std::stoul(a.pos[0]);
    ny = std::stoul(a.pos[1]);
    if (KG_DIM == 3) nz = std::stoul(a.pos[2]);
    Lx = std::stod(a.pos[2 + o]);
    Ly = std::stod(a.pos[3 + o]);
    if (KG_DIM == 3) (void)std::stod(a.pos[5]);  // Lz (unused by the reference)
    T = std::stod(a.pos[8 + 2 * o]);
    nt = std::stoul(a.pos[9 + 2 * o]);
    ns = std::stoul(a.pos[10 + 2 * o]);
    m = cli::flag_int(a, "m", 10);  // kg_driver_dev_3d.cpp:145
    device = cli::flag_int(a, "device", -1);
  } catch (const std::exception &e) {
    std::cerr << "Error: bad argument (" << e.what() << ")\n";
    print_usage(argv[0]);
    return 1;
  }
  const std::string u_file = a.pos[4 + 2 * o], v_file = a.pos[5 + 2 * o];
  const std::string out_u = a.pos[6 + 2 * o], out_v = a.pos[7 + 2 * o];
  const std::string m_file = a.pos[11 + 2 * o], c_file = a.pos[12 + 2 * o];
  if (nx < 3 || ny < 3 || (KG_DIM == 3 && nz < 3) || nt < 1 || ns < 1) {
    std::cerr << "Error: need grid extents >= 3 and nt, num_snapshots >= 1\n";
    return 1;
  }
  const double dx = 2 * Lx / (nx - 1), dy = 2 * Ly / (ny - 1);
  (void)dy;
  const double dt = T / nt;
  const uint32_t freq = nt / ns;
  if (freq == 0) {
    std::cerr << "Error: num_snapshots (" << ns << ") > nt (" << nt << ")\n";
    return 1;
  }
  std::vector<uint64_t> ushape, vshape;
  std::vector<double> u0, v0;
  try {
    u0 = npy::load<double>(u_file, ushape);
    v0 = npy::load<double>(v_file, vshape);
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
#if KG_DIM == 3
  const std::vector<uint64_t> fshape = {nz, ny, nx}, mshape = fshape, cshape = fshape;
  const bool true_shape = a.flags.count("true-shape") > 0;
  const std::vector<uint64_t> out_shape =
      true_shape ? std::vector<uint64_t>{ns, nz, ny, nx} : std::vector<uint64_t>{ns, ny, nx};
#else
  // kg_driver_dev_2d.cpp:63,77,92 -- consistent only on the square grids the
  // builder asserts (laplacians.hpp:63)
  const std::vector<uint64_t> fshape = {nx, ny}, mshape = {ny, nx}, cshape = {nx, ny};
  const std::vector<uint64_t> out_shape = {ns, ny, nx};
#endif
  if (ushape != fshape || vshape.size() != fshape.size() || v0.size() != u0.size()) {
    std::cerr << "Error: Input array dimensions mismatch\n";
    std::cerr << "Expected: " << ny << "x" << nx << "\n";
    std::cerr << "Got: " << shape_text(ushape) << "\n";
    return 1;
  }
  std::vector<double> mfield, cfield;
  if (!load_field(m_file, mshape, "m", mfield)) return 1;
  if (!load_field(c_file, cshape, "c", cfield)) return 1;

  try {
    const uint64_t payload = (uint64_t)ns * nz * ny * nx;
    npy::Writer wu = npy::Writer::open<double>(out_u, out_shape, payload);
    npy::Writer wv = npy::Writer::open<double>(out_v, out_shape, payload);
    nls::Grid g;
    g.dim = KG_DIM;
#if KG_DIM == 3
    g.nx = nx;
    g.ny = ny;
    g.nz = nz;
    g.dy = dx;
#else
    g.nx = (uint32_t)fshape[1];  // C layout of the arrays
    g.ny = (uint32_t)fshape[0];
    g.dy = dy;
#endif
    g.dx = dx;
    uint32_t next = 0;
    nls::KGESolverDevice solver(
        g, u0.data(), v0.data(), mfield.data(), cfield.data(), dt, ns, (uint32_t)m,
        [&](uint32_t idx, const double *u, const double *v, uint64_t n) {
          if (idx != next) throw std::runtime_error("snapshot order");
          wu.append(u, n * sizeof(double));
          wv.append(v, n * sizeof(double));
          ++next;
        },
        device);
    for (uint32_t i = 1; i < nt; ++i) {
      solver.step();
      solver.apply_bc();
      if (i % freq == 0) solver.store_snapshot(i / freq);
    }
    wu.close();
    wv.close();
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
