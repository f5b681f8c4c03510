// nlse_call_3d -- 3D counterpart of nlse_call on the MI355X library (G1
// semantics of nlse_driver_3d.cpp: build_laplacian_noflux_3d incl. the y-wrap,
// scale 1/dx^2, mass normalised with dx*dy*dz, tau = 1j*dt).  The reference
// has no 3D G1 CLI (nlse_driver_3d.cpp hard-codes its parameters); the argv
// follows nlse_call with a z extent added:
//
//   prog nx ny nz Lx Ly Lz input_u0.npy output_traj.npy T nt num_snapshots
//        [--m=10] [--device=-1] [--cq] [--sigma1=re,im] [--sigma2=re,im]
//
// input complex128 [nz, ny, nx]; output complex128 [num_snapshots, nz, ny, nx].
#include <chrono>
#include <cstdlib>
#include <complex>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "cli_common.hpp"
#include "nls_solver.hpp"
#include "npy.hpp"

static void print_usage(const char *p) {
  std::cerr << "Usage: " << p
            << " nx ny nz Lx Ly Lz input_u0.npy output_traj.npy T nt num_snapshots\n";
}

static std::complex<double> parse_c(const std::string &s) {
  const size_t c = s.find(',');
  if (c == std::string::npos) return {std::stod(s), 0.0};
  return {std::stod(s.substr(0, c)), std::stod(s.substr(c + 1))};
}

int main(int argc, char **argv) {
  const cli::Args a = cli::parse(argc, argv);
  if (a.pos.size() != 11) {
    print_usage(argv[0]);
    return 1;
  }
  uint32_t nx, ny, nz, nt, ns;
  double Lx, Ly, Lz, T;
  int m, device, eq;
  std::complex<double> s1, s2;
  try {
    nx = std::stoul(a.pos[0]);
    ny = std::stoul(a.pos[1]);
    nz = std::stoul(a.pos[2]);
    Lx = std::stod(a.pos[3]);
    Ly = std::stod(a.pos[4]);
    Lz = std::stod(a.pos[5]);
    T = std::stod(a.pos[8]);
    nt = std::stoul(a.pos[9]);
    ns = std::stoul(a.pos[10]);
    m = cli::flag_int(a, "m", 10);
    device = cli::flag_int(a, "device", -1);
    eq = a.flags.count("cq") ? NLS_NLSE_CQ : NLS_NLSE_CUBIC;
    s1 = parse_c(cli::flag_str(a, "sigma1", "0,0.5"));
    s2 = parse_c(cli::flag_str(a, "sigma2", "-0.5,0"));
  } catch (const std::exception &e) {
    std::cerr << "Error: bad argument (" << e.what() << ")\n";
    print_usage(argv[0]);
    return 1;
  }
  if (nx < 2 || ny < 2 || nz < 2 || nt < 1 || ns < 1) {
    std::cerr << "Error: need nx, ny, nz >= 2 and nt, num_snapshots >= 1\n";
    return 1;
  }
  const double dx = 2 * Lx / (nx - 1), dy = 2 * Ly / (ny - 1), dz = 2 * Lz / (nz - 1);
  const double dt = T / nt;
  const uint32_t freq = nt / ns;
  if (freq == 0) {
    std::cerr << "Error: num_snapshots (" << ns << ") > nt (" << nt << ")\n";
    return 1;
  }
  std::vector<uint64_t> shape;
  std::vector<std::complex<double>> u0;
  try {
    u0 = npy::load<std::complex<double>>(a.pos[6], shape);
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  if (shape.size() != 3 || shape[0] != nz || shape[1] != ny || shape[2] != nx) {
    std::cerr << "Error: Input array dimensions mismatch\n";
    std::cerr << "Expected: " << nz << "x" << ny << "x" << nx << "\n";
    return 1;
  }
  double mass = 0.0;  // nlse_driver_3d.cpp:185-189
  for (const auto &v : u0) mass += std::norm(v) * dx * dy * dz;
  const double norm = std::sqrt(mass);
  for (auto &v : u0) v /= norm;

  auto start = std::chrono::high_resolution_clock::now();
  double elapsed = 0.0;
  const bool phase_times = std::getenv("NLS_DRIVER_TIMING") != nullptr;
  auto lap = [&](const char *what) {
    if (phase_times)
      std::cerr << what << " " << std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - start).count() << " s\n";
  };
  try {
    npy::Writer out = npy::Writer::open<std::complex<double>>(
        a.pos[7], {ns, (uint64_t)nz, (uint64_t)ny, (uint64_t)nx});
    nls::Grid g;
    g.dim = 3;
    g.nx = nx;
    g.ny = ny;
    g.nz = nz;
    g.dx = dx;
    g.dy = dy;
    nls::NLSESolverDevice::Parameters params(ns, freq, (uint32_t)m);
    nls::NLSESolverDevice solver(
        g, u0.data(), params,
        [&](uint32_t, const std::complex<double> *u, uint64_t n) {  // writer thread
          out.append(u, n * sizeof(std::complex<double>));
        },
        eq, device, s1, s2);
    lap("constructed");
    for (uint32_t i = 1; i < nt; ++i) solver.step({0.0, dt}, i);
    lap("enqueued");
    solver.sync();
    elapsed = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - start).count();
    lap("synced");
    solver.finish();
    out.close();
    lap("written");
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  std::cout << std::scientific << std::setprecision(4);
  std::cout << "Trajectory took: " << elapsed << "s\n";
  return 0;
}
