// nlse_call / nlse_cq_call -- drop-in replacement of the reference drivers
// device/nlse_call.cpp and device/nlse_cq_call.cpp on the MI355X library.
//
//   prog nx ny Lx Ly input_u0.npy output_traj.npy T nt num_snapshots
//        [--m=10] [--device=-1] [--sigma1=re,im] [--sigma2=re,im]   (extensions)
//
// Same argv, exit codes, stdout line and .npy layout as the reference
// (device/nlse_call.cpp:13-88): u0 complex128 [ny, nx] normalised to unit
// mass sum |u|^2 dx dy; nt-1 SS2 steps with tau = 1j*T/nt; a snapshot every
// nt/num_snapshots steps; output complex128 [num_snapshots, ny, nx].
// Snapshots are streamed to the output file as they are produced.
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

#ifndef NLSE_EQUATION
#define NLSE_EQUATION NLS_NLSE_CUBIC
#endif

static void print_usage(const char *program_name) {
  std::cerr << "Usage: " << program_name
            << " nx ny Lx Ly input_u0.npy output_traj.npy T nt num_snapshots\n";
  std::cerr << "Example: " << program_name
            << " 256 256 10.0 10.0 initial.npy evolution.npy 1.5 500 100\n";
}

static std::complex<double> parse_c(const std::string &s) {
  const size_t c = s.find(',');
  if (c == std::string::npos) return {std::stod(s), 0.0};
  return {std::stod(s.substr(0, c)), std::stod(s.substr(c + 1))};
}

int main(int argc, char **argv) {
  const cli::Args a = cli::parse(argc, argv);
  if (a.pos.size() != 9) {
    print_usage(argv[0]);
    return 1;
  }
  uint32_t nx, ny, nt, num_snapshots;
  double Lx, Ly, T;
  int m, device;
  std::complex<double> s1, s2;
  try {
    nx = std::stoul(a.pos[0]);
    ny = std::stoul(a.pos[1]);
    Lx = std::stod(a.pos[2]);
    Ly = std::stod(a.pos[3]);
    T = std::stod(a.pos[6]);
    nt = std::stoul(a.pos[7]);
    num_snapshots = std::stoul(a.pos[8]);
    m = cli::flag_int(a, "m", 10);
    device = cli::flag_int(a, "device", -1);
    s1 = parse_c(cli::flag_str(a, "sigma1", "0,0.5"));
    s2 = parse_c(cli::flag_str(a, "sigma2", "-0.5,0"));
  } catch (const std::exception &e) {
    std::cerr << "Error: bad argument (" << e.what() << ")\n";
    print_usage(argv[0]);
    return 1;
  }
  const std::string input_file = a.pos[4];
  const std::string output_file = a.pos[5];
  if (nx < 2 || ny < 2 || nt < 1 || num_snapshots < 1) {
    std::cerr << "Error: need nx, ny >= 2 and nt, num_snapshots >= 1\n";
    return 1;
  }

  const double dx = 2 * Lx / (nx - 1);
  const double dy = 2 * Ly / (ny - 1);
  const double dt = T / nt;
  const uint32_t freq = nt / num_snapshots;
  const std::complex<double> dti(0, dt);
  if (freq == 0) {  // the reference divides by zero here (i % freq)
    std::cerr << "Error: num_snapshots (" << num_snapshots << ") > nt (" << nt << ")\n";
    return 1;
  }

  std::vector<uint64_t> input_shape;
  std::vector<std::complex<double>> u0;
  try {
    u0 = npy::load<std::complex<double>>(input_file, input_shape);
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  if (input_shape.size() != 2 || input_shape[0] != ny || input_shape[1] != nx) {
    std::cerr << "Error: Input array dimensions mismatch\n";
    std::cerr << "Expected: " << ny << "x" << nx << "\n";
    std::cerr << "Got: " << (input_shape.size() > 0 ? input_shape[0] : 0) << "x"
              << (input_shape.size() > 1 ? input_shape[1] : 0) << "\n";
    return 1;
  }
  // u0 /= sqrt(sum conj(u) u dx dy)   (nlse_call.cpp:41-49)
  double mass = 0.0;
  for (const auto &v : u0) mass += (std::conj(v) * v).real() * dx * dy;
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
        output_file, {num_snapshots, (uint64_t)ny, (uint64_t)nx});
    nls::Grid g;
    g.dim = 2;
    g.nx = nx;
    g.ny = ny;
    g.dx = dx;
    g.dy = dy;
    nls::NLSESolverDevice::Parameters params(num_snapshots, freq, (uint32_t)m);
    nls::NLSESolverDevice solver(
        g, u0.data(), params,
        [&](uint32_t, const std::complex<double> *u, uint64_t n) {  // writer thread
          out.append(u, n * sizeof(std::complex<double>));
        },
        NLSE_EQUATION, device, s1, s2);
    lap("constructed");
    for (uint32_t i = 1; i < nt; ++i) solver.step(dti, i);
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
  // as the reference (device/nlse_call.cpp:63-79): construction, steps and all
  // snapshot transfers.  The .npy writing overlaps the loop on the snapshot
  // writer thread; whatever of it the loop had to wait for is included.
  const double compute_time = elapsed;

  std::cout << std::scientific << std::setprecision(4);
  std::cout << "Trajectory took: " << compute_time << "s\n";
  return 0;
}
