// sg_driver_dev -- drop-in for the reference device/sg_driver_dev.cpp on the
// MI355X library: no arguments runs the reference experiment (2D sine-Gordon,
// nx = ny = 256, L = 3, T = 5, nt = 500, 100 snapshots, u0 = 2 atan(exp(3 - 5r)),
// v0 = 0, m = -1, Gautschi with Krylov m = 10; sg_driver_dev.cpp:23-80) and
// writes evolution_sg_u_device.npy [100, 256, 256] (float64).  The reference
// also runs its Eigen CPU path and prints CPU-vs-GPU diffs; that comparison
// lives in tests/ (against the oracle) -- product binaries never link it.
//
// Optional flags (extensions): --nx=N --L=3 --T=5 --nt=500 --ns=100 --m=10
//   --device=-1 --prefix=evolution_sg  (also writes <prefix>_v_device.npy)
#include <chrono>
#include <cmath>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "cli_common.hpp"
#include "nls_solver.hpp"
#include "npy.hpp"

int main(int argc, char **argv) {
  const cli::Args a = cli::parse(argc, argv);
  if (!a.pos.empty()) {
    std::cerr << "Usage: " << argv[0]
              << " [--nx=256] [--L=3] [--T=5] [--nt=500] [--ns=100] [--m=10] [--device=-1]"
                 " [--prefix=evolution_sg]\n";
    return 1;
  }
  uint32_t nx, nt, ns;
  double L, T;
  int m, device;
  std::string prefix;
  try {
    nx = (uint32_t)cli::flag_int(a, "nx", 256);
    L = cli::flag_double(a, "L", 3.0);
    T = cli::flag_double(a, "T", 5.0);
    nt = (uint32_t)cli::flag_int(a, "nt", 500);
    ns = (uint32_t)cli::flag_int(a, "ns", 100);
    m = cli::flag_int(a, "m", 10);
    device = cli::flag_int(a, "device", -1);
    prefix = cli::flag_str(a, "prefix", "evolution_sg");
  } catch (const std::exception &e) {
    std::cerr << "Error: bad flag (" << e.what() << ")\n";
    return 1;
  }
  const uint32_t ny = nx;
  if (nx < 2 || nt < 1 || ns < 1 || nt / ns == 0) {
    std::cerr << "Error: need nx >= 2 and 1 <= ns <= nt\n";
    return 1;
  }
  const double dx = 2 * L / (nx - 1), dy = 2 * L / (ny - 1);
  const uint32_t freq = nt / ns;
  const double dt = T / nt;

  // apply_function_uniform (sg_driver_dev.cpp:8-21): u[i*nx + j] = f(x[i], y[j])
  const uint64_t n = (uint64_t)nx * ny;
  std::vector<double> u0(n), v0(n, 0.0), mf(n, -1.0);
  for (uint32_t i = 0; i < ny; ++i) {
    const double x = ny > 1 ? -L + 2 * L * i / (ny - 1) : -L;
    for (uint32_t j = 0; j < nx; ++j) {
      const double y = -L + 2 * L * j / (nx - 1);
      u0[(uint64_t)i * nx + j] = 2. * std::atan(std::exp(3. - 5. * std::sqrt(x * x + y * y)));
    }
  }

  double io_seconds = 0.0;
  auto start = std::chrono::high_resolution_clock::now();
  try {
    npy::Writer wu = npy::Writer::open<double>(prefix + "_u_device.npy", {ns, (uint64_t)nx, (uint64_t)ny});
    npy::Writer wv = npy::Writer::open<double>(prefix + "_v_device.npy", {ns, (uint64_t)nx, (uint64_t)ny});
    nls::Grid g;
    g.dim = 2;
    g.nx = nx;
    g.ny = ny;
    g.dx = dx;
    g.dy = dy;
    nls::SGESolverDevice solver(
        g, u0.data(), v0.data(), mf.data(), dt, ns, freq, (uint32_t)m,
        [&](uint32_t, const double *u, const double *v, uint64_t cnt) {
          auto t0 = std::chrono::high_resolution_clock::now();
          wu.append(u, cnt * sizeof(double));
          wv.append(v, cnt * sizeof(double));
          io_seconds += std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
        },
        device);
    for (uint32_t i = 1; i < nt; ++i) solver.step(dt, i);
    wu.close();
    wv.close();
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  auto end = std::chrono::high_resolution_clock::now();
  const double us = (std::chrono::duration<double>(end - start).count() - io_seconds) * 1e6;
  std::cout << std::scientific << std::setprecision(4);
  std::cout << "device time: " << (long long)us << " us\n";
  return 0;
}
