// npy_tool -- exercises the driver .npy codec (used by the CPU test-suite):
//   npy_tool copy-c16 in.npy out.npy   read complex128, write it back (streamed in 2 chunks)
//   npy_tool copy-f8  in.npy out.npy   same for float64
//   npy_tool shape    in.npy           print the shape (complex128 or float64)
#include <complex>
#include <iostream>
#include <string>

#include "npy.hpp"

template <class T> int copy(const std::string &in, const std::string &out) {
  std::vector<uint64_t> shape;
  std::vector<T> d = npy::load<T>(in, shape);
  npy::Writer w = npy::Writer::open<T>(out, shape);
  const size_t half = d.size() / 2;
  w.append(d.data(), half * sizeof(T));
  w.append(d.data() + half, (d.size() - half) * sizeof(T));
  w.close();
  return 0;
}

int main(int argc, char **argv) {
  try {
    if (argc == 4 && std::string(argv[1]) == "copy-c16") return copy<std::complex<double>>(argv[2], argv[3]);
    if (argc == 4 && std::string(argv[1]) == "copy-f8") return copy<double>(argv[2], argv[3]);
    if (argc == 3 && std::string(argv[1]) == "shape") {
      std::vector<uint64_t> shape;
      try {
        npy::load<std::complex<double>>(argv[2], shape);
      } catch (...) {
        npy::load<double>(argv[2], shape);
      }
      for (auto s : shape) std::cout << s << " ";
      std::cout << "\n";
      return 0;
    }
  } catch (const std::exception &e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
  std::cerr << "usage: npy_tool copy-c16|copy-f8 in out | shape in\n";
  return 1;
}
