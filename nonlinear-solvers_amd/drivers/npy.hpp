// npy.hpp -- minimal .npy reader/writer (format versions 1.0-3.0, C order,
// little-endian '<c16' / '<f8').  Replaces the reference's libnpy submodule
// (.gitmodules:1-3, absent offline) behind the same save/read contract as
// util.hpp:25-50.  The writer supports streaming: write the header for the
// final shape, then append records (snapshots) as they are produced.
#pragma once
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace npy {

template <class T> const char *descr();
template <> inline const char *descr<double>() { return "<f8"; }
template <> inline const char *descr<std::complex<double>>() { return "<c16"; }

inline std::string shape_str(const std::vector<uint64_t> &shape) {
  std::string s = "(";
  for (size_t i = 0; i < shape.size(); ++i) {
    s += std::to_string(shape[i]);
    if (shape.size() == 1 || i + 1 < shape.size()) s += ",";
    if (i + 1 < shape.size()) s += " ";
  }
  return s + ")";
}

// Header as numpy writes it: v1.0, dict padded with spaces so that the data
// starts at a multiple of 64 bytes, terminated by '\n'.
inline std::string make_header(const char *dsc, const std::vector<uint64_t> &shape) {
  std::string dict = std::string("{'descr': '") + dsc + "', 'fortran_order': False, 'shape': " +
                     shape_str(shape) + ", }";
  const size_t pre = 10;  // magic(6) + version(2) + len(2)
  size_t total = pre + dict.size() + 1;
  const size_t padded = (total + 63) / 64 * 64;
  dict.append(padded - total, ' ');
  dict.push_back('\n');
  std::string h("\x93NUMPY\x01\x00", 8);
  const uint16_t len = (uint16_t)dict.size();
  h.push_back((char)(len & 0xff));
  h.push_back((char)(len >> 8));
  return h + dict;
}

class Writer {
 public:
  template <class T>
  static Writer open(const std::string &path, const std::vector<uint64_t> &shape) {
    uint64_t n = 1;
    for (auto d : shape) n *= d;
    return open<T>(path, shape, n);
  }
  // header `shape`, payload of `elems` values: the reference's 3D Klein-Gordon
  // driver writes the header [ns, ny, nx] for ns*nz*ny*nx values
  // (kg_driver_dev_3d.cpp:161-163; libnpy writes the whole vector)
  template <class T>
  static Writer open(const std::string &path, const std::vector<uint64_t> &shape, uint64_t elems) {
    Writer w;
    w.f_ = std::fopen(path.c_str(), "wb");
    if (!w.f_) throw std::runtime_error("cannot open " + path + " for writing");
    const std::string h = make_header(descr<T>(), shape);
    if (std::fwrite(h.data(), 1, h.size(), w.f_) != h.size()) throw std::runtime_error("write failed");
    w.expect_ = sizeof(T) * elems;
    return w;
  }
  Writer() = default;
  Writer(Writer &&o) noexcept : f_(o.f_), expect_(o.expect_), written_(o.written_) { o.f_ = nullptr; }
  Writer &operator=(Writer &&o) noexcept {
    std::swap(f_, o.f_);
    expect_ = o.expect_;
    written_ = o.written_;
    return *this;
  }
  ~Writer() {
    if (f_) std::fclose(f_);
  }
  void append(const void *data, size_t bytes) {
    if (written_ + bytes > expect_) throw std::runtime_error("npy: more data than the declared shape");
    if (std::fwrite(data, 1, bytes, f_) != bytes) throw std::runtime_error("npy: write failed");
    written_ += bytes;
  }
  // pad with zeros up to the declared size (unfilled snapshot slots), close
  void close() {
    if (!f_) return;
    std::vector<char> z(1 << 16, 0);
    while (written_ < expect_) {
      const size_t n = std::min<size_t>(z.size(), expect_ - written_);
      append(z.data(), n);
    }
    std::fclose(f_);
    f_ = nullptr;
  }

 private:
  FILE *f_ = nullptr;
  uint64_t expect_ = 0, written_ = 0;
};

template <class T>
void save(const std::string &path, const T *data, const std::vector<uint64_t> &shape) {
  Writer w = Writer::open<T>(path, shape);
  uint64_t n = 1;
  for (auto d : shape) n *= d;
  w.append(data, n * sizeof(T));
  w.close();
}

// Read a C-order array of dtype T; shape returned in `shape`.
template <class T>
std::vector<T> load(const std::string &path, std::vector<uint64_t> &shape) {
  FILE *f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  struct Closer {
    FILE *f;
    ~Closer() { std::fclose(f); }
  } closer{f};
  char magic[8];
  if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, "\x93NUMPY", 6) != 0)
    throw std::runtime_error(path + ": not a .npy file");
  const int major = (unsigned char)magic[6];
  uint32_t hlen = 0;
  if (major == 1) {
    unsigned char b[2];
    if (std::fread(b, 1, 2, f) != 2) throw std::runtime_error("truncated header");
    hlen = b[0] | (b[1] << 8);
  } else if (major == 2 || major == 3) {
    unsigned char b[4];
    if (std::fread(b, 1, 4, f) != 4) throw std::runtime_error("truncated header");
    hlen = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
  } else {
    throw std::runtime_error(path + ": unsupported .npy version");
  }
  std::string h(hlen, '\0');
  if (std::fread(&h[0], 1, hlen, f) != hlen) throw std::runtime_error("truncated header");
  auto field = [&](const char *key) -> std::string {
    const size_t k = h.find(key);
    if (k == std::string::npos) throw std::runtime_error(std::string("npy header lacks ") + key);
    return h.substr(k + std::strlen(key));
  };
  std::string d = field("'descr':");
  const size_t q0 = d.find('\''), q1 = d.find('\'', q0 + 1);
  const std::string dsc = d.substr(q0 + 1, q1 - q0 - 1);
  if (dsc != descr<T>() && !(dsc == "|c16" && std::string(descr<T>()) == "<c16"))
    throw std::runtime_error(path + ": dtype " + dsc + ", expected " + descr<T>());
  std::string fo = field("'fortran_order':");
  if (fo.find("True") < fo.find(','))
    throw std::runtime_error(path + ": fortran_order arrays are not supported");
  std::string sh = field("'shape':");
  const size_t p0 = sh.find('('), p1 = sh.find(')');
  sh = sh.substr(p0 + 1, p1 - p0 - 1);
  shape.clear();
  size_t pos = 0;
  while (pos < sh.size()) {
    while (pos < sh.size() && (sh[pos] == ' ' || sh[pos] == ',')) ++pos;
    if (pos >= sh.size()) break;
    size_t e = pos;
    while (e < sh.size() && sh[e] >= '0' && sh[e] <= '9') ++e;
    if (e == pos) throw std::runtime_error("bad shape in npy header");
    shape.push_back(std::stoull(sh.substr(pos, e - pos)));
    pos = e;
  }
  uint64_t n = 1;
  for (auto s : shape) n *= s;
  std::vector<T> out(n);
  if (n && std::fread(out.data(), sizeof(T), n, f) != n) throw std::runtime_error(path + ": truncated data");
  return out;
}

}  // namespace npy
