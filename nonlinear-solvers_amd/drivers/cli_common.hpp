// cli_common.hpp -- shared argv helpers of the drop-in drivers.
#pragma once
#include <cstdlib>
#include <iostream>
#include <map>
#include <string>
#include <vector>

namespace cli {

// Split argv into positional arguments and trailing --key=value flags (the
// reference CLIs are purely positional; flags are an optional extension).
struct Args {
  std::vector<std::string> pos;
  std::map<std::string, std::string> flags;
  bool bad_flag = false;
};

inline Args parse(int argc, char **argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    if (s.rfind("--", 0) == 0) {
      const size_t eq = s.find('=');
      if (eq == std::string::npos) {
        a.flags[s.substr(2)] = "1";
      } else {
        a.flags[s.substr(2, eq - 2)] = s.substr(eq + 1);
      }
    } else {
      a.pos.push_back(s);
    }
  }
  return a;
}

inline int flag_int(const Args &a, const std::string &k, int def) {
  auto it = a.flags.find(k);
  return it == a.flags.end() ? def : std::stoi(it->second);
}
inline double flag_double(const Args &a, const std::string &k, double def) {
  auto it = a.flags.find(k);
  return it == a.flags.end() ? def : std::stod(it->second);
}
inline std::string flag_str(const Args &a, const std::string &k, const std::string &def) {
  auto it = a.flags.find(k);
  return it == a.flags.end() ? def : it->second;
}

}  // namespace cli
