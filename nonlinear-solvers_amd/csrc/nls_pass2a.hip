// nls_pass2a.hip -- instantiations of the LDS-DMA two-vector pass k_p2d for the G2
// anisotropic operator div(c grad) (nls_pass2d.hpp, A = true): 3D complex fields,
// J = 0, 2, .., 22 (m <= 26; the G2 NLSE driver runs m = 25), and 3D real fields as
// pairs of cells (the Klein-Gordon Gautschi step), J = 0, 2, .., 14; with and without Z.
#define NLS_NO_P2_KERNELS  // k_p2coef / k_p2tail / k_p2tfin live in nls_kernels.hip
#include "nls_reduce.hpp"
#include "nls_kernels.hpp"
#include "nls_pass2d.hpp"

namespace nls {

const void *kernel_pass2a(int J, bool hz, bool pr) {
  if (pr) {  // real fields as pairs of cells (Klein-Gordon), J <= P2D_JMAX_A2
    switch (J) {
#define X(J)                                                                        \
  case J:                                                                           \
    return hz ? reinterpret_cast<const void *>(&k_p2d<J, true, false, true, true>)  \
              : reinterpret_cast<const void *>(&k_p2d<J, false, false, true, true>);
      X(0) X(2) X(4) X(6) X(8) X(10) X(12) X(14)
#undef X
      default: return nullptr;
    }
  }
  switch (J) {
#define X(J)                                                                          \
  case J:                                                                             \
    return hz ? reinterpret_cast<const void *>(&k_p2d<J, true, false, false, true>)   \
              : reinterpret_cast<const void *>(&k_p2d<J, false, false, false, true>);
    X(0) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(22)
#undef X
    default: return nullptr;
  }
}

}  // namespace nls
