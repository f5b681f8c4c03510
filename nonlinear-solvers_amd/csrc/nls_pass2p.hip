// nls_pass2p.hip -- instantiations of the LDS-DMA two-vector pass k_p2d with the
// peer-store epilogue (nls_pass2d.hpp, PEER = true; NLS_PEER=1 multi-rank handles,
// DESIGN.md section 5): 3D isotropic complex fields, J = 0, 2, .., 14, with and
// without Z.  A separate object: the plain instantiations keep their march loop.
#define NLS_NO_P2_KERNELS  // k_p2coef / k_p2tail / k_p2tfin live in nls_kernels.hip
#include "nls_reduce.hpp"
#include "nls_kernels.hpp"
#include "nls_pass2d.hpp"

namespace nls {

const void *kernel_pass2_peer(int J, bool hz) {
  switch (J) {
#define X(J)                                                                                \
  case J:                                                                                   \
    return hz ? reinterpret_cast<const void *>(&k_p2d<J, true, false, false, false, true>)  \
              : reinterpret_cast<const void *>(&k_p2d<J, false, false, false, false, true>);
    X(0) X(2) X(4) X(6) X(8) X(10) X(12) X(14)
#undef X
    default: return nullptr;
  }
}

}  // namespace nls
