// nls_pass2g.hip -- instantiations of the march two-vector pass k_p2m (nls_pass2g.hpp):
// 2D / 3D, isotropic / G2 anisotropic, J = 0, 2, .., 28 (m <= 32), with and without Z.
#define NLS_NO_P2_KERNELS  // k_p2coef / k_p2tail / k_p2tfin live in nls_kernels.hip
#include "nls_reduce.hpp"  // (device helpers only; nls_stencil.hpp uses them)
#include "nls_kernels.hpp"
#include "nls_pass2g.hpp"

namespace nls {

namespace {
template <int DIM, bool ANI> const void *p2m_j(int J, bool hz) {
  switch (J) {
#define X(J) \
  case J: return hz ? reinterpret_cast<const void *>(&k_p2m<DIM, J, true, ANI>) \
                    : reinterpret_cast<const void *>(&k_p2m<DIM, J, false, ANI>);
    X(0) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(22) X(24) X(26) X(28)
#undef X
    default: return nullptr;
  }
}
}  // namespace

const void *kernel_p2m(int dim, int J, bool hz, bool ani) {
  if (dim == 3) return ani ? p2m_j<3, true>(J, hz) : p2m_j<3, false>(J, hz);
  return ani ? p2m_j<2, true>(J, hz) : p2m_j<2, false>(J, hz);
}
int p2m_rows_per_thread(int J) {
  switch (J) {
#define X(J) case J: return P2mRB<J>::v;
    X(0) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(22) X(24) X(26) X(28)
#undef X
    default: return 1;
  }
}

}  // namespace nls
