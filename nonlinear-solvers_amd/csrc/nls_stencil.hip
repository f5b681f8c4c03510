// nls_stencil.hip -- kernel tables of the stencil passes (k_update<J>, k_alpha,
// k_lap, k_alpha_l2, k_final_fused) for ONE operator variant and dimension.  The Makefile compiles this
// file four times (NLS_ANI = 0/1 x NLS_DIM = 2/3) so the ~250 instantiations
// build in parallel; nls_kernels.hip dispatches between the four tables.
//   NLS_ANI 0: G1 isotropic operator, f64 (sine-Gordon) and c128 (NLSE)
//   NLS_ANI 1: G2 anisotropic div(c grad) operator, c128 (NLSE) and f64 (Klein-Gordon)
#include "nls_stencil.hpp"
#include "nls_kernels.hpp"

#include <type_traits>

#if !defined(NLS_ANI) || !defined(NLS_DIM) || !defined(NLS_TABLE)
#error "compile with -DNLS_ANI=0|1 -DNLS_DIM=2|3 -DNLS_TABLE=<name>"
#endif

namespace nls {

namespace {
template <class S> const void *update_fn(int J) {
  switch (J) {
#define X(J) case J: return reinterpret_cast<const void *>(&k_update<S, NLS_DIM, J, (NLS_ANI != 0)>);
    NLS_J_LIST(X)
#undef X
    default: return nullptr;
  }
}
const void *fused_fn(int M) {
  switch (M) {
#define X(M) case M: return reinterpret_cast<const void *>(&k_final_fused<NLS_DIM, M, (NLS_ANI != 0)>);
    NLS_MF_LIST(X)
#undef X
    default: return nullptr;
  }
}
template <class S> const void *pick(int kind, int J) {
  switch (kind) {
    case NLS_KIND_ALPHA_L2: return reinterpret_cast<const void *>(&k_alpha_l2<S, NLS_DIM, (NLS_ANI != 0)>);
    case NLS_KIND_FINAL: return std::is_same<S, cplx>::value ? fused_fn(J) : nullptr;
    case NLS_KIND_UPDATE: return update_fn<S>(J);
    case NLS_KIND_ALPHA: return reinterpret_cast<const void *>(&k_alpha<S, NLS_DIM, (NLS_ANI != 0)>);
    case NLS_KIND_LAP: return reinterpret_cast<const void *>(&k_lap<S, NLS_DIM, (NLS_ANI != 0)>);
    default: return nullptr;
  }
}
}  // namespace

const void *NLS_TABLE(int kind, bool complex_, int J) {
  return complex_ ? pick<cplx>(kind, J) : pick<double>(kind, J);
}

}  // namespace nls
