// nls_stencil.hip -- kernel tables of the stencil passes (k_update<J>, k_alpha,
// k_lap, k_alpha_l2, k_tail) for ONE operator variant and dimension.  The Makefile compiles this
// file four times (NLS_ANI = 0/1 x NLS_DIM = 2/3) so the ~250 instantiations
// build in parallel; nls_kernels.hip dispatches between the four tables.
//   NLS_ANI 0: G1 isotropic operator, f64 (sine-Gordon) and c128 (NLSE)
//   NLS_ANI 1: G2 anisotropic div(c grad) operator, c128 (NLSE) and f64 (Klein-Gordon)
#include "nls_reduce.hpp"
#include "nls_stencil.hpp"
#include "nls_kernels.hpp"

#include <type_traits>

#if !defined(NLS_ANI) || !defined(NLS_DIM) || !defined(NLS_TABLE)
#error "compile with -DNLS_ANI=0|1 -DNLS_DIM=2|3 -DNLS_TABLE=<name>"
#endif

namespace nls {

namespace {
// J encodes qa * 64 + J (qa: the next alpha folded into the pass, march_q)
template <class S> const void *update_fn(int code) {
  const int J = code % 64;
  if (code >= 64) {
    switch (J) {
#define X(J) case J: return reinterpret_cast<const void *>(&k_update<S, NLS_DIM, J, (NLS_ANI != 0), true>);
      NLS_J_LIST(X)
#undef X
      default: return nullptr;
    }
  }
  switch (J) {
#define X(J) case J: return reinterpret_cast<const void *>(&k_update<S, NLS_DIM, J, (NLS_ANI != 0)>);
    NLS_J_LIST(X)
#undef X
    default: return nullptr;
  }
}
// tail kernels: J encodes mode * 64 + M.  G1 (iso) tables hold the NLSE,
// sine-Gordon and G2 Gautschi-family tails, G2 (ani) tables the NLSE,
// Klein-Gordon and sEWI tails.
template <class S, int MODE> const void *tail_m(int M) {
  switch (M) {
#define X(M) case M: return reinterpret_cast<const void *>(&k_tail<S, NLS_DIM, M, (NLS_ANI != 0), MODE>);
    NLS_MF_LIST(X)
#undef X
    default: return nullptr;
  }
}
const void *tail_fn(bool complex_, int code) {
  const int mode = code / 64, M = code % 64;
  if (mode == TAIL_COMBINE)  // every variant: nls_krylov_apply on a basis that stores m-1 vectors
    return complex_ ? tail_m<cplx, TAIL_COMBINE>(M) : tail_m<double, TAIL_COMBINE>(M);
  if (complex_) {
    switch (mode) {
      case TAIL_NLSE: return tail_m<cplx, TAIL_NLSE>(M);
#if NLS_ANI
      case TAIL_COMBINE_W0: return tail_m<cplx, TAIL_COMBINE_W0>(M);
      case TAIL_SEWI_END: return tail_m<cplx, TAIL_SEWI_END>(M);
#endif
      default: return nullptr;
    }
  }
  switch (mode) {
#if NLS_ANI
    case TAIL_KG_END: return tail_m<double, TAIL_KG_END>(M);
    case TAIL_KG_END1: return tail_m<double, TAIL_KG_END1>(M);
    case TAIL_COMBINE_W0: return tail_m<double, TAIL_COMBINE_W0>(M);
#else
    case TAIL_SG_MID: return tail_m<double, TAIL_SG_MID>(M);
    case TAIL_GG_MID: return tail_m<double, TAIL_GG_MID>(M);
    case TAIL_SG_END: return tail_m<double, TAIL_SG_END>(M);
#endif
    default: return nullptr;
  }
}
template <class S> const void *pick(int kind, int J) {
  switch (kind) {
    case NLS_KIND_XPAIRS: return reinterpret_cast<const void *>(&k_xpairs<S, NLS_DIM, (NLS_ANI != 0)>);
    case NLS_KIND_REDUCE_QA: return reinterpret_cast<const void *>(&k_reduce_qa<S, NLS_DIM, (NLS_ANI != 0)>);
    case NLS_KIND_ALPHA_L2:  // J = 1: the pipelined march (3D)
      return J && NLS_DIM == 3 ? reinterpret_cast<const void *>(&k_alpha_l2<S, NLS_DIM, (NLS_ANI != 0), true>)
                               : reinterpret_cast<const void *>(&k_alpha_l2<S, NLS_DIM, (NLS_ANI != 0)>);
    case NLS_KIND_FINAL: return tail_fn(std::is_same<S, cplx>::value, J);
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
