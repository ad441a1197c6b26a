// pluss_fa_uni.hip — the faithful scan pipeline (pluss_faithful.h) instantiated
// for the uniform key-order lists generated inside the pass (pluss_uniform.h),
// in a translation unit of its own.
#include "pluss_faithful.h"

namespace pluss {

void fa_launch_uni(const FaLaunch& L) {
  if (L.p2) fa_launch_t<SRC_UNI, false, true>(L);
  else fa_launch_t<SRC_UNI, false, false>(L);
}

}  // namespace pluss
