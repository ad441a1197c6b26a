// pluss_fa_smp.hip — the faithful scan pipeline (pluss_faithful.h) instantiated
// for one element source, in a translation unit of its own.
#include "pluss_faithful.h"

namespace pluss {

void fa_launch_smp(const FaLaunch& L) {
  if (L.p2) fa_launch_t<SRC_SAMPLES, true, true>(L);
  else fa_launch_t<SRC_SAMPLES, true, false>(L);
}

}  // namespace pluss
