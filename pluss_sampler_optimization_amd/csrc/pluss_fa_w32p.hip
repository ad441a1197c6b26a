// pluss_fa_w32p.hip — the faithful scan pipeline (pluss_faithful.h) instantiated
// for one element source, in a translation unit of its own: the radix sort's
// 4-byte payloads with their parents' digits put back (SRC_W32P).
#include "pluss_faithful.h"

namespace pluss {

void fa_launch_w32p(const FaLaunch& L) {
  if (L.p2) fa_launch_t<SRC_W32P, false, true>(L);
  else fa_launch_t<SRC_W32P, false, false>(L);
}

}  // namespace pluss
