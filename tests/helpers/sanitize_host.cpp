// Drives libpluss_host's functions (csrc/host/pluss_host.cpp) on synthetic
// raw histograms, from several threads at once, for the ASan/UBSan and TSan
// builds (tests/test_sanitizers.py): the host pipeline keeps no global state.
// Test-only.
#include <cstdio>
#include <thread>
#include <vector>

#include "pluss_host.h"

static int run(int seed) {
  std::vector<pluss_hist_entry> raw;
  for (int ref = 0; ref < 6; ++ref)
    for (int x = 0; x < 40; ++x) {
      const int64_t ri = x == 0 ? -1 : (int64_t)(1 + ((x * 7919 + seed * 31) % 70000));
      raw.push_back(pluss_hist_entry{ref, (ref == 3 && ri > 33000) ? 1 : 0, ri, (uint64_t)(1 + x * 3 + seed)});
    }
  std::vector<pluss_kv> out(1 << 16), merged(1 << 16), mrc(400000);
  std::vector<char> text(1 << 22);
  uint64_t n = 0, nm = 0, nmrc = 0, len = 0;
  std::vector<pluss_kv> all;
  for (int ref = 0; ref < 6; ++ref) {
    std::vector<pluss_hist_entry> one;
    for (auto& e : raw)
      if (e.ref == ref) one.push_back(e);
    if (pluss_cri_r10(4, one.data(), one.size(), out.data(), out.size(), &n)) return 1;
    all.insert(all.end(), out.begin(), out.begin() + n);
  }
  if (pluss_log2_merge(all.data(), all.size(), merged.data(), merged.size(), &nm)) return 2;
  if (pluss_aet(merged.data(), nm, mrc.data(), mrc.size(), &nmrc)) return 3;
  if (pluss_format_hist("reuse", merged.data(), nm, text.data(), text.size(), &len)) return 4;
  if (pluss_format_mrc(mrc.data(), nmrc, text.data(), text.size(), &len)) return 5;
  if (pluss_cri_v1(4, raw.data(), raw.size(), out.data(), out.size(), &n)) return 6;
  // r10's host half in one call: six CRI threads, merge, AET, text
  {
    pluss_hist h = {raw.data(), raw.size(), raw.size(), {0}};
    std::vector<pluss_kv> reuse(1 << 16), m2(400000);
    uint64_t nr = 0, nm2 = 0, tl = 0;
    if (pluss_r10_host_pipeline(4, &h, 6, reuse.data(), reuse.size(), &nr, m2.data(), m2.size(), &nm2, text.data(),
                                text.size(), &tl))
      return 8;
    if (nm2 == 0 || tl == 0) return 9;
  }
  // a buffer too small: an error code, nothing written past it, the needed length reported
  char small[9];
  small[8] = 'X';
  if (pluss_format_hist("tiny", out.data(), n, small, 8, &len) == 0 || small[8] != 'X' || len < 8) return 7;
  return 0;
}

int main() {
  std::vector<std::thread> th;
  std::vector<int> rc(4, -1);
  for (int t = 0; t < 4; ++t) th.emplace_back([&, t] { rc[t] = run(t); });
  for (auto& x : th) x.join();
  for (int r : rc)
    if (r) {
      std::printf("host driver failed: %d\n", r);
      return 1;
    }
  std::printf("host sanitizer driver ok\n");
  return 0;
}
