// The library's pluss_aet (its walk in jumps of equal additions) against the
// reference's pluss_AET walk restated step by step (pluss_utils.h:758-804), on
// random histograms: every point must be equal bit for bit.  Test-only
// (tests/test_host_pipeline.py).  usage: aet_check CASES SEED
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <vector>

#include "pluss_host.h"

// pluss_AET, one addition per t (the reference's loop, pluss_utils.h:786-803)
static std::vector<pluss_kv> aet_stepping(const std::map<long, double>& h) {
  std::vector<pluss_kv> out;
  double total = 0;
  long max_rt = 0;
  for (auto& kv : h) {
    total += kv.second;
    if (max_rt < kv.first) max_rt = kv.first;
  }
  std::map<uint64_t, double> P;
  double acc = 0;
  if (h.count(-1)) acc = h.at(-1);
  for (auto it = h.rbegin(); it != h.rend(); ++it) {
    if (it->first == -1) break;
    P[(uint64_t)it->first] = acc / total;
    acc += it->second;
  }
  P[0] = 1.0;
  double sum_p = 0, pred = -1.0;
  uint64_t t = 0, prev_t = 0;
  const uint64_t cs = 2560 * 1024 / sizeof(double);
  for (uint64_t c = 0; (long)c <= max_rt && c <= cs; c++) {
    while (sum_p < (double)c && (long)t <= max_rt) {
      auto f = P.find(t);
      if (f != P.end()) {
        sum_p += f->second;
        prev_t = t;
      } else {
        sum_p += P[prev_t];
      }
      t++;
    }
    if (pred != -1.0 || pred - P[prev_t] < 0.0001) {
      if (pred == -1.0) pred = P[prev_t];
      out.push_back(pluss_kv{(int64_t)c, P[prev_t]});
    }
  }
  return out;
}

int main(int argc, char** argv) {
  const int cases = argc > 1 ? atoi(argv[1]) : 200;
  std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
  int bad = 0;
  for (int k = 0; k < cases; ++k) {
    std::map<long, double> h;
    const int nb = 1 + (int)(rng() % 24);
    const long span = 1L << (4 + rng() % 26);  // keys up to 2^29: walks of up to a few 10^8 steps
    for (int b = 0; b < nb; ++b) {
      long key = (long)(rng() % (uint64_t)span);
      if (rng() % 3 == 0) key = 1L << (rng() % 29);  // powers of two, as the log2 bins are
      double v = (double)(1 + rng() % 1000000);
      if (rng() % 4 == 0) v = std::ldexp((double)(1 + rng() % 1000), -(int)(rng() % 20));  // fractional (CRI outputs)
      h[key] += v;
    }
    if (rng() % 2) h[-1] += (double)(rng() % 100000);
    std::vector<pluss_kv> in;
    for (auto& kv : h) in.push_back(pluss_kv{kv.first, kv.second});
    const std::vector<pluss_kv> want = aet_stepping(h);
    std::vector<pluss_kv> got(want.size() + 1);
    uint64_t n = 0;
    const int rc = pluss_aet(in.data(), in.size(), got.data(), got.size(), &n);
    bool ok = rc == 0 && n == want.size();
    for (uint64_t i = 0; ok && i < n; ++i)
      ok = got[i].key == want[i].key && std::memcmp(&got[i].value, &want[i].value, sizeof(double)) == 0;
    if (!ok) {
      ++bad;
      std::printf("MISMATCH case %d (%zu keys, %zu points, got %llu)\n", k, h.size(), want.size(),
                  (unsigned long long)n);
    }
  }
  std::printf("%s %d cases\n", bad ? "FAIL" : "ok", cases);
  return bad ? 1 : 0;
}
