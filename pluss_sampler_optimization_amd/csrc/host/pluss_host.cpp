// pluss_host.cpp — CRI distribution, AET and text formats (include/pluss_host.h).
//
// Host-only by design: these functions run once per sampler over histograms
// of a few thousand bins.  They follow the reference line for line in what they
// compute (including its quirks), but iterate ordered
// maps where the reference iterates unordered ones, so floating-point sums may
// differ from a given libstdc++ build in the last ulp.
#include "../../../include/pluss_host.h"

#include <cmath>
#include <cstring>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

using Hist = std::map<long, double>;

// log |Gamma(x)| without touching glibc's global `signgam` (std::lgamma writes
// it: a data race when two threads run the pipeline, found by the TSan build
// in tests/test_sanitizers.py)
double lgam(double x) {
  int sign = 0;
  return ::lgamma_r(x, &sign);
}

// gsl_ran_negative_binomial_pdf(k, p, n) (GSL randist/nbinomial.c form)
double nbd_pdf(unsigned int k, double p, double n) {
  const double f = lgam((double)k + n), a = lgam(n), b = lgam((double)k + 1.0);
  return std::exp(f - a - b + n * std::log(p) + (double)k * std::log1p(-p));
}

long floor_pow2(long x) {  // _polybench_to_highest_power_of_two (pluss_utils.h:665-679)
  x |= x >> 1; x |= x >> 2; x |= x >> 4; x |= x >> 8; x |= x >> 16; x |= x >> 32;
  return x ^ (x >> 1);
}

void add(Hist& h, long k, double c) { h[k] += c; }
void add_log(Hist& h, long k, double c) { add(h, k > 0 ? floor_pow2(k) : k, c); }  // pluss_histogram_update

// r10 simulate_negative_binomial (r10:42-64).  `thread_cnt` is an int: the
// share path passes 1.0/THREAD_NUM, which truncates to 0 (Q5).
void nbd_r10(int thread_cnt, long threads_macro, long n, std::vector<std::pair<long, double>>& dist) {
  const double p = 1.0 / thread_cnt;
  if (n >= (4000. * (thread_cnt - 1)) / thread_cnt) {
    const int i = (int)std::log2((double)n);
    const long bin = (long)std::pow(2.0, i);
    dist.emplace_back(threads_macro * bin, 1.0);
    return;
  }
  uint64_t k = 0;
  double prob_sum = 0.0;
  while (true) {
    const double pr = nbd_pdf((unsigned int)k, p, (double)n);
    prob_sum += pr;
    dist.emplace_back((long)(k + n), pr);
    if (prob_sum > 0.999) break;
    k += 1;
  }
}

// v1 _pluss_cri_nbd (pluss_utils.h:987-1009)
void nbd_v1(int thread_cnt, long threads_macro, long n, std::vector<std::pair<long, double>>& dist) {
  const double p = 1.0 / thread_cnt;
  if (n >= (4000. * (thread_cnt - 1)) / thread_cnt) {
    dist.emplace_back(threads_macro * n, 1.0);
    return;
  }
  long k = 0;
  double prob_sum = 0.0;
  while (true) {
    const double pr = nbd_pdf((unsigned int)k, p, (double)n);
    prob_sum += pr;
    dist.emplace_back(k + n, pr);
    if (prob_sum > 0.9999) break;
    k += 1;
  }
}

// racetrack split of one (ri, count) over power-of-two bins (r10:101-123 with
// exponent n-1; pluss_utils.h:1076-1098 with exponent n).
template <typename AddFn>
void racetrack(long ri, double cnt, double expo, AddFn addfn) {
  std::map<int, double> prob;
  double prob_sum = 0.0;
  int i = 1;
  while (true) {
    if (std::pow(2.0, (double)i) > ri) break;
    prob[i] = std::pow(1 - (std::pow(2.0, (double)i - 1) / ri), expo) - std::pow(1 - (std::pow(2.0, (double)i) / ri), expo);
    prob_sum += prob[i];
    i++;
    if (prob_sum == 1.0) break;
  }
  if (prob_sum != 1.0) prob[i - 1] = 1 - prob_sum;
  for (auto& b : prob) addfn((long)std::pow(2.0, b.first - 1), b.second * cnt);
}

int emit(const Hist& h, pluss_kv* out, uint64_t cap, uint64_t* n_out) {
  if (n_out) *n_out = h.size();
  if (h.size() > cap) return PLUSS_ERR_CAPACITY;
  uint64_t i = 0;
  for (auto& kv : h) {
    out[i].key = kv.first;
    out[i].value = kv.second;
    ++i;
  }
  return PLUSS_OK;
}

int emit_text(const std::string& s, char* buf, uint64_t cap, uint64_t* len) {
  if (len) *len = s.size();
  if (!buf || cap == 0) return s.empty() ? PLUSS_OK : PLUSS_ERR_CAPACITY;
  if (s.size() + 1 > cap) {
    std::memcpy(buf, s.data(), cap - 1);
    buf[cap - 1] = 0;
    return PLUSS_ERR_CAPACITY;
  }
  std::memcpy(buf, s.data(), s.size() + 1);
  return PLUSS_OK;
}


// pluss_AET (pluss_utils.h:758-804), the reference's walk of t with its
// additions in its order; the points go straight to the output array (one per
// cache size c = 0..min(max RI, 327680), in c order: no map of 327,681 points).
int aet_impl(const pluss_kv* hist, uint64_t n, pluss_kv* mrc, uint64_t cap, uint64_t* n_out) {
  if (n && !hist) return PLUSS_ERR_CONFIG;
  Hist h;
  double total = 0;
  long max_rt = 0;
  for (uint64_t i = 0; i < n; ++i) {
    total += hist[i].value;
    h[(long)hist[i].key] += hist[i].value;
    if (max_rt < hist[i].key) max_rt = (long)hist[i].key;
  }
  std::map<uint64_t, double> P;
  double acc = 0.;
  auto m1 = h.find(-1);
  if (m1 != h.end()) acc = m1->second;
  for (auto it = h.rbegin(); it != h.rend(); ++it) {
    if (it->first == -1) break;
    P[(uint64_t)it->first] = acc / total;
    acc += it->second;
  }
  P[0] = 1.0;
  // walk t = 0..max_rt like the reference (same additions, same order)
  std::vector<std::pair<uint64_t, double>> pv(P.begin(), P.end());
  size_t pi = 0;
  double sum_p = 0, pred = -1.0, cur = pv[0].second;
  uint64_t t = 0;
  const uint64_t cs = 2560 * 1024 / sizeof(double);
  const uint64_t top = (uint64_t)max_rt < cs ? (uint64_t)max_rt : cs;  // c = 0..top
  const uint64_t nout = max_rt >= 0 ? top + 1 : 0;
  if (n_out) *n_out = nout;
  if (nout > cap) return PLUSS_ERR_CAPACITY;
  uint64_t k = 0;
  for (uint64_t c = 0; c <= (uint64_t)max_rt && c <= cs; c++) {
    while (sum_p < (double)c && t <= (uint64_t)max_rt) {
      while (pi < pv.size() && pv[pi].first < t) ++pi;
      if (pi < pv.size() && pv[pi].first == t) {
        sum_p += pv[pi].second;
        cur = pv[pi].second;
        t++;
      } else {
        sum_p += cur;
        t++;
      }
    }
    if (pred != -1.0 || pred - cur < 0.0001) {  // (the reference's test: every c is written)
      if (pred == -1.0) pred = cur;
      mrc[k].key = (int64_t)c;
      mrc[k].value = cur;
      ++k;
    }
  }
  if (n_out) *n_out = k;
  return PLUSS_OK;
}

}  // namespace

extern "C" {

int pluss_cri_r10(int64_t threads, const pluss_hist_entry* raw, uint64_t n, pluss_kv* out, uint64_t cap,
                  uint64_t* n_out) {
  if (threads < 1 || (n && !raw)) return PLUSS_ERR_CONFIG;
  Hist noshare, share;
  for (uint64_t i = 0; i < n; ++i) (raw[i].kind ? share : noshare)[(long)raw[i].ri] += (double)raw[i].count;
  Hist target;
  std::vector<std::pair<long, double>> dist;
  // no_share_distribute (r10:65-84)
  for (auto& e : noshare) {
    if (e.first < 0) {
      add(target, e.first, e.second);
      continue;
    }
    if (threads > 1) {
      dist.clear();
      nbd_r10((int)threads, threads, e.first, dist);
      for (auto& d : dist) add(target, d.first, e.second * d.second);
    } else {
      add(target, e.first, e.second);
    }
  }
  // share_distribute (r10:85-131); share ratio n = THREAD_NUM-1 (r10:2483)
  const double nratio = (double)(threads - 1);
  for (auto& e : share) {
    if (threads > 1) {
      dist.clear();
      nbd_r10((int)(1.0 / threads), threads, e.first, dist);
      for (auto& d : dist)
        racetrack(d.first, e.second * d.second, nratio - 1, [&](long k, double v) { add(target, k, v); });
    } else {
      add(target, e.first, e.second);
    }
  }
  return emit(target, out, cap, n_out);
}

int pluss_cri_v1(int64_t threads, const pluss_hist_entry* raw, uint64_t n, pluss_kv* out, uint64_t cap,
                 uint64_t* n_out) {
  if (threads < 1 || (n && !raw)) return PLUSS_ERR_CONFIG;
  Hist noshare, share;
  for (uint64_t i = 0; i < n; ++i) {
    const long ri = (long)raw[i].ri;
    if (raw[i].kind) share[ri] += (double)raw[i].count;                          // raw (pluss_utils.h:928-937)
    else noshare[ri > 0 ? floor_pow2(ri) : ri] += (double)raw[i].count;           // binned at record (:924-927)
  }
  Hist rih;
  std::vector<std::pair<long, double>> dist;
  for (auto& e : noshare) {  // _pluss_cri_noshare_distribute (:1010-1039)
    if (e.first < 0) {
      add_log(rih, e.first, e.second);
      continue;
    }
    if (threads > 1) {
      dist.clear();
      nbd_v1((int)threads, threads, e.first, dist);
      for (auto& d : dist) add_log(rih, d.first, e.second * d.second);
    } else {
      add_log(rih, e.first, e.second);
    }
  }
  const double nratio = (double)(threads - 1);  // _pluss_cri_racetrack (:1040-1131)
  for (auto& e : share) {
    if (threads > 1) {
      dist.clear();
      nbd_v1((int)threads, threads, e.first, dist);
      for (auto& d : dist)
        racetrack(d.first, e.second * d.second, nratio, [&](long k, double v) { add_log(rih, k, v); });
    } else {
      add_log(rih, e.first, e.second);
    }
  }
  return emit(rih, out, cap, n_out);
}

int pluss_log2_merge(const pluss_kv* in, uint64_t n, pluss_kv* out, uint64_t cap, uint64_t* n_out) {
  if (n && !in) return PLUSS_ERR_CONFIG;
  Hist h;
  for (uint64_t i = 0; i < n; ++i) add_log(h, (long)in[i].key, in[i].value);
  return emit(h, out, cap, n_out);
}

int pluss_aet(const pluss_kv* hist, uint64_t n, pluss_kv* mrc, uint64_t cap, uint64_t* n_out) {
  return aet_impl(hist, n, mrc, cap, n_out);
}

int pluss_format_hist(const char* title, const pluss_kv* hist, uint64_t n, char* buf, uint64_t cap, uint64_t* len) {
  // _pluss_histogram_print (pluss_utils.h:690-702)
  std::ostringstream os;
  os << (title ? title : "") << "\n";
  double sum = 0.;
  Hist tmp;
  for (uint64_t i = 0; i < n; ++i) {
    sum += hist[i].value;
    tmp[(long)hist[i].key] = hist[i].value;
  }
  for (auto& kv : tmp) os << kv.first << "," << kv.second << "," << kv.second / sum << "\n";
  return emit_text(os.str(), buf, cap, len);
}

int pluss_format_mrc(const pluss_kv* mrc, uint64_t n, char* buf, uint64_t cap, uint64_t* len) {
  // pluss_print_mrc (pluss_utils.h:851-883): plateaus printed as first/last point.
  // The points in key order (pluss_aet's output already is: no map needed).
  std::vector<std::pair<uint64_t, double>> m;
  m.reserve(n);
  bool sorted = true;
  for (uint64_t i = 0; i < n; ++i) {
    if (i && (uint64_t)mrc[i].key <= (uint64_t)mrc[i - 1].key) sorted = false;
    m.emplace_back((uint64_t)mrc[i].key, mrc[i].value);
  }
  if (!sorted) {
    std::map<uint64_t, double> mm;
    for (uint64_t i = 0; i < n; ++i) mm[(uint64_t)mrc[i].key] = mrc[i].value;
    m.assign(mm.begin(), mm.end());
  }
  std::ostringstream os;
  os << "miss ratio\n";
  size_t i1 = 0, i2 = 0;
  while (i1 < m.size()) {
    while (i2 + 1 < m.size() && m[i1].second - m[i2 + 1].second < 0.00001) ++i2;
    os << m[i1].first << ", " << m[i1].second << "\n";
    if (i1 != i2) os << m[i2].first << ", " << m[i2].second << "\n";
    i1 = ++i2;
  }
  return emit_text(os.str(), buf, cap, len);
}

}  // extern "C"
