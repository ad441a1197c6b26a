// pluss_host.cpp — CRI distribution, AET and text formats (include/pluss_host.h).
//
// Host-only by design: these functions run once per sampler over histograms
// of a few thousand bins.  They follow the reference line for line in what they
// compute (including its quirks), but iterate ordered
// maps where the reference iterates unordered ones, so floating-point sums may
// differ from a given libstdc++ build in the last ulp.
#include "../../../include/pluss_host.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <sstream>
#include <string>
#include <thread>
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


// s after n repeated additions s = fl(s + d), exactly as the additions one by
// one leave it.  While s stays inside one binade [2^(e-1), 2^e), adding d adds
// the same whole number of ulps each time: round(d / ulp), or, when d / ulp
// ends in exactly one half (a tie, rounded to the even neighbour), the even
// choice once s is even -- after one addition it always is.  Runs of such
// additions are taken in one jump (integer arithmetic in ulps); every other
// addition (from s == 0, the first of a tie, the ones near the binade's end,
// the last few) is made as the walk makes it.
double advance(double s, const double d, uint64_t n) {
  constexpr uint64_t TOP = (1ull << 53) - 2;
  while (n) {
    if (n <= 4 || !(s > 0.0) || !(d > 0.0)) {
      s += d;
      --n;
      continue;
    }
    int e = 0;
    (void)std::frexp(s, &e);
    const double u = std::ldexp(1.0, e - 53);  // ulp(s)
    const double q = d / u;                    // (exact: scaling by a power of two)
    if (q >= 4.0e15) {  // an increment about as large as the binade: one by one
      s += d;
      --n;
      continue;
    }
    const uint64_t k = (uint64_t)(s / u);
    const double qf = std::floor(q), f = q - qf;
    const uint64_t qi = (uint64_t)qf;
    uint64_t st;
    if (f == 0.5) {
      if (k & 1) {  // the first addition of a tie makes s even
        s += d;
        --n;
        continue;
      }
      st = qi + (qi & 1);
    } else {
      st = qi + (f > 0.5 ? 1u : 0u);
    }
    if (st == 0) return s;  // fl(s + d) == s: nothing moves s out of this binade again
    const uint64_t qc = (uint64_t)std::ceil(q);
    if (k + qc + st > TOP) {  // the next addition may leave the binade
      s += d;
      --n;
      continue;
    }
    uint64_t j = (TOP - k - qc) / st;  // additions whose exact sums stay 2 ulps below the binade's end
    j = j < n ? j : n;
    s = (double)(k + j * st) * u;
    n -= j;
  }
  return s;
}

// pluss_AET (pluss_utils.h:758-804): the reference's walk of t with its
// additions in its order.  From one key of P to the next every step adds the
// same P value and leaves it as the current miss ratio, so a segment of steps
// is taken at once (advance) and every cache size c its sum passes gets that
// value -- the c the walk stops at inside the segment.  The curve comes out as
// runs of equal points [c0, c1] (one per c = 0..min(max RI, 327680) in all,
// in c order): 327,681 points are written only where a caller asks for them.
struct Run {
  uint64_t c0, c1;  // its first and last point's cache size
  double v;
};
void aet_runs(const Hist& h, std::vector<Run>& runs) {
  runs.clear();
  double total = 0;
  long max_rt = 0;
  for (auto& kv : h) {
    total += kv.second;
    if (max_rt < kv.first) max_rt = kv.first;
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
  const std::vector<std::pair<uint64_t, double>> pv(P.begin(), P.end());
  const uint64_t cs = 2560 * 1024 / sizeof(double);
  if (max_rt < 0) return;
  const uint64_t tmax = (uint64_t)max_rt;  // the walk's t <= max_RT
  const uint64_t top = tmax < cs ? tmax : cs;
  size_t seg = 0;  // pv[seg].first <= t < pv[seg + 1].first
  double sum_p = 0, cur = pv[0].second;
  uint64_t t = 0, c = 0;
  auto put = [&](uint64_t c1) {  // points c..c1 take the current value
    if (!runs.empty() && runs.back().v == cur && runs.back().c1 + 1 == c) runs.back().c1 = c1;
    else runs.push_back(Run{c, c1, cur});
    c = c1 + 1;
  };
  // (the reference writes every c: its test `pred != -1 || pred - cur < 0.0001` always holds)
  while (c <= top) {
    if (t > tmax) {  // the walk makes no more steps
      put(top);
      break;
    }
    if (sum_p >= (double)c) {  // no step for c, nor for any c up to sum_p
      const double f = std::floor(sum_p);
      put(f < (double)top ? (uint64_t)f : top);
      continue;
    }
    while (seg + 1 < pv.size() && pv[seg + 1].first <= t) ++seg;
    const uint64_t tend = seg + 1 < pv.size() && pv[seg + 1].first <= tmax ? pv[seg + 1].first : tmax + 1;
    cur = pv[seg].second;  // (at t == the key the walk adds P[t] and takes it as current; past it, the same)
    sum_p = advance(sum_p, cur, tend - t);
    t = tend;
  }
}

uint64_t run_points(const std::vector<Run>& runs) { return runs.empty() ? 0 : runs.back().c1 + 1; }

void fill_points(const std::vector<Run>& runs, pluss_kv* out) {
  for (auto& r : runs)
    for (uint64_t c = r.c0; c <= r.c1; ++c) out[c] = pluss_kv{(int64_t)c, r.v};
}

int aet_impl(const pluss_kv* hist, uint64_t n, pluss_kv* mrc, uint64_t cap, uint64_t* n_out) {
  if (n && !hist) return PLUSS_ERR_CONFIG;
  Hist h;
  for (uint64_t i = 0; i < n; ++i) h[(long)hist[i].key] += hist[i].value;
  std::vector<Run> runs;
  aet_runs(h, runs);
  const uint64_t np = run_points(runs);
  if (n_out) *n_out = np;
  if (np > cap) return PLUSS_ERR_CAPACITY;
  if (np) fill_points(runs, mrc);
  return PLUSS_OK;
}

// pluss_print_mrc (pluss_utils.h:851-883) over runs of equal points in c
// order: a plateau (points within 0.00001 of its first) extends over whole
// runs, printed as its first and last point
std::string mrc_text(const std::vector<Run>& runs) {
  std::ostringstream os;
  os << "miss ratio\n";
  size_t r1 = 0;
  while (r1 < runs.size()) {
    size_t r2 = r1;
    while (r2 + 1 < runs.size() && runs[r1].v - runs[r2 + 1].v < 0.00001) ++r2;
    const uint64_t c_first = runs[r1].c0, c_last = runs[r2].c1;
    os << c_first << ", " << runs[r1].v << "\n";
    if (c_last != c_first) os << c_last << ", " << runs[r2].v << "\n";
    r1 = r2 + 1;
  }
  return os.str();
}

// r10's per-reference CRI (no_share_distribute + share_distribute, r10:65-131)
// of the raw entries of reference `ref` (-1: every entry)
Hist cri_r10(int64_t threads, const pluss_hist_entry* raw, uint64_t n, int ref) {
  Hist noshare, share;
  for (uint64_t i = 0; i < n; ++i)
    if (ref < 0 || raw[i].ref == ref) (raw[i].kind ? share : noshare)[(long)raw[i].ri] += (double)raw[i].count;
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
  return target;
}


}  // namespace

extern "C" {

int pluss_cri_r10(int64_t threads, const pluss_hist_entry* raw, uint64_t n, pluss_kv* out, uint64_t cap,
                  uint64_t* n_out) {
  if (threads < 1 || (n && !raw)) return PLUSS_ERR_CONFIG;
  return emit(cri_r10(threads, raw, n, -1), out, cap, n_out);
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
  // pluss_print_mrc (pluss_utils.h:851-883): the points in key order
  // (pluss_aet's output already is: no map needed), as runs of equal values
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
  std::vector<Run> runs;
  for (auto& p : m) {
    if (!runs.empty() && runs.back().v == p.second) runs.back().c1 = p.first;
    else runs.push_back(Run{p.first, p.first, p.second});
  }
  return emit_text(mrc_text(runs), buf, cap, len);
}

int pluss_r10_host_pipeline(int64_t threads, const pluss_hist* raw, int32_t workers, pluss_kv* reuse,
                            uint64_t reuse_cap, uint64_t* n_reuse, pluss_kv* mrc, uint64_t mrc_cap, uint64_t* n_mrc,
                            char* text, uint64_t text_cap, uint64_t* text_len) {
  if (threads < 1 || !raw || (raw->n_entries && !raw->entries) || workers < 0) return PLUSS_ERR_CONFIG;
  // the six sampler_<REF> outputs (r10:690-691, inside r10's six sampler threads, r10:3203-3257)
  static const int ORDER[6] = {PLUSS_C3, PLUSS_C2, PLUSS_A0, PLUSS_C0, PLUSS_B0, PLUSS_C1};  // r10:3259-3276
  bool present[6] = {false, false, false, false, false, false};
  for (uint64_t i = 0; i < raw->n_entries; ++i)
    if (raw->entries[i].ref >= 0 && raw->entries[i].ref < 6) present[raw->entries[i].ref] = true;
  Hist per[6];
  auto one = [&](int r) { per[r] = cri_r10(threads, raw->entries, raw->n_entries, r); };
  std::vector<int> refs;
  for (int r : ORDER)
    if (present[r]) refs.push_back(r);
  const size_t nw = workers == 0 ? refs.size() : std::min<size_t>((size_t)workers, refs.size());
  if (nw <= 1) {
    for (int r : refs) one(r);
  } else {
    std::vector<std::thread> pool;
    for (size_t w = 0; w < nw; ++w)
      pool.emplace_back([&, w]() {
        for (size_t i = w; i < refs.size(); i += nw) one(refs[i]);
      });
    for (auto& th : pool) th.join();
  }
  // merged into the reuse histogram, floor-log2 binned, in r10's reference order
  Hist rih;
  for (int r : ORDER)
    for (auto& kv : per[r]) add_log(rih, kv.first, kv.second);
  int rc = PLUSS_OK;
  if (n_reuse || reuse) {
    uint64_t nr = 0;
    const int e = emit(rih, reuse ? reuse : nullptr, reuse ? reuse_cap : 0, &nr);
    if (n_reuse) *n_reuse = nr;
    if (reuse && e) rc = e;
  }
  std::vector<Run> runs;
  aet_runs(rih, runs);  // pluss_AET
  const uint64_t np = run_points(runs);
  if (n_mrc) *n_mrc = np;
  if (mrc) {
    if (np > mrc_cap) rc = PLUSS_ERR_CAPACITY;
    else fill_points(runs, mrc);
  }
  if (text || text_len) {  // pluss_print_mrc
    const int e = emit_text(mrc_text(runs), text, text_cap, text_len);
    if (text && e) rc = e;
  }
  return rc;
}

}  // extern "C"
