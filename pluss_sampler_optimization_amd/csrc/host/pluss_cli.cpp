// pluss_cli — the reference's drivers on top of the two C ABIs.
//
//   pluss_cli acc    [opts]   full trace + CRI + AET + prints   (seq main `acc`, …-ri-omp-seq.cpp:336-350)
//   pluss_cli speed  [opts]   10 timed full-trace runs           (seq main `speed`, :351-360)
//   pluss_cli sample [opts]   six r10 samplers + merge + AET     (r10 main, r10:3191-3293)
//   pluss_cli replay FILE     like `sample`, on a given list of "SAMPLE <REF> c0 c1 [c2]" lines
//
// opts: --n N --threads T --chunk CS --ds DS --cls CLS --seed S --total K --device D
//       --trace FILE  (sample / replay) one line per sample: "ref c0 c1 c2 ri sink_key"
//                     (the RI and sink the reference derives at r10:333/558; ri -1 = cold)
//       --json FILE   the same results as one machine-readable JSON object
// Output formats are the reference's (_pluss_histogram_print, pluss_print_mrc).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/pluss_gpu.h"
#include "../../../include/pluss_host.h"

namespace {

const char* REFNAME[6] = {"C0", "C1", "A0", "B0", "C2", "C3"};
const int PRINT_ORDER[6] = {PLUSS_C3, PLUSS_C2, PLUSS_A0, PLUSS_C0, PLUSS_B0, PLUSS_C1};  // r10:3280-3285

void die(const char* what, int rc) {
  std::cerr << what << " failed (" << rc << "): " << pluss_last_error() << "\n";
  std::exit(1);
}

std::string text_hist(const char* title, const std::vector<pluss_kv>& h) {
  uint64_t len = 0;
  pluss_format_hist(title, h.data(), h.size(), nullptr, 0, &len);
  std::string s(len + 1, '\0');
  pluss_format_hist(title, h.data(), h.size(), &s[0], len + 1, &len);
  s.resize(len);
  return s;
}

std::string text_mrc(const std::vector<pluss_kv>& m) {
  uint64_t len = 0;
  pluss_format_mrc(m.data(), m.size(), nullptr, 0, &len);
  std::string s(len + 1, '\0');
  pluss_format_mrc(m.data(), m.size(), &s[0], len + 1, &len);
  s.resize(len);
  return s;
}

template <typename F, typename... A>
std::vector<pluss_kv> call_kv(F fn, A... args) {
  std::vector<pluss_kv> out(1 << 16);
  uint64_t n = 0;
  int rc = fn(args..., out.data(), out.size(), &n);
  if (rc == PLUSS_ERR_CAPACITY) {
    out.resize(n);
    rc = fn(args..., out.data(), out.size(), &n);
  }
  if (rc) die("host pipeline", rc);
  out.resize(n);
  return out;
}

std::vector<pluss_hist_entry> fetch(pluss_hist& h, std::vector<pluss_hist_entry>& buf) {
  return std::vector<pluss_hist_entry>(buf.begin(), buf.begin() + h.n_entries);
}

struct Opts {
  pluss_cfg cfg{128, 4, 4, 8, 64, PLUSS_MODE_CLEAN, PLUSS_THR_R10, 0, 0};
  uint64_t seed = 0x5EED0001;
  uint64_t total = 0;  // 0: the reference's counts (164 / 2098 at any N)
  std::string trace, json;
};

Opts parse(int argc, char** argv, int first) {
  Opts o;
  for (int i = first; i + 1 < argc; i += 2) {
    std::string k = argv[i];
    if (k == "--trace") {
      o.trace = argv[i + 1];
      continue;
    }
    if (k == "--json") {
      o.json = argv[i + 1];
      continue;
    }
    long long v = std::strtoll(argv[i + 1], nullptr, 0);
    if (k == "--n") o.cfg.n = v;
    else if (k == "--threads") o.cfg.threads = v;
    else if (k == "--chunk") o.cfg.chunk = v;
    else if (k == "--ds") o.cfg.ds = v;
    else if (k == "--cls") o.cfg.cls = v;
    else if (k == "--seed") o.seed = (uint64_t)v;
    else if (k == "--total") o.total = (uint64_t)v;
    else if (k == "--device") o.cfg.device = (int32_t)v;
  }
  return o;
}

// ---- machine-readable output: {"histograms": {name: [[key, value], ...]}, "mrc": [[c, mr], ...], ...}
std::string json_kv(const std::vector<pluss_kv>& v) {
  std::ostringstream o;
  o.precision(17);
  o << "[";
  for (size_t i = 0; i < v.size(); ++i) o << (i ? ", " : "") << "[" << v[i].key << ", " << v[i].value << "]";
  o << "]";
  return o.str();
}

void write_json(const std::string& path, const Opts& o, const char* mode,
                const std::vector<std::pair<std::string, std::vector<pluss_kv>>>& hists, const std::vector<pluss_kv>& mrc,
                const std::vector<uint64_t>& traversed, double seconds) {
  std::ofstream f(path);
  if (!f) {
    std::cerr << "cannot write " << path << "\n";
    std::exit(1);
  }
  f.precision(17);
  // sampler: which semantics the histograms follow (acc: the full trace; sample/replay: r10's
  // queue semantics -- samples after its Q1 exit are not recorded, colds count for tid 0 only)
  const bool full = std::string(mode) == "acc";
  f << "{\"mode\": \"" << mode << "\", \"sampler\": \"" << (full ? "full trace" : "faithful (r10 queue semantics)")
    << "\", \"n\": " << o.cfg.n << ", \"threads\": " << o.cfg.threads
    << ", \"chunk\": " << o.cfg.chunk << ", \"ds\": " << o.cfg.ds << ", \"cls\": " << o.cfg.cls
    << ", \"seconds\": " << seconds << ",\n \"histograms\": {";
  for (size_t i = 0; i < hists.size(); ++i)
    f << (i ? ",\n  " : "\n  ") << "\"" << hists[i].first << "\": " << json_kv(hists[i].second);
  f << "},\n \"mrc\": " << json_kv(mrc) << ",\n \"traversed\": [";
  for (size_t i = 0; i < traversed.size(); ++i) f << (i ? ", " : "") << traversed[i];
  f << "]}\n";
}

// per-sample RI / sink dump (--trace)
void write_trace(const std::string& path, const pluss_cfg& cfg, const std::vector<uint64_t>& samples) {
  pluss_cfg c = cfg;
  c.mode = PLUSS_MODE_CLEAN;
  std::vector<int64_t> ri(samples.size());
  std::vector<uint64_t> sink(samples.size());
  if (!samples.empty())
    if (int rc = pluss_gemm_sampled_ri(&c, samples.data(), samples.size(), ri.data(), sink.data()))
      die("pluss_gemm_sampled_ri", rc);
  std::ofstream f(path);
  if (!f) {
    std::cerr << "cannot write " << path << "\n";
    std::exit(1);
  }
  // The RI of each sample is its own next reuse (clean mode).  In a faithful
  // (r10) run the histograms leave out the samples after r10's Q1 exit and
  // count cold samples of tid 0 only, so the trace says so in its header.
  if (cfg.mode == PLUSS_MODE_FAITHFUL)
    f << "# ref c0 c1 c2 ri sink_key: per-sample reuse (clean); the faithful histograms skip samples after r10's "
         "Q1 exit and count cold samples of tid 0 only\n";
  const uint64_t M = (1ull << 20) - 1;
  for (size_t i = 0; i < samples.size(); ++i) {
    const uint64_t x = samples[i];
    f << REFNAME[(x >> 60) & 7] << " " << ((x >> 40) & M) << " " << ((x >> 20) & M) << " " << (x & M) << " " << ri[i]
      << " " << (int64_t)sink[i] << "\n";
  }
}

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// full trace: seq sampler() + pluss_cri_distribute(THREAD_NUM) [+ AET]
std::vector<pluss_hist_entry> fulltrace(pluss_cfg cfg, uint64_t* traversed) {
  cfg.thr_variant = PLUSS_THR_V1;  // seq.cpp:203
  std::vector<pluss_hist_entry> buf(1 << 14);
  pluss_hist h{buf.data(), buf.size(), 0, {0}};
  if (int rc = pluss_gemm_fulltrace_hist(&cfg, &h)) die("pluss_gemm_fulltrace_hist", rc);
  *traversed = h.traversed[0];
  return fetch(h, buf);
}

int run_acc(const Opts& o) {
  const double t0 = now();
  uint64_t trav = 0;
  auto raw = fulltrace(o.cfg, &trav);
  auto rih = call_kv(pluss_cri_v1, (int64_t)o.cfg.threads, raw.data(), (uint64_t)raw.size());
  auto mrc = call_kv(pluss_aet, rih.data(), (uint64_t)rih.size());
  const double t1 = now();
  std::map<long, double> ns, sh;
  for (auto& e : raw) {
    if (e.kind) sh[(long)e.ri] += (double)e.count;
    else {
      long k = (long)e.ri;
      if (k > 0) {  // pluss_cri_noshare_histogram_update bins floor-log2 (pluss_utils.h:924-927)
        long x = k;
        x |= x >> 1; x |= x >> 2; x |= x >> 4; x |= x >> 8; x |= x >> 16; x |= x >> 32;
        k = x ^ (x >> 1);
      }
      ns[k] += (double)e.count;
    }
  }
  std::vector<pluss_kv> vns, vsh;
  for (auto& kv : ns) vns.push_back({kv.first, kv.second});
  for (auto& kv : sh) vsh.push_back({kv.first, kv.second});
  std::cout << "MI355X: " << (t1 - t0) << "\n";
  std::cout << text_hist("Start to dump noshare private reuse time", vns);
  std::cout << text_hist("Start to dump share private reuse time", vsh);
  std::cout << text_hist("Start to dump reuse time", rih);
  std::cout << text_mrc(mrc);
  std::cout << "max iteration traversed\n" << trav << "\n\n";
  if (!o.json.empty())
    write_json(o.json, o, "acc", {{"noshare", vns}, {"share", vsh}, {"reuse", rih}}, mrc, {trav}, t1 - t0);
  return 0;
}

int run_speed(const Opts& o) {
  std::cout << "MI355X:\n";
  for (int i = 0; i < 10; ++i) {
    const double t0 = now();
    uint64_t trav = 0;
    auto raw = fulltrace(o.cfg, &trav);
    auto rih = call_kv(pluss_cri_v1, (int64_t)o.cfg.threads, raw.data(), (uint64_t)raw.size());
    (void)rih;
    std::cout << (now() - t0) << "\n";
  }
  std::cout << "\n";
  return 0;
}

int run_samplers(const Opts& o, const std::vector<uint64_t>* given) {
  pluss_cfg cfg = o.cfg;
  cfg.mode = PLUSS_MODE_FAITHFUL;
  std::vector<uint64_t> samples;
  if (given) {
    samples = *given;
  } else {
    uint64_t counts[6];
    if (o.total) {
      if (int rc = pluss_default_counts(cfg.n, o.total, counts)) die("pluss_default_counts", rc);
    } else {
      for (int r = 0; r < 6; ++r) counts[r] = (r == PLUSS_C0 || r == PLUSS_C1) ? 164 : 2098;  // r10:156,1688
    }
    for (int r = 0; r < 6; ++r) {
      std::vector<uint64_t> s(counts[r]);
      if (int rc = pluss_expand_samples(&cfg, o.seed, r, 0, counts[r], s.data())) die("pluss_expand_samples", rc);
      samples.insert(samples.end(), s.begin(), s.end());
    }
  }
  const double t0 = now();
  std::vector<pluss_hist_entry> buf(1 << 16);
  pluss_hist h{buf.data(), buf.size(), 0, {0}};
  if (int rc = pluss_gemm_sampled_hist(&cfg, samples.data(), samples.size(), &h)) die("pluss_gemm_sampled_hist", rc);
  auto raw = fetch(h, buf);
  // r10's host half in one call: the six CRI steps on host threads, the merge, AET, the MRC text
  uint64_t nr = 0, nm = 0, nt = 0;
  if (int rc = pluss_r10_host_pipeline(cfg.threads, &h, 0, nullptr, 0, &nr, nullptr, 0, &nm, nullptr, 0, &nt))
    die("pluss_r10_host_pipeline", rc);
  std::vector<pluss_kv> rih(nr ? nr : 1), mrc(nm ? nm : 1);
  std::string mrc_txt(nt + 1, '\0');
  if (int rc = pluss_r10_host_pipeline(cfg.threads, &h, 0, rih.data(), rih.size(), &nr, mrc.data(), mrc.size(), &nm,
                                       &mrc_txt[0], nt + 1, &nt))
    die("pluss_r10_host_pipeline", rc);
  rih.resize(nr);
  mrc.resize(nm);
  mrc_txt.resize(nt);
  std::cout << (now() - t0) << "\n";
  std::vector<std::vector<pluss_kv>> per(6);  // each sampler_<REF>'s output, for its printout
  for (int r = 0; r < 6; ++r) {
    std::vector<pluss_hist_entry> mine;
    for (auto& e : raw)
      if (e.ref == r) mine.push_back(e);
    if (!mine.empty()) per[r] = call_kv(pluss_cri_r10, (int64_t)cfg.threads, mine.data(), (uint64_t)mine.size());
  }
  for (int r : PRINT_ORDER) std::cout << text_hist(REFNAME[r], per[r]);
  std::cout << text_hist("Start to dump reuse time", rih);
  std::cout << mrc_txt;
  uint64_t mx = 0;
  for (int r = 0; r < 6; ++r) mx = h.traversed[r] > mx ? h.traversed[r] : mx;
  std::cout << "max iteration traversed\n" << mx << "\n";
  const double t1 = now();
  if (!o.json.empty()) {
    std::vector<std::pair<std::string, std::vector<pluss_kv>>> hs;
    for (int r = 0; r < 6; ++r) hs.push_back({REFNAME[r], per[r]});
    hs.push_back({"reuse", rih});
    write_json(o.json, o, given ? "replay" : "sample", hs, mrc, std::vector<uint64_t>(h.traversed, h.traversed + 6),
               t1 - t0);
  }
  if (!o.trace.empty()) write_trace(o.trace, cfg, samples);
  return 0;
}

std::vector<uint64_t> read_samples(const char* path) {
  std::ifstream f(path);
  if (!f) {
    std::cerr << "cannot open " << path << "\n";
    std::exit(1);
  }
  std::vector<uint64_t> out;
  std::string tag, ref;
  while (f >> tag) {
    if (tag != "SAMPLE") {
      std::string rest;
      std::getline(f, rest);
      continue;
    }
    std::string line;
    std::getline(f, line);
    std::istringstream is(line);
    is >> ref;
    uint64_t c[3] = {0, 0, 0};
    for (int i = 0; i < 3 && (is >> c[i]); ++i) {
    }
    int r = -1;
    for (int k = 0; k < 6; ++k)
      if (ref == REFNAME[k]) r = k;
    if (r < 0) continue;
    out.push_back(((uint64_t)r << 60) | (c[0] << 40) | (c[1] << 20) | c[2]);
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::cerr << "usage: pluss_cli acc|speed|sample [--n N --threads T ...] | replay FILE [opts]\n";
    return 2;
  }
  const std::string mode = argv[1];
  if (mode == "acc") return run_acc(parse(argc, argv, 2));
  if (mode == "speed") return run_speed(parse(argc, argv, 2));
  if (mode == "sample") return run_samplers(parse(argc, argv, 2), nullptr);
  if (mode == "replay" && argc >= 3) {
    auto s = read_samples(argv[2]);
    return run_samplers(parse(argc, argv, 3), &s);
  }
  std::cerr << "unknown mode " << mode << "\n";
  return 2;
}
