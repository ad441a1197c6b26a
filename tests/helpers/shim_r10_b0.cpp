// INTEGRATION.md §2, compiled: the reference's r10 entry point
//   void sampler_B0(std::unordered_map<long, double>& histogram)
//   (c_lib/test/sampler/gemm-t4-pluss-pro-model-rs-ri-opt-r10.cpp:2221)
// with its body replaced by calls into libpluss_gpu (faithful raw histogram)
// and libpluss_host (r10's no_share_distribute + share_distribute).  The
// driver replays a reference sample list (one "c0 c1 c2" line per sample) and
// prints the histogram the way r10's main prints a reference's result
// (title, then "ri,count,fraction" rows: _pluss_histogram_print), plus the
// traversed count.  Test-only (tests/test_integration_shim.py).
#include <cstdio>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "pluss_gpu.h"
#include "pluss_host.h"

static int64_t N = 128, THREAD_NUM = 4;
static const int64_t CHUNK_SIZE = 4, DS = 8, CLS = 64;
static std::vector<uint64_t> g_samples;                 // the replayed B0 samples (packed)
static std::map<std::string, long> iteration_traversed_map;  // r10's per-reference traversed counts
static int g_rc = 0;

void sampler_B0(std::unordered_map<long, double>& histogram) {
  pluss_cfg cfg = {N, THREAD_NUM, CHUNK_SIZE, DS, CLS, PLUSS_MODE_FAITHFUL, PLUSS_THR_R10, 0, 0};
  std::vector<pluss_hist_entry> raw(1 << 14);
  pluss_hist h = {raw.data(), raw.size(), 0, {0}};
  if ((g_rc = pluss_gemm_sampled_hist(&cfg, g_samples.data(), g_samples.size(), &h))) {
    std::fprintf(stderr, "pluss_gemm_sampled_hist: %s\n", pluss_last_error());
    return;
  }
  std::vector<pluss_kv> out(1 << 16);
  uint64_t n = 0;
  if ((g_rc = pluss_cri_r10(THREAD_NUM, raw.data(), h.n_entries, out.data(), out.size(), &n))) return;
  for (uint64_t i = 0; i < n; ++i) histogram[out[i].key] += out[i].value;
  iteration_traversed_map["B0"] = (long)h.traversed[PLUSS_B0];
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s N THREADS samples.txt\n", argv[0]);
    return 2;
  }
  N = std::stoll(argv[1]);
  THREAD_NUM = std::stoll(argv[2]);
  FILE* f = std::fopen(argv[3], "r");
  if (!f) return 2;
  unsigned long long c0, c1, c2;
  while (std::fscanf(f, "%llu %llu %llu", &c0, &c1, &c2) == 3)
    g_samples.push_back(((uint64_t)PLUSS_B0 << 60) | (c0 << 40) | (c1 << 20) | c2);
  std::fclose(f);
  std::unordered_map<long, double> histogram;
  sampler_B0(histogram);
  if (g_rc) return 1;
  std::vector<pluss_kv> kv;
  for (auto& e : histogram) kv.push_back(pluss_kv{e.first, e.second});
  std::vector<char> text(1 << 20);
  uint64_t len = 0;
  if (pluss_format_hist("B0", kv.data(), kv.size(), text.data(), text.size(), &len)) return 1;
  std::fputs(text.data(), stdout);
  std::printf("traversed %ld\n", iteration_traversed_map["B0"]);
  return 0;
}
