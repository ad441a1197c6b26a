// Probe (diagnostics, not product): rocPRIM radix sort of one reference's
// worth of 32-bit faithful-mode words (4,189,071 at config 2) on gfx950,
// default config vs onesweep digit widths / tile shapes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <rocprim/device/device_radix_sort.hpp>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);          \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <class Cfg>
int run(const char* name, uint32_t* in, uint32_t* out, size_t n, unsigned end_bit) {
  size_t tmp = 0;
  CK(rocprim::radix_sort_keys<Cfg>(nullptr, tmp, in, out, n, 0, end_bit, 0));
  void* t = nullptr;
  CK(hipMalloc(&t, tmp));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) CK(rocprim::radix_sort_keys<Cfg>(t, tmp, in, out, n, 0, end_bit, 0));
  CK(hipEventRecord(a, 0));
  const int R = 20;
  for (int r = 0; r < R; ++r) CK(rocprim::radix_sort_keys<Cfg>(t, tmp, in, out, n, 0, end_bit, 0));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  std::vector<uint32_t> h(n);
  CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
  const uint32_t mask = end_bit >= 32 ? ~0u : ((1u << end_bit) - 1);
  bool ok = true;
  for (size_t i = 1; i < n; ++i)
    if ((h[i - 1] & mask) > (h[i] & mask)) {
      ok = false;
      break;
    }
  printf("{\"cfg\": \"%s\", \"n\": %zu, \"end_bit\": %u, \"us\": %.2f, \"sorted\": %d}\n", name, n, end_bit,
         ms * 1000 / R, ok);
  fflush(stdout);
  CK(hipFree(t));
  return 0;
}

using namespace rocprim;
template <int HB, int HI, int SB, int SI, int BITS>
using OS = radix_sort_config<default_config, default_config,
                             radix_sort_onesweep_config<kernel_config<HB, HI>, kernel_config<SB, SI>, BITS,
                                                                        block_radix_rank_algorithm::match>>;

int main() {
  const size_t n = 4189071;
  std::vector<uint32_t> h(n);
  std::mt19937 g(1);
  for (auto& x : h) x = g();
  uint32_t *in, *out;
  CK(hipMalloc(&in, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice));
  run<default_config>("default", in, out, n, 32);
  run<default_config>("default_30bit", in, out, n, 30);
  run<OS<256, 12, 256, 12, 11>>("os11_256x12", in, out, n, 32);
  run<OS<512, 16, 512, 16, 11>>("os11_512x16", in, out, n, 32);
  run<OS<1024, 32, 1024, 12, 8>>("os8_1024x12", in, out, n, 32);
  run<OS<1024, 32, 1024, 16, 8>>("os8_1024x16", in, out, n, 32);
  run<OS<512, 16, 512, 16, 10>>("os10_512x16_30bit", in, out, n, 30);
  return 0;
}
