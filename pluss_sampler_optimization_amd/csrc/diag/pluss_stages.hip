// pluss_stages.hip -- the diagnostic build's stage markers (build.py
// variant "stages", -DPLUSS_DEBUG_STAGES; never part of the product library,
// which reads no environment variable).  See PLUSS_STAGE in pluss_internal.h.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../pluss_internal.h"

namespace pluss {

// Modes (environment PLUSS_STAGE_MODE): "sync" drains the stream at every
// stage and prints its outcome; "off" does nothing (the product's timing);
// otherwise ("mark") each stage enqueues a marker
// kernel that writes its sequence number into pinned host memory, with no
// host wait (the streams' timing stays close to the product's), and
// pluss_debug_stage_dump() lists which stages' markers ran -- after a device
// fault, the last stage each stream completed.
__global__ void k_stage_mark(volatile unsigned long long* slot, unsigned long long v) { *slot = v; }
static std::vector<std::pair<std::string, const void*>> g_stage_names;
static unsigned long long* g_stage_marks = nullptr;
constexpr size_t STAGE_CAP = 1 << 16;
void debug_stage(hipStream_t s, const char* what) {
  static int mode = -1;
  static const char* only = nullptr;
  if (mode < 0) {
    const char* e = std::getenv("PLUSS_STAGE_MODE");  // sync | off | mark (the default)
    mode = e && std::strcmp(e, "sync") == 0 ? 1 : e && std::strcmp(e, "off") == 0 ? 2 : 0;
    only = std::getenv("PLUSS_STAGE_ONLY");  // mark only the stages whose names contain this
  }
  if (mode == 2 || (only && !std::strstr(what, only))) return;
  if (mode == 1) {
    static unsigned long long seq = 0;
    hipError_t e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipPeekAtLastError();
    std::fprintf(stderr, "[stage %llu] %s: %s\n", ++seq, what, e == hipSuccess ? "ok" : hipGetErrorString(e));
    std::fflush(stderr);
    return;
  }
  if (!g_stage_marks) {
    if (hipHostMalloc((void**)&g_stage_marks, STAGE_CAP * 8, hipHostMallocMapped) != hipSuccess) return;
    std::memset(g_stage_marks, 0, STAGE_CAP * 8);
  }
  const size_t i = g_stage_names.size();
  if (i >= STAGE_CAP) return;
  g_stage_names.emplace_back(what, (const void*)s);
  hipLaunchKernelGGL(k_stage_mark, dim3(1), dim3(1), 0, s, g_stage_marks + i, (unsigned long long)(i + 1));
}
int debug_knob(const char* name) {
  const std::string k = std::string("PLUSS_KNOB_") + name;
  const char* e = std::getenv(k.c_str());
  return e ? std::atoi(e) : 0;
}
}  // namespace pluss

extern "C" void pluss_debug_stage_dump(int last) {
  using namespace pluss;
  const size_t n = g_stage_names.size(), a = last > 0 && (size_t)last < n ? n - (size_t)last : 0;
  for (size_t i = a; i < n; ++i)
    std::fprintf(stderr, "[mark %zu] %s on stream %p: %s\n", i + 1, g_stage_names[i].first.c_str(),
                 g_stage_names[i].second, g_stage_marks && g_stage_marks[i] == i + 1 ? "ran" : "NOT RUN");
  std::fflush(stderr);
}
