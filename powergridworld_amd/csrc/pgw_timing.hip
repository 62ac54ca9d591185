// Sampled kernel timing for the benchmark's roofline: while enabled, every
// `every`-th launch of each timed kernel is issued with hipExtLaunchKernelGGL
// and a start/stop event pair, timestamped by that kernel's dispatch on its own
// stream (the interval rocprofv3 reports).  Not thread-safe: one timing session
// per process, as bench.py uses it.
#include <vector>

#include "pgw_common.h"

namespace pgw {

namespace {
struct Sample {
  int kernel;
  hipEvent_t start, stop;
};
bool g_on = false;
int g_every = 1;
int64_t g_calls[PGW_T_COUNT] = {};
std::vector<hipEvent_t> g_pool;
std::vector<Sample> g_samples;
size_t g_pool_used = 0;
constexpr size_t kPrealloc = 512;   // events ready before a session (256 samples)

hipEvent_t next_event() {
  if (g_pool_used == g_pool.size()) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return nullptr;
    g_pool.push_back(ev);
  }
  return g_pool[g_pool_used++];
}
}  // namespace

TimingSlot timing_begin(int kernel) {
  TimingSlot s;
  if (!g_on || kernel < 0 || kernel >= PGW_T_COUNT) return s;
  if (g_calls[kernel]++ % g_every != 0) return s;
  s.start = next_event();
  s.stop = next_event();
  if (!s.start || !s.stop) s.start = s.stop = nullptr;
  return s;
}

void timing_commit(int kernel, const TimingSlot& s) {
  if (s.start && s.stop) g_samples.push_back({kernel, s.start, s.stop});
}

}  // namespace pgw

using namespace pgw;

extern "C" {

int32_t pgw_timing_start(int32_t every) {
  PGW_REQUIRE(every >= 1, "pgw_timing_start: every < 1");
  g_on = true;
  g_every = every;
  for (auto& c : g_calls) c = 0;
  g_samples.clear();
  g_pool_used = 0;
  // events are created here, not on the first timed launches: hipEventCreate
  // inside the timed region costs host time per sample (the short bench's
  // 10 samples x 2 kernels would otherwise create 40 events while timing)
  while (g_pool.size() < kPrealloc) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) break;
    g_pool.push_back(ev);
  }
  g_samples.reserve(kPrealloc / 2);
  return PGW_OK;
}

int32_t pgw_timing_stop(double* total_ms, int64_t* count) {
  PGW_REQUIRE(total_ms && count, "pgw_timing_stop: null argument");
  for (int k = 0; k < PGW_T_COUNT; ++k) {
    total_ms[k] = 0.0;
    count[k] = 0;
  }
  for (const Sample& s : g_samples) {
    float ms = 0.f;
    if (hipEventSynchronize(s.stop) != hipSuccess || hipEventElapsedTime(&ms, s.start, s.stop) != hipSuccess) {
      set_error("pgw_timing_stop: event query failed");
      g_on = false;
      return PGW_ERR_HIP;
    }
    total_ms[s.kernel] += ms;
    count[s.kernel] += 1;
  }
  g_on = false;
  g_samples.clear();
  g_pool_used = 0;
  return PGW_OK;
}

}  // extern "C"
