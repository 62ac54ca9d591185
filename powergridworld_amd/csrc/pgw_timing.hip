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

// STREAM-style copy for the bench's measured HBM ceiling: 16 B per lane, four
// loads in flight per lane before their stores, grid-stride over the buffer,
// nontemporal both ways (a copy's data is never re-read).
constexpr int kCopyUnroll = 4;
typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(kBlock) k_stream_copy(const dv2* __restrict__ src,
                                                        dv2* __restrict__ dst, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * kBlock * kCopyUnroll;
  for (int64_t base = (int64_t)blockIdx.x * kBlock * kCopyUnroll + threadIdx.x; base < n16; base += stride) {
    dv2 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const int64_t i = base + (int64_t)u * kBlock;
      if (i < n16) v[u] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const int64_t i = base + (int64_t)u * kBlock;
      if (i < n16) __builtin_nontemporal_store(v[u], dst + i);
    }
  }
}

}  // namespace pgw

using namespace pgw;

extern "C" {

int32_t pgw_stream_copy(const void* src, void* dst, int64_t bytes, int32_t reps, float* ms_out,
                        void* stream) {
  PGW_REQUIRE(src && dst && ms_out && reps >= 1 && bytes > 0 && bytes % 16 == 0,
              "pgw_stream_copy: bad argument");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t n16 = bytes / 16;
  // 32 blocks per CU, grid-stride: the best of the grids and cache policies
  // tools/micro/copy_peak.hip measured (profiles/r02/copy_peak.txt: 6.06 TB/s;
  // read-only 6.2-6.4, write-only 4.1-4.6)
  const unsigned grid = 8192;
  auto launch = [&] {
    hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(kBlock), 0, st,
                       static_cast<const dv2*>(src), static_cast<dv2*>(dst), n16);
  };
  launch();   // warm: page tables, clocks
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return check_launch("pgw_stream_copy");
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return check_launch("pgw_stream_copy");
  }
  (void)hipEventRecord(e0, st);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(e1, st);
  float ms = 0.f;
  const bool ok = hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (!ok) {
    set_error("pgw_stream_copy: event query failed");
    return PGW_ERR_HIP;
  }
  *ms_out = ms / reps;
  return check_launch("pgw_stream_copy");
}

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
