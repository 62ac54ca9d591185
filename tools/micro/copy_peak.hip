// Device-copy ceiling on one MI355X: 1 GiB copies with 16-B lanes, varying the
// load/store cache policy, the loads in flight per lane and the grid, to pick
// the bench's measured HBM peak (pgw_stream_copy) honestly.  Also a read-only
// and a write-only stream.   ./copy_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dv2 __attribute__((ext_vector_type(2)));

template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_copy(const dv2* __restrict__ src, dv2* __restrict__ dst, long n) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long base = (long)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
    dv2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + (long)u * 256;
      if (i < n) v[u] = NTL ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + (long)u * 256;
      if (i < n) {
        if (NTS) __builtin_nontemporal_store(v[u], dst + i);
        else dst[i] = v[u];
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_read(const dv2* __restrict__ src, dv2* __restrict__ sink, long n) {
  dv2 acc = {0, 0};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) acc += src[i];
  if (acc.x == 12345.0) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_write(dv2* __restrict__ dst, long n) {
  const dv2 v = {1.0, 2.0};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(v, dst + i);
}

template <class F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const long bytes = 1L << 30, n = bytes / 16;
  dv2 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  (void)hipMemset(a, 0, bytes);
  (void)hipMemset(b, 0, bytes);
  const int reps = 30;
  for (int grid : {1024, 2048, 4096, 8192}) {
#define RUN(U, NTL, NTS)                                                                              \
  {                                                                                                 \
    float ms = time_ms([&] { hipLaunchKernelGGL((k_copy<U, NTL, NTS>), dim3(grid), dim3(256), 0, 0, a, b, n); }, reps); \
    printf("copy grid %5d unroll %d nt_load %d nt_store %d: %7.1f GB/s\n", grid, U, NTL, NTS, 2.0 * bytes / (ms * 1e6)); \
  }
    RUN(4, true, true) RUN(4, false, true) RUN(4, false, false) RUN(8, false, true) RUN(2, false, true)
    float ms = time_ms([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, b, n); }, reps);
    printf("read  grid %5d: %7.1f GB/s\n", grid, bytes / (ms * 1e6));
    ms = time_ms([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, b, n); }, reps);
    printf("write grid %5d: %7.1f GB/s\n", grid, bytes / (ms * 1e6));
  }
  return 0;
}
