// Kernel-argument latency probe: a wave-uniform chain of dependent loads
// (idx = tab[idx], scalar loads) from (a) a 3 KB by-value kernel argument,
// (b) the same table in an ordinary device buffer, (c) kernarg but only one
// independent load.  1024 one-wave blocks (the k_ma_step shape at 65 536 envs)
// and 256 four-wave blocks; HIP events around 200 launches each.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kTab = 768;   // 3 KB of int32
struct Big {
  int tab[kTab];
};

template <int DEP>
__global__ void k_arg(Big a, int* out) {
  int idx = 0;
#pragma unroll
  for (int i = 0; i < DEP; ++i) idx = a.tab[(idx + i * 37) % kTab];
  out[blockIdx.x * blockDim.x + threadIdx.x] = idx;
}

template <int DEP>
__global__ void k_buf(const int* __restrict__ tab, int* out) {
  int idx = 0;
#pragma unroll
  for (int i = 0; i < DEP; ++i) idx = tab[(idx + i * 37) % kTab];
  out[blockIdx.x * blockDim.x + threadIdx.x] = idx;
}

template <class F>
static float time_it(F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) launch();
  hipEventRecord(a);
  const int reps = 200;
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps;
}

int main() {
  Big h;
  for (int i = 0; i < kTab; ++i) h.tab[i] = (i * 7 + 3) % kTab;
  int *tab, *out;
  hipMalloc(&tab, sizeof(h));
  hipMalloc(&out, 65536 * sizeof(int) * 4);
  hipMemcpy(tab, &h, sizeof(h), hipMemcpyHostToDevice);
  for (int bs : {64, 256}) {
    const int grid = 65536 / bs;
    printf("block %3d x %4d:  kernarg dep1 %.2f us  dep4 %.2f  dep16 %.2f | buffer dep1 %.2f  dep4 %.2f  dep16 %.2f\n",
           bs, grid,
           time_it([&] { hipLaunchKernelGGL(k_arg<1>, dim3(grid), dim3(bs), 0, 0, h, out); }),
           time_it([&] { hipLaunchKernelGGL(k_arg<4>, dim3(grid), dim3(bs), 0, 0, h, out); }),
           time_it([&] { hipLaunchKernelGGL(k_arg<16>, dim3(grid), dim3(bs), 0, 0, h, out); }),
           time_it([&] { hipLaunchKernelGGL(k_buf<1>, dim3(grid), dim3(bs), 0, 0, tab, out); }),
           time_it([&] { hipLaunchKernelGGL(k_buf<4>, dim3(grid), dim3(bs), 0, 0, tab, out); }),
           time_it([&] { hipLaunchKernelGGL(k_buf<16>, dim3(grid), dim3(bs), 0, 0, tab, out); }));
  }
  return 0;
}
