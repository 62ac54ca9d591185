// HBM ceiling for the agents kernel's traffic: per (env, agent) item read R
// doubles and write W doubles, env-minor rows (8 B/lane coalesced), trivial
// compute.  Reports GB/s for the agents mix (R=14, W=25) and reference mixes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int R, int W>
__global__ void __launch_bounds__(256) k_mix(const double* __restrict__ in, double* __restrict__ out,
                                              long n) {
  long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < R; ++j) acc += in[j * n + e];
#pragma unroll
  for (int j = 0; j < W; ++j) out[j * n + e] = acc + j;
}

template <int R, int W>
void run(const char* name, long n, const double* in, double* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  dim3 g((n + 255) / 256);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k_mix<R, W>), g, dim3(256), 0, 0, in, out, n);
  const int it = 50;
  hipEventRecord(a);
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((k_mix<R, W>), g, dim3(256), 0, 0, in, out, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double us = ms * 1e3 / it, bytes = 8.0 * (R + W) * n;
  printf("%-22s n=%ld  %.2f us  %.0f GB/s\n", name, n, us, bytes / (us * 1e-6) / 1e9);
}

int main() {
  const long n = 65536L * 5;
  double *in, *out;
  hipMalloc(&in, 8L * 32 * n);
  hipMalloc(&out, 8L * 32 * n);
  hipMemset(in, 0, 8L * 32 * n);
  run<14, 25>("agents mix R14 W25", n, in, out);
  run<14, 0>("read only R14", n, in, out);
  run<0, 25>("write only W25", n, in, out);
  run<16, 16>("copy-like R16 W16", n, in, out);
  run<14, 25>("agents mix x4 n", 4 * n > 0 ? n : n, in, out);
  hipFree(in);
  hipFree(out);
  return 0;
}
