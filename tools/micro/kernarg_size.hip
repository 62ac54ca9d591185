// Micro-probe: does the size of a kernel's by-value argument block cost GPU time
// per launch?  Back-to-back launches of a tiny kernel (1 block per launch... and
// a 1024-block grid) with a 64 B / 1 KB / 2.3 KB / 3.6 KB struct argument; HIP
// events around 2000 launches on one stream -> us per launch (throughput).
// Build: hipcc --offload-arch=gfx950 -O3 kernarg_size.hip -o kernarg_size
#include <hip/hip_runtime.h>
#include <cstdio>

template <int B>
struct Args {
  double v[B / 8];
};

template <int B>
__global__ void k_args(Args<B> a, double* out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0) out[0] = a.v[B / 8 - 1];     // touch the last field
}

template <int B>
static void run(int blocks, double* out, hipStream_t st) {
  Args<B> a;
  for (int i = 0; i < B / 8; ++i) a.v[i] = i;
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_args<B>, dim3(blocks), dim3(256), 0, st, a, out);
  hipEventRecord(t0, st);
  const int N = 2000;
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_args<B>, dim3(blocks), dim3(256), 0, st, a, out);
  hipEventRecord(t1, st);
  hipEventSynchronize(t1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, t0, t1);
  printf("args %5d B, %5d blocks: %.2f us per launch\n", B, blocks, ms * 1e3 / N);
  hipEventDestroy(t0);
  hipEventDestroy(t1);
}

int main() {
  double* out;
  hipMalloc(&out, 64);
  hipStream_t st;
  hipStreamCreate(&st);
  for (int blocks : {1, 1024}) {
    run<64>(blocks, out, st);
    run<1024>(blocks, out, st);
    run<2304>(blocks, out, st);
    run<3584>(blocks, out, st);
  }
  hipFree(out);
  return 0;
}
