// Host-side cost of one kernel launch on MI355X vs kernel-argument size and
// stream (null vs created), the GPU kept far behind by a long first kernel.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

template <int B> struct Args { char b[B]; };

template <int B>
__global__ void k_empty(Args<B> a, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.b[0] == 42) out[0] = 1;
}
__global__ void k_spin(long long cycles) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
}

template <int B>
double bench(hipStream_t st, int* out, int n) {
  Args<B> a = {};
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st, 2000000000LL / 10);  // GPU busy ~ tens of ms
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty<B>, dim3(256), dim3(256), 0, st, a, out);
  auto t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(st);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  int* out;
  hipMalloc(&out, 64);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int rep = 0; rep < 2; ++rep) {
    printf("null stream : args 16 B %.2f us, 1 KB %.2f us, 2.5 KB %.2f us\n", bench<16>(0, out, 500),
           bench<1024>(0, out, 500), bench<2560>(0, out, 500));
    printf("own stream  : args 16 B %.2f us, 1 KB %.2f us, 2.5 KB %.2f us\n", bench<16>(s, out, 500),
           bench<1024>(s, out, 500), bench<2560>(s, out, 500));
  }
  return 0;
}
