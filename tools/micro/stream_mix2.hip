// Structure study for the agents kernel (R=14 reads, W=25 writes of fp64 per
// item, 327 680 items, env-minor rows), with an emulated compute phase of C
// fp64 FMAs per item (4 independent chains) between the loads and the stores:
//   flat  : one item per thread (k_coord_agents_std's structure)
//   nt    : flat + nontemporal stores
//   loop  : G waves per SIMD, each thread loops over items with the next
//           item's loads issued before the current item's compute (prefetch)
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int R = 14, W = 25;

template <int C>
__device__ __forceinline__ void compute(const double (&x)[R], double (&y)[4]) {
  double a0 = x[0], a1 = x[1], a2 = x[2], a3 = x[3];
#pragma unroll
  for (int j = 4; j < R; ++j) a0 += x[j];
#pragma unroll
  for (int k = 0; k < C / 4; ++k) {
    a0 = fma(a0, 1.0000001, 0.5);
    a1 = fma(a1, 0.9999999, 0.25);
    a2 = fma(a2, 1.0000002, 0.125);
    a3 = fma(a3, 0.9999998, 0.0625);
  }
  y[0] = a0; y[1] = a1; y[2] = a2; y[3] = a3;
}

template <int C, bool NT>
__global__ void __launch_bounds__(256) k_flat(const double* __restrict__ in, double* __restrict__ out, int n) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  double x[R], y[4];
#pragma unroll
  for (int j = 0; j < R; ++j) x[j] = in[(long)j * n + e];
  compute<C>(x, y);
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const double v = y[j & 3] + j;
    if (NT) __builtin_nontemporal_store(v, &out[(long)j * n + e]);
    else out[(long)j * n + e] = v;
  }
}

template <int C, bool NT>
__global__ void __launch_bounds__(256) k_loop(const double* __restrict__ in, double* __restrict__ out, int n) {
  const int T = gridDim.x * 256;
  int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  double nx[R];
#pragma unroll
  for (int j = 0; j < R; ++j) nx[j] = in[(long)j * n + e];
  for (;;) {
    double x[R], y[4];
#pragma unroll
    for (int j = 0; j < R; ++j) x[j] = nx[j];
    const int en = e + T;
    if (en < n) {
#pragma unroll
      for (int j = 0; j < R; ++j) nx[j] = in[(long)j * n + en];
    }
    compute<C>(x, y);
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const double v = y[j & 3] + j;
      if (NT) __builtin_nontemporal_store(v, &out[(long)j * n + e]);
      else out[(long)j * n + e] = v;
    }
    if (en >= n) break;
    e = en;
  }
}

// pooled: 8 of the 14 rows come from one of 64 cycled action batches (HBM,
// not MALL-resident: 1.3 GB), the other 6 are state rows re-read every launch
template <int C, bool LOOP>
__global__ void __launch_bounds__(256) k_pool(const double* __restrict__ act, const double* __restrict__ st,
                                              double* __restrict__ out, int n) {
  const int T = LOOP ? gridDim.x * 256 : n;
  int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  for (;;) {
    double x[R], y[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = act[(long)j * n + e];
#pragma unroll
    for (int j = 8; j < R; ++j) x[j] = st[(long)(j - 8) * n + e];
    compute<C>(x, y);
#pragma unroll
    for (int j = 0; j < W; ++j) out[(long)j * n + e] = y[j & 3] + j;
    e += T;
    if (!LOOP || e >= n) break;
  }
}

template <typename K>
void run_pool(const char* name, K kern, int blocks, int n, const double* act, const double* st, double* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const long pool = 8L * n;
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, act, st, out, n);
  const int it = 128;
  hipEventRecord(a);
  for (int i = 0; i < it; ++i)
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, act + (i % 64) * pool, st, out, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / it, bytes = 8.0 * (R + W) * n;
  printf("%-28s blocks=%5d  %.2f us  %.0f GB/s\n", name, blocks, us, bytes / (us * 1e-6) / 1e9);
}

template <typename K>
void run(const char* name, K kern, int blocks, int n, const double* in, double* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, in, out, n);
  const int it = 50;
  hipEventRecord(a);
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, in, out, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / it, bytes = 8.0 * (R + W) * n;
  printf("%-28s blocks=%5d  %.2f us  %.0f GB/s\n", name, blocks, us, bytes / (us * 1e-6) / 1e9);
}

template <int C>
void suite(int n, const double* in, double* out) {
  char nm[64];
  const int flat = (n + 255) / 256;
  printf("-- compute %d FMAs per item\n", C);
  snprintf(nm, 64, "flat C%d", C); run(nm, k_flat<C, false>, flat, n, in, out);
  snprintf(nm, 64, "flat nt C%d", C); run(nm, k_flat<C, true>, flat, n, in, out);
  for (int blocks : {256, 512, 640, 768, 1024}) {
    snprintf(nm, 64, "loop C%d", C); run(nm, k_loop<C, false>, blocks, n, in, out);
  }
  snprintf(nm, 64, "loop nt C%d", C); run(nm, k_loop<C, true>, 512, n, in, out);
}

int main() {
  const int n = 65536 * 5;
  double *in, *out;
  hipMalloc(&in, 8L * R * n);
  hipMalloc(&out, 8L * W * n);
  hipMemset(in, 0, 8L * R * n);
  suite<0>(n, in, out);
  suite<200>(n, in, out);
  suite<400>(n, in, out);
  double* act;
  hipMalloc(&act, 8L * 8 * n * 64);
  hipMemset(act, 0, 8L * 8 * n * 64);
  printf("-- pooled actions (64 batches cycled), C = 400\n");
  run_pool("pool flat C400", k_pool<400, false>, (n + 255) / 256, n, act, in, out);
  for (int blocks : {512, 768, 1024})
    run_pool("pool loop C400", k_pool<400, true>, blocks, n, act, in, out);
  hipFree(act);
  hipFree(in);
  hipFree(out);
  return 0;
}
