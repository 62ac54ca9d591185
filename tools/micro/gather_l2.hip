// Gather cost of the PF predictor records: 65 536 lanes (one wave per SIMD,
// 64-thread... 256-thread blocks) each need one record of C 16-byte chunks
// from a 3 201-record table at random indices.
//   lane   : every lane loads its own record (C scattered dwordx4 per lane)
//   coop   : the wave moves its 64 records with coalesced LDS-DMA (RPI whole
//            records per wave-instruction, odd-padded slots), then each lane
//            reads its record from LDS
// Timed back to back (table L2-warm if L2 survives launches) and behind a
// 128 MB streaming kernel (table evicted from L2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>

typedef __attribute__((address_space(3))) char lds_char;
typedef float fv4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) fv4 lds_fv4;

template <int C>
__global__ void __launch_bounds__(256) k_lane(const fv4* __restrict__ tab, const int* __restrict__ idx, fv4* __restrict__ out, int n) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const fv4* r = tab + (long)idx[e] * C;
  fv4 v[C];
#pragma unroll
  for (int k = 0; k < C; ++k) v[k] = r[k];
  fv4 acc = v[0];
#pragma unroll
  for (int k = 1; k < C; ++k) acc += v[k];
  out[e] = acc;
}

template <int C>
__global__ void __launch_bounds__(256) k_coop(const fv4* __restrict__ tab, const int* __restrict__ idx, fv4* __restrict__ out, int n) {
  constexpr int S = C + 1, RPI = 64 / S, NI = (64 + RPI - 1) / RPI;
  __shared__ __attribute__((aligned(16))) char lds[4 * 64 * S * 16];
  const int e = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
  lds_char* slab = (lds_char*)lds + (threadIdx.x >> 6) * 64 * S * 16;
  const int c = idx[e];
  const int sub = lane / S, q = lane - sub * S;
  const bool act = sub < RPI && q < C;
  const char* base = reinterpret_cast<const char*>(tab) + q * 16;
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    int cr = __builtin_amdgcn_readlane(c, k * RPI);
#pragma unroll
    for (int j = 1; j < RPI; ++j)
      if (k * RPI + j < 64) cr = sub == j ? __builtin_amdgcn_readlane(c, k * RPI + j) : cr;
    if (act && k * RPI + sub < 64)
      __builtin_amdgcn_global_load_lds(base + (long)cr * C * 16, slab + k * RPI * S * 16, 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const lds_fv4* r = (const lds_fv4*)(slab + lane * S * 16);
  fv4 acc = r[0];
#pragma unroll
  for (int k = 1; k < C; ++k) acc += r[k];
  out[e] = acc;
}

__global__ void k_stream(const double* __restrict__ in, double* __restrict__ o, long m) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) o[i] = in[i] * 1.5;
}

int main() {
  const int n = 65536, P = 3201, CMAX = 28;
  fv4 *tab, *out;
  int* idx;
  double *sa, *sb;
  const long sn = 8L << 20;
  hipMalloc(&tab, (long)P * CMAX * 16);
  hipMalloc(&out, n * 16L);
  hipMalloc(&idx, n * 4L);
  hipMalloc(&sa, sn * 8);
  hipMalloc(&sb, sn * 8);
  hipMemset(tab, 0, (long)P * CMAX * 16);
  hipMemset(sa, 0, sn * 8);
  std::vector<int> h(n);
  std::mt19937 g(1);
  for (auto& v : h) v = g() % P;
  hipMemcpy(idx, h.data(), n * 4L, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto stream = [&]() {
    hipLaunchKernelGGL(k_stream, dim3(sn / 256), dim3(256), 0, 0, (const double*)sa, sb, sn);
  };
  auto timed = [&](auto f, int it) {
    f(); f();
    hipEventRecord(a);
    for (int i = 0; i < it; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3 / it;
  };
  const double s = timed(stream, 20);
  auto report = [&](const char* name, auto kern) {
    auto run = [&] { hipLaunchKernelGGL(kern, dim3(n / 256), dim3(256), 0, 0, (const fv4*)tab, (const int*)idx, out, n); };
    const double warm = timed(run, 50);
    const double cold = timed([&] { stream(); run(); }, 20) - s;
    printf("%-14s warm %6.2f us   after 128 MB stream %6.2f us\n", name, warm, cold);
  };
  printf("stream alone %.2f us\n", s);
  report("lane C1", k_lane<1>);
  report("lane C14", k_lane<14>);
  report("lane C21", k_lane<21>);
  report("lane C28", k_lane<28>);
  report("coop C14", k_coop<14>);
  report("coop C21", k_coop<21>);
  report("coop C28", k_coop<28>);
  return 0;
}
