// Does a gathered table stay in L2 across kernel launches?  65 536 lanes each
// gather one 448-byte record (28 x 16 B, lane-scattered, like the PF
// predictor) from a 1.43 MB table at random indices.  Timed: back-to-back
// gathers (table warm if L2 survives launches) vs a gather behind a 128 MB
// streaming kernel (table evicted), and the latency-only chain (1 record).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>

constexpr int REC = 448 / 16;   // float4 chunks per record

__global__ void k_gather(const float4* __restrict__ tab, const int* __restrict__ idx, float4* __restrict__ out, int n, int nchunk) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float4* r = tab + (long)idx[e] * REC;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int k = 0; k < nchunk; ++k) {
    const float4 v = r[k];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  out[e] = acc;
}

__global__ void k_stream(const double* __restrict__ in, double* __restrict__ out, long n) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) out[e] = in[e] * 1.5;
}

int main() {
  const int n = 65536, P = 3201;
  float4 *tab, *out;
  int* idx;
  double *sa, *sb;
  const long sn = 8L << 20;   // 64 MB each
  hipMalloc(&tab, (long)P * REC * 16);
  hipMalloc(&out, n * 16L);
  hipMalloc(&idx, n * 4L);
  hipMalloc(&sa, sn * 8);
  hipMalloc(&sb, sn * 8);
  hipMemset(tab, 0, (long)P * REC * 16);
  hipMemset(sa, 0, sn * 8);
  std::vector<int> h(n);
  std::mt19937 g(1);
  for (auto& v : h) v = g() % P;
  hipMemcpy(idx, h.data(), n * 4L, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto gather = [&](int nchunk) { hipLaunchKernelGGL(k_gather, dim3(n / 64), dim3(64), 0, 0, tab, idx, out, n, nchunk); };
  auto stream = [&]() { hipLaunchKernelGGL(k_stream, dim3(sn / 256), dim3(256), 0, 0, sa, sb, sn); };
  auto timed = [&](const char* name, auto f, int it) {
    f(); f();
    hipEventRecord(a);
    for (int i = 0; i < it; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-40s %.2f us\n", name, ms * 1e3 / it);
    return ms * 1e3 / it;
  };
  for (int nchunk : {REC, 1}) {
    printf("-- %d chunks per lane\n", nchunk);
    timed("gather back to back", [&] { gather(nchunk); }, 50);
    const double s = timed("stream 128 MB alone", [&] { stream(); }, 20);
    const double sg = timed("stream + gather", [&] { stream(); gather(nchunk); }, 20);
    printf("%-40s %.2f us\n", "=> gather after stream", sg - s);
  }
  return 0;
}
