// Probe: fragment layout and throughput of v_mfma_f64_16x16x4f64 vs v_fma_f64 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>

typedef double double4_t __attribute__((ext_vector_type(4)));

__global__ void layout(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  // hypothesis: A[i][k] with i = l%16, k = l/16 ; B[k][j] with k = l/16, j = l%16
  double a = A[(l % 16) * 4 + (l / 16)];
  double b = B[(l / 16) * 16 + (l % 16)];
  double4_t c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}

__global__ void mfma_loop(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double4_t c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

__global__ void fma_loop(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double c[8] = {0, 1, 2, 3, 4, 5, 6, 7};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = fma(a, c[k], b);
  }
  double s = 0;
  for (int k = 0; k < 8; ++k) s += c[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  std::vector<double> A(64), B(64), D(256);
  for (int i = 0; i < 64; ++i) { A[i] = i + 1; B[i] = (i % 7) - 3 + 0.5 * (i / 16); }
  double *dA, *dB, *dD, *dO;
  hipMalloc(&dA, 64 * 8); hipMalloc(&dB, 64 * 8); hipMalloc(&dD, 256 * 8);
  hipMemcpy(dA, A.data(), 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 64 * 8, hipMemcpyHostToDevice);
  layout<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(D.data(), dD, 256 * 8, hipMemcpyDeviceToHost);
  // reference C = A(16x4) B(4x16); check hypothesis D[l][r] = C[4*(l/16)+r][l%16]
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      int i = 4 * (l / 16) + r, j = l % 16;
      double ref = 0;
      for (int k = 0; k < 4; ++k) ref += A[i * 4 + k] * B[k * 16 + j];
      if (std::fabs(ref - D[l * 4 + r]) > 1e-9) ++bad;
    }
  printf("layout hypothesis mismatches: %d / 256\n", bad);
  int blocks = 256 * 8, threads = 256, iters = 2000;
  hipMalloc(&dO, blocks * threads * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    mfma_loop<<<blocks, threads>>>(dO, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = 2.0 * 16 * 16 * 4 * 4.0 * iters * (blocks * threads / 64);
    printf("mfma_f64_16x16x4: %.3f ms  %.1f TFLOP/s\n", ms, flops / ms / 1e9);
    hipEventRecord(e0);
    fma_loop<<<blocks, threads>>>(dO, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    flops = 2.0 * 8 * iters * (double)(blocks * threads);
    printf("v_fma_f64: %.3f ms  %.1f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  return 0;
}
