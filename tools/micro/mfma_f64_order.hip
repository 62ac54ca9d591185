// In which order does v_mfma_f64_16x16x4f64 accumulate?  Random operands with
// spread exponents; each D[i][j] is compared bit for bit with candidate
// host evaluations of C + sum_k A[i][k] B[k][j]:
//   seq    c = fma(a_k, b_k, c) for k = 0..3
//   rev    the same for k = 3..0
//   pair   c + ((a0 b0 + a1 b1) + (a2 b2 + a3 b3)), every op rounded
//   once   the exact value rounded once (long double sum of exact products)
// Operand layout (tools/micro/mfma_f64_layout.hip): A lane l = A[l%16][l/16],
// B lane l = B[l/16][l%16], D lane l reg r = D[l/16 + 4r][l%16].
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef double double4_t __attribute__((ext_vector_type(4)));

__global__ void k(const double* A, const double* B, const double* C, double* D, int trials) {
  const int t = blockIdx.x, l = threadIdx.x;
  if (t >= trials) return;
  const double a = A[t * 64 + (l % 16) * 4 + l / 16];
  const double b = B[t * 64 + (l / 16) * 16 + l % 16];
  double4_t c;
  for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + (l / 16 + 4 * r) * 16 + l % 16];
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[t * 256 + (l / 16 + 4 * r) * 16 + l % 16] = c[r];
}

int main() {
  const int T = 256;
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  std::uniform_int_distribution<int> ex(-30, 30);
  std::vector<double> A(T * 64), B(T * 64), C(T * 256), D(T * 256);
  for (auto& x : A) x = std::ldexp(u(g), ex(g));
  for (auto& x : B) x = std::ldexp(u(g), ex(g));
  for (auto& x : C) x = std::ldexp(u(g), ex(g));
  double *dA, *dB, *dC, *dD;
  hipMalloc(&dA, A.size() * 8);
  hipMalloc(&dB, B.size() * 8);
  hipMalloc(&dC, C.size() * 8);
  hipMalloc(&dD, D.size() * 8);
  hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD, T);
  hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost);
  long seq = 0, rev = 0, pair = 0, once = 0, total = 0;
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        const double* a = &A[t * 64 + i * 4];
        double b[4];
        for (int kk = 0; kk < 4; ++kk) b[kk] = B[t * 64 + kk * 16 + j];
        const double c = C[t * 256 + i * 16 + j], d = D[t * 256 + i * 16 + j];
        double s = c;
        for (int kk = 0; kk < 4; ++kk) s = std::fma(a[kk], b[kk], s);
        double r2 = c;
        for (int kk = 3; kk >= 0; --kk) r2 = std::fma(a[kk], b[kk], r2);
        const double p = c + ((a[0] * b[0] + a[1] * b[1]) + (a[2] * b[2] + a[3] * b[3]));
        long double ex_ = (long double)c;
        for (int kk = 0; kk < 4; ++kk) ex_ += (long double)a[kk] * (long double)b[kk];
        seq += (s == d);
        rev += (r2 == d);
        pair += (p == d);
        once += ((double)ex_ == d);
        ++total;
      }
  printf("v_mfma_f64_16x16x4f64: %ld outputs; bit-equal to: seq fma k=0..3 %ld, rev fma k=3..0 %ld, "
         "pairwise %ld, rounded-once (long double) %ld\n", total, seq, rev, pair, once);
  return 0;
}
