// Decode the v_mfma_f64_16x16x4f64 operand/result lane layout: wave w = (t, u)
// sets a = [lane==t], b = [lane==u]; D is dumped.  D is non-zero exactly where
// A(lane t) and B(lane u) share the K index.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double double4_t __attribute__((ext_vector_type(4)));
__global__ void k(double* D) {
  int w = blockIdx.x, l = threadIdx.x, t = w / 64, u = w % 64;
  double a = (l == t) ? 1.0 : 0.0, b = (l == u) ? 1.0 : 0.0;
  double4_t c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(size_t)w * 256 + l * 4 + r] = c[r];
}
int main() {
  double* d; hipMalloc(&d, 4096 * 256 * 8);
  k<<<4096, 64>>>(d);
  std::vector<double> h(4096 * 256);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  FILE* f = fopen("gpurun_out/mfma_f64_layout.txt", "w");
  for (int w = 0; w < 4096; ++w)
    for (int p = 0; p < 256; ++p)
      if (h[(size_t)w * 256 + p] != 0.0) fprintf(f, "%d %d %d %g\n", w / 64, w % 64, p, h[(size_t)w * 256 + p]);
  fclose(f);
  printf("done\n");
  return 0;
}
