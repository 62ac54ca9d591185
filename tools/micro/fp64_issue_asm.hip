// fp64 VALU issue rate (inline-asm variant of fp64_issue.hip) of one vs two waves per SIMD, plain and DPP-broadcast
// operands (the question behind the PF kernels' one-lane-per-env layout):
// each lane runs ITERS x 16 independent v_fmac_f64 (16 accumulators), the B
// operand plain or through row_newbcast.  Prints cycles per instruction per
// SIMD for waves-per-SIMD = 1, 2, 4.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITERS = 4096;

template <int DPP>
__global__ void __launch_bounds__(256) k_fma(double* out, double seed) {
  double acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = seed * (threadIdx.x + j);
  double a = seed + threadIdx.x, b = seed * 0.5;
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (DPP) {
      asm volatile(
          "s_nop 1\n"
          "v_fmac_f64_dpp %0, %16, %17 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %1, %16, %17 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %2, %16, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %3, %16, %17 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %4, %16, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %5, %16, %17 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %6, %16, %17 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %7, %16, %17 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %8, %16, %17 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %9, %16, %17 row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %10, %16, %17 row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %11, %16, %17 row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %12, %16, %17 row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %13, %16, %17 row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %14, %16, %17 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
          "v_fmac_f64_dpp %15, %16, %17 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
          : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
            "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]), "+v"(acc[12]),
            "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15])
          : "v"(a), "v"(b));
    } else {
      asm volatile(
          "v_fmac_f64_e32 %0, %16, %17\n"
          "v_fmac_f64_e32 %1, %16, %17\n"
          "v_fmac_f64_e32 %2, %16, %17\n"
          "v_fmac_f64_e32 %3, %16, %17\n"
          "v_fmac_f64_e32 %4, %16, %17\n"
          "v_fmac_f64_e32 %5, %16, %17\n"
          "v_fmac_f64_e32 %6, %16, %17\n"
          "v_fmac_f64_e32 %7, %16, %17\n"
          "v_fmac_f64_e32 %8, %16, %17\n"
          "v_fmac_f64_e32 %9, %16, %17\n"
          "v_fmac_f64_e32 %10, %16, %17\n"
          "v_fmac_f64_e32 %11, %16, %17\n"
          "v_fmac_f64_e32 %12, %16, %17\n"
          "v_fmac_f64_e32 %13, %16, %17\n"
          "v_fmac_f64_e32 %14, %16, %17\n"
          "v_fmac_f64_e32 %15, %16, %17\n"
          : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
            "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]), "+v"(acc[12]),
            "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15])
          : "v"(a), "v"(b));
    }
  }
  double s = 0.0;
  for (int j = 0; j < 16; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

template <int DPP>
static void run(int cus, double clk_ghz, double* out) {
  for (int wps : {1, 2, 4}) {
    const int waves = cus * 4 * wps;          // 4 SIMDs per CU
    const int blocks = waves / 4;             // 256 threads = 4 waves per block
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    k_fma<DPP><<<blocks, 256>>>(out, 1.0);
    CHECK(hipEventRecord(a));
    k_fma<DPP><<<blocks, 256>>>(out, 1.0);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double instr = (double)ITERS * 16 * wps;   // per SIMD
    printf("%s waves/SIMD=%d  %.3f ms  %.2f cycles per fp64 FMA instr per SIMD  (%.1f TFLOP/s)\n",
           DPP ? "dpp  " : "plain", wps, ms, ms * 1e-3 * clk_ghz * 1e9 / instr,
           2.0 * 64 * instr * cus * 4 / (ms * 1e-3) * 1e-12);
  }
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const double clk = p.clockRate * 1e-6;   // kHz -> GHz
  printf("%s CUs=%d clock=%.2f GHz\n", p.gcnArchName, cus, clk);
  double* out;
  CHECK(hipMalloc(&out, (size_t)cus * 4 * 4 * 64 * sizeof(double)));
  run<0>(cus, clk, out);
  run<1>(cus, clk, out);
  CHECK(hipFree(out));
  return 0;
}
