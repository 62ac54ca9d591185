// fp64 FMA issue rate of ONE wave per SIMD (the PF kernels' occupancy at
// 65 536 envs): 256 blocks x 256 threads, every wave running R independent
// accumulation chains for ITER rounds, as
//   plain  v_fmac_f64 with VGPR operands,
//   dpp    v_fmac_f64_dpp ... row_newbcast (the PF's resident-operand form),
// and the same with 2 and 4 waves per SIMD (more blocks) for comparison.
// Prints ns per wave-instruction and the implied cycles at the measured clock.
// Build: hipcc -O3 --offload-arch=gfx950 fp64_issue.hip -o fp64_issue
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;

template <int R>
__global__ void __launch_bounds__(256) k_plain(double* out, double a, double b) {
  double acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = threadIdx.x * 1e-3 + r;
  double x = a + threadIdx.x * 1e-9;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = __builtin_fma(x, b, acc[r]);
  }
  double s = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) s += acc[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int R>
__global__ void __launch_bounds__(256) k_dpp(double* out, double a, double b) {
  double acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = threadIdx.x * 1e-3 + r;
  double w = a + (threadIdx.x & 15) * 1e-9;   // resident operand, broadcast by DPP
  double x = b;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf"
                   : "+v"(acc[r]) : "v"(w), "v"(x));
  }
  double s = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) s += acc[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
static float time_kernel(K kern, int blocks, double* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 0.9999999);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 0.9999999);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return best;
}

template <int R>
static void run(double* out, int clock_khz) {
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int blocks = 256 * wps;                 // 4 waves per block, 256 CUs
    const double instr = (double)ITER * R;        // FMAs per wave
    const float tp = time_kernel(k_plain<R>, blocks, out);
    const float td = time_kernel(k_dpp<R>, blocks, out);
    // per SIMD: wps waves x instr instructions
    const double per_p = tp * 1e6 / (wps * instr), per_d = td * 1e6 / (wps * instr);
    printf("R=%2d chains, %d wave(s)/SIMD: plain %.3f ns/instr (%.2f cyc), dpp %.3f ns/instr (%.2f cyc)\n", R, wps,
           per_p, per_p * clock_khz * 1e-6, per_d, per_d * clock_khz * 1e-6);
  }
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("%s, %d CUs, clock %d kHz\n", p.name, p.multiProcessorCount, p.clockRate);
  double* out;
  hipMalloc(&out, 4 * 256 * 256 * sizeof(double));
  run<1>(out, p.clockRate);
  run<2>(out, p.clockRate);
  run<4>(out, p.clockRate);
  run<8>(out, p.clockRate);
  hipFree(out);
  return 0;
}
