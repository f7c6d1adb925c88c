// Measured fp64 VALU throughput of one MI355X (the guide has no FP64 row):
// every SIMD busy with independent v_fma_f64 chains, HIP events around the
// launch.  Reports FLOP/s (2 per FMA lane) and the wave-instruction issue
// rate per SIMD, for bench.py's roofline.fp64 (profiles/r05_fp64_peak.json).
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/fp64_peak tools/micro/fp64_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CH 8  // independent chains per lane

template <int ITER>
__global__ __launch_bounds__(256) void k_fma(double* sink, double c, double b) {
  double e[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) e[j] = (double)(threadIdx.x + j);
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int j = 0; j < CH; ++j) e[j] = fma(e[j], c, b);
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < CH; ++j) s += e[j];
  if (s == 12345.678) sink[threadIdx.x] = s;  // never true: keeps the chains live
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  double* sink;
  hipMalloc(&sink, 256 * sizeof(double));
  hipEvent_t a, z;
  hipEventCreate(&a);
  hipEventCreate(&z);
  constexpr int ITER = 32768;
  std::printf("device %s, %d CUs, clock %d kHz\n", p.name, cus, p.clockRate);
  std::printf("%-10s %-10s %12s %14s %16s\n", "waves/SIMD", "blocks", "ms", "TFLOP/s", "instr/SIMD/clk");
  double best = 0.0;
  for (int wps : {1, 2, 4, 8, 16}) {
    const int blocks = cus * wps;  // 256 threads = 4 waves per block: one per SIMD
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_fma<ITER>, dim3(blocks), dim3(256), 0, 0, sink, 1.0000001, 1e-9);
    hipDeviceSynchronize();
    float ms_best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_fma<ITER>, dim3(blocks), dim3(256), 0, 0, sink, 1.0000001, 1e-9);
      hipEventRecord(z);
      hipEventSynchronize(z);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, z);
      if (ms < ms_best) ms_best = ms;
    }
    const double fmas = (double)blocks * 256 * CH * ITER;
    const double tf = 2.0 * fmas / (ms_best * 1e-3) / 1e12;
    const double winstr = fmas / 64.0;  // wave64 instructions
    const double per_simd_clk = winstr / (cus * 4.0) / (ms_best * 1e-3 * p.clockRate * 1e3);
    std::printf("%-10d %-10d %12.4f %14.2f %16.4f\n", wps, blocks, ms_best, tf, per_simd_clk);
    if (tf > best) best = tf;
  }
  std::printf("peak_fp64_fma_tflops %.3f\n", best);
  return 0;
}
