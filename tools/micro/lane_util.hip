// Calibration of the VALU lane-utilisation counters (tools/pmc_lanes.sh):
// the same fp64 FMA loop run by every lane of a wave (k_full), by 8 lanes
// (k_8: lanes 0..7, like one trial group of the line search) and by 7 lanes
// (k_7: the 7x7 LLT / BoxQP rows of the backward pass).  Under
// `rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES`
// the ratio THREAD_CYCLES_VALU / ACTIVE_INST_VALU of k_full is the full-lane
// figure, and k_8 / k_7 must come out at 8/64 and 7/64 of it.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/micro/lane_util tools/micro/lane_util.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int LANES>
__global__ __launch_bounds__(64) void k_lanes(double* sink, double c, double b, int iters) {
  const int l = threadIdx.x;
  double e = (double)l;
  if (l < LANES) {
    for (int i = 0; i < iters; ++i) {
      e = fma(e, c, b);
      e = fma(e, c, b);
      e = fma(e, c, b);
      e = fma(e, c, b);
    }
  }
  if (e == 12345.678) sink[l] = e;  // never true: keeps the chain live
}

int main() {
  double* sink;
  if (hipMalloc(&sink, 64 * sizeof(double)) != hipSuccess) return 1;
  const int blocks = 1024, iters = 4096;
  hipLaunchKernelGGL((k_lanes<64>), dim3(blocks), dim3(64), 0, 0, sink, 0.999, 1e-3, iters);
  hipLaunchKernelGGL((k_lanes<8>), dim3(blocks), dim3(64), 0, 0, sink, 0.999, 1e-3, iters);
  hipLaunchKernelGGL((k_lanes<7>), dim3(blocks), dim3(64), 0, 0, sink, 0.999, 1e-3, iters);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("lane_util calibration kernels done (%d blocks x 64 lanes, %d x 4 FMA per active lane)\n", blocks, iters);
  (void)hipFree(sink);
  return 0;
}
