// Semantics check of gfx950's v_permlane16_swap_b32 (__builtin_amdgcn_permlane16_swap)
// for the backward pass (a DPP row's values copied to the next row): prints,
// for input = lane id in both operands, the two results per lane.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/micro/permlane_swap tools/micro/permlane_swap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_swap(unsigned* o) {
  const unsigned x = threadIdx.x, y = 100 + threadIdx.x;
  const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  o[threadIdx.x] = r[0];
  o[64 + threadIdx.x] = r[1];
}

int main() {
  unsigned* d;
  unsigned h[128];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_swap, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  std::printf("vdst=lane, vsrc=100+lane\nr0:");
  for (int i = 0; i < 64; ++i) std::printf(" %u", h[i]);
  std::printf("\nr1:");
  for (int i = 0; i < 64; ++i) std::printf(" %u", h[64 + i]);
  std::printf("\n");
  (void)hipFree(d);
  return 0;
}
