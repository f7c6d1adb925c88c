#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out, int n) {
  const int l = threadIdx.x;
  int v = l + 100;
  asm volatile("" : "+v"(v));
  int r = -1, r2 = -1;
  if ((l & 15) < n) {  // lanes 8..15 of each row disabled
    r = __builtin_amdgcn_mov_dpp(v, 0x101, 0xf, 0xf, true);   // row_shl:1, bound_ctrl
    r2 = __builtin_amdgcn_mov_dpp(v, 0x104, 0xf, 0xf, true);  // row_shl:4
  }
  out[l] = r;
  out[64 + l] = r2;
}
int main() {
  int* o; hipMalloc(&o, 128 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, 8);
  int h[128]; hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
  printf("row_shl:1 lanes 0..15: "); for (int i = 0; i < 16; ++i) printf("%d ", h[i]); printf("\n");
  printf("row_shl:4 lanes 0..15: "); for (int i = 0; i < 16; ++i) printf("%d ", h[64 + i]); printf("\n");
  return 0;
}
