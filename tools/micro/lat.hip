// Microbenchmarks of single-wave instruction latency / issue on gfx950 (one
// wave per launch, s_memtime deltas): dependent / independent fp64 FMA
// chains, DPP moves, ds_swizzle, readlane broadcasts, LDS round trips.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 256
__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define PIN(x) asm volatile("" : "+v"(x))
template <int CTRL> __device__ __forceinline__ double dpp64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__global__ void k(unsigned long long* out, double* sink, double s) {
  __shared__ double L[64 * 4];
  const int l = threadIdx.x;
  double a = s + l, b = s * 0.5, c = 1.0000001;
  unsigned long long t0, t1;
  // 1. dependent fp64 FMA chain
  PIN(a); PIN(b); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N; ++i) a = fma(a, c, b);
  PIN(a); t1 = clk(); out[0] = t1 - t0;
  // 2. 4 independent fp64 FMA chains
  double a0 = a, a1 = a + 1, a2 = a + 2, a3 = a + 3;
  PIN(a0); PIN(a1); PIN(a2); PIN(a3); t0 = clk();
#pragma unroll
  for (int i = 0; i < N / 4; ++i) { a0 = fma(a0, c, b); a1 = fma(a1, c, b); a2 = fma(a2, c, b); a3 = fma(a3, c, b); }
  PIN(a0); PIN(a1); PIN(a2); PIN(a3); t1 = clk(); out[1] = t1 - t0; a = a0 + a1 + a2 + a3;
  // 3. dependent DPP (row_shr:1) + add chain
  PIN(a); PIN(b); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N; ++i) a = a + dpp64<0x111>(a);
  PIN(a); t1 = clk(); out[2] = t1 - t0;
  // 4. dependent ds_swizzle broadcast + add
  PIN(a); PIN(b); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(a), 0x18 | (3 << 5));
    const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(a), 0x18 | (3 << 5));
    a = a + __hiloint2double(hi, lo);
  }
  PIN(a); t1 = clk(); out[3] = (t1 - t0) * 4;
  // 5. dependent readlane broadcast + add
  PIN(a); PIN(b); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(a), 5);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(a), 5);
    a = a + __hiloint2double(hi, lo);
  }
  PIN(a); t1 = clk(); out[4] = (t1 - t0) * 4;
  // 6. dependent LDS store -> load round trip
  PIN(a); PIN(b); t0 = clk(); PIN(a);
#pragma unroll 1
  for (int i = 0; i < N / 4; ++i) {
    L[l] = a;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    a = a + L[(l + 1) & 63];
  }
  PIN(a); t1 = clk(); out[5] = (t1 - t0) * 4;
  // 7. dependent fp64 multiply-add with 2 inputs from the chain (x = x*x + b)
  PIN(a); PIN(b); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N; ++i) a = a * c + b;
  PIN(a); t1 = clk(); out[6] = t1 - t0;
  // 8. rsqrt_f64 dependent chain
  PIN(a); PIN(b); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) a = __builtin_amdgcn_rsq(a) + 1.0;
  PIN(a); t1 = clk(); out[7] = (t1 - t0) * 4;
  // 9. 8 independent DPP moves then adds (issue rate of dpp)
  double d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = a + j;
  for (int j = 0; j < 8; ++j) PIN(d[j]);
  t0 = clk();
  for (int j = 0; j < 8; ++j) PIN(d[j]);
#pragma unroll
  for (int i = 0; i < N / 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = dpp64<0x111>(d[j]);
  for (int j = 0; j < 8; ++j) PIN(d[j]);
  t1 = clk(); out[8] = t1 - t0;
  for (int j = 0; j < 8; ++j) a += d[j];
  // 10. fp64 division chain
  PIN(a); PIN(b); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N / 8; ++i) a = b / a + 1.0;
  PIN(a); t1 = clk(); out[9] = (t1 - t0) * 8;
  // 11. 8 independent fp64 FMA chains (issue rate)
  double e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = a + j;
  for (int j = 0; j < 8; ++j) PIN(e[j]);
  t0 = clk();
  for (int j = 0; j < 8; ++j) PIN(e[j]);
#pragma unroll
  for (int i = 0; i < N / 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = fma(e[j], c, b);
  for (int j = 0; j < 8; ++j) PIN(e[j]);
  t1 = clk(); out[10] = t1 - t0;
  for (int j = 0; j < 8; ++j) a += e[j];
  // 12. 8 independent 64-bit row_newbcast moves (issue rate of v_mov_b64_dpp)
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = a + j;
  for (int j = 0; j < 8; ++j) PIN(e[j]);
  t0 = clk();
  for (int j = 0; j < 8; ++j) PIN(e[j]);
#pragma unroll
  for (int i = 0; i < N / 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long long x = __builtin_bit_cast(long long, e[j]);
      const long long y = __builtin_amdgcn_update_dpp(x, x, 0x153, 0xf, 0xf, true);
      e[j] = __builtin_bit_cast(double, y);
    }
  for (int j = 0; j < 8; ++j) PIN(e[j]);
  t1 = clk(); out[11] = t1 - t0;
  for (int j = 0; j < 8; ++j) a += e[j];
  // 13. dependent row_newbcast + add
  PIN(a); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    const long long x = __builtin_bit_cast(long long, a);
    const long long y = __builtin_amdgcn_update_dpp(x, x, 0x153, 0xf, 0xf, true);
    a = a + __builtin_bit_cast(double, y);
  }
  PIN(a); t1 = clk(); out[12] = (t1 - t0) * 4;
  // 14. 8 independent v_cndmask-style selects on 64-bit values (per select)
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = a + j;
  for (int j = 0; j < 8; ++j) PIN(e[j]);
  const bool cond = (l & 1) != 0;
  t0 = clk();
  for (int j = 0; j < 8; ++j) PIN(e[j]);
#pragma unroll
  for (int i = 0; i < N / 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { e[j] = cond ? e[j] : b; PIN(e[j]); }
  t1 = clk(); out[13] = t1 - t0;
  for (int j = 0; j < 8; ++j) a += e[j];
  // 15. 8 independent fp64 adds (issue rate)
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = a + j;
  for (int j = 0; j < 8; ++j) PIN(e[j]);
  t0 = clk();
  for (int j = 0; j < 8; ++j) PIN(e[j]);
#pragma unroll
  for (int i = 0; i < N / 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = e[j] + b;
  for (int j = 0; j < 8; ++j) PIN(e[j]);
  t1 = clk(); out[14] = t1 - t0;
  for (int j = 0; j < 8; ++j) a += e[j];
  // 16. dependent g8_bc (two bank-masked newbcast moves) + add
  PIN(a); t0 = clk(); PIN(a);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    const long long x = __builtin_bit_cast(long long, a);
    const long long t = __builtin_amdgcn_mov_dpp(x, 0x158 + 3, 0xf, 0xC, false);
    const long long r = __builtin_amdgcn_update_dpp(t, x, 0x150 + 3, 0xf, 0x3, false);
    a = a + __builtin_bit_cast(double, r);
  }
  PIN(a); t1 = clk(); out[15] = (t1 - t0) * 4;
  sink[l] = a;
}
int main() {
  unsigned long long* o; double* s;
  hipMalloc(&o, 64 * 8); hipMalloc(&s, 64 * 8);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, s, 1.5);
    hipDeviceSynchronize();
  }
  unsigned long long h[16];
  hipMemcpy(h, o, 16 * 8, hipMemcpyDeviceToHost);
  const char* names[] = {"dep fma", "4 indep fma (per fma)", "dpp+add dep", "swizzle bcast+add dep", "readlane bcast+add dep",
                         "lds st/bar/ld round trip", "dep mul+add (2 ops)", "rsq+add dep", "indep dpp64 (per dpp64)", "div+add dep",
                         "8 indep fma (per fma)", "indep b64 newbcast (per op)", "newbcast+add dep", "select64 (per op)",
                         "8 indep add (per add)", "g8_bc+add dep"};
  for (int i = 0; i < 16; ++i) printf("%-28s %7.1f cycles per op\n", names[i], (double)h[i] / N);
  return 0;
}
