// ffddp_prof.hpp — development-only phase timers (compiled in with -DFFDDP_PHASE_PROF)
#pragma once
#include <hip/hip_runtime.h>
namespace ffddp {
#ifdef FFDDP_PHASE_PROF
// development instrumentation: per-phase shader-clock sums of instance 0
__device__ unsigned long long g_pp[32];
#define PP_INIT()                                                                       \
  unsigned long long pp_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};                \
  unsigned long long pp_last = (unsigned long long)__builtin_readcyclecounter()
#define PP(k)                                                                           \
  do {                                                                                  \
    const unsigned long long t_ = (unsigned long long)__builtin_readcyclecounter();      \
    pp_acc[k] += t_ - pp_last;                                                          \
    pp_last = t_;                                                                       \
  } while (0)
#define PP_FLUSH_AT(base)                                                               \
  do {                                                                                  \
    if (pp_on && (threadIdx.x & 63) == 0)                                               \
      for (int k_ = 0; k_ < 12; ++k_) g_pp[(base) + k_] += pp_acc[k_];                  \
  } while (0)
#define PP_FLUSH() PP_FLUSH_AT(0)
#else
#define PP_INIT() (void)0
#define PP(k) (void)0
#define PP_FLUSH() (void)0
#define PP_FLUSH_AT(base) (void)0
#endif

}  // namespace ffddp
