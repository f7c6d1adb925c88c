// ffddp_prof.hpp — development-only phase timers (compiled in with -DFFDDP_PHASE_PROF)
#pragma once
#include <hip/hip_runtime.h>
namespace ffddp {
#ifdef FFDDP_PHASE_PROF
// development instrumentation: per-phase shader-clock sums of instance 0
__device__ unsigned long long g_pp[48];  // 32..39: BoxQP split (boxqp_lanes, two-wave backward)
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
// BoxQP split: time per part and counts into pq[0..7] (nullptr: off)
#define BQ_T0() unsigned long long bq_t = (unsigned long long)__builtin_readcyclecounter()
#define BQ_ACC(k)                                                                  \
  do {                                                                             \
    if (pq) {                                                                      \
      const unsigned long long t_ = (unsigned long long)__builtin_readcyclecounter(); \
      pq[k] += t_ - bq_t;                                                          \
      bq_t = t_;                                                                   \
    }                                                                              \
  } while (0)
#define BQ_CNT(k)        \
  do {                   \
    if (pq) pq[k] += 1;  \
  } while (0)
#else
#define BQ_T0() (void)0
#define BQ_ACC(k) (void)0
#define BQ_CNT(k) (void)0
#define PP_INIT() (void)0
#define PP(k) (void)0
#define PP_FLUSH() (void)0
#define PP_FLUSH_AT(base) (void)0
#endif

}  // namespace ffddp
