// MEASUREMENT TOOL (not product code, not linked by anything else): fp64
// operation counts of the scalar C++ CPU baseline (oracle/cpu/ffddp_cpu.cpp:
// the product's node models compiled for the host + a sequential,
// Crocoddyl-style dense backward pass and line search) per solve phase.
//
// The whole translation unit is compiled with `double` replaced by a counting
// type, so every fp64 add / sub / mul / div / fma / sqrt the scalar
// implementation executes is tallied under the phase it runs in:
//   node      calc + calcDiff of one node (node_diff)
//   backward  the backward pass (per node of its t loop; the terminal
//             node's Vxx / Vx set-up is charged to the pass)
//   forward   the line search's rollout (per trial node)
// These are the useful (algorithmic) flops per unit that bench.py prices the
// GPU's time with (roofline.fp64.useful): one scalar instance, no SIMD lanes,
// no idle or duplicate lanes.  flops = add + sub + mul + div + 2 fma + sqrt.
// Driven by tools/flop_count.py (ctypes).
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>

namespace fc {
enum { ADD, MUL, DIV, FMA, SQRT, TRANS, NKIND };
constexpr int NPH = 4;  // other, node, backward, forward
unsigned long long g_cnt[NPH][NKIND];
unsigned long long g_units[NPH];
int g_ph = 0;

struct D {
  double v;
  D() = default;
  constexpr D(double x) : v(x) {}
  explicit operator double() const { return v; }
  explicit operator int() const { return (int)v; }
  explicit operator long long() const { return (long long)v; }
  explicit operator bool() const { return v != 0.0; }
};
static_assert(sizeof(D) == 8, "layout");
inline void tick(int k, unsigned long long n = 1) { g_cnt[g_ph][k] += n; }
inline D operator+(D a, D b) { tick(ADD); return D(a.v + b.v); }
inline D operator-(D a, D b) { tick(ADD); return D(a.v - b.v); }
inline D operator*(D a, D b) { tick(MUL); return D(a.v * b.v); }
inline D operator/(D a, D b) { tick(DIV); return D(a.v / b.v); }
inline D operator-(D a) { return D(-a.v); }
inline D operator+(D a) { return a; }
inline D& operator+=(D& a, D b) { tick(ADD); a.v += b.v; return a; }
inline D& operator-=(D& a, D b) { tick(ADD); a.v -= b.v; return a; }
inline D& operator*=(D& a, D b) { tick(MUL); a.v *= b.v; return a; }
inline D& operator/=(D& a, D b) { tick(DIV); a.v /= b.v; return a; }
inline bool operator<(D a, D b) { return a.v < b.v; }
inline bool operator>(D a, D b) { return a.v > b.v; }
inline bool operator<=(D a, D b) { return a.v <= b.v; }
inline bool operator>=(D a, D b) { return a.v >= b.v; }
inline bool operator==(D a, D b) { return a.v == b.v; }
inline bool operator!=(D a, D b) { return a.v != b.v; }
inline D fma(D a, D b, D c) { tick(FMA); return D(std::fma(a.v, b.v, c.v)); }
inline D sqrt(D a) { tick(SQRT); return D(std::sqrt(a.v)); }
inline D fabs(D a) { return D(std::fabs(a.v)); }
inline D rint(D a) { return D(std::rint(a.v)); }
struct PhaseScope {
  int prev;
  explicit PhaseScope(int p) : prev(g_ph) { g_ph = p; }
  ~PhaseScope() { g_ph = prev; }
};
}  // namespace fc

namespace std {
inline fc::D fma(fc::D a, fc::D b, fc::D c) { return fc::fma(a, b, c); }
inline fc::D sqrt(fc::D a) { return fc::sqrt(a); }
inline fc::D fabs(fc::D a) { return fc::fabs(a); }
inline fc::D sin(fc::D a) { fc::tick(fc::TRANS); return fc::D(std::sin(a.v)); }
inline fc::D cos(fc::D a) { fc::tick(fc::TRANS); return fc::D(std::cos(a.v)); }
inline bool isnan(fc::D a) { return std::isnan(a.v); }
inline bool isinf(fc::D a) { return std::isinf(a.v); }
inline fc::D min(fc::D a, fc::D b) { return b < a ? b : a; }
inline fc::D max(fc::D a, fc::D b) { return a < b ? b : a; }
}  // namespace std
using fc::fma;
using fc::sqrt;
using fc::fabs;

#define __builtin_rint(x) fc::rint(x)
#define FFDDP_CPU_PHASE_SCOPE(p) fc::PhaseScope fc_scope_(p)
#define FFDDP_CPU_UNIT(p) (++fc::g_units[p])
#define double fc::D
#include "../../oracle/cpu/ffddp_cpu.cpp"
#undef double

extern "C" {
// Solve B instances (ffddp_cpu_solve_batch's arguments, one thread) and
// return the counts: cnt[4][6] (phase x {add/sub, mul, div, fma, sqrt,
// transcendental}) and units[4] (phase: node stages, backward nodes, trial nodes).
int flop_count_solve(const void* robot, const void* cfg, int B, const double* x0, const double* node_ref,
                     const double* inst_ref, const uint8_t* surface, const double* xs_init, const double* us_init,
                     int maxiter, double* xs, double* us, double* K, double* cost, int32_t* iters, uint8_t* ok,
                     int32_t* stats, unsigned long long* cnt, unsigned long long* units) {
  std::memset(fc::g_cnt, 0, sizeof(fc::g_cnt));
  std::memset(fc::g_units, 0, sizeof(fc::g_units));
  using DD = fc::D;
  const int rc = ffddp_cpu_solve_batch((const ffddp_robot*)robot, (const ffddp_ocp_config*)cfg, B, (const DD*)x0,
                                       (const DD*)node_ref, (const DD*)inst_ref, surface, (const DD*)xs_init,
                                       (const DD*)us_init, maxiter, 0, (DD*)xs, (DD*)us, (DD*)K, (DD*)cost, iters, ok,
                                       stats, nullptr, 1);
  std::memcpy(cnt, fc::g_cnt, sizeof(fc::g_cnt));
  std::memcpy(units, fc::g_units, sizeof(fc::g_units));
  return rc;
}
}
