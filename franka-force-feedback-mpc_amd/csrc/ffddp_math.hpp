// ffddp_math.hpp — fixed-size fp64 algebra for the 7-DoF arm, generic over a
// scalar T in {double, Dual}.  Dual carries ONE forward-mode tangent: in the
// calcDiff kernel every lane of a 16-lane node group propagates a different
// state direction through the same primal code, so each lane produces one
// column of the analytic Jacobians (Pinocchio's computeRNEADerivatives /
// getFrame{Velocity,Acceleration}Derivatives, which the reference reaches via
// Crocoddyl, crocoddyl_classical.py:619, 722).
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#define FFD_HD __host__ __device__ __forceinline__

namespace ffddp {

struct Dual {
  double v, d;
};

FFD_HD Dual operator+(Dual a, Dual b) { return {a.v + b.v, a.d + b.d}; }
FFD_HD Dual operator-(Dual a, Dual b) { return {a.v - b.v, a.d - b.d}; }
FFD_HD Dual operator-(Dual a) { return {-a.v, -a.d}; }
FFD_HD Dual operator*(Dual a, Dual b) { return {a.v * b.v, a.v * b.d + a.d * b.v}; }
FFD_HD Dual operator*(double s, Dual a) { return {s * a.v, s * a.d}; }
FFD_HD Dual operator*(Dual a, double s) { return {s * a.v, s * a.d}; }
FFD_HD Dual operator+(Dual a, double s) { return {a.v + s, a.d}; }
FFD_HD Dual operator+(double s, Dual a) { return {a.v + s, a.d}; }
FFD_HD Dual operator-(Dual a, double s) { return {a.v - s, a.d}; }
FFD_HD Dual operator-(double s, Dual a) { return {s - a.v, -a.d}; }
FFD_HD Dual& operator+=(Dual& a, Dual b) { a.v += b.v; a.d += b.d; return a; }
FFD_HD Dual& operator-=(Dual& a, Dual b) { a.v -= b.v; a.d -= b.d; return a; }

FFD_HD double val(double x) { return x; }
FFD_HD double val(Dual x) { return x.v; }
FFD_HD double tng(double) { return 0.0; }
FFD_HD double tng(Dual x) { return x.d; }

template <class T> FFD_HD T mk(double v, double d);
template <> FFD_HD double mk<double>(double v, double) { return v; }
template <> FFD_HD Dual mk<Dual>(double v, double d) { return {v, d}; }

// ---------------------------------------------------------------------------
// Lean fp64 sin/cos and acos.  Every VALU op costs a wave 4 cycles, and on the
// latency-bound rollout chain the library versions (full-range Payne-Hanek
// reduction for sin/cos, several branches for acos) were ~20 % of the line
// search's instructions.  The arguments here are joint angles and rotation
// angles, so: Cody-Waite reduction by pi/2 with three FMA terms (the products
// are exact inside the FMAs, so the reduction stays accurate far beyond any
// joint or rotation angle; NaN and inf propagate to NaN as in the library),
// the fdlibm minimax kernels on [-pi/4, pi/4] (< 1 ulp) and fdlibm's rational
// acos, evaluated branch-free.  Max error vs libm: 2 ulp sin/cos, 1 ulp acos.
// ---------------------------------------------------------------------------
// Horner step a * b + k with the coefficient k in an SGPR pair: one
// v_fma_f64.  The compiler otherwise keeps the coefficients in VGPRs and
// emits v_fmac_f64 (accumulator tied to the addend) plus a v_mov_b64 copying
// the coefficient into the accumulator for every step.  Same single rounding
// as the contracted a * b + k.
FFD_HD double hfma(double a, double b, double k) {
#ifdef __HIP_DEVICE_COMPILE__
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
#else
  return a * b + k;  // host builds (oracle/cpu): the expression as written
#endif
}

FFD_HD void sincos_(double x, double& s, double& c) {
  const double n = __builtin_rint(x * 0.63661977236758134308);  // 2 / pi
  double y = fma(-n, 1.5707963267948966, x);                   // pi/2 in three parts
  y = fma(-n, 6.123233995736766e-17, y);
  y = fma(-n, -1.4973849048591698e-33, y);
  const double z = y * y;
  const double ps = hfma(z, hfma(z, hfma(z, hfma(z, hfma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                                   2.75573137070700676789e-06),
                                         -1.98412698298579493134e-04),
                               8.33333333332248946124e-03),
                     -1.66666666666666324348e-01);
  const double pc = hfma(z, hfma(z, hfma(z, hfma(z, hfma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                                   -2.75573143513906633035e-07),
                                         2.48015872894767294178e-05),
                               -1.38888888888741095749e-03),
                     4.16666666666666019037e-02);
  const double sp = fma(y * z, ps, y);
  const double cp = fma(z * z, pc, 1.0 - 0.5 * z);
  const int qd = (int)((long long)n & 3);
  s = (qd == 0) ? sp : ((qd == 1) ? cp : ((qd == 2) ? -sp : -cp));
  c = (qd == 0) ? cp : ((qd == 1) ? -sp : ((qd == 2) ? -cp : sp));
}

// acos on [-1, 1] (fdlibm e_acos.c's rational approximation of asin,
// branch-free: one P/Q for the three argument ranges)
FFD_HD double acos_(double x) {
  const double ax = fabs(x);
  const bool mid = ax < 0.5;
  const double z = mid ? x * x : (1.0 - ax) * 0.5;
  const double p = z * hfma(z, hfma(z, hfma(z, hfma(z, hfma(z, 3.47933107596021167570e-05, 7.91534994289814532176e-04),
                                                    -4.00555345006794114027e-02),
                                          2.01212532134862925881e-01),
                                -3.25565818622400915405e-01),
                      1.66666666666666657415e-01);
  const double q = hfma(z, hfma(z, hfma(z, hfma(z, 7.70381505559019352791e-02, -6.88283971605453293030e-01),
                                        2.02094576023350569471e+00),
                              -2.40339491173441421878e+00),
                    1.0);
  const double r = p / q;
  const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
  if (mid) return pio2_hi - (x - (pio2_lo - x * r));
  const double s = sqrt(z);
  if (x < 0.0) return 2.0 * pio2_hi - 2.0 * (s + (r * s - pio2_lo));
  return 2.0 * (s + r * s);
}
FFD_HD void sincos_(Dual q, Dual& s, Dual& c) {
  double sv, cv;
  sincos_(q.v, sv, cv);
  s = {sv, q.d * cv};
  c = {cv, -q.d * sv};
}

template <class T> struct V3 {
  T x, y, z;
};

template <class T> FFD_HD V3<T> operator+(V3<T> a, V3<T> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <class T> FFD_HD V3<T> operator-(V3<T> a, V3<T> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <class T> FFD_HD V3<T> operator*(T s, V3<T> a) { return {s * a.x, s * a.y, s * a.z}; }
template <class T> FFD_HD V3<T> scale(V3<T> a, double s) { return {a.x * s, a.y * s, a.z * s}; }
template <class T> FFD_HD V3<T> cross(V3<T> a, V3<T> b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <class T> FFD_HD T dot(V3<T> a, V3<T> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <class T> FFD_HD V3<T> v3zero() { return {T{}, T{}, T{}}; }
template <class T> FFD_HD V3<T> v3c(const double* p) {
  return {mk<T>(p[0], 0.0), mk<T>(p[1], 0.0), mk<T>(p[2], 0.0)};
}

// 3x3, row-major
template <class T> struct M3 {
  T m[9];
};
template <class T> FFD_HD M3<T> m3eye() {
  M3<T> r;
  for (int i = 0; i < 9; ++i) r.m[i] = mk<T>((i % 4 == 0) ? 1.0 : 0.0, 0.0);
  return r;
}
template <class T> FFD_HD V3<T> mul(const M3<T>& A, V3<T> x) {
  return {A.m[0] * x.x + A.m[1] * x.y + A.m[2] * x.z, A.m[3] * x.x + A.m[4] * x.y + A.m[5] * x.z,
          A.m[6] * x.x + A.m[7] * x.y + A.m[8] * x.z};
}
template <class T> FFD_HD V3<T> mulT(const M3<T>& A, V3<T> x) {
  return {A.m[0] * x.x + A.m[3] * x.y + A.m[6] * x.z, A.m[1] * x.x + A.m[4] * x.y + A.m[7] * x.z,
          A.m[2] * x.x + A.m[5] * x.y + A.m[8] * x.z};
}
// A (T) * B (double constant)
template <class T> FFD_HD M3<T> mulc(const M3<T>& A, const double* B) {
  M3<T> r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      r.m[3 * i + j] = A.m[3 * i + 0] * B[0 * 3 + j] + A.m[3 * i + 1] * B[1 * 3 + j] + A.m[3 * i + 2] * B[2 * 3 + j];
  return r;
}
template <class T> FFD_HD V3<T> mulc_v(const M3<T>& A, const double* p) {
  return {A.m[0] * p[0] + A.m[1] * p[1] + A.m[2] * p[2], A.m[3] * p[0] + A.m[4] * p[1] + A.m[5] * p[2],
          A.m[6] * p[0] + A.m[7] * p[1] + A.m[8] * p[2]};
}
// constant symmetric 3x3 (row-major, double) times vector
template <class T> FFD_HD V3<T> cmul(const double* I, V3<T> x) {
  return {I[0] * x.x + I[1] * x.y + I[2] * x.z, I[3] * x.x + I[4] * x.y + I[5] * x.z,
          I[6] * x.x + I[7] * x.y + I[8] * x.z};
}

// ---------------------------------------------------------------------------
// packed lower-triangular Cholesky (Eigen::LLT semantics: fail if pivot <= 0).
// Storage: off-diagonal L_ij (i > j) as usual, the DIAGONAL HOLDS 1 / L_ii so
// that the triangular solves multiply instead of divide (fp64 division is a
// ~10-instruction dependent sequence on CDNA; the solves sit on the critical
// path of every kernel).
// ---------------------------------------------------------------------------
FFD_HD int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// 1/sqrt(d) for d > 0: hardware estimate refined by two Newton steps (full
// double precision, within an ulp or so of the correctly rounded quotient)
// instead of a correctly rounded sqrt followed by a division; both are long
// dependent sequences on CDNA and sit on the critical path of every LLT.
FFD_HD double rsqrt_nr(double d) {
#ifdef __HIP_DEVICE_COMPILE__
  double y = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  y = y * (1.5 - h * y * y);
  y = y * (1.5 - h * y * y);
  return y;
#else
  return 1.0 / sqrt(d);
#endif
}

template <int N> FFD_HD bool chol_packed(double* A /* packed lower, in-place */) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double d = A[tri(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= A[tri(j, k)] * A[tri(j, k)];
    if (!(d > 0.0)) return false;
    const double il = rsqrt_nr(d);
    A[tri(j, j)] = il;
#pragma unroll
    for (int i = j + 1; i < N; ++i) {
      double s = A[tri(i, j)];
#pragma unroll
      for (int k = 0; k < j; ++k) s -= A[tri(i, k)] * A[tri(j, k)];
      A[tri(i, j)] = s * il;
    }
  }
  return true;
}
// solve L y = b in place
template <int N> FFD_HD void fwd_sub(const double* L, double* b) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= L[tri(i, k)] * b[k];
    b[i] = s * L[tri(i, i)];
  }
}
// solve L^T x = y in place
template <int N> FFD_HD void bwd_sub(const double* L, double* b) {
#pragma unroll
  for (int i = N - 1; i >= 0; --i) {
    double s = b[i];
#pragma unroll
    for (int k = i + 1; k < N; ++k) s -= L[tri(k, i)] * b[k];
    b[i] = s * L[tri(i, i)];
  }
}
template <int N> FFD_HD void chol_solve(const double* L, double* b) {
  fwd_sub<N>(L, b);
  bwd_sub<N>(L, b);
}

}  // namespace ffddp
