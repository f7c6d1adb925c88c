// ffddp_rollout.hpp — the line search's node calc (forward-pass primal,
// SolverFDDP::forwardPass -> IntegratedActionModelEuler::calc ->
// DifferentialActionModelContactFwdDynamics::calc) on an
// 8-lane group: lane i < 7 owns joint i, lane 7 the end-effector frame (the
// scans of ffddp_group.hpp).
//
// Two lane layouts run the same arithmetic:
//   ROW = false  two groups per 16-lane DPP row (lanes 0..7 and 8..15): the
//                throughput layout.  A group broadcast is two bank-masked
//                row_newbcast moves and the scans mask the lanes whose
//                source falls in the other group.
//   ROW = true   one group per DPP row (lanes 0..7; lanes 8..15 are a
//                phantom group with zero mass): the latency layout for passes
//                with few trials.  A broadcast is one row_newbcast move, and
//                the additive scans need no mask (a source outside the row
//                reads 0; the phantom lanes add exact zeros to the suffix
//                sums).
// Every product-sum in this file is written as explicit fma() under
// `fp contract(off)`, so the compiler cannot contract the two instantiations
// differently: both layouts give the same bits (up to the sign of a zero),
// and the layout can be chosen per pass without making an instance's result
// depend on its batch.  Same physics and cost stack as
// node_primal (ffddp_node.hpp); only the evaluation order differs.
#pragma once

#include "ffddp_group.hpp"

#pragma clang fp contract(off)

// the rollout's contact solve: one backward substitution through the Schur
// complement (1) or two solves (0)
#ifndef FFDDP_LS_SCHUR
#define FFDDP_LS_SCHUR 1
#endif

namespace ffddp {

// ---- the rollout's cost flags ----
// Read from DevConsts inside the node loop, each flag was re-loaded by a
// scalar load right before its branch (the scalar registers cannot hold every
// DevConsts value the loop reads) and waited for at once.  As one bit mask
// held in a scalar register for the whole kernel the branches need no load
// (9 fewer scalar-memory waits per node; line search at C5 -0.6 %).  The
// weights stay in DevConsts: staged in LDS they were hoisted out of the node
// loop into ~80 held registers (270 -> 356 per lane, so the wave no longer
// shares its SIMD with another stream's node or backward wave: B = 4096
// -3.5 %; still 314 when re-read per node).
enum : unsigned {
  RF_STATE = 1u,    // state regularisation (classical, or FF's inner_state_reg)
  RF_QSOFT = 2u,    // q soft limits
  RF_TAU = 4u,      // torque regularisation (classical, or FF's inner_tau_reg)
  RF_TSOFT = 8u,    // torque soft limits
  RF_PZ = 16u,      // plane-z cost in contact
  RF_VZ = 32u,      // normal-velocity cost in contact
  RF_FC = 64u,      // friction cone
  RF_UNI = 128u,    // unilateral force barrier
  RF_FN = 256u,     // normal-force tracking
  RF_BOX = 512u,    // control box clamp
};
__device__ __forceinline__ unsigned ls_flags(const DevConsts& C) {
  unsigned f = 0;
  f |= (C.variant == FFDDP_CLASSICAL || C.inner_state_reg) ? RF_STATE : 0u;
  f |= C.has_qsoft ? RF_QSOFT : 0u;
  f |= (C.variant == FFDDP_CLASSICAL || C.inner_tau_reg) ? RF_TAU : 0u;
  f |= C.has_tsoft ? RF_TSOFT : 0u;
  f |= C.has_pz ? RF_PZ : 0u;
  f |= C.has_vz ? RF_VZ : 0u;
  f |= C.has_fc ? RF_FC : 0u;
  f |= C.has_uni ? RF_UNI : 0u;
  f |= C.has_fn ? RF_FN : 0u;
  f |= C.use_box ? RF_BOX : 0u;
  asm volatile("" : "+s"(f));  // a register value from here on, not a re-loadable one
  return f;
}
// ---- scalar helpers, explicit fma ----
__device__ __forceinline__ double ls_dot3(double a0, double b0, double a1, double b1, double a2, double b2) {
  return fma(a2, b2, fma(a1, b1, a0 * b0));
}
__device__ __forceinline__ void ls_cross(const double* a, const double* b, double* c) {
  c[0] = fma(a[1], b[2], -(a[2] * b[1]));
  c[1] = fma(a[2], b[0], -(a[0] * b[2]));
  c[2] = fma(a[0], b[1], -(a[1] * b[0]));
}
__device__ __forceinline__ double ls_rsqrt(double d) {
  double y = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  y = y * fma(-(h * y), y, 1.5);
  y = y * fma(-(h * y), y, 1.5);
  return y;
}
// sincos_ / acos_ of ffddp_math.hpp (same kernels), explicit fma
__device__ __forceinline__ void ls_sincos(double x, double& s, double& c) {
  const double n = __builtin_rint(x * 0.63661977236758134308);
  double y = fma(-n, 1.5707963267948966, x);
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
  const double cp = fma(z * z, pc, fma(-0.5, z, 1.0));
  const int qd = (int)((long long)n & 3);
  s = (qd == 0) ? sp : ((qd == 1) ? cp : ((qd == 2) ? -sp : -cp));
  c = (qd == 0) ? cp : ((qd == 1) ? -sp : ((qd == 2) ? -cp : sp));
}
__device__ __forceinline__ double ls_acos(double x) {
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
  if (mid) return pio2_hi - (x - fma(-x, r, pio2_lo));
  const double s = sqrt(z);
  if (x < 0.0) return 2.0 * pio2_hi - 2.0 * (s + fma(r, s, -pio2_lo));
  return 2.0 * fma(r, s, s);
}
// log3 of ffddp_node.hpp (pinocchio::log3): angle and scaled axis
__device__ __forceinline__ void ls_log3(const double* R, double* r) {
  const double tr = R[0] + R[4] + R[8];
  double c = (tr - 1.0) / 2.0;
  c = c > 1.0 ? 1.0 : (c < -1.0 ? -1.0 : c);
  const double th = ls_acos(c);
  const double eps3 = 6.0554544523933395e-06;
  double st, ct;
  ls_sincos(th, st, ct);
  const double t = (th > eps3 ? th / st : 1.0) / 2.0;
  r[0] = t * (R[7] - R[5]);
  r[1] = t * (R[2] - R[6]);
  r[2] = t * (R[3] - R[1]);
}
// QuadraticBarrier cost value 1/2 |max(r - ub, 0)|^2 + 1/2 |min(r - lb, 0)|^2
__device__ __forceinline__ double ls_barrier(double r, double lb, double ub) {
  const double dl = r - lb, du = r - ub;
  const double rl = dl < 0.0 ? dl : 0.0;
  const double ru = du > 0.0 ? du : 0.0;
  return 0.5 * fma(ru, ru, rl * rl);
}
// friction-cone cost (ffddp_node.hpp friction_cone, value only)
__device__ __forceinline__ double ls_friction_cone(const DevConsts& C, const double* lam) {
  double c = 0.0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const double* A = C.fc_A[k];
    c += ls_barrier(ls_dot3(A[0], lam[0], A[1], lam[1], A[2], lam[2]), C.fc_lb[k], C.fc_ub[k]);
  }
  return C.w_fc * c;
}

// ---- group primitives per layout ----
template <bool ROW> __device__ __forceinline__ double ls_get(double v, int src) { return g8_get<ROW>(v, src); }
// prefix-scan step over n values: x += x[li - d] (lanes li < d keep x).
// SHARED: one exec-masked block (three scalar instructions for the block,
// not a select per value).  ROW: unmasked (a source outside the row reads 0).
template <bool ROW, int NV> __device__ __forceinline__ void ls_up_add(double (&x)[NV], int d, int li) {
  double t[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) t[k] = g8_up(x[k], d);
  if (ROW || li >= d) {
#pragma unroll
    for (int k = 0; k < NV; ++k) x[k] += t[k];
  }
}
// suffix-scan step: x += x[li + d] (lanes li + d >= 8 keep x; ROW: the
// phantom lanes 8..15 hold exact zeros)
template <bool ROW, int NV> __device__ __forceinline__ void ls_down_add(double (&x)[NV], int d, int li) {
  double t[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) t[k] = g8_down(x[k], d);
  if (ROW || li + d < G8) {
#pragma unroll
    for (int k = 0; k < NV; ++k) x[k] += t[k];
  }
}

// LLT with row i on group lane i (g8_chol_rows, explicit fma)
template <bool ROW> __device__ __forceinline__ void ls_chol_rows(double (&a)[NQ], int li) {
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    double d = a[k];
#pragma unroll
    for (int m = 0; m < k; ++m) d = fma(-a[m], a[m], d);
    const double il = ls_rsqrt(ls_get<ROW>(d, k));
    double s = a[k];
#pragma unroll
    for (int m = 0; m < k; ++m) s = fma(-a[m], ls_get<ROW>(a[m], k), s);
    a[k] = (li == k) ? il : ((li > k) ? s * il : a[k]);
  }
}
// L y = r (rows on lanes): y (group-uniform, all NQ entries)
template <bool ROW> __device__ __forceinline__ void ls_fwd(const double (&Lr)[NQ], double r, double (&y)[NQ]) {
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    double s = r;
#pragma unroll
    for (int m = 0; m < k; ++m) s = fma(-Lr[m], y[m], s);
    y[k] = ls_get<ROW>(s * Lr[k], k);
  }
}
// L^T x = y (y group-uniform): this lane's x
template <bool ROW> __device__ __forceinline__ double ls_bwd(const double (&Lt)[NQ][NQ], const double (&y)[NQ], int li) {
  double x[NQ];
#pragma unroll
  for (int k = NQ - 1; k >= 0; --k) {
    double s = y[k];
#pragma unroll
    for (int m = k + 1; m < NQ; ++m) s = fma(-Lt[k][m], x[m], s);
    x[k] = s * Lt[k][k];
  }
  double out = 0.0;
#pragma unroll
  for (int k = 0; k < NQ; ++k) out = (li == k) ? x[k] : out;
  return out;
}

// Inner node calc (DAM + Euler step) on an 8-lane group, explicit fma.
//   lane i < 7 inputs: q, v (joint i), u (inner control / tau), xq, xv (posture
//   reference), tr (torque reference);  ref: p_ref(3), v_ref(3) of the node.
//   outputs: qn, vn (joint i of the Euler step; x itself for MODE_TERMINAL_X),
//   cpart (this lane's share of the unscaled DAM cost: g8_sum gives the cost),
//   lam (contact force, group-uniform; zero in free mode).
// Contact: a = L^-T (y1 - Y lambda'), y1 = L^-1 (u - tau), Y = L^-1 Jc^T,
// lambda' = S^-1 (gamma + Y' y1), S = Y'Y + eps (the KKT of
// DifferentialActionModelContactFwdDynamics by its Schur complement; one
// backward substitution instead of two full solves).
template <int NC, bool ROW>
__device__ __forceinline__ void ls_node_calc(const DevConsts& C, unsigned fl, const LaneK& K, int mode, bool surface, double q,
                                             double v, double u, double xq, double xv, double tr, const double* ref,
                                             double& qn, double& vn, double& cpart, double (&lam)[3]
#ifdef FFDDP_PHASE_PROF
                                             , unsigned long long (&pp_acc)[12], unsigned long long& pp_last
#endif
) {
  const int li = g8_lane();
  const bool J = li < NQ;
  const bool with_dyn = mode != MODE_TERMINAL_X;
  const bool terminal = mode != MODE_RUNNING;
  if (!J) q = v = u = 0.0;

  // ---- forward kinematics: prefix scan of transforms ----
  double R[9], o[3];
  if (J) {
    double s, c;
    ls_sincos(q, s, c);
    const double* Jr = K.R;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      R[3 * r + 0] = fma(s, Jr[3 * r + 1], c * Jr[3 * r + 0]);
      R[3 * r + 1] = fma(-s, Jr[3 * r + 0], c * Jr[3 * r + 1]);
      R[3 * r + 2] = Jr[3 * r + 2];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = K.R[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) o[k] = K.p[k];
#pragma unroll
  for (int d = 1; d < G8; d <<= 1) {
    double Rp[9], op[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) Rp[k] = g8_up(R[k], d);
#pragma unroll
    for (int k = 0; k < 3; ++k) op[k] = g8_up(o[k], d);
    // composed on every lane.  SHARED: kept where the source lane is in the
    // group (a select per value).  ROW: a lane whose source is outside the
    // row reads 0 for every entry; composing with the identity instead gives
    // R and o back exactly, so only the three diagonal entries need the
    // select (the off-diagonal ones and the offset of the identity are 0)
    const bool take = li >= d;
    if (ROW) {
      Rp[0] = take ? Rp[0] : 1.0;
      Rp[4] = take ? Rp[4] : 1.0;
      Rp[8] = take ? Rp[8] : 1.0;
    }
    double Rn[9], on[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) Rn[3 * r + c] = ls_dot3(Rp[3 * r + 0], R[c], Rp[3 * r + 1], R[3 + c], Rp[3 * r + 2], R[6 + c]);
      on[r] = op[r] + ls_dot3(Rp[3 * r + 0], o[0], Rp[3 * r + 1], o[1], Rp[3 * r + 2], o[2]);
    }
    if (ROW) {
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = Rn[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) o[k] = on[k];
    } else {
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = take ? Rn[k] : R[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) o[k] = take ? on[k] : o[k];
    }
  }
  // joint axis (world) and spatial motion subspace S = (o x z, z)
  double z[3] = {J ? R[2] : 0.0, J ? R[5] : 0.0, J ? R[8] : 0.0};
  double Sv[3];
  ls_cross(o, z, Sv);
  PP(0);
  // ---- velocities: prefix sum of S qd ----
  const double Svq[3] = {Sv[0] * v, Sv[1] * v, Sv[2] * v};
  const double zq[3] = {z[0] * v, z[1] * v, z[2] * v};
  double vw[6] = {Svq[0], Svq[1], Svq[2], zq[0], zq[1], zq[2]};  // (vO, w)
#pragma unroll
  for (int d = 1; d < G8; d <<= 1) ls_up_add<ROW>(vw, d, li);
  const double vO[3] = {vw[0], vw[1], vw[2]}, w[3] = {vw[3], vw[4], vw[5]};
  // ---- bias accelerations (qdd = 0): prefix sum of V_i x (S_i qd_i) ----
  double aa[6];  // (aO, al)
  {
    double c1[3], c2[3], c3[3];
    ls_cross(w, Svq, c1);
    ls_cross(vO, zq, c2);
    ls_cross(w, zq, c3);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      aa[k] = c1[k] + c2[k];
      aa[3 + k] = c3[k];
    }
  }
#pragma unroll
  for (int d = 1; d < G8; d <<= 1) ls_up_add<ROW>(aa, d, li);
  const double aO[3] = {aa[0], aa[1], aa[2]}, al[3] = {aa[3], aa[4], aa[5]};
  PP(1);
  // ---- end-effector frame (lane 7 holds it after the scans) ----
  double pee[3], vp[3], wee[3], ap[3], Ree[9];
  {
    double vpl[3], apl[3], c1[3], c2[3];
    ls_cross(w, o, c1);  // w x p  (lane 7: o = p_ee)
#pragma unroll
    for (int k = 0; k < 3; ++k) vpl[k] = vO[k] + c1[k];
    ls_cross(al, o, c1);
    ls_cross(w, vpl, c2);
#pragma unroll
    for (int k = 0; k < 3; ++k) apl[k] = aO[k] + (c1[k] + c2[k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pee[k] = ls_get<ROW>(o[k], 7);
      vp[k] = ls_get<ROW>(vpl[k], 7);
      wee[k] = ls_get<ROW>(w[k], 7);
      ap[k] = ls_get<ROW>(apl[k], 7);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) Ree[k] = ls_get<ROW>(R[k], 7);
  }
  PP(2);
  // ---- costs that do not depend on the dynamics (group-uniform operands) ----
  double cee;  // EE cost except the contact-force terms (uniform in the group)
  {
    double Rrel[9], rr[3];
#pragma unroll
    for (int a_ = 0; a_ < 3; ++a_)
#pragma unroll
      for (int b_ = 0; b_ < 3; ++b_)
        Rrel[3 * a_ + b_] = ls_dot3(C.Rdes[0 * 3 + a_], Ree[0 * 3 + b_], C.Rdes[1 * 3 + a_], Ree[1 * 3 + b_],
                                    C.Rdes[2 * 3 + a_], Ree[2 * 3 + b_]);
    ls_log3(Rrel, rr);
    cee = C.w_ori * (0.5 * ls_dot3(C.ori_w[0] * rr[0], rr[0], C.ori_w[1] * rr[1], rr[1], C.ori_w[2] * rr[2], rr[2]));
    cee = fma(C.w_wd, 0.5 * ls_dot3(C.wd_w[0] * wee[0], wee[0], C.wd_w[1] * wee[1], wee[1], C.wd_w[2] * wee[2], wee[2]),
              cee);
    const double rx = pee[0] - ref[0], ry = pee[1] - ref[1], rz = pee[2] - ref[2];
    const double cfree =
        C.w_ee_pos * (0.5 * ls_dot3(C.ee_pos_w[0] * rx, rx, C.ee_pos_w[1] * ry, ry, C.ee_pos_w[2] * rz, rz));
    const double vx = vp[0] - ref[3], vy = vp[1] - ref[4];
    double ccon = fma(C.w_tv, 0.5 * fma(vy, vy, vx * vx), C.w_tp * (0.5 * fma(ry, ry, rx * rx)));
    if (fl & RF_PZ) {
      const double pz = pee[2] - (ref[2] - C.z_press);
      ccon = fma(C.w_pz, 0.5 * (pz * pz), ccon);
    }
    if (fl & RF_VZ) ccon = fma(C.w_vz, 0.5 * (vp[2] * vp[2]), ccon);
    cee += surface ? ccon : cfree;
  }
  double cj = 0.0;  // this joint's state / control costs
  if (J) {
    if (fl & RF_STATE) {
      const double rq = q - xq, rv = v - xv;
      cj = C.w_post * (0.5 * fma(rv, rv, rq * rq));
      cj = fma(C.w_v, 0.5 * ((K.vdw * v) * v), cj);
    }
    if (fl & RF_QSOFT) cj = fma(C.w_qs, ls_barrier(q - K.qsx, K.qslb, K.qsub), cj);
    if (!terminal && (fl & RF_TAU)) {
      const double r = u - tr;
      cj = fma(C.w_tau, 0.5 * (r * r), cj);
      if (fl & RF_TSOFT) cj = fma(C.w_ts, ls_barrier(u, K.tslb, K.tsub), cj);
    }
  }
  lam[0] = lam[1] = lam[2] = 0.0;
  double a = 0.0;
  if (with_dyn) {
    // ---- link forces (RNEA, qdd = 0) and CRBA tuples ----
    // every lane, unmasked: lane 7 (the EE frame) and the ROW layout's
    // phantom lanes have zero mass and inertia in LaneK, so their link force
    // and CRBA tuple come out zero
    double sf[16];  // suffix-summed tuple: fl(3) fa(3) th(3) tI(6) tm
    {
      const double m = K.m;
      const double* Ic = K.I;
      double cw[3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
        cw[r] = o[r] + ls_dot3(R[3 * r + 0], K.com[0], R[3 * r + 1], K.com[1], R[3 * r + 2], K.com[2]);
      // world inertia Iw = R Ic R^T (symmetric: six entries)
      double IcR[9], Iw[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          IcR[3 * r + c] = ls_dot3(Ic[3 * r + 0], R[3 * c + 0], Ic[3 * r + 1], R[3 * c + 1], Ic[3 * r + 2], R[3 * c + 2]);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = r; c < 3; ++c) {
          Iw[3 * r + c] = ls_dot3(R[3 * r + 0], IcR[0 * 3 + c], R[3 * r + 1], IcR[1 * 3 + c], R[3 * r + 2], IcR[2 * 3 + c]);
          Iw[3 * c + r] = Iw[3 * r + c];
        }
      double Iww[3], Ial[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        Iww[r] = ls_dot3(Iw[3 * r + 0], w[0], Iw[3 * r + 1], w[1], Iw[3 * r + 2], w[2]);
        Ial[r] = ls_dot3(Iw[3 * r + 0], al[0], Iw[3 * r + 1], al[1], Iw[3 * r + 2], al[2]);
      }
      double t1[3], hl[3], ha[3], f1[3], n1[3];
      ls_cross(cw, w, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) hl[k] = m * (vO[k] - t1[k]);
      ls_cross(cw, hl, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) ha[k] = t1[k] + Iww[k];
      ls_cross(cw, al, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) f1[k] = m * ((aO[k] - C.rb.gravity[k]) - t1[k]);
      ls_cross(cw, f1, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) n1[k] = t1[k] + Ial[k];
      double c1[3], c2[3], c3[3];
      ls_cross(w, hl, c1);
      ls_cross(w, ha, c2);
      ls_cross(vO, hl, c3);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        sf[k] = f1[k] + c1[k];
        sf[3 + k] = n1[k] + (c2[k] + c3[k]);
      }
      const double mc[3] = {m * cw[0], m * cw[1], m * cw[2]};
      const double c2n = ls_dot3(cw[0], cw[0], cw[1], cw[1], cw[2], cw[2]);
      sf[6] = mc[0];
      sf[7] = mc[1];
      sf[8] = mc[2];
      sf[9] = fma(m, c2n, fma(-mc[0], cw[0], Iw[0]));
      sf[10] = fma(-mc[0], cw[1], Iw[1]);
      sf[11] = fma(-mc[0], cw[2], Iw[2]);
      sf[12] = fma(m, c2n, fma(-mc[1], cw[1], Iw[4]));
      sf[13] = fma(-mc[1], cw[2], Iw[5]);
      sf[14] = fma(m, c2n, fma(-mc[2], cw[2], Iw[8]));
      sf[15] = m;
    }
    // suffix sums (lane 7 and the phantom lanes contribute zero)
#pragma unroll
    for (int d = 1; d < G8; d <<= 1) ls_down_add<ROW>(sf, d, li);
    const double fl[3] = {sf[0], sf[1], sf[2]}, fa[3] = {sf[3], sf[4], sf[5]}, th[3] = {sf[6], sf[7], sf[8]};
    const double tI[6] = {sf[9], sf[10], sf[11], sf[12], sf[13], sf[14]}, tm = sf[15];
    const double tau = fma(z[2], fa[2], fma(z[1], fa[1], fma(z[0], fa[0], ls_dot3(Sv[0], fl[0], Sv[1], fl[1], Sv[2], fl[2]))));
    PP(3);
    // CRBA column: F = Ic_j S_j ; M[k][j] = S_k . F  (k <= j), row j of the lower triangle on lane j
    double Fl[3], Fa[3];
    {
      double hz[3], hs[3];
      ls_cross(th, z, hz);
      ls_cross(th, Sv, hs);
#pragma unroll
      for (int k = 0; k < 3; ++k) Fl[k] = fma(tm, Sv[k], -hz[k]);
      Fa[0] = hs[0] + ls_dot3(tI[0], z[0], tI[1], z[1], tI[2], z[2]);
      Fa[1] = hs[1] + ls_dot3(tI[1], z[0], tI[3], z[1], tI[4], z[2]);
      Fa[2] = hs[2] + ls_dot3(tI[2], z[0], tI[4], z[1], tI[5], z[2]);
    }
    double Lr[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const double sx = ls_get<ROW>(Sv[0], k), sy = ls_get<ROW>(Sv[1], k), sz = ls_get<ROW>(Sv[2], k);
      const double zx = ls_get<ROW>(z[0], k), zy = ls_get<ROW>(z[1], k), zz = ls_get<ROW>(z[2], k);
      const double mkj = fma(zz, Fa[2], fma(zy, Fa[1], fma(zx, Fa[0], ls_dot3(sx, Fl[0], sy, Fl[1], sz, Fl[2]))));
      Lr[k] = (k <= li) ? mkj : (li == k ? 1.0 : 0.0);
    }
    if (!J) {
#pragma unroll
      for (int k = 0; k < NQ; ++k) Lr[k] = 0.0;
    }
    PP(4);
    ls_chol_rows<ROW>(Lr, li);
    // L^T by rows, group-uniform: Lt[k][m] = L[m][k] (m >= k) from lane m
    double Lt[NQ][NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k)
#pragma unroll
      for (int m = k; m < NQ; ++m) Lt[k][m] = ls_get<ROW>(Lr[k], m);
    double y1[NQ];
    ls_fwd<ROW>(Lr, u - tau, y1);
    PP(5);
    if (surface) {
      constexpr int c0 = NC == 1 ? 2 : 0;
      const double pstar[3] = {ref[0], ref[1], ref[2] - C.z_press};
      double rel[3] = {pee[0] - o[0], pee[1] - o[1], pee[2] - o[2]};
      double jcol[3];
      ls_cross(z, rel, jcol);  // z_i x (p - o_i): LWA linear Jacobian column i
      double Y[3][NQ], gam[3];
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        const double Jc = J ? jcol[c0 + r] : 0.0;
        gam[r] = fma(C.Kd, vp[c0 + r], fma(C.Kp, pee[c0 + r] - pstar[c0 + r], ap[c0 + r]));
        ls_fwd<ROW>(Lr, Jc, Y[r]);
      }
      // S = Y'Y + eps I and yl = gamma + Y'y1 from the group-uniform
      // forward solutions (no cross-lane sums)
      double S[6], yl[3];
#pragma unroll
      for (int r = 0; r < NC; ++r) {
#pragma unroll
        for (int s2 = 0; s2 <= r; ++s2) {
          double acc = Y[r][0] * Y[s2][0];
#pragma unroll
          for (int k = 1; k < NQ; ++k) acc = fma(Y[r][k], Y[s2][k], acc);
          S[tri(r, s2)] = acc + (r == s2 ? C.eps : 0.0);
        }
        double acc = Y[r][0] * y1[0];
#pragma unroll
        for (int k = 1; k < NQ; ++k) acc = fma(Y[r][k], y1[k], acc);
        yl[r] = gam[r] + acc;
      }
      // chol_packed / chol_solve<NC> of ffddp_math.hpp, explicit fma
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        double dd = S[tri(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) dd = fma(-S[tri(j, k)], S[tri(j, k)], dd);
        const double il = ls_rsqrt(dd);
        S[tri(j, j)] = il;
#pragma unroll
        for (int i = j + 1; i < NC; ++i) {
          double s = S[tri(i, j)];
#pragma unroll
          for (int k = 0; k < j; ++k) s = fma(-S[tri(i, k)], S[tri(j, k)], s);
          S[tri(i, j)] = s * il;
        }
      }
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        double s = yl[i];
#pragma unroll
        for (int k = 0; k < i; ++k) s = fma(-S[tri(i, k)], yl[k], s);
        yl[i] = s * S[tri(i, i)];
      }
#pragma unroll
      for (int i = NC - 1; i >= 0; --i) {
        double s = yl[i];
#pragma unroll
        for (int k = i + 1; k < NC; ++k) s = fma(-S[tri(k, i)], yl[k], s);
        yl[i] = s * S[tri(i, i)];
      }
#if FFDDP_LS_SCHUR
      // a = L^-T (y1 - Y yl), lambda = -yl
      double y2[NQ];
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        double s = y1[k];
#pragma unroll
        for (int r = 0; r < NC; ++r) s = fma(-Y[r][k], yl[r], s);
        y2[k] = s;
      }
      a = ls_bwd<ROW>(Lt, y2, li);
#else
      // two solves: a = L^-T y1 + M^-1 Jc^T (-yl)
      double rhs = 0.0;
#pragma unroll
      for (int r = 0; r < NC; ++r) rhs = fma(J ? jcol[c0 + r] : 0.0, -yl[r], rhs);
      double y3[NQ];
      ls_fwd<ROW>(Lr, rhs, y3);
      a = ls_bwd<ROW>(Lt, y1, li) + ls_bwd<ROW>(Lt, y3, li);
#endif
#pragma unroll
      for (int r = 0; r < NC; ++r) lam[r] = -yl[r];
    } else {
      a = ls_bwd<ROW>(Lt, y1, li);
    }
  }
  PP(6);
  // ---- Euler step ----
  if (with_dyn) {
    const double dt = C.dt;
    qn = q + fma(a * dt, dt, v * dt);
    vn = fma(a, dt, v);
  } else {
    qn = q;
    vn = v;
  }
  // ---- contact-force costs (need lambda), then this lane's share ----
  double cf = 0.0;
  if (surface) {
    double lm[3] = {0, 0, 0};
    if (mode != MODE_TERMINAL_X)
#pragma unroll
      for (int r = 0; r < NC; ++r) lm[r] = lam[r];
    if (NC == 3 && (fl & RF_FC)) cf += ls_friction_cone(C, lm);
    if (fl & RF_UNI) {
#pragma unroll
      for (int r = 0; r < NC; ++r) cf = fma(C.w_uni, ls_barrier(lm[r], C.uni_lb[r], C.uni_ub[r]), cf);
    }
    if (fl & RF_FN) {
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        const double e = lm[r] - C.fn_ref[r];
        cf = fma(C.w_fn, 0.5 * ((C.fn_w[r] * e) * e), cf);
      }
    }
  }
  const double c = J ? cj : cee + cf;
  cpart = c;
  PP(7);
}

}  // namespace ffddp

#pragma clang fp contract(fast)
