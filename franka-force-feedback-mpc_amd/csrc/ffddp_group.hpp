// ffddp_group.hpp — the node calc (forward-pass primal) spread over an
// 8-lane group: lane i < 7 owns joint i, lane 7 owns the end-effector frame.
//
// The serial chains of the rigid-body algorithms become log-depth scans:
//   * forward kinematics  = inclusive prefix scan of joint transforms
//     (R, o)_i = (R, o)_{i-1} o (R_joint Rz(q_i), p_joint)  (lane 7: EE offset)
//   * spatial velocity    = prefix sum of S_i qd_i
//   * bias acceleration   = prefix sum of V_i x (S_i qd_i)
//   * RNEA torques        = suffix sum of link forces, tau_i = S_i . F_i
//   * CRBA                = suffix sum of (m, m c, I_O) tuples, M_ij = S_i . (Ic_j S_j)
//   * LLT of M / solves   = one row per lane (chol_rows layout)
// so one rollout step of a line-search trial costs ~log2(8) dependent
// exchange steps per stage instead of 7 serial joint steps on one lane.
// Same physics and cost stack as node_primal (ffddp_node.hpp); only the
// evaluation order (hence rounding) differs.
#pragma once

#include "ffddp_node.hpp"
#include "ffddp_prof.hpp"

namespace ffddp {

constexpr int G8 = 8;

__device__ __forceinline__ int g8_lane() { return (int)(threadIdx.x & 7); }

// Cross-lane moves inside the 8-lane group without going through LDS:
// DPP row_shr / row_shl for the scans (groups are 8-aligned inside 16-lane
// DPP rows; lanes whose source falls outside the group are masked by the
// callers), DPP row_newbcast for broadcasts, DPP half-mirror and quad
// permutes for the sums.
// bound_ctrl: a lane whose source is outside the row reads 0 (what the scans
// need), and no "old" operand has to be zeroed first: one v_mov_b32_dpp per
// 32-bit half and nothing else (with update_dpp(0, ...) every move also cost
// two v_mov_b32 of the zero old value; a VALU op is 4 cycles of the wave
// either way, so those were a third of every scan step)
template <int CTRL> __device__ __forceinline__ double dpp64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
template <int CTRL> __device__ __forceinline__ int dpp32(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, true);
}
// Broadcast of group lane K: row_newbcast of lane K and of lane 8 + K under
// bank masks (one v_mov_b64_dpp each: both 8-lane groups of the 16-lane DPP
// row get their own lane K).  Measured faster in the line search than
// ds_swizzle BROADCAST(8, K) through the LDS pipe, and than four 32-bit
// quad_perm / row_shr moves (negative results).
template <int K> __device__ __forceinline__ double g8_rowb(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const long long r = __builtin_amdgcn_update_dpp(x, x, 0x150 + K, 0xf, 0xf, true);
  return __builtin_bit_cast(double, r);
}
template <int K> __device__ __forceinline__ double g8_bc(double v) {
  // row_newbcast of lane 8 + K into banks 2-3 (lanes 8..15), then of lane K
  // into banks 0-1 (lanes 0..7) of the same register: two v_mov_b64_dpp, no select
  const long long x = __builtin_bit_cast(long long, v);
  const long long t = __builtin_amdgcn_mov_dpp(x, 0x158 + K, 0xf, 0xC, false);
  const long long r = __builtin_amdgcn_update_dpp(t, x, 0x150 + K, 0xf, 0x3, false);
  return __builtin_bit_cast(double, r);
}
// ROW: the group is lanes 0..7 of a 16-lane DPP row whose lanes 8..15 do
// not take part (k_node's calc): one row_newbcast move per broadcast
template <bool ROW = false> __device__ __forceinline__ double g8_get(double v, int src) {
  if (ROW) {
    switch (src) {
      case 0: return g8_rowb<0>(v);
      case 1: return g8_rowb<1>(v);
      case 2: return g8_rowb<2>(v);
      case 3: return g8_rowb<3>(v);
      case 4: return g8_rowb<4>(v);
      case 5: return g8_rowb<5>(v);
      case 6: return g8_rowb<6>(v);
      default: return g8_rowb<7>(v);
    }
  }
  switch (src) {
    case 0: return g8_bc<0>(v);
    case 1: return g8_bc<1>(v);
    case 2: return g8_bc<2>(v);
    case 3: return g8_bc<3>(v);
    case 4: return g8_bc<4>(v);
    case 5: return g8_bc<5>(v);
    case 6: return g8_bc<6>(v);
    default: return g8_bc<7>(v);
  }
}
__device__ __forceinline__ double g8_up(double v, int d) {
  return d == 1 ? dpp64<0x111>(v) : (d == 2 ? dpp64<0x112>(v) : dpp64<0x114>(v));
}
__device__ __forceinline__ double g8_down(double v, int d) {
  return d == 1 ? dpp64<0x101>(v) : (d == 2 ? dpp64<0x102>(v) : dpp64<0x104>(v));
}
__device__ __forceinline__ double g8_sum(double v) {
  v += dpp64<0x141>(v);  // row_half_mirror: lane i <-> 7 - i
  v += dpp64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp64<0x4E>(v);   // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ int g8_or(int v) {
  v |= dpp32<0x141>(v);
  v |= dpp32<0xB1>(v);
  v |= dpp32<0x4E>(v);
  return v;
}

// LLT with row i on group lane i (lanes 0..6); reciprocal diagonal as in chol_packed
template <bool ROW = false> __device__ __forceinline__ void g8_chol_rows(double (&a)[NQ], int li) {
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    double d = a[k];
#pragma unroll
    for (int m = 0; m < k; ++m) d -= a[m] * a[m];
    const double il = rsqrt_nr(g8_get<ROW>(d, k));
    double s = a[k];
#pragma unroll
    for (int m = 0; m < k; ++m) s -= a[m] * g8_get<ROW>(a[m], k);
    a[k] = (li == k) ? il : ((li > k) ? s * il : a[k]);
  }
}

// forward substitution L y = r (row layout), result per lane
template <bool ROW = false> __device__ __forceinline__ double g8_fwd(const double (&Lr)[NQ], double r, int li) {
  double y[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    double s = r;
#pragma unroll
    for (int m = 0; m < k; ++m) s -= Lr[m] * y[m];
    y[k] = g8_get<ROW>(s * Lr[k], k);
  }
  double out = 0.0;
#pragma unroll
  for (int k = 0; k < NQ; ++k) out = (li == k) ? y[k] : out;
  return out;
}

// L L^T x = r (row layout)
template <bool ROW = false> __device__ __forceinline__ double g8_solve(const double (&Lr)[NQ], double r, int li) {
  double y[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    double s = r;
#pragma unroll
    for (int m = 0; m < k; ++m) s -= Lr[m] * y[m];
    y[k] = g8_get<ROW>(s * Lr[k], k);
  }
  double x[NQ];
#pragma unroll
  for (int k = NQ - 1; k >= 0; --k) {
    double s = y[k];
#pragma unroll
    for (int m = k + 1; m < NQ; ++m) s -= g8_get<ROW>(Lr[k], m) * x[m];
    x[k] = s * g8_get<ROW>(Lr[k], k);
  }
  double out = 0.0;
#pragma unroll
  for (int k = 0; k < NQ; ++k) out = (li == k) ? x[k] : out;
  return out;
}

// Per-lane (joint) constants of the group calc, staged once per block in LDS
// (lane 7: the end-effector offset in R / p, zero inertia).  Read from the
// constant struct with lane-indexed addresses they were vector-memory loads
// inside the rollout's node loop, and since vmcnt counts loads and stores
// together every such load also waited for the next node's prefetch and the
// trial's stores.
struct LaneK {
  double R[9], p[3], com[3], I[9];
  double m, vdw, qsx, qslb, qsub, tslb, tsub, ulb, uub, wy2q, wy2v, wy2t, wslim;
};

// lane li < 8 of the block fills LK[li]; the caller synchronises
__device__ __forceinline__ void lane_consts_fill(const DevConsts& C, LaneK* LK, int li) {
  if (li >= G8) return;
  const ffddp_robot& rb = C.rb;
  LaneK& k = LK[li];
  const bool J = li < NQ;
  const int j = J ? li : NQ - 1;
  for (int e = 0; e < 9; ++e) {
    k.R[e] = J ? rb.joint_R[j][e] : rb.ee_R[e];
    k.I[e] = J ? rb.inertia[j][e] : 0.0;
  }
  for (int e = 0; e < 3; ++e) {
    k.p[e] = J ? rb.joint_p[j][e] : rb.ee_p[e];
    k.com[e] = J ? rb.com[j][e] : 0.0;
  }
  k.m = J ? rb.mass[j] : 0.0;
  k.vdw = C.vdw[j];
  k.qsx = C.qs_xref[j];
  k.qslb = C.qs_lb[j];
  k.qsub = C.qs_ub[j];
  k.tslb = C.ts_lb[j];
  k.tsub = C.ts_ub[j];
  k.ulb = C.u_lb[j];
  k.uub = C.u_ub[j];
  k.wy2q = C.Wy2[j];
  k.wy2v = C.Wy2[7 + j];
  k.wy2t = C.Wy2[14 + j];
  k.wslim = C.ws_lim[j];
}

// ROW line-search layout (ffddp_rollout.hpp): lanes 8..15 of the block fill
// LK[8..15], the phantom group of each DPP row: the joint frames of lanes
// 0..7 (finite kinematics) with zero mass, inertia and centre of mass, so its
// link forces and CRBA tuples are exact zeros in the real group's suffix sums
__device__ __forceinline__ void lane_consts_fill_phantom(const DevConsts& C, LaneK* LK, int li16) {
  if (li16 < G8 || li16 >= 2 * G8) return;
  lane_consts_fill(C, LK + G8, li16 - G8);
  LaneK& k = LK[li16];
  k.m = 0.0;
  for (int e = 0; e < 9; ++e) k.I[e] = 0.0;
  for (int e = 0; e < 3; ++e) k.com[e] = 0.0;
}

__device__ __forceinline__ void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// Inner node calc (DAM + Euler step) on an 8-lane group.
//   lane i < 7 inputs: q, v (joint i), u (inner control / tau), xq, xv (posture
//   reference), tr (torque reference);  ref: p_ref(3), v_ref(3) of the node.
//   outputs: qn, vn (joint i of the Euler step; x itself for MODE_TERMINAL_X),
//   cpart (this lane's share of the unscaled DAM cost: g8_sum gives P.cost),
//   lam (contact force, group-uniform; zero in free mode).
template <int NC>
__device__ __forceinline__ void node_calc_g8(const DevConsts& C, const LaneK& K, int mode, bool surface, double q,
                                             double v, double u, double xq, double xv, double tr, const double* ref,
                                             double& qn, double& vn, double& cpart, double (&lam)[3]
#ifdef FFDDP_PHASE_PROF
                                             , unsigned long long (&pp_acc)[12], unsigned long long& pp_last
#endif
) {
  const ffddp_robot& rb = C.rb;
  const int li = g8_lane();
  const bool J = li < NQ;
  const int ji = J ? li : NQ - 1;  // clamped joint index for parameter loads
  const bool with_dyn = mode != MODE_TERMINAL_X;
  const bool terminal = mode != MODE_RUNNING;
  if (!J) q = v = u = 0.0;

  // ---- forward kinematics: prefix scan of transforms ----
  double R[9], o[3];
  if (J) {
    double s, c;
    sincos_(q, s, c);
    const double* Jr = K.R;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      R[3 * r + 0] = c * Jr[3 * r + 0] + s * Jr[3 * r + 1];
      R[3 * r + 1] = c * Jr[3 * r + 1] - s * Jr[3 * r + 0];
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
    // composed on every lane, kept where the source lane is in the group: a
    // select per value instead of an exec-masked block, whose results the
    // compiler copied out of and back into the loop-carried registers
    // (two moves per value and step)
    const bool take = li >= d;
    double Rn[9], on[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) Rn[3 * r + c] = Rp[3 * r + 0] * R[c] + Rp[3 * r + 1] * R[3 + c] + Rp[3 * r + 2] * R[6 + c];
      on[r] = op[r] + (Rp[3 * r + 0] * o[0] + Rp[3 * r + 1] * o[1] + Rp[3 * r + 2] * o[2]);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = take ? Rn[k] : R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) o[k] = take ? on[k] : o[k];
  }
  // joint axis (world) and spatial motion subspace S = (o x z, z)
  double z[3] = {J ? R[2] : 0.0, J ? R[5] : 0.0, J ? R[8] : 0.0};
  double Sv[3];
  cross3(o, z, Sv);
  PP(0);
  // ---- velocities: prefix sum of S qd ----
  const double Svq[3] = {Sv[0] * v, Sv[1] * v, Sv[2] * v};
  const double zq[3] = {z[0] * v, z[1] * v, z[2] * v};
  double vO[3] = {Svq[0], Svq[1], Svq[2]}, w[3] = {zq[0], zq[1], zq[2]};
#pragma unroll
  for (int d = 1; d < G8; d <<= 1) {
    double t[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      t[k] = g8_up(vO[k], d);
      t[3 + k] = g8_up(w[k], d);
    }
    if (li >= d) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        vO[k] += t[k];
        w[k] += t[3 + k];
      }
    }
  }
  // ---- bias accelerations (qdd = 0): prefix sum of V_i x (S_i qd_i) ----
  double aO[3], al[3];
  {
    double c1[3], c2[3], c3[3];
    cross3(w, Svq, c1);
    cross3(vO, zq, c2);
    cross3(w, zq, c3);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      aO[k] = c1[k] + c2[k];
      al[k] = c3[k];
    }
  }
#pragma unroll
  for (int d = 1; d < G8; d <<= 1) {
    double t[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      t[k] = g8_up(aO[k], d);
      t[3 + k] = g8_up(al[k], d);
    }
    if (li >= d) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        aO[k] += t[k];
        al[k] += t[3 + k];
      }
    }
  }
  PP(1);
  // ---- end-effector frame (lane 7 holds it after the scans) ----
  double pee[3], vp[3], wee[3], ap[3], Ree[9];
  {
    double vpl[3], apl[3], c1[3], c2[3];
    cross3(w, o, c1);  // w x p  (lane 7: o = p_ee)
#pragma unroll
    for (int k = 0; k < 3; ++k) vpl[k] = vO[k] + c1[k];
    cross3(al, o, c1);
    cross3(w, vpl, c2);
#pragma unroll
    for (int k = 0; k < 3; ++k) apl[k] = aO[k] + c1[k] + c2[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pee[k] = g8_get(o[k], 7);
      vp[k] = g8_get(vpl[k], 7);
      wee[k] = g8_get(w[k], 7);
      ap[k] = g8_get(apl[k], 7);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) Ree[k] = g8_get(R[k], 7);
  }

  PP(2);
  // ---- costs that do not depend on the dynamics, computed by every lane with
  // the same (broadcast) operands: no divergent EE-only block, so the
  // scheduler can overlap them with the dynamics below ----
  double cee;  // EE cost except the contact-force terms (uniform in the group)
  {
    double Rrel[9], rr[3], th;
#pragma unroll
    for (int a_ = 0; a_ < 3; ++a_)
#pragma unroll
      for (int b_ = 0; b_ < 3; ++b_)
        Rrel[3 * a_ + b_] = C.Rdes[0 * 3 + a_] * Ree[0 * 3 + b_] + C.Rdes[1 * 3 + a_] * Ree[1 * 3 + b_] +
                            C.Rdes[2 * 3 + a_] * Ree[2 * 3 + b_];
    log3(Rrel, rr, th);
    cee = C.w_ori * (0.5 * (C.ori_w[0] * rr[0] * rr[0] + C.ori_w[1] * rr[1] * rr[1] + C.ori_w[2] * rr[2] * rr[2]));
    cee += C.w_wd * (0.5 * (C.wd_w[0] * wee[0] * wee[0] + C.wd_w[1] * wee[1] * wee[1] + C.wd_w[2] * wee[2] * wee[2]));
    const double rx = pee[0] - ref[0], ry = pee[1] - ref[1], rz = pee[2] - ref[2];
    const double cfree = C.w_ee_pos * (0.5 * (C.ee_pos_w[0] * rx * rx + C.ee_pos_w[1] * ry * ry + C.ee_pos_w[2] * rz * rz));
    const double vx = vp[0] - ref[3], vy = vp[1] - ref[4];
    double ccon = C.w_tp * (0.5 * (rx * rx + ry * ry)) + C.w_tv * (0.5 * (vx * vx + vy * vy));
    if (C.has_pz) {
      const double pz = pee[2] - (ref[2] - C.z_press);
      ccon += C.w_pz * (0.5 * pz * pz);
    }
    if (C.has_vz) ccon += C.w_vz * (0.5 * vp[2] * vp[2]);
    cee += surface ? ccon : cfree;
  }
  double cj = 0.0;  // this joint's state / control costs
  if (J) {
    if (C.variant == FFDDP_CLASSICAL || C.inner_state_reg) {
      const double rq = q - xq, rv = v - xv;
      cj += C.w_post * (0.5 * (rq * rq + rv * rv));
      cj += C.w_v * (0.5 * (K.vdw * v * v));
    }
    if (C.has_qsoft) {
      double ai, Ar, Arr;
      barrier(q - K.qsx, K.qslb, K.qsub, ai, Ar, Arr);
      cj += C.w_qs * ai;
    }
    if (!terminal && (C.variant == FFDDP_CLASSICAL || C.inner_tau_reg)) {
      const double r = u - tr;
      cj += C.w_tau * (0.5 * r * r);
      if (C.has_tsoft) {
        double ai, Ar, Arr;
        barrier(u, K.tslb, K.tsub, ai, Ar, Arr);
        cj += C.w_ts * ai;
      }
    }
  }
  lam[0] = lam[1] = lam[2] = 0.0;
  double a = 0.0;
  if (with_dyn) {
    // ---- link forces (RNEA, qdd = 0) and CRBA tuples ----
    // every lane, unmasked: lane 7 (the EE frame) has zero mass and inertia
    // in LaneK, so its link force and CRBA tuple come out zero (its frame
    // is finite whenever the joint lanes are); an exec-masked block made the
    // compiler zero-fill and copy the 16 outputs around it
    double fl[3], fa[3];
    double tm, th[3], tI[6];
    {
      const double m = K.m;
      const double* Ic = K.I;
      double cw[3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
        cw[r] = o[r] + (R[3 * r + 0] * K.com[0] + R[3 * r + 1] * K.com[1] + R[3 * r + 2] * K.com[2]);
      // world inertia Iw = R Ic R^T
      double IcR[9], Iw[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          IcR[3 * r + c] = Ic[3 * r + 0] * R[3 * c + 0] + Ic[3 * r + 1] * R[3 * c + 1] + Ic[3 * r + 2] * R[3 * c + 2];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          Iw[3 * r + c] = R[3 * r + 0] * IcR[0 * 3 + c] + R[3 * r + 1] * IcR[1 * 3 + c] + R[3 * r + 2] * IcR[2 * 3 + c];
      double Iww[3], Ial[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        Iww[r] = Iw[3 * r + 0] * w[0] + Iw[3 * r + 1] * w[1] + Iw[3 * r + 2] * w[2];
        Ial[r] = Iw[3 * r + 0] * al[0] + Iw[3 * r + 1] * al[1] + Iw[3 * r + 2] * al[2];
      }
      double t1[3], hl[3], ha[3], f1[3], n1[3];
      cross3(cw, w, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) hl[k] = m * (vO[k] - t1[k]);
      cross3(cw, hl, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) ha[k] = t1[k] + Iww[k];
      cross3(cw, al, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) f1[k] = m * ((aO[k] - rb.gravity[k]) - t1[k]);
      cross3(cw, f1, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) n1[k] = t1[k] + Ial[k];
      double c1[3], c2[3], c3[3];
      cross3(w, hl, c1);
      cross3(w, ha, c2);
      cross3(vO, hl, c3);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        fl[k] = f1[k] + c1[k];
        fa[k] = n1[k] + c2[k] + c3[k];
      }
      const double c2n = cw[0] * cw[0] + cw[1] * cw[1] + cw[2] * cw[2];
      tm = m;
      th[0] = m * cw[0];
      th[1] = m * cw[1];
      th[2] = m * cw[2];
      tI[0] = Iw[0] + m * (c2n - cw[0] * cw[0]);
      tI[1] = Iw[1] - m * cw[0] * cw[1];
      tI[2] = Iw[2] - m * cw[0] * cw[2];
      tI[3] = Iw[4] + m * (c2n - cw[1] * cw[1]);
      tI[4] = Iw[5] - m * cw[1] * cw[2];
      tI[5] = Iw[8] + m * (c2n - cw[2] * cw[2]);
    }
    // suffix sums (lane 7 contributes zero)
#pragma unroll
    for (int d = 1; d < G8; d <<= 1) {
      double t[16];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        t[k] = g8_down(fl[k], d);
        t[3 + k] = g8_down(fa[k], d);
        t[6 + k] = g8_down(th[k], d);
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) t[9 + k] = g8_down(tI[k], d);
      t[15] = g8_down(tm, d);
      if (li + d < G8) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          fl[k] += t[k];
          fa[k] += t[3 + k];
          th[k] += t[6 + k];
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) tI[k] += t[9 + k];
        tm += t[15];
      }
    }
    const double tau = Sv[0] * fl[0] + Sv[1] * fl[1] + Sv[2] * fl[2] + z[0] * fa[0] + z[1] * fa[1] + z[2] * fa[2];
    PP(3);
    // CRBA column: F = Ic_j S_j ; M[k][j] = S_k . F  (k <= j), row j of the lower triangle on lane j
    double Fl[3], Fa[3];
    {
      double hz[3], hs[3];
      cross3(th, z, hz);
      cross3(th, Sv, hs);
#pragma unroll
      for (int k = 0; k < 3; ++k) Fl[k] = tm * Sv[k] - hz[k];
      Fa[0] = hs[0] + tI[0] * z[0] + tI[1] * z[1] + tI[2] * z[2];
      Fa[1] = hs[1] + tI[1] * z[0] + tI[3] * z[1] + tI[4] * z[2];
      Fa[2] = hs[2] + tI[2] * z[0] + tI[4] * z[1] + tI[5] * z[2];
    }
    double Lr[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const double sx = g8_get(Sv[0], k), sy = g8_get(Sv[1], k), sz = g8_get(Sv[2], k);
      const double zx = g8_get(z[0], k), zy = g8_get(z[1], k), zz = g8_get(z[2], k);
      const double mkj = sx * Fl[0] + sy * Fl[1] + sz * Fl[2] + zx * Fa[0] + zy * Fa[1] + zz * Fa[2];
      Lr[k] = (k <= li) ? mkj : (li == k ? 1.0 : 0.0);
    }
    if (!J) {
#pragma unroll
      for (int k = 0; k < NQ; ++k) Lr[k] = 0.0;
    }
    PP(4);
    g8_chol_rows(Lr, li);
    double af = g8_solve(Lr, u - tau, li);
    PP(5);
    if (surface) {
      constexpr int c0 = NC == 1 ? 2 : 0;
      const double pstar[3] = {ref[0], ref[1], ref[2] - C.z_press};
      double rel[3] = {pee[0] - o[0], pee[1] - o[1], pee[2] - o[2]};
      double jcol[3];
      cross3(z, rel, jcol);  // z_i x (p - o_i): LWA linear Jacobian column i
      double Jc[3], Y[3], gam[3];
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        Jc[r] = J ? jcol[c0 + r] : 0.0;
        gam[r] = ap[c0 + r] + C.Kp * (pee[c0 + r] - pstar[c0 + r]) + C.Kd * vp[c0 + r];
        Y[r] = g8_fwd(Lr, Jc[r], li);
      }
      double S[6], yl[3];
#pragma unroll
      for (int r = 0; r < NC; ++r) {
#pragma unroll
        for (int s2 = 0; s2 <= r; ++s2) S[tri(r, s2)] = g8_sum(J ? Y[r] * Y[s2] : 0.0) + (r == s2 ? C.eps : 0.0);
        yl[r] = gam[r] + g8_sum(J ? Jc[r] * af : 0.0);
      }
      chol_packed<NC>(S);
      chol_solve<NC>(S, yl);
      double rhs = 0.0;
#pragma unroll
      for (int r = 0; r < NC; ++r) rhs += Jc[r] * (-yl[r]);
      a = af + g8_solve(Lr, rhs, li);
#pragma unroll
      for (int r = 0; r < NC; ++r) lam[r] = -yl[r];
    } else {
      a = af;
    }
  }
  PP(6);
  // ---- Euler step ----
  if (with_dyn) {
    const double dt = C.dt;
    qn = q + (v * dt + a * dt * dt);
    vn = v + a * dt;
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
    if (NC == 3 && C.has_fc) cf += friction_cone(C, lm, nullptr, nullptr, nullptr);
    if (C.has_uni) {
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        double ai, Ar, Arr;
        barrier(lm[r], C.uni_lb[r], C.uni_ub[r], ai, Ar, Arr);
        cf += C.w_uni * ai;
      }
    }
    if (C.has_fn) {
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        const double e = lm[r] - C.fn_ref[r];
        cf += C.w_fn * (0.5 * C.fn_w[r] * e * e);
      }
    }
  }
  const double c = J ? cj : cee + cf;
  cpart = c;
  PP(7);
}

}  // namespace ffddp
