// ffddp_group.hpp — 8-lane group primitives of the node calcs (k_node's
// calc, ffddp_primal_g8.hpp; the line search's, ffddp_rollout.hpp): lane
// i < 7 owns joint i, lane 7 owns the end-effector frame.
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

// L y = r (row layout): y group-uniform (all NQ entries)
template <bool ROW = false> __device__ __forceinline__ void g8_fwd_all(const double (&Lr)[NQ], double r, double (&y)[NQ]) {
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    double s = r;
#pragma unroll
    for (int m = 0; m < k; ++m) s -= Lr[m] * y[m];
    y[k] = g8_get<ROW>(s * Lr[k], k);
  }
}
// L^T x = y (y group-uniform, row layout): this lane's x
template <bool ROW = false> __device__ __forceinline__ double g8_bwd_all(const double (&Lr)[NQ], const double (&y)[NQ], int li) {
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

}  // namespace ffddp
