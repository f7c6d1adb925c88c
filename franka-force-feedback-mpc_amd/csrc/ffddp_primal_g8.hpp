// ffddp_primal_g8.hpp — the calc of calcDiff (node_primal + rb_links of
// ffddp_node.hpp / ffddp_robot.hpp) spread over an 8-lane group: lane i < 7
// owns joint i, lane 7 the end-effector frame (same scans as node_calc_g8).
// It writes what k_node consumes: the Primal record (dynamics, contact
// factorisation, kinematics, Gauss-Newton weights, cost, Euler step) and the
// per-link world-frame data at (q, v, qdd = a) of rb_links, each lane its own
// joint's / link's share.  Same physics and cost stack as node_primal; only
// the evaluation order (hence rounding) differs.
#pragma once

// k_node's contact solve: one backward substitution through the Schur
// complement (1) or the two-solve form (0, default: on configs[1]'s random-x0
// spread the Schur form doubled the distance of `us` from an
// extended-precision solve, 1.7e-7 -> 3.3e-7, tools/ext_budget.py)
#ifndef FFDDP_KN_SCHUR
#define FFDDP_KN_SCHUR 0
#endif

#include "ffddp_group.hpp"

namespace ffddp {

// gp: this node's Primal in global memory; lk: its link record (LK_* layout).
// Returns (group-uniform) the unscaled DAM cost and the contact force.
template <int NC>
__device__ __forceinline__ double node_primal_g8(const DevConsts& C, int mode, bool surface, double q, double v, double u,
                                                 double xq, double xv, double tr, const double* ref,
                                                 Primal* __restrict__ gp, double* __restrict__ lk, double (&lam)[3]) {
  const ffddp_robot& rb = C.rb;
  const int li = g8_lane();
  const bool J = li < NQ;
  const int ji = J ? li : NQ - 1;
  const bool with_dyn = mode != MODE_TERMINAL_X;
  const bool terminal = mode != MODE_RUNNING;
  if (!J) q = v = u = 0.0;

  // ---- forward kinematics: prefix scan of transforms ----
  double R[9], o[3];
  if (J) {
    double s, c;
    sincos_(q, s, c);
    const double* Jr = rb.joint_R[ji];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      R[3 * r + 0] = c * Jr[3 * r + 0] + s * Jr[3 * r + 1];
      R[3 * r + 1] = c * Jr[3 * r + 1] - s * Jr[3 * r + 0];
      R[3 * r + 2] = Jr[3 * r + 2];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) o[k] = rb.joint_p[ji][k];
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = rb.ee_R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) o[k] = rb.ee_p[k];
  }
#pragma unroll
  for (int d = 1; d < G8; d <<= 1) {
    double Rp[9], op[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) Rp[k] = g8_up(R[k], d);
#pragma unroll
    for (int k = 0; k < 3; ++k) op[k] = g8_up(o[k], d);
    if (li >= d) {
      double Rn[9], on[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) Rn[3 * r + c] = Rp[3 * r + 0] * R[c] + Rp[3 * r + 1] * R[3 + c] + Rp[3 * r + 2] * R[6 + c];
        on[r] = op[r] + (Rp[3 * r + 0] * o[0] + Rp[3 * r + 1] * o[1] + Rp[3 * r + 2] * o[2]);
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = Rn[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) o[k] = on[k];
    }
  }
  double z[3] = {J ? R[2] : 0.0, J ? R[5] : 0.0, J ? R[8] : 0.0};
  double Sv[3];
  cross3(o, z, Sv);
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
  // ---- end-effector frame (lane 7) ----
  double pee[3], vp[3], wee[3], ap0[3], Ree[9];
  {
    double vpl[3], apl[3], c1[3], c2[3];
    cross3(w, o, c1);
#pragma unroll
    for (int k = 0; k < 3; ++k) vpl[k] = vO[k] + c1[k];
    cross3(al, o, c1);
    cross3(w, vpl, c2);
#pragma unroll
    for (int k = 0; k < 3; ++k) apl[k] = aO[k] + c1[k] + c2[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pee[k] = g8_get<true>(o[k], 7);
      vp[k] = g8_get<true>(vpl[k], 7);
      wee[k] = g8_get<true>(w[k], 7);
      ap0[k] = g8_get<true>(apl[k], 7);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) Ree[k] = g8_get<true>(R[k], 7);
  }
  if (J) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      gp->z[li][k] = z[k];
      gp->o[li][k] = o[k];
    }
  }
  if (li == 7) {
#pragma unroll
    for (int k = 0; k < 3; ++k) gp->pee[k] = pee[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) gp->Ree[k] = Ree[k];
  }
  // ---- per-link inertia (world) : m, h = m c, I_O, and Iw for the link forces ----
  double m = 0.0, cw[3] = {0, 0, 0}, Iw[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (J) {
    m = rb.mass[ji];
    const double* Ic = rb.inertia[ji];
#pragma unroll
    for (int r = 0; r < 3; ++r)
      cw[r] = o[r] + (R[3 * r + 0] * rb.com[ji][0] + R[3 * r + 1] * rb.com[ji][1] + R[3 * r + 2] * rb.com[ji][2]);
    double IcR[9];
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
  }
  const double c2n = cw[0] * cw[0] + cw[1] * cw[1] + cw[2] * cw[2];
  const double IO[6] = {Iw[0] + m * (c2n - cw[0] * cw[0]), Iw[1] - m * cw[0] * cw[1], Iw[2] - m * cw[0] * cw[2],
                        Iw[4] + m * (c2n - cw[1] * cw[1]), Iw[5] - m * cw[1] * cw[2], Iw[8] + m * (c2n - cw[2] * cw[2])};
  const double hh[3] = {m * cw[0], m * cw[1], m * cw[2]};
  auto IOmul = [&](const double* x3, double* y3) {
    y3[0] = IO[0] * x3[0] + IO[1] * x3[1] + IO[2] * x3[2];
    y3[1] = IO[1] * x3[0] + IO[3] * x3[1] + IO[4] * x3[2];
    y3[2] = IO[2] * x3[0] + IO[4] * x3[1] + IO[5] * x3[2];
  };
  // momentum H = I V (per link)
  double hl[3], ha[3];
  {
    double t1[3], t2[3], Iwv[3];
    cross3(hh, w, t1);
#pragma unroll
    for (int k = 0; k < 3; ++k) hl[k] = m * vO[k] - t1[k];
    cross3(hh, vO, t2);
    IOmul(w, Iwv);
#pragma unroll
    for (int k = 0; k < 3; ++k) ha[k] = t2[k] + Iwv[k];
  }
  lam[0] = lam[1] = lam[2] = 0.0;
  double a = 0.0;
  if (with_dyn) {
    // ---- RNEA at qdd = 0 (bias torques) and CRBA tuples: suffix sums ----
    double fl[3], fa[3];
    {
      const double g0[3] = {rb.gravity[0], rb.gravity[1], rb.gravity[2]};
      double ag[3], t1[3], f1[3], n1[3], Ial[3], c1[3], c2[3], c3[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) ag[k] = aO[k] - g0[k];
      cross3(hh, al, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) f1[k] = m * ag[k] - t1[k];
      cross3(hh, ag, t1);
      IOmul(al, Ial);
#pragma unroll
      for (int k = 0; k < 3; ++k) n1[k] = t1[k] + Ial[k];
      cross3(w, hl, c1);
      cross3(w, ha, c2);
      cross3(vO, hl, c3);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        fl[k] = J ? f1[k] + c1[k] : 0.0;
        fa[k] = J ? n1[k] + c2[k] + c3[k] : 0.0;
      }
    }
    double tm = m, th[3] = {hh[0], hh[1], hh[2]}, tI[6] = {IO[0], IO[1], IO[2], IO[3], IO[4], IO[5]};
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
      const double sx = g8_get<true>(Sv[0], k), sy = g8_get<true>(Sv[1], k), sz = g8_get<true>(Sv[2], k);
      const double zx = g8_get<true>(z[0], k), zy = g8_get<true>(z[1], k), zz = g8_get<true>(z[2], k);
      const double mkj = sx * Fl[0] + sy * Fl[1] + sz * Fl[2] + zx * Fa[0] + zy * Fa[1] + zz * Fa[2];
      Lr[k] = (k <= li) ? mkj : (li == k ? 1.0 : 0.0);
    }
    if (!J) {
#pragma unroll
      for (int k = 0; k < NQ; ++k) Lr[k] = (k == NQ - 1) ? 1.0 : 0.0;  // harmless identity row (not stored)
    }
    g8_chol_rows<true>(Lr, li);
    if (J) {
#pragma unroll
      for (int k = 0; k < NQ; ++k)
        if (k <= li) gp->L[tri(li, k)] = Lr[k];
    }
#if FFDDP_KN_SCHUR
    // y1 = L^-1 (u - tau); free: a = L^-T y1.  Contact (the KKT by its Schur
    // complement): Y = L^-1 Jc^T, S = Y'Y + eps, yl = S^-1 (gamma + Y'y1),
    // a = L^-T (y1 - Y yl), lambda = -yl: one backward substitution, and the
    // Schur sums from the group-uniform forward solutions (no cross-lane sums)
    double y1[NQ];
    g8_fwd_all<true>(Lr, u - tau, y1);
    if (surface) {
      constexpr int c0 = NC == 1 ? 2 : 0;
      const double pstar[3] = {ref[0], ref[1], ref[2] - C.z_press};
      double rel[3] = {pee[0] - o[0], pee[1] - o[1], pee[2] - o[2]};
      double jcol[3];
      cross3(z, rel, jcol);
      double Yu[3][NQ], gam[3];
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        const double Jc = J ? jcol[c0 + r] : 0.0;
        gam[r] = ap0[c0 + r] + C.Kp * (pee[c0 + r] - pstar[c0 + r]) + C.Kd * vp[c0 + r];
        g8_fwd_all<true>(Lr, Jc, Yu[r]);
        double yown = 0.0;
#pragma unroll
        for (int k = 0; k < NQ; ++k) yown = (li == k) ? Yu[r][k] : yown;
        if (J) {
          gp->Jc[r][li] = Jc;
          gp->Y[r][li] = yown;
        }
      }
      double S[6], yl[3];
#pragma unroll
      for (int r = 0; r < NC; ++r) {
#pragma unroll
        for (int s2 = 0; s2 <= r; ++s2) {
          double acc = Yu[r][0] * Yu[s2][0];
#pragma unroll
          for (int k = 1; k < NQ; ++k) acc += Yu[r][k] * Yu[s2][k];
          S[tri(r, s2)] = acc + (r == s2 ? C.eps : 0.0);
        }
        double acc = Yu[r][0] * y1[0];
#pragma unroll
        for (int k = 1; k < NQ; ++k) acc += Yu[r][k] * y1[k];
        yl[r] = gam[r] + acc;
      }
      chol_packed<NC>(S);
      if (li == 0) {
#pragma unroll
        for (int e = 0; e < NC * (NC + 1) / 2; ++e) gp->Ls[e] = S[e];
      }
      chol_solve<NC>(S, yl);
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
#pragma unroll
        for (int r = 0; r < NC; ++r) y1[k] -= Yu[r][k] * yl[r];
      }
#pragma unroll
      for (int r = 0; r < NC; ++r) lam[r] = -yl[r];
    }
    a = g8_bwd_all<true>(Lr, y1, li);
#else
    // FFDDP_KN_SCHUR=0: the two-solve form (a = af + M^-1 Jc^T (-yl),
    // af = M^-1 (u - tau), Schur sums across the group's lanes)
    const double af = g8_solve<true>(Lr, u - tau, li);
    if (surface) {
      constexpr int c0 = NC == 1 ? 2 : 0;
      const double pstar[3] = {ref[0], ref[1], ref[2] - C.z_press};
      double rel[3] = {pee[0] - o[0], pee[1] - o[1], pee[2] - o[2]};
      double jcol[3];
      cross3(z, rel, jcol);
      double Jc[3], Y[3], gam[3];
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        Jc[r] = J ? jcol[c0 + r] : 0.0;
        gam[r] = ap0[c0 + r] + C.Kp * (pee[c0 + r] - pstar[c0 + r]) + C.Kd * vp[c0 + r];
        Y[r] = g8_fwd<true>(Lr, Jc[r], li);
        if (J) {
          gp->Jc[r][li] = Jc[r];
          gp->Y[r][li] = Y[r];
        }
      }
      double S[6], yl[3];
#pragma unroll
      for (int r = 0; r < NC; ++r) {
#pragma unroll
        for (int s2 = 0; s2 <= r; ++s2) S[tri(r, s2)] = g8_sum(J ? Y[r] * Y[s2] : 0.0) + (r == s2 ? C.eps : 0.0);
        yl[r] = gam[r] + g8_sum(J ? Jc[r] * af : 0.0);
      }
      chol_packed<NC>(S);
      if (li == 0) {
#pragma unroll
        for (int e = 0; e < NC * (NC + 1) / 2; ++e) gp->Ls[e] = S[e];
      }
      chol_solve<NC>(S, yl);
      double rhs = 0.0;
#pragma unroll
      for (int r = 0; r < NC; ++r) rhs += Jc[r] * (-yl[r]);
      a = af + g8_solve<true>(Lr, rhs, li);
#pragma unroll
      for (int r = 0; r < NC; ++r) lam[r] = -yl[r];
    } else {
      a = af;
    }
#endif
  }
  if (!J) a = 0.0;
  if (J) gp->a[li] = a;
  if (li == 0) {
#pragma unroll
    for (int r = 0; r < 3; ++r) gp->lam[r] = lam[r];
  }
  // ---- link data at qdd = a: accelerations += prefix sum of S a ----
  {
    double aa[6] = {Sv[0] * a, Sv[1] * a, Sv[2] * a, z[0] * a, z[1] * a, z[2] * a};
#pragma unroll
    for (int d = 1; d < G8; d <<= 1) {
      double t[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) t[k] = g8_up(aa[k], d);
      if (li >= d) {
#pragma unroll
        for (int k = 0; k < 6; ++k) aa[k] += t[k];
      }
    }
    double aOa[3], ala[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      aOa[k] = aO[k] + aa[k];
      ala[k] = al[k] + aa[3 + k];
    }
    if (J) {
      double* L = lk + li * LK_STRIDE;
      const double g0[3] = {rb.gravity[0], rb.gravity[1], rb.gravity[2]};
      double ag[3], t1[3], f1[3], n1[3], Ial[3], c1[3], c2[3], c3[3], f[3], n[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) ag[k] = aOa[k] - g0[k];
      cross3(hh, ala, t1);
#pragma unroll
      for (int k = 0; k < 3; ++k) f1[k] = m * ag[k] - t1[k];
      cross3(hh, ag, t1);
      IOmul(ala, Ial);
#pragma unroll
      for (int k = 0; k < 3; ++k) n1[k] = t1[k] + Ial[k];
      cross3(w, hl, c1);
      cross3(w, ha, c2);
      cross3(vO, hl, c3);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        f[k] = f1[k] + c1[k];
        n[k] = n1[k] + c2[k] + c3[k];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        L[LK_SV + k] = Sv[k];
        L[LK_Z + k] = z[k];
        L[LK_O + k] = o[k];
        L[LK_VO + k] = vO[k];
        L[LK_W + k] = w[k];
        L[LK_AO + k] = aOa[k];
        L[LK_AL + k] = ala[k];
        L[LK_F + k] = f[k];
        L[LK_N + k] = n[k];
        L[LK_HL + k] = hl[k];
        L[LK_HA + k] = ha[k];
        L[LK_H + k] = hh[k];
      }
      L[LK_M] = m;
#pragma unroll
      for (int e = 0; e < 6; ++e) L[LK_IO + e] = IO[e];
    } else {
      // EE (lane 7 carries link 7's cumulative V, A): p, v_p, w, classical a_p at qdd = a
      double c1[3], c2[3], apa[3];
      cross3(ala, o, c1);
      cross3(w, vp, c2);
#pragma unroll
      for (int k = 0; k < 3; ++k) apa[k] = aOa[k] + c1[k] + c2[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        lk[LK_EE + k] = pee[k];
        lk[LK_EE + 3 + k] = vp[k];
        lk[LK_EE + 6 + k] = w[k];
        lk[LK_EE + 9 + k] = apa[k];
      }
    }
  }
  // ---- costs (CostModelSum, _make_dam order) with their Gauss-Newton weights ----
  double cj = 0.0;  // this lane's state / control costs
  {
    double dxq = 0.0, gxq = 0.0, dxv = 0.0, gxv = 0.0, du = 0.0, gu = 0.0;
    if (J) {
      if (C.variant == FFDDP_CLASSICAL || C.inner_state_reg) {
        const double rq = q - xq, rv = v - xv;
        dxq += C.w_post;
        gxq += C.w_post * rq;
        dxv += C.w_post;
        gxv += C.w_post * rv;
        cj += C.w_post * (0.5 * (rq * rq + rv * rv));
        const double wi = C.vdw[ji];
        dxv += C.w_v * wi;
        gxv += C.w_v * wi * v;
        cj += C.w_v * (0.5 * (wi * v * v));
      }
      if (C.has_qsoft) {
        double ai, Ar, Arr, bi, Br, Brr;
        barrier(q - C.qs_xref[ji], C.qs_lb[ji], C.qs_ub[ji], ai, Ar, Arr);
        barrier(v - C.qs_xref[7 + ji], C.qs_lb[7 + ji], C.qs_ub[7 + ji], bi, Br, Brr);
        dxq += C.w_qs * Arr;
        gxq += C.w_qs * Ar;
        dxv += C.w_qs * Brr;
        gxv += C.w_qs * Br;
        cj += C.w_qs * (ai + bi);
      }
      if (!terminal && (C.variant == FFDDP_CLASSICAL || C.inner_tau_reg)) {
        const double r = u - tr;
        du += C.w_tau;
        gu += C.w_tau * r;
        cj += C.w_tau * (0.5 * r * r);
        if (C.has_tsoft) {
          double ai, Ar, Arr;
          barrier(u, C.ts_lb[ji], C.ts_ub[ji], ai, Ar, Arr);
          du += C.w_ts * Arr;
          gu += C.w_ts * Ar;
          cj += C.w_ts * ai;
        }
      }
      gp->Dx[li] = dxq;
      gp->gx[li] = gxq;
      gp->Dx[7 + li] = dxv;
      gp->gx[7 + li] = gxv;
      gp->Du[li] = du;
      gp->gu[li] = gu;
    }
  }
  // EE / contact residuals: every lane computes them (group-uniform operands);
  // lane k < NDENSE_MAX stores dense row k's weights
  double Dd[NDENSE_MAX], gd[NDENSE_MAX];
#pragma unroll
  for (int k = 0; k < NDENSE_MAX; ++k) Dd[k] = gd[k] = 0.0;
  double cee = 0.0;
  double rr[3], th;
  {
    double Rrel[9];
#pragma unroll
    for (int a_ = 0; a_ < 3; ++a_)
#pragma unroll
      for (int b_ = 0; b_ < 3; ++b_)
        Rrel[3 * a_ + b_] = C.Rdes[0 * 3 + a_] * Ree[0 * 3 + b_] + C.Rdes[1 * 3 + a_] * Ree[1 * 3 + b_] +
                            C.Rdes[2 * 3 + a_] * Ree[2 * 3 + b_];
    log3(Rrel, rr, th);
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      s += C.ori_w[i] * rr[i] * rr[i];
      Dd[3 + i] += C.w_ori * C.ori_w[i];
      gd[3 + i] += C.w_ori * C.ori_w[i] * rr[i];
    }
    cee += C.w_ori * (0.5 * s);
  }
  {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      s += C.wd_w[i] * wee[i] * wee[i];
      Dd[9 + i] += C.w_wd * C.wd_w[i];
      gd[9 + i] += C.w_wd * C.wd_w[i] * wee[i];
    }
    cee += C.w_wd * (0.5 * s);
  }
  if (!surface) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double r = pee[i] - ref[i];
      s += C.ee_pos_w[i] * r * r;
      Dd[i] += C.w_ee_pos * C.ee_pos_w[i];
      gd[i] += C.w_ee_pos * C.ee_pos_w[i] * r;
    }
    cee += C.w_ee_pos * (0.5 * s);
  } else {
    const double pstar2 = ref[2] - C.z_press;
    {
      const double rx = pee[0] - ref[0], ry = pee[1] - ref[1], rz = pee[2] - ref[2];
      const double s = rx * rx + ry * ry + 0.0 * rz * rz;
      Dd[0] += C.w_tp;
      Dd[1] += C.w_tp;
      gd[0] += C.w_tp * rx;
      gd[1] += C.w_tp * ry;
      cee += C.w_tp * (0.5 * s);
    }
    {
      const double rx = vp[0] - ref[3], ry = vp[1] - ref[4];
      Dd[6] += C.w_tv;
      Dd[7] += C.w_tv;
      gd[6] += C.w_tv * rx;
      gd[7] += C.w_tv * ry;
      cee += C.w_tv * (0.5 * (rx * rx + ry * ry));
    }
    if (C.has_pz) {
      const double rz = pee[2] - pstar2;
      Dd[2] += C.w_pz;
      gd[2] += C.w_pz * rz;
      cee += C.w_pz * (0.5 * rz * rz);
    }
    if (C.has_vz) {
      Dd[8] += C.w_vz;
      gd[8] += C.w_vz * vp[2];
      cee += C.w_vz * (0.5 * vp[2] * vp[2]);
    }
    double lm[3] = {0, 0, 0};
    if (mode != MODE_TERMINAL_X)
#pragma unroll
      for (int r = 0; r < NC; ++r) lm[r] = lam[r];
    if (NC == 3 && C.has_fc) {
      double gl[3], Hd[3], Ho[3];
      cee += friction_cone(C, lm, gl, Hd, Ho);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        Dd[12 + r] += Hd[r];
        gd[12 + r] += gl[r];
      }
      if (li == 0) {
#pragma unroll
        for (int r = 0; r < 3; ++r) gp->Dfo[r] = Ho[r];
      }
    } else if (li == 0) {
#pragma unroll
      for (int r = 0; r < 3; ++r) gp->Dfo[r] = 0.0;
    }
    if (C.has_uni) {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        double ai, Ar, Arr;
        barrier(lm[r], C.uni_lb[r], C.uni_ub[r], ai, Ar, Arr);
        s += ai;
        Dd[12 + r] += C.w_uni * Arr;
        gd[12 + r] += C.w_uni * Ar;
      }
      cee += C.w_uni * s;
    }
    if (C.has_fn) {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        const double e = lm[r] - C.fn_ref[r];
        s += C.fn_w[r] * e * e;
        Dd[12 + r] += C.w_fn * C.fn_w[r];
        gd[12 + r] += C.w_fn * C.fn_w[r] * e;
      }
      cee += C.w_fn * (0.5 * s);
    }
  }
  if (li == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) gp->r_rot[i] = rr[i];
    gp->th_rot = th;
    if (!surface) {
#pragma unroll
      for (int r = 0; r < 3; ++r) gp->Dfo[r] = 0.0;
    }
  }
  // rows split over the 8 lanes (static indices: lane li stores rows li and li + 8)
#pragma unroll
  for (int k = 0; k < NDENSE_MAX; ++k)
    if ((k & 7) == li) {
      gp->D[k] = Dd[k];
      gp->g[k] = gd[k];
    }
  const double cost = g8_sum(J ? cj : 0.0) + cee;
  if (li == 0) gp->cost = cost;
  // ---- Euler step ----
  if (J) {
    if (with_dyn) {
      const double dt = C.dt;
      gp->xnext[li] = q + (v * dt + a * dt * dt);
      gp->xnext[NQ + li] = v + a * dt;
    } else {
      gp->xnext[li] = q;
      gp->xnext[NQ + li] = v;
    }
  }
  return cost;
}

}  // namespace ffddp
