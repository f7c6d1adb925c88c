// ffddp_plant.hpp — closed-loop plant stand-in.
//
// Replaces the MuJoCo plant of the reference's closed loop
// (src/sim/franka_sim.py:144-169 step(), torque mode; scene
// assets/scenes/panda_table_scene.xml, robot assets/scenes/panda_robot.xml)
// for the arm + tool sphere + table-plane contact, one thread per instance:
//
//   per physics substep h (model.opt.timestep, n_substeps per control step):
//     bias = rnea(q, v, 0) (gravity + Coriolis, qfrc_bias); M_a = crba(q) + armature
//     f_s  = tau - bias - damping v                            (qfrc_smooth)
//     qacc_s = M_a^-1 f_s
//     tool sphere (radius r, at the ee_site) vs the table_contact plane:
//       dist = n . (p_site - p_plane) - r, active when dist < margin (condim 1)
//       J_n = n^T J_site, A = J_n M_a^-1 J_n^T, a_unc = J_n qacc_s + n . a_site(qdd=0)
//       MuJoCo soft constraint (solref = (timeconst, dampratio), solimp):
//         pos = dist - margin, imp = solimp(|pos|),
//         a_ref = -B (J_n v) - K imp pos, K = 1/(dmax^2 tc^2 dr^2), B = 2/(dmax tc)
//         R = (1 - imp)/imp * A  (MuJoCo uses the body-weight approximation of A)
//         f = max(0, (a_ref - a_unc) / (A + R)),  qfrc_c = J_n^T f
//     implicitfast: (M_a + h D) qacc = f_s + qfrc_c ; v += h qacc ; q += h v
//
// Observation semantics follow mj_step: kinematics, bias and contact force
// are those of the last substep's mj_forward (pre-integration state); q, v are
// post-integration.  Parity with MuJoCo is unpinned (MuJoCo is absent); the
// numpy restatement in oracle/plant.py is the checker.
#pragma once

#include "ffddp_robot.hpp"

namespace ffddp {

// observation record layout (FFDDP_PLANT_OBS words per instance)
enum {
  PO_Q = 0, PO_DQ = 7, PO_BIAS = 14, PO_TAUC = 21, PO_EE_P = 28, PO_EE_V = 31, PO_EE_R = 34, PO_FW = 43, PO_FN = 46,
  PO_NCON = 47, PO_J = 48 /* 3x7 site linear Jacobian, MJ world */, PO_WORDS = 69
};

// MuJoCo solimp impedance (mju_impedance semantics for |pos| <= width)
FFD_HD double plant_imp(const ffddp_plant_params& P, double pos) {
  const double d0 = P.solimp[0], dmax = P.solimp[1], width = P.solimp[2], mid = P.solimp[3], pw = P.solimp[4];
  double x = fabs(pos) / (width > 0.0 ? width : 1.0);
  if (x >= 1.0 || width <= 0.0) return dmax;
  double y;
  if (pw == 1.0) {
    y = x;
  } else if (x <= mid) {
    y = pow(x, pw) / pow(mid, pw - 1.0);
  } else {
    y = 1.0 - pow(1.0 - x, pw) / pow(1.0 - mid, pw - 1.0);
  }
  return d0 + y * (dmax - d0);
}

// in-place solve with a packed LLT (reciprocal diagonal), 7x7
FFD_HD void plant_solve(const double* L, double* b) { chol_solve<FFDDP_NQ>(L, b); }

// One control step (n_substeps physics steps) of one instance.  q, v in/out;
// tau applied torque (qfrc_applied); n_mj, p0_mj: table plane normal / point
// (MuJoCo world); obs: PO_WORDS.  Returns false on a non-SPD mass matrix.
FFD_HD bool plant_step(const ffddp_robot& rb, const ffddp_plant_params& P, double* q, double* v, const double* tau,
                       const double n_mj[3], const double p0_mj[3], int integrate, double* obs) {
  constexpr int NQ = FFDDP_NQ;
  // MuJoCo world = R_MJ_FROM_PIN . Pinocchio/link0 world, R = diag(-1, -1, 1)
  const double n[3] = {-n_mj[0], -n_mj[1], n_mj[2]};
  const double p0[3] = {-p0_mj[0], -p0_mj[1], p0_mj[2]};
  const int nsub = integrate ? (P.n_substeps > 0 ? P.n_substeps : 1) : 1;
  const double h = P.timestep;
  for (int s = 0; s < nsub; ++s) {
    const double zero[NQ] = {0, 0, 0, 0, 0, 0, 0};
    RBOut<double> o;
    double M[28];
    rb_pass<double, true, true>(rb, q, v, zero, nullptr, o, M);
    double fs[NQ];
    for (int i = 0; i < NQ; ++i) {
      M[tri(i, i)] += P.armature[i];
      fs[i] = tau[i] - o.tau[i] - P.damping[i] * v[i];
    }
    double La[28];
    for (int e = 0; e < 28; ++e) La[e] = M[e];
    if (!chol_packed<NQ>(La)) return false;
    double qs[NQ];
    for (int i = 0; i < NQ; ++i) qs[i] = fs[i];
    plant_solve(La, qs);
    // site Jacobian (linear, Pinocchio world) and contact
    const double pe[3] = {o.pee.x, o.pee.y, o.pee.z};
    double Jl[3][NQ];
    for (int i = 0; i < NQ; ++i) {
      const double rx = pe[0] - o.o[i].x, ry = pe[1] - o.o[i].y, rz = pe[2] - o.o[i].z;
      const double zx = o.z[i].x, zy = o.z[i].y, zz = o.z[i].z;
      Jl[0][i] = zy * rz - zz * ry;
      Jl[1][i] = zz * rx - zx * rz;
      Jl[2][i] = zx * ry - zy * rx;
    }
    const double dist = n[0] * (pe[0] - p0[0]) + n[1] * (pe[1] - p0[1]) + n[2] * (pe[2] - p0[2]) - P.r_tool;
    double f = 0.0, qc[NQ] = {0, 0, 0, 0, 0, 0, 0};
    const bool active = dist < P.margin;
    if (active) {
      double Jn[NQ], y[NQ];
      for (int i = 0; i < NQ; ++i) {
        Jn[i] = n[0] * Jl[0][i] + n[1] * Jl[1][i] + n[2] * Jl[2][i];
        y[i] = Jn[i];
      }
      plant_solve(La, y);
      double A = 0.0, au = 0.0, vel = 0.0;
      for (int i = 0; i < NQ; ++i) {
        A += Jn[i] * y[i];
        au += Jn[i] * qs[i];
        vel += Jn[i] * v[i];
      }
      au += n[0] * o.ap.x + n[1] * o.ap.y + n[2] * o.ap.z;
      const double pos = dist - P.margin;
      const double imp = plant_imp(P, pos);
      const double dmax = P.solimp[1];
      const double tc = P.solref[0], dr = P.solref[1];
      const double K = 1.0 / (dmax * dmax * tc * tc * dr * dr), Bd = 2.0 / (dmax * tc);
      const double aref = -Bd * vel - K * imp * pos;
      const double R = (1.0 - imp) / imp * A;
      f = (aref - au) / (A + R);
      f = f > 0.0 ? f : 0.0;
      for (int i = 0; i < NQ; ++i) qc[i] = Jn[i] * f;
    }
    if (s == nsub - 1) {
      // observation of this substep's forward pass (MuJoCo frame)
      for (int i = 0; i < NQ; ++i) {
        obs[PO_BIAS + i] = o.tau[i];
        obs[PO_TAUC + i] = qc[i];
      }
      obs[PO_EE_P + 0] = -pe[0];
      obs[PO_EE_P + 1] = -pe[1];
      obs[PO_EE_P + 2] = pe[2];
      // site rotation R_mj = R . Ree . R_site_from_ee (tool body quat, panda_robot.xml:189)
      const double c = P.site_R[0], sn = P.site_R[1];
      for (int r = 0; r < 3; ++r) {
        const double sgn = r < 2 ? -1.0 : 1.0;
        const double a0 = o.Ree.m[3 * r + 0], a1 = o.Ree.m[3 * r + 1], a2 = o.Ree.m[3 * r + 2];
        obs[PO_EE_R + 3 * r + 0] = sgn * (a0 * c + a1 * sn);
        obs[PO_EE_R + 3 * r + 1] = sgn * (-a0 * sn + a1 * c);
        obs[PO_EE_R + 3 * r + 2] = sgn * a2;
      }
      for (int r = 0; r < 3; ++r) {
        const double sgn = r < 2 ? -1.0 : 1.0;
        for (int i = 0; i < NQ; ++i) obs[PO_J + r * NQ + i] = sgn * Jl[r][i];
        obs[PO_FW + r] = n_mj[r] * f;  // force on the tool (table pushes along +n)
      }
      obs[PO_FN] = f;
      obs[PO_NCON] = active ? 1.0 : 0.0;
    }
    if (!integrate) break;
    // implicitfast: (M_a + h D) qacc = f_s + qfrc_c
    double Li[28], qa[NQ];
    for (int e = 0; e < 28; ++e) Li[e] = M[e];
    for (int i = 0; i < NQ; ++i) {
      Li[tri(i, i)] += h * P.damping[i];
      qa[i] = fs[i] + qc[i];
    }
    if (!chol_packed<NQ>(Li)) return false;
    plant_solve(Li, qa);
    for (int i = 0; i < NQ; ++i) {
      v[i] += h * qa[i];
      q[i] += h * v[i];
    }
  }
  for (int i = 0; i < NQ; ++i) {
    obs[PO_Q + i] = q[i];
    obs[PO_DQ + i] = v[i];
  }
  // ee_vel = J_site (last forward) . qvel (post-integration), MuJoCo frame
  for (int r = 0; r < 3; ++r) {
    double a = 0.0;
    for (int i = 0; i < NQ; ++i) a += obs[PO_J + r * NQ + i] * v[i];
    obs[PO_EE_V + r] = a;
  }
  return true;
}

}  // namespace ffddp
