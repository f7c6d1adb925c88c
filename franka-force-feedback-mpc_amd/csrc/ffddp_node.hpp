// ffddp_node.hpp — one shooting node: IntegratedActionModelEuler around
// DifferentialActionModel{Free,Contact}FwdDynamics with the reference cost
// stack (crocoddyl_classical.py:558-728; FF :838-1009), plus the
// _AugmentedLPFActionModel wrapper (crocoddyl_force_feedback.py:149-290).
//
// Split in three pieces so the kernels can schedule them differently:
//   node_primal()  : calc — dynamics (ABA / contact KKT), residuals,
//                    activations, cost, Euler step.  T = double.
//   node_tangent() : one forward-mode direction of calcDiff (a lane of the
//                    node group): d a / d x_j, d lambda / d x_j and the
//                    residual-Jacobian column j.
//   Gauss-Newton assembly across lanes lives in the kernel (LDS).
#pragma once

#include "ffddp_robot.hpp"

namespace ffddp {

constexpr int NQ = FFDDP_NQ;
constexpr int NU = FFDDP_NU;
constexpr int NDIR = 21;  // inner directions: 14 state + 7 inner control
constexpr int NDENSE_MAX = 12 + FFDDP_MAX_NC;
constexpr int NTRIALS = 10;

// Node modes
enum { MODE_RUNNING = 0, MODE_TERMINAL_X = 1, MODE_TERMINAL_U = 2 };

// Host-precomputed constants, uniform across the batch (scalar loads).
struct DevConsts {
  ffddp_robot rb;
  int variant, N, nc, use_box, nx;
  int has_qsoft, has_tsoft, has_pz, has_vz, has_uni, has_fn, inner_state_reg, inner_tau_reg;
  double dt;
  // state costs
  double w_post, w_v, vdw[7], w_qs, qs_xref[14], qs_lb[14], qs_ub[14];
  // frame costs
  double w_ori, ori_w[3], w_wd, wd_w[3], w_ee_pos, ee_pos_w[3];
  double w_tp, w_tv, w_pz, w_vz;
  double Rdes[9];
  // force costs
  double w_uni, uni_lb[3], uni_ub[3], w_fn, fn_w[3], fn_ref[3];
  // friction cone (nc = 3): r = A lambda, QuadraticBarrier(lb, ub)
  int has_fc;
  double w_fc, fc_A[5][3], fc_lb[5], fc_ub[5];
  // control costs
  double w_tau, w_ts, ts_lb[7], ts_ub[7];
  // contact
  double Kp, Kd, eps, z_press;
  double u_lb[7], u_ub[7];
  // force feedback
  double alpha, beta, w_w, w_ws, ws_lim[7], w_y, Wy2[21];
  // solver constants (crocoddyl SolverBoxFDDP / BoxQP)
  double th_stop, th_grad, th_acceptstep, th_acceptnegstep, th_stepdec, th_stepinc;
  double reg_min, reg_max, reg_inc, reg_dec;
  int neg_rule;  // FFDDP_NEGSTEP_* : ascent-direction acceptance comparator
  double alphas[NTRIALS];
  int qp_maxiter;
  double qp_th_acceptstep, qp_th_grad, qp_reg;
};

// record layout (doubles) of one node's calcDiff output
FFD_HD int rec_off_A() { return 0; }                        // [21][7]  A[dir][i] = d a_i / d dir
FFD_HD int rec_off_Lxx(int) { return 147; }                 // [nx][nx]
FFD_HD int rec_off_Lxu(int nx) { return 147 + nx * nx; }    // [nx][7]
FFD_HD int rec_off_Luu(int nx) { return 147 + nx * nx + nx * 7; }
FFD_HD int rec_off_Lx(int nx) { return rec_off_Luu(nx) + 49; }
FFD_HD int rec_off_Lu(int nx) { return rec_off_Lx(nx) + nx; }
FFD_HD int rec_off_cost(int nx) { return rec_off_Lu(nx) + 7; }
FFD_HD int rec_off_lam(int nx) { return rec_off_cost(nx) + 1; }
// padded to a multiple of 16 words (128 B): every node record starts on a
// cache-line boundary, so k_node's record writes cover whole lines
FFD_HD int rec_size(int nx) { return (rec_off_lam(nx) + 3 + 15) & ~15; }

// ---------------------------------------------------------------------------
// log3 / Jlog3 (pinocchio)
// ---------------------------------------------------------------------------
FFD_HD void log3(const double* R, double* r, double& th) {
  const double tr = R[0] + R[4] + R[8];
  double c = (tr - 1.0) / 2.0;
  c = c > 1.0 ? 1.0 : (c < -1.0 ? -1.0 : c);
  th = acos_(c);
  const double eps3 = 6.0554544523933395e-06;  // eps^(1/3)
  double st, ct;
  sincos_(th, st, ct);
  const double t = (th > eps3 ? th / st : 1.0) / 2.0;
  r[0] = t * (R[7] - R[5]);
  r[1] = t * (R[2] - R[6]);
  r[2] = t * (R[3] - R[1]);
}

FFD_HD void jlog3(const double* r, double th, double* J) {
  const double eps3 = 6.0554544523933395e-06;
  double alpha, beta;
  if (th >= eps3) {
    double st, ct;
    sincos_(th, st, ct);
    const double st_1mct = st / (1.0 - ct);
    alpha = th * st_1mct / 2.0;
    beta = 1.0 / (th * th) - st_1mct / (2.0 * th);
  } else {
    alpha = 1.0;
    beta = 1.0 / 12.0;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) J[3 * i + j] = beta * r[i] * r[j] + (i == j ? alpha : 0.0);
  J[1] += -0.5 * r[2];
  J[2] += 0.5 * r[1];
  J[3] += 0.5 * r[2];
  J[5] += -0.5 * r[0];
  J[6] += -0.5 * r[1];
  J[7] += 0.5 * r[0];
}

FFD_HD void barrier(double r, double lb, double ub, double& a, double& Ar, double& Arr) {
  const double dl = r - lb, du = r - ub;
  const double rl = dl < 0.0 ? dl : 0.0;
  const double ru = du > 0.0 ? du : 0.0;
  a = 0.5 * rl * rl + 0.5 * ru * ru;
  Ar = rl + ru;
  Arr = (dl <= 0.0 ? 1.0 : 0.0) + (du >= 0.0 ? 1.0 : 0.0);
}

// Friction-cone cost on the world-aligned contact force lam (nc = 3):
// ResidualModelContactFrictionCone r = A lam over crocoddyl.FrictionCone(I, mu,
// nf = 4, inner = False) with a QuadraticBarrier narrowed by friction_margin
// (crocoddyl_classical.py:678-687, 891-903, 999-1018; FF :959-966).  Returns
// the weighted cost and, if gl != nullptr, the Gauss-Newton gradient gl[3] =
// w A^T A_r and Hessian w A^T diag(A_rr) A (diagonal Hd[3], off-diagonal
// Ho[3] = (1,0), (2,0), (2,1)) in lambda space.
FFD_HD double friction_cone(const DevConsts& C, const double* lam, double* gl, double* Hd, double* Ho) {
  double c = 0.0;
  double g0 = 0.0, g1 = 0.0, g2 = 0.0, h00 = 0.0, h11 = 0.0, h22 = 0.0, h10 = 0.0, h20 = 0.0, h21 = 0.0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const double* A = C.fc_A[k];
    const double r = A[0] * lam[0] + A[1] * lam[1] + A[2] * lam[2];
    double ai, Ar, Arr;
    barrier(r, C.fc_lb[k], C.fc_ub[k], ai, Ar, Arr);
    c += ai;
    g0 += A[0] * Ar;
    g1 += A[1] * Ar;
    g2 += A[2] * Ar;
    h00 += A[0] * Arr * A[0];
    h11 += A[1] * Arr * A[1];
    h22 += A[2] * Arr * A[2];
    h10 += A[1] * Arr * A[0];
    h20 += A[2] * Arr * A[0];
    h21 += A[2] * Arr * A[1];
  }
  if (gl != nullptr) {
    const double w = C.w_fc;
    gl[0] = w * g0;
    gl[1] = w * g1;
    gl[2] = w * g2;
    Hd[0] = w * h00;
    Hd[1] = w * h11;
    Hd[2] = w * h22;
    Ho[0] = w * h10;
    Ho[1] = w * h20;
    Ho[2] = w * h21;
  }
  return C.w_fc * c;
}

// ---------------------------------------------------------------------------
// primal
// ---------------------------------------------------------------------------
struct Primal {
  // dynamics
  double a[NQ], lam[3];
  double L[28];      // chol(M) packed
  double Jc[3][NQ];  // contact Jacobian rows
  double Y[3][NQ];   // L^-1 Jc^T  (column per contact dim)
  double Ls[6];      // chol(S), S = Jc M^-1 Jc^T + eps I
  // kinematics needed by the tangent / residual Jacobians
  double z[NQ][3], o[NQ][3], pee[3], Ree[9];
  double r_rot[3], th_rot;
  // Gauss-Newton data: dense rows 0..2 translation, 3..5 rotation, 6..11
  // frame velocity (lin, ang), 12.. force;  D = w * A_rr,  g = w * A_r.
  // The force block's Hessian is not diagonal once the friction cone couples
  // the components: Dfo holds its off-diagonal (1,0), (2,0), (2,1) entries.
  double D[NDENSE_MAX], g[NDENSE_MAX];
  double Dfo[3];
  double Dx[14], gx[14];  // state-residual costs (R_x = I)
  double Du[7], gu[7];    // control-residual costs (R_u = I)
  double cost;            // DAM cost (unscaled)
  double xnext[14];
};

// field-wise copy (static indices only, so a register-resident Primal is not
// forced into scratch memory by a whole-struct memcpy)
FFD_HD void copy_primal(const Primal& s, Primal& d) {
#pragma unroll
  for (int i = 0; i < NQ; ++i) d.a[i] = s.a[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) d.lam[i] = s.lam[i];
#pragma unroll
  for (int i = 0; i < 28; ++i) d.L[i] = s.L[i];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      d.Jc[r][i] = s.Jc[r][i];
      d.Y[r][i] = s.Y[r][i];
    }
#pragma unroll
  for (int i = 0; i < 6; ++i) d.Ls[i] = s.Ls[i];
#pragma unroll
  for (int i = 0; i < NQ; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      d.z[i][k] = s.z[i][k];
      d.o[i][k] = s.o[i][k];
    }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    d.pee[i] = s.pee[i];
    d.r_rot[i] = s.r_rot[i];
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) d.Ree[i] = s.Ree[i];
  d.th_rot = s.th_rot;
#pragma unroll
  for (int i = 0; i < NDENSE_MAX; ++i) {
    d.D[i] = s.D[i];
    d.g[i] = s.g[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) d.Dfo[i] = s.Dfo[i];
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    d.Dx[i] = s.Dx[i];
    d.gx[i] = s.gx[i];
    d.xnext[i] = s.xnext[i];
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    d.Du[i] = s.Du[i];
    d.gu[i] = s.gu[i];
  }
  d.cost = s.cost;
}

// n-dim force vector in world coordinates from lambda
template <int NC> FFD_HD void force_world(const double* lam, double* fw) {
  if (NC == 1) {
    fw[0] = 0.0;
    fw[1] = 0.0;
    fw[2] = lam[0];
  } else {
    fw[0] = lam[0];
    fw[1] = lam[1];
    fw[2] = lam[2];
  }
}

// x: inner state (14), u: inner control (7, ignored for MODE_TERMINAL_X),
// ref: p_ref(3), v_ref(3) for this node, xreg (14), tau_ref (7).
template <int NC>
FFD_HD void node_primal(const DevConsts& C, int mode, bool surface, const double* x, const double* u,
                        const double* ref, const double* xreg, const double* tauref, Primal& P,
                        Primal* gout = nullptr) {
  // gout: each block of fields is stored as soon as it is final, so the
  // registers holding it can be reused (a whole-struct copy at the end would
  // keep all ~225 words live to the last instruction).
  constexpr int nc = NC;
  const bool with_dyn = mode != MODE_TERMINAL_X;
  const bool terminal = mode != MODE_RUNNING;
  const double* q = x;
  const double* v = x + NQ;
  double zero[NQ] = {0, 0, 0, 0, 0, 0, 0};
  RBOut<double> K;
  double M[28];
  if (with_dyn) {
    rb_pass<double, true, true>(C.rb, q, v, zero, nullptr, K, M);
  } else {
    rb_pass<double, false, false>(C.rb, q, v, zero, nullptr, K, nullptr);
  }
  #pragma unroll
  for (int i = 0; i < NQ; ++i) {
    P.z[i][0] = K.z[i].x;
    P.z[i][1] = K.z[i].y;
    P.z[i][2] = K.z[i].z;
    P.o[i][0] = K.o[i].x;
    P.o[i][1] = K.o[i].y;
    P.o[i][2] = K.o[i].z;
  }
  P.pee[0] = K.pee.x;
  P.pee[1] = K.pee.y;
  P.pee[2] = K.pee.z;
  #pragma unroll
  for (int k = 0; k < 9; ++k) P.Ree[k] = K.Ree.m[k];
  if (gout) {
  #pragma unroll
    for (int i = 0; i < NQ; ++i)
  #pragma unroll
      for (int k = 0; k < 3; ++k) {
        gout->z[i][k] = P.z[i][k];
        gout->o[i][k] = P.o[i][k];
      }
  #pragma unroll
    for (int k = 0; k < 3; ++k) gout->pee[k] = P.pee[k];
  #pragma unroll
    for (int k = 0; k < 9; ++k) gout->Ree[k] = P.Ree[k];
  }
  const double pstar[3] = {ref[0], ref[1], ref[2] - C.z_press};
  P.lam[0] = P.lam[1] = P.lam[2] = 0.0;
  if (with_dyn) {
    #pragma unroll
    for (int k = 0; k < 28; ++k) P.L[k] = M[k];
    chol_packed<NQ>(P.L);  // M is SPD for the arm
    double af[NQ];
    #pragma unroll
    for (int i = 0; i < NQ; ++i) af[i] = u[i] - K.tau[i];
    chol_solve<NQ>(P.L, af);
    if (surface) {
      // contact Jacobian rows (LWA linear, components z or xyz): z_i x (p - o_i)
      constexpr int c0 = NC == 1 ? 2 : 0;
      double gam[3];
      const double ap[3] = {K.ap.x, K.ap.y, K.ap.z};
      const double vp[3] = {K.vp.x, K.vp.y, K.vp.z};
      #pragma unroll
      for (int r = 0; r < nc; ++r) {
        const int cmp = c0 + r;
        gam[r] = ap[cmp] + C.Kp * (P.pee[cmp] - pstar[cmp]) + C.Kd * vp[cmp];
        #pragma unroll
        for (int i = 0; i < NQ; ++i) {
          const double dx = P.pee[0] - P.o[i][0], dy = P.pee[1] - P.o[i][1], dz = P.pee[2] - P.o[i][2];
          const double cr[3] = {P.z[i][1] * dz - P.z[i][2] * dy, P.z[i][2] * dx - P.z[i][0] * dz,
                                P.z[i][0] * dy - P.z[i][1] * dx};
          P.Jc[r][i] = cr[cmp];
        }
      }
      // Y = L^-1 Jc^T, S = Y^T Y + eps I
      #pragma unroll
      for (int r = 0; r < nc; ++r) {
        #pragma unroll
        for (int i = 0; i < NQ; ++i) P.Y[r][i] = P.Jc[r][i];
        fwd_sub<NQ>(P.L, P.Y[r]);
      }
      double S[6];
      #pragma unroll
      for (int r = 0; r < nc; ++r)
        #pragma unroll
        for (int s = 0; s <= r; ++s) {
          double acc = 0.0;
          #pragma unroll
          for (int i = 0; i < NQ; ++i) acc += P.Y[r][i] * P.Y[s][i];
          S[tri(r, s)] = acc + (r == s ? C.eps : 0.0);
        }
      #pragma unroll
      for (int k = 0; k < 6; ++k) P.Ls[k] = S[k];
      double yl[3];
      #pragma unroll
      for (int r = 0; r < nc; ++r) {
        double acc = gam[r];
        #pragma unroll
        for (int i = 0; i < NQ; ++i) acc += P.Jc[r][i] * af[i];
        yl[r] = acc;
      }
      chol_packed<NC>(P.Ls);
      chol_solve<NC>(P.Ls, yl);
      // lambda = -y_l ;  a = af + M^-1 Jc^T lambda
      double t7[NQ];
      #pragma unroll
      for (int i = 0; i < NQ; ++i) {
        double acc = 0.0;
        #pragma unroll
        for (int r = 0; r < nc; ++r) acc += P.Jc[r][i] * (-yl[r]);
        t7[i] = acc;
      }
      chol_solve<NQ>(P.L, t7);
      #pragma unroll
      for (int i = 0; i < NQ; ++i) P.a[i] = af[i] + t7[i];
      #pragma unroll
      for (int r = 0; r < nc; ++r) P.lam[r] = -yl[r];
    } else {
      #pragma unroll
      for (int i = 0; i < NQ; ++i) P.a[i] = af[i];
    }
  }

  if (gout) {
  #pragma unroll
    for (int i = 0; i < NQ; ++i) gout->a[i] = P.a[i];
  #pragma unroll
    for (int i = 0; i < 3; ++i) gout->lam[i] = P.lam[i];
  #pragma unroll
    for (int i = 0; i < 28; ++i) gout->L[i] = P.L[i];
  #pragma unroll
    for (int r = 0; r < 3; ++r)
  #pragma unroll
      for (int i = 0; i < NQ; ++i) {
        gout->Jc[r][i] = P.Jc[r][i];
        gout->Y[r][i] = P.Y[r][i];
      }
  #pragma unroll
    for (int i = 0; i < 6; ++i) gout->Ls[i] = P.Ls[i];
  }
  // ---------------- costs (CostModelSum, in _make_dam order) ----------------
  double cost = 0.0;
  #pragma unroll
  for (int k = 0; k < NDENSE_MAX; ++k) P.D[k] = P.g[k] = 0.0;
  P.Dfo[0] = P.Dfo[1] = P.Dfo[2] = 0.0;
  #pragma unroll
  for (int k = 0; k < 14; ++k) P.Dx[k] = P.gx[k] = 0.0;
  #pragma unroll
  for (int k = 0; k < 7; ++k) P.Du[k] = P.gu[k] = 0.0;
  if (C.variant == FFDDP_CLASSICAL || C.inner_state_reg) {
    // posture: Quad on x - x_reg_ref
    double a = 0.0;
    #pragma unroll
    for (int i = 0; i < 14; ++i) {
      const double r = x[i] - xreg[i];
      a += r * r;
      P.Dx[i] += C.w_post;
      P.gx[i] += C.w_post * r;
    }
    cost += C.w_post * (0.5 * a);
    // v_damp: WeightedQuad [0*7, vdw] on x - 0
    a = 0.0;
    #pragma unroll
    for (int i = 0; i < 14; ++i) {
      const double wi = i < 7 ? 0.0 : C.vdw[i - 7];
      a += wi * x[i] * x[i];
      P.Dx[i] += C.w_v * wi;
      P.gx[i] += C.w_v * wi * x[i];
    }
    cost += C.w_v * (0.5 * a);
  }
  if (C.has_qsoft) {
    double a = 0.0;
    #pragma unroll
    for (int i = 0; i < 14; ++i) {
      double ai, Ar, Arr;
      barrier(x[i] - C.qs_xref[i], C.qs_lb[i], C.qs_ub[i], ai, Ar, Arr);
      a += ai;
      P.Dx[i] += C.w_qs * Arr;
      P.gx[i] += C.w_qs * Ar;
    }
    cost += C.w_qs * a;
  }
  {  // ee_ori: FrameRotation(R_des), WeightedQuad(ori_weights)
    double Rrel[9];
    #pragma unroll
    for (int i = 0; i < 3; ++i)
      #pragma unroll
      for (int j = 0; j < 3; ++j)
        Rrel[3 * i + j] = C.Rdes[0 * 3 + i] * P.Ree[0 * 3 + j] + C.Rdes[1 * 3 + i] * P.Ree[1 * 3 + j] +
                          C.Rdes[2 * 3 + i] * P.Ree[2 * 3 + j];
    log3(Rrel, P.r_rot, P.th_rot);
    double a = 0.0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
      a += C.ori_w[i] * P.r_rot[i] * P.r_rot[i];
      P.D[3 + i] += C.w_ori * C.ori_w[i];
      P.g[3 + i] += C.w_ori * C.ori_w[i] * P.r_rot[i];
    }
    cost += C.w_ori * (0.5 * a);
  }
  const double vel[6] = {K.vp.x, K.vp.y, K.vp.z, K.w.x, K.w.y, K.w.z};
  {  // w_damp: FrameVelocity(0, LWA), WeightedQuad [0,0,0, ww]
    double a = 0.0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
      a += C.wd_w[i] * vel[3 + i] * vel[3 + i];
      P.D[9 + i] += C.w_wd * C.wd_w[i];
      P.g[9 + i] += C.w_wd * C.wd_w[i] * vel[3 + i];
    }
    cost += C.w_wd * (0.5 * a);
  }
  if (!terminal && (C.variant == FFDDP_CLASSICAL || C.inner_tau_reg)) {
    double a = 0.0;
    #pragma unroll
    for (int i = 0; i < 7; ++i) {
      const double r = u[i] - tauref[i];
      a += r * r;
      P.Du[i] += C.w_tau;
      P.gu[i] += C.w_tau * r;
    }
    cost += C.w_tau * (0.5 * a);
    if (C.has_tsoft) {
      a = 0.0;
      #pragma unroll
      for (int i = 0; i < 7; ++i) {
        double ai, Ar, Arr;
        barrier(u[i], C.ts_lb[i], C.ts_ub[i], ai, Ar, Arr);
        a += ai;
        P.Du[i] += C.w_ts * Arr;
        P.gu[i] += C.w_ts * Ar;
      }
      cost += C.w_ts * a;
    }
  }
  if (!surface) {
    // ee_pos: FrameTranslation(p_ref), WeightedQuad [1,1,2.5]
    double a = 0.0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double r = P.pee[i] - ref[i];
      a += C.ee_pos_w[i] * r * r;
      P.D[i] += C.w_ee_pos * C.ee_pos_w[i];
      P.g[i] += C.w_ee_pos * C.ee_pos_w[i] * r;
    }
    cost += C.w_ee_pos * (0.5 * a);
  } else {
    {  // ee_xy: FrameTranslation(p_ref), WeightedQuad [1,1,0]
      const double rx = P.pee[0] - ref[0], ry = P.pee[1] - ref[1], rz = P.pee[2] - ref[2];
      const double a = rx * rx + ry * ry + 0.0 * rz * rz;
      P.D[0] += C.w_tp;
      P.D[1] += C.w_tp;
      P.g[0] += C.w_tp * rx;
      P.g[1] += C.w_tp * ry;
      cost += C.w_tp * (0.5 * a);
    }
    {  // ee_vxy: FrameVelocity([v_ref_xy, 0; 0], LWA), WeightedQuad [1,1,0,0,0,0]
      const double rx = vel[0] - ref[3], ry = vel[1] - ref[4];
      const double a = rx * rx + ry * ry;
      P.D[6] += C.w_tv;
      P.D[7] += C.w_tv;
      P.g[6] += C.w_tv * rx;
      P.g[7] += C.w_tv * ry;
      cost += C.w_tv * (0.5 * a);
    }
    if (C.has_pz) {  // plane_z: FrameTranslation(p_contact), WeightedQuad [0,0,1]
      const double rz = P.pee[2] - pstar[2];
      P.D[2] += C.w_pz;
      P.g[2] += C.w_pz * rz;
      cost += C.w_pz * (0.5 * rz * rz);
    }
    if (C.has_vz) {  // vz_damp: FrameVelocity(0, LWA), WeightedQuad [0,0,1,0,0,0]
      P.D[8] += C.w_vz;
      P.g[8] += C.w_vz * vel[2];
      cost += C.w_vz * (0.5 * vel[2] * vel[2]);
    }
    // contact force: lambda (classical terminal calc(x): zero-initialised data, R2)
    double lam[3] = {0, 0, 0};
    if (mode != MODE_TERMINAL_X)
      #pragma unroll
      for (int r = 0; r < nc; ++r) lam[r] = P.lam[r];
    if (NC == 3 && C.has_fc) {
      double gl[3], Hd[3], Ho[3];
      cost += friction_cone(C, lam, gl, Hd, Ho);
      #pragma unroll
      for (int r = 0; r < 3; ++r) {
        P.D[12 + r] += Hd[r];
        P.g[12 + r] += gl[r];
        P.Dfo[r] = Ho[r];
      }
    }
    if (C.has_uni) {
      double a = 0.0;
      #pragma unroll
      for (int r = 0; r < nc; ++r) {
        double ai, Ar, Arr;
        barrier(lam[r], C.uni_lb[r], C.uni_ub[r], ai, Ar, Arr);
        a += ai;
        P.D[12 + r] += C.w_uni * Arr;
        P.g[12 + r] += C.w_uni * Ar;
      }
      cost += C.w_uni * a;
    }
    if (C.has_fn) {
      double a = 0.0;
      #pragma unroll
      for (int r = 0; r < nc; ++r) {
        const double rr = lam[r] - C.fn_ref[r];
        a += C.fn_w[r] * rr * rr;
        P.D[12 + r] += C.w_fn * C.fn_w[r];
        P.g[12 + r] += C.w_fn * C.fn_w[r] * rr;
      }
      cost += C.w_fn * (0.5 * a);
    }
  }
  P.cost = cost;
  if (with_dyn) {
    const double dt = C.dt;
    #pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const double vn = v[i] + P.a[i] * dt;
      P.xnext[i] = q[i] + (v[i] * dt + P.a[i] * dt * dt);
      P.xnext[NQ + i] = vn;
    }
  } else {
    #pragma unroll
    for (int i = 0; i < 14; ++i) P.xnext[i] = x[i];
  }
  if (gout) {
  #pragma unroll
    for (int i = 0; i < 3; ++i) gout->r_rot[i] = P.r_rot[i];
    gout->th_rot = P.th_rot;
  #pragma unroll
    for (int i = 0; i < NDENSE_MAX; ++i) {
      gout->D[i] = P.D[i];
      gout->g[i] = P.g[i];
    }
  #pragma unroll
    for (int i = 0; i < 3; ++i) gout->Dfo[i] = P.Dfo[i];
  #pragma unroll
    for (int i = 0; i < 14; ++i) {
      gout->Dx[i] = P.Dx[i];
      gout->gx[i] = P.gx[i];
      gout->xnext[i] = P.xnext[i];
    }
  #pragma unroll
    for (int i = 0; i < 7; ++i) {
      gout->Du[i] = P.Du[i];
      gout->gu[i] = P.gu[i];
    }
    gout->cost = P.cost;
  }
}

// ---------------------------------------------------------------------------
// Closed-form state tangent (replaces the forward-mode dual pass above in the
// calcDiff kernel).  World-frame spatial algebra, S_j = (o_j x z_j, z_j):
//   q_j : every link k >= j rotates about S_j, so
//         dV_k = S_j x (V_k - V_{j-1}),
//         dA_k = S_j x (A_k - A_{j-1}) + cV x (V_k - V_{j-1}),  cV = -S_j x V_{j-1}
//         dF_k = S_j x* F_k + I_k Y_k + T x* H_k + V_k x* (I_k T),
//                Y_k = cA + cV x (V_k - V_{j-1}), cA = -S_j x (A_{j-1} - G), T = cV
//   v_j : dV_k = S_j, dA_k = S_j x (V_k - 2 V_{j-1}),
//         dF_k = I_k Y_k + T x* H_k + V_k x* (I_k T),
//                Y_k = -S_j x V_{j-1} + S_j x (V_k - V_{j-1}), T = S_j
// (F = I (A - G) + V x* (I V), H = I V; x = motion cross, x* = force cross),
// then d tau_i = dS_i . Ftot_i + S_i . dFtot_i over the suffix sums (the
// contact force is a world-fixed vector at the moving EE point).  Same
// outputs as node_tangent_state: da, dlam, residual-Jacobian column.
// ---------------------------------------------------------------------------
FFD_HD void sp_mcross(const double* sv, const double* sw, const double* xv, const double* xw, double* ov, double* ow) {
  // (sw x xv + sv x xw, sw x xw)
  ov[0] = sw[1] * xv[2] - sw[2] * xv[1] + sv[1] * xw[2] - sv[2] * xw[1];
  ov[1] = sw[2] * xv[0] - sw[0] * xv[2] + sv[2] * xw[0] - sv[0] * xw[2];
  ov[2] = sw[0] * xv[1] - sw[1] * xv[0] + sv[0] * xw[1] - sv[1] * xw[0];
  ow[0] = sw[1] * xw[2] - sw[2] * xw[1];
  ow[1] = sw[2] * xw[0] - sw[0] * xw[2];
  ow[2] = sw[0] * xw[1] - sw[1] * xw[0];
}
FFD_HD void sp_fcross(const double* xv, const double* xw, const double* f, const double* n, double* of, double* on) {
  // (xw x f, xw x n + xv x f)
  of[0] = xw[1] * f[2] - xw[2] * f[1];
  of[1] = xw[2] * f[0] - xw[0] * f[2];
  of[2] = xw[0] * f[1] - xw[1] * f[0];
  on[0] = xw[1] * n[2] - xw[2] * n[1] + xv[1] * f[2] - xv[2] * f[1];
  on[1] = xw[2] * n[0] - xw[0] * n[2] + xv[2] * f[0] - xv[0] * f[2];
  on[2] = xw[0] * n[1] - xw[1] * n[0] + xv[0] * f[1] - xv[1] * f[0];
}
FFD_HD void sp_imul(double m, const double* h, const double* IO, const double* xv, const double* xw, double* of,
                    double* on) {
  // (m xv - h x xw, h x xv + I_O xw)
  of[0] = m * xv[0] - (h[1] * xw[2] - h[2] * xw[1]);
  of[1] = m * xv[1] - (h[2] * xw[0] - h[0] * xw[2]);
  of[2] = m * xv[2] - (h[0] * xw[1] - h[1] * xw[0]);
  on[0] = (h[1] * xv[2] - h[2] * xv[1]) + IO[0] * xw[0] + IO[1] * xw[1] + IO[2] * xw[2];
  on[1] = (h[2] * xv[0] - h[0] * xv[2]) + IO[1] * xw[0] + IO[3] * xw[1] + IO[4] * xw[2];
  on[2] = (h[0] * xv[1] - h[1] * xv[0]) + IO[2] * xw[0] + IO[4] * xw[1] + IO[5] * xw[2];
}

// Two parts, so a kernel can store the residual-Jacobian column between them
// (k_node: the column is not live across the contact solves):
//   node_tangent_state_links    link-record part: the column (force rows 0),
//                               d tau (r1) and dh; reads LK and P
//   node_tangent_state_contact  contact solves: da, dlam, force rows; reads P only
template <int NC>
FFD_HD void node_tangent_state_links(const DevConsts& C, int mode, bool surface, const double* LK, const Primal& P,
                                     int dir, double* r1, double* dh, double* col) {
  constexpr int nc = NC;
  const bool with_dyn = mode != MODE_TERMINAL_X;
  const bool isq = dir < NQ;
  const int j = isq ? dir : dir - NQ;
  const double* Lj = LK + j * LK_STRIDE;
  const double* Lp = LK + (j > 0 ? j - 1 : 0) * LK_STRIDE;
  const double pz = j > 0 ? 1.0 : 0.0;
  double Sv[3], Sz[3], oj[3], Vpv[3], Vpw[3], Apv[3], Apw[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    Sv[k] = Lj[LK_SV + k];
    Sz[k] = Lj[LK_Z + k];
    oj[k] = Lj[LK_O + k];
    Vpv[k] = pz * Lp[LK_VO + k];
    Vpw[k] = pz * Lp[LK_W + k];
    Apv[k] = pz * Lp[LK_AO + k] - C.rb.gravity[k];  // A_{j-1} - G
    Apw[k] = pz * Lp[LK_AL + k];
  }
  const double* E = LK + LK_EE;
  const double pee[3] = {E[0], E[1], E[2]}, vp[3] = {E[3], E[4], E[5]}, wee[3] = {E[6], E[7], E[8]};
  const double* L6 = LK + (NQ - 1) * LK_STRIDE;
  const double qs = isq ? 1.0 : 0.0;
  // cV = -S_j x V_{j-1} ; T = q ? cV : S_j ; Cc = q ? -S_j x (A_{j-1} - G) : cV
  double cVv[3], cVw[3], cAv[3], cAw[3];
  sp_mcross(Sv, Sz, Vpv, Vpw, cVv, cVw);
  sp_mcross(Sv, Sz, Apv, Apw, cAv, cAw);
  double Tv[3], Tw[3], Ccv[3], Ccw[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    cVv[k] = -cVv[k];
    cVw[k] = -cVw[k];
    Tv[k] = isq ? cVv[k] : Sv[k];
    Tw[k] = isq ? cVw[k] : Sz[k];
    Ccv[k] = isq ? -cAv[k] : cVv[k];
    Ccw[k] = isq ? -cAw[k] : cVw[k];
  }
  // Dm = q ? cV : S_j  (multiplies (V_k - V_{j-1}) in Y_k); for v_j Y_k = cV + S_j x (V_k - V_{j-1})
  // ---- end-effector tangents ----
  double dpee[3] = {0, 0, 0};
  {
    const double r[3] = {pee[0] - oj[0], pee[1] - oj[1], pee[2] - oj[2]};
    dpee[0] = qs * (Sz[1] * r[2] - Sz[2] * r[1]);
    dpee[1] = qs * (Sz[2] * r[0] - Sz[0] * r[2]);
    dpee[2] = qs * (Sz[0] * r[1] - Sz[1] * r[0]);
  }
  double d6v[3], d6w[3];  // dV_6
  double dA6v[3], dA6w[3];
  {
    const double D6v[3] = {L6[LK_VO] - Vpv[0], L6[LK_VO + 1] - Vpv[1], L6[LK_VO + 2] - Vpv[2]};
    const double D6w[3] = {L6[LK_W] - Vpw[0], L6[LK_W + 1] - Vpw[1], L6[LK_W + 2] - Vpw[2]};
    double t1v[3], t1w[3];
    sp_mcross(Sv, Sz, D6v, D6w, t1v, t1w);  // S_j x (V_6 - V_{j-1})
    // A_6 - A_{j-1}  (gravity cancels)
    const double DAv[3] = {L6[LK_AO] - pz * Lp[LK_AO], L6[LK_AO + 1] - pz * Lp[LK_AO + 1], L6[LK_AO + 2] - pz * Lp[LK_AO + 2]};
    const double DAw[3] = {L6[LK_AL] - Apw[0], L6[LK_AL + 1] - Apw[1], L6[LK_AL + 2] - Apw[2]};
    double t2v[3], t2w[3], t3v[3], t3w[3];
    sp_mcross(Sv, Sz, DAv, DAw, t2v, t2w);   // S_j x (A_6 - A_{j-1})
    sp_mcross(cVv, cVw, D6v, D6w, t3v, t3w);  // cV x (V_6 - V_{j-1})
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      d6v[k] = isq ? t1v[k] : Sv[k];
      d6w[k] = isq ? t1w[k] : Sz[k];
      // q: S x (A6 - Ap) + cV x (V6 - Vp) ; v: S x (V6 - Vp) + cV  x ... = S x (V6 - 2 Vp) = t1 + cV
      dA6v[k] = isq ? t2v[k] + t3v[k] : t1v[k] + cVv[k];
      dA6w[k] = isq ? t2w[k] + t3w[k] : t1w[k] + cVw[k];
    }
  }
  double dvp[3], dap[3];
  {
    double c1[3], c2[3];
    const double* w6 = wee;
    // dvp = dvO + dw x p + w x dp
    c1[0] = d6w[1] * pee[2] - d6w[2] * pee[1];
    c1[1] = d6w[2] * pee[0] - d6w[0] * pee[2];
    c1[2] = d6w[0] * pee[1] - d6w[1] * pee[0];
    c2[0] = w6[1] * dpee[2] - w6[2] * dpee[1];
    c2[1] = w6[2] * dpee[0] - w6[0] * dpee[2];
    c2[2] = w6[0] * dpee[1] - w6[1] * dpee[0];
#pragma unroll
    for (int k = 0; k < 3; ++k) dvp[k] = d6v[k] + c1[k] + c2[k];
    // dap = daO + dal x p + al x dp + dw x vp + w x dvp
    const double al6[3] = {L6[LK_AL], L6[LK_AL + 1], L6[LK_AL + 2]};
    double c3[3], c4[3], c5[3], c6[3];
    c3[0] = dA6w[1] * pee[2] - dA6w[2] * pee[1];
    c3[1] = dA6w[2] * pee[0] - dA6w[0] * pee[2];
    c3[2] = dA6w[0] * pee[1] - dA6w[1] * pee[0];
    c4[0] = al6[1] * dpee[2] - al6[2] * dpee[1];
    c4[1] = al6[2] * dpee[0] - al6[0] * dpee[2];
    c4[2] = al6[0] * dpee[1] - al6[1] * dpee[0];
    c5[0] = d6w[1] * vp[2] - d6w[2] * vp[1];
    c5[1] = d6w[2] * vp[0] - d6w[0] * vp[2];
    c5[2] = d6w[0] * vp[1] - d6w[1] * vp[0];
    c6[0] = w6[1] * dvp[2] - w6[2] * dvp[1];
    c6[1] = w6[2] * dvp[0] - w6[0] * dvp[2];
    c6[2] = w6[0] * dvp[1] - w6[1] * dvp[0];
#pragma unroll
    for (int k = 0; k < 3; ++k) dap[k] = dA6v[k] + c3[k] + c4[k] + c5[k] + c6[k];
  }
  // dh = d (classical acc + Kp (p - p*) + Kd v_p) / d x_j
  {
    constexpr int c0 = NC == 1 ? 2 : 0;
#pragma unroll
    for (int r = 0; r < nc; ++r) dh[r] = dap[c0 + r] + C.Kp * dpee[c0 + r] + C.Kd * dvp[c0 + r];
  }
  // ---- residual-Jacobian column ----
  {
    double wl[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) wl[i] = qs * (P.Ree[0 * 3 + i] * Sz[0] + P.Ree[1 * 3 + i] * Sz[1] + P.Ree[2 * 3 + i] * Sz[2]);
    col[0] = dpee[0];
    col[1] = dpee[1];
    col[2] = dpee[2];
    double Jlog[9];
    jlog3(P.r_rot, P.th_rot, Jlog);
#pragma unroll
    for (int i = 0; i < 3; ++i) col[3 + i] = Jlog[3 * i + 0] * wl[0] + Jlog[3 * i + 1] * wl[1] + Jlog[3 * i + 2] * wl[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      col[6 + i] = dvp[i];
      col[9 + i] = d6w[i];
    }
#pragma unroll
    for (int r = 0; r < nc; ++r) col[12 + r] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < NQ; ++i) r1[i] = 0.0;
  if (!with_dyn) return;
  // ---- d tau = d RNEA(q, v, a, fext = lambda) / d x_j at fixed a, lambda ----
  double lw[3] = {0, 0, 0};
  if (surface) force_world<NC>(P.lam, lw);
  double Fe[3], dFe[3];  // moment parts of Fext and dFext (linear parts: lw and 0)
  Fe[0] = pee[1] * lw[2] - pee[2] * lw[1];
  Fe[1] = pee[2] * lw[0] - pee[0] * lw[2];
  Fe[2] = pee[0] * lw[1] - pee[1] * lw[0];
  dFe[0] = dpee[1] * lw[2] - dpee[2] * lw[1];
  dFe[1] = dpee[2] * lw[0] - dpee[0] * lw[2];
  dFe[2] = dpee[0] * lw[1] - dpee[1] * lw[0];
  double FSf[3] = {0, 0, 0}, FSn[3] = {0, 0, 0}, dSf[3] = {0, 0, 0}, dSn[3] = {0, 0, 0};
#pragma unroll
  for (int k = NQ - 1; k >= 0; --k) {
    const double* Lk = LK + k * LK_STRIDE;
    const double* Vk = Lk + LK_VO;
    const double* Wk = Lk + LK_W;
    const double* Fk = Lk + LK_F;
    const double* Nk = Lk + LK_N;
    const double* Hl = Lk + LK_HL;
    const double* Ha = Lk + LK_HA;
    const double m = Lk[LK_M];
    const double* h = Lk + LK_H;
    const double* IO = Lk + LK_IO;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      FSf[e] += Fk[e];
      FSn[e] += Nk[e];
    }
    const double mk = (k >= j) ? 1.0 : 0.0;
    // Y = Cc + Dm x (V_k - V_{j-1}),  Dm = q ? cV : S_j
    const double Dv[3] = {Vk[0] - Vpv[0], Vk[1] - Vpv[1], Vk[2] - Vpv[2]};
    const double Dw[3] = {Wk[0] - Vpw[0], Wk[1] - Vpw[1], Wk[2] - Vpw[2]};
    double Dmv[3], Dmw[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      Dmv[e] = isq ? cVv[e] : Sv[e];
      Dmw[e] = isq ? cVw[e] : Sz[e];
    }
    double Yv[3], Yw[3];
    sp_mcross(Dmv, Dmw, Dv, Dw, Yv, Yw);
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      Yv[e] += Ccv[e];
      Yw[e] += Ccw[e];
    }
    double a1f[3], a1n[3], a2f[3], a2n[3], a3f[3], a3n[3], ITf[3], ITn[3], a4f[3], a4n[3];
    sp_imul(m, h, IO, Yv, Yw, a1f, a1n);      // I_k Y
    sp_fcross(Tv, Tw, Hl, Ha, a2f, a2n);      // T x* H_k
    sp_imul(m, h, IO, Tv, Tw, ITf, ITn);      // I_k T
    sp_fcross(Vk, Wk, ITf, ITn, a3f, a3n);    // V_k x* (I_k T)
    sp_fcross(Sv, Sz, Fk, Nk, a4f, a4n);      // S_j x* F_k   (q only)
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      dSf[e] += mk * (a1f[e] + a2f[e] + a3f[e] + qs * a4f[e]);
      dSn[e] += mk * (a1n[e] + a2n[e] + a3n[e] + qs * a4n[e]);
    }
    // dS_k = S_j x S_k for q_j, k > j
    const double* Svk = Lk + LK_SV;
    const double* Szk = Lk + LK_Z;
    double dSv[3], dSw[3];
    sp_mcross(Sv, Sz, Svk, Szk, dSv, dSw);
    const double ms = (isq && k > j) ? 1.0 : 0.0;
    const double Ftf[3] = {FSf[0] - lw[0], FSf[1] - lw[1], FSf[2] - lw[2]};
    const double Ftn[3] = {FSn[0] - Fe[0], FSn[1] - Fe[1], FSn[2] - Fe[2]};
    const double dFtn[3] = {dSn[0] - dFe[0], dSn[1] - dFe[1], dSn[2] - dFe[2]};
    const double dtau = ms * (dSv[0] * Ftf[0] + dSv[1] * Ftf[1] + dSv[2] * Ftf[2] + dSw[0] * Ftn[0] + dSw[1] * Ftn[1] +
                              dSw[2] * Ftn[2]) +
                        (Svk[0] * dSf[0] + Svk[1] * dSf[1] + Svk[2] * dSf[2] + Szk[0] * dFtn[0] + Szk[1] * dFtn[1] +
                         Szk[2] * dFtn[2]);
    r1[k] = -dtau;
  }
}

template <int NC>
FFD_HD void node_tangent_state_contact(int mode, bool surface, const Primal& P, const double* r1, const double* dh,
                                       double* da, double* dlam, double* col) {
  constexpr int nc = NC;
  dlam[0] = dlam[1] = dlam[2] = 0.0;
  if (mode == MODE_TERMINAL_X) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) da[i] = 0.0;
    return;
  }
  if (!surface) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) da[i] = r1[i];
    chol_solve<NQ>(P.L, da);
    return;
  }
  double mr[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) mr[i] = r1[i];
  chol_solve<NQ>(P.L, mr);
  double yl[3];
#pragma unroll
  for (int r = 0; r < nc; ++r) {
    double acc = dh[r];
#pragma unroll
    for (int i = 0; i < NQ; ++i) acc += P.Jc[r][i] * mr[i];
    yl[r] = acc;
  }
  chol_solve<NC>(P.Ls, yl);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    double acc = r1[i];
#pragma unroll
    for (int r = 0; r < nc; ++r) acc -= P.Jc[r][i] * yl[r];
    da[i] = acc;
  }
  chol_solve<NQ>(P.L, da);
#pragma unroll
  for (int r = 0; r < nc; ++r) {
    dlam[r] = -yl[r];
    col[12 + r] = dlam[r];
  }
}

// da = d a / d x_dir, dlam, residual-Jacobian column dir (both parts)
template <int NC>
FFD_HD void node_tangent_state_an(const DevConsts& C, int mode, bool surface, const double* LK, const Primal& P,
                                  int dir, double* da, double* dlam, double* col) {
  double r1[NQ], dh[3];
  node_tangent_state_links<NC>(C, mode, surface, LK, P, dir, r1, dh, col);
  node_tangent_state_contact<NC>(mode, surface, P, r1, dh, da, dlam, col);
}

// control direction k in [0,7): dg = -e_k, dh = 0
template <int NC>
FFD_HD void node_tangent_control(const DevConsts& C, bool surface, const Primal& P, int k, double* da, double* dlam) {
  constexpr int nc = NC;
  double r1[NQ];
  for (int i = 0; i < NQ; ++i) r1[i] = (i == k) ? 1.0 : 0.0;
  dlam[0] = dlam[1] = dlam[2] = 0.0;
  if (!surface) {
    chol_solve<NQ>(P.L, r1);
    for (int i = 0; i < NQ; ++i) da[i] = r1[i];
    return;
  }
  double mr[NQ];
  for (int i = 0; i < NQ; ++i) mr[i] = r1[i];
  chol_solve<NQ>(P.L, mr);
  double yl[3];
  for (int r = 0; r < nc; ++r) {
    double acc = 0.0;
    for (int i = 0; i < NQ; ++i) acc += P.Jc[r][i] * mr[i];
    yl[r] = acc;
  }
  chol_solve<NC>(P.Ls, yl);
  for (int i = 0; i < NQ; ++i) {
    double acc = r1[i];
    for (int r = 0; r < nc; ++r) acc -= P.Jc[r][i] * yl[r];
    da[i] = acc;
  }
  chol_solve<NQ>(P.L, da);
  for (int r = 0; r < nc; ++r) dlam[r] = -yl[r];
}

// Full node calc for the forward pass (variant-aware): y (nx), w (7) ->
// ynext (nx), cost.  Terminal: w ignored.  Returns lambda in P.lam.
template <int NC, bool FF>
FFD_HD void node_calc(const DevConsts& C, bool terminal, bool surface, const double* y, const double* w,
                      const double* ref, const double* xreg, const double* tauref, const double* yref, Primal& P,
                      double* ynext, double& cost) {
  if (!FF) {
    node_primal<NC>(C, terminal ? MODE_TERMINAL_X : MODE_RUNNING, surface, y, w, ref, xreg, tauref, P);
    for (int i = 0; i < 14; ++i) ynext[i] = P.xnext[i];
    cost = terminal ? P.cost : C.dt * P.cost;
    return;
  }
  const double* tau = y + 14;
  double wz[7] = {0, 0, 0, 0, 0, 0, 0};
  const double* ww = terminal ? wz : w;
  node_primal<NC>(C, terminal ? MODE_TERMINAL_U : MODE_RUNNING, surface, y, tau, ref, xreg, tauref, P);
  for (int i = 0; i < 14; ++i) ynext[i] = P.xnext[i];
  for (int i = 0; i < 7; ++i) ynext[14 + i] = C.alpha * tau[i] + C.beta * ww[i];
  double c = C.dt * P.cost;
  if (C.w_y > 0.0) {
    double a = 0.0;
    for (int i = 0; i < 21; ++i) {
      const double d = y[i] - yref[i];
      a += C.Wy2[i] * d * d;
    }
    c += 0.5 * C.w_y * a;
  }
  if (C.w_w > 0.0) {
    double a = 0.0;
    for (int i = 0; i < 7; ++i) a += ww[i] * ww[i];
    c += 0.5 * C.w_w * a;
  }
  if (C.w_ws > 0.0) {
    double a = 0.0;
    for (int i = 0; i < 7; ++i) {
      const double ov = fabs(ww[i]) - C.ws_lim[i];
      const double o = ov > 0.0 ? ov : 0.0;
      a += o * o;
    }
    c += C.w_ws * (0.5 * a);
  }
  cost = c;
}

}  // namespace ffddp
