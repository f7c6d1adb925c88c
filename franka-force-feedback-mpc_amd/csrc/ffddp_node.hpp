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
FFD_HD int rec_size(int nx) { return (rec_off_lam(nx) + 3 + 7) & ~7; }

// ---------------------------------------------------------------------------
// log3 / Jlog3 (pinocchio)
// ---------------------------------------------------------------------------
FFD_HD void log3(const double* R, double* r, double& th) {
  const double tr = R[0] + R[4] + R[8];
  double c = (tr - 1.0) / 2.0;
  c = c > 1.0 ? 1.0 : (c < -1.0 ? -1.0 : c);
  th = acos(c);
  const double eps3 = 6.0554544523933395e-06;  // eps^(1/3)
  const double t = (th > eps3 ? th / sin(th) : 1.0) / 2.0;
  r[0] = t * (R[7] - R[5]);
  r[1] = t * (R[2] - R[6]);
  r[2] = t * (R[3] - R[1]);
}

FFD_HD void jlog3(const double* r, double th, double* J) {
  const double eps3 = 6.0554544523933395e-06;
  double alpha, beta;
  if (th >= eps3) {
    const double st = sin(th), ct = cos(th);
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
  // frame velocity (lin, ang), 12.. force;  D = w * A_rr,  g = w * A_r
  double D[NDENSE_MAX], g[NDENSE_MAX];
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
                        const double* ref, const double* xreg, const double* tauref, Primal& P) {
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

  // ---------------- costs (CostModelSum, in _make_dam order) ----------------
  double cost = 0.0;
  #pragma unroll
  for (int k = 0; k < NDENSE_MAX; ++k) P.D[k] = P.g[k] = 0.0;
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
}

// ---------------------------------------------------------------------------
// tangent: state direction j in [0,14) of the inner model
//   da[7], dlam[nc], col = residual-Jacobian column j over the dense rows
// ---------------------------------------------------------------------------
template <int NC>
FFD_HD void node_tangent_state(const DevConsts& C, int mode, bool surface, const double* x, const double* ref,
                               const Primal& P, int j, double* da, double* dlam, double* col) {
  constexpr int nc = NC;
  const bool with_dyn = mode != MODE_TERMINAL_X;
  Dual q[NQ], v[NQ];
  for (int i = 0; i < NQ; ++i) {
    q[i] = {x[i], i == j ? 1.0 : 0.0};
    v[i] = {x[NQ + i], NQ + i == j ? 1.0 : 0.0};
  }
  RBOut<Dual> K;
  double fw[3];
  force_world<NC>(P.lam, fw);
  if (with_dyn) {
    rb_pass<Dual, true, false>(C.rb, q, v, P.a, surface ? fw : nullptr, K, nullptr);
  } else {
    const double zero[NQ] = {0, 0, 0, 0, 0, 0, 0};
    rb_pass<Dual, false, false>(C.rb, q, v, zero, nullptr, K, nullptr);
  }
  // residual-Jacobian column j over the dense rows
  const bool isq = j < NQ;
  double Jl[3] = {0, 0, 0}, wl[3] = {0, 0, 0};
  if (isq) {
    // LWA linear Jacobian column z_j x (p - o_j);  local angular R_ee^T z_j
    const double dx = P.pee[0] - P.o[j][0], dy = P.pee[1] - P.o[j][1], dz = P.pee[2] - P.o[j][2];
    Jl[0] = P.z[j][1] * dz - P.z[j][2] * dy;
    Jl[1] = P.z[j][2] * dx - P.z[j][0] * dz;
    Jl[2] = P.z[j][0] * dy - P.z[j][1] * dx;
    for (int i = 0; i < 3; ++i) wl[i] = P.Ree[0 * 3 + i] * P.z[j][0] + P.Ree[1 * 3 + i] * P.z[j][1] + P.Ree[2 * 3 + i] * P.z[j][2];
  }
  col[0] = Jl[0];
  col[1] = Jl[1];
  col[2] = Jl[2];
  double Jlog[9];
  jlog3(P.r_rot, P.th_rot, Jlog);
  for (int i = 0; i < 3; ++i) col[3 + i] = Jlog[3 * i + 0] * wl[0] + Jlog[3 * i + 1] * wl[1] + Jlog[3 * i + 2] * wl[2];
  col[6] = K.vp.x.d;
  col[7] = K.vp.y.d;
  col[8] = K.vp.z.d;
  col[9] = K.w.x.d;
  col[10] = K.w.y.d;
  col[11] = K.w.z.d;
  for (int r = 0; r < nc; ++r) col[12 + r] = 0.0;
  for (int i = 0; i < NQ; ++i) da[i] = 0.0;
  dlam[0] = dlam[1] = dlam[2] = 0.0;
  if (!with_dyn) return;
  // dg = d RNEA(q, v, a, fext = lambda) / d x_j  (at fixed a, lambda)
  double r1[NQ];
  for (int i = 0; i < NQ; ++i) r1[i] = -K.tau[i].d;
  if (!surface) {
    chol_solve<NQ>(P.L, r1);
    for (int i = 0; i < NQ; ++i) da[i] = r1[i];
    return;
  }
  // dh = d (classical acc + Kp (p - p*) + Kd v_p) / d x_j
  constexpr int c0 = NC == 1 ? 2 : 0;
  const double dap[3] = {K.ap.x.d, K.ap.y.d, K.ap.z.d};
  const double dvp[3] = {K.vp.x.d, K.vp.y.d, K.vp.z.d};
  const double dpe[3] = {K.pee.x.d, K.pee.y.d, K.pee.z.d};
  double dh[3];
  for (int r = 0; r < nc; ++r) dh[r] = dap[c0 + r] + C.Kp * dpe[c0 + r] + C.Kd * dvp[c0 + r];
  // K [da; -dlam] = -[dg; dh]:  y_l = S^-1 (Jc M^-1 (-dg) + dh), da = M^-1 (-dg - Jc^T y_l), dlam = -y_l
  double mr[NQ];
  for (int i = 0; i < NQ; ++i) mr[i] = r1[i];
  chol_solve<NQ>(P.L, mr);
  double yl[3];
  for (int r = 0; r < nc; ++r) {
    double acc = dh[r];
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
  for (int r = 0; r < nc; ++r) {
    dlam[r] = -yl[r];
    col[12 + r] = (mode == MODE_TERMINAL_X) ? 0.0 : dlam[r];
  }
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
