// ffddp_consts.hpp — ffddp_ocp_config (the C-ABI's OCP definition) -> the
// DevConsts every node model reads: weights, activation bounds, contact and
// friction-cone data, force-feedback filter constants and the solver
// constants of crocoddyl::SolverBoxFDDP / SolverFDDP / BoxQP.  Host code;
// shared by the HIP library and the CPU baseline (oracle/cpu).
#pragma once

#include <cmath>
#include <cstring>

#include "ffddp_node.hpp"

namespace ffddp {

inline void fill_consts(const ffddp_robot& rb, const ffddp_ocp_config& c, DevConsts& k) {
  std::memset(&k, 0, sizeof(k));
  k.rb = rb;
  k.variant = c.variant;
  k.N = c.horizon;
  k.nc = c.nc;
  k.use_box = c.use_box;
  k.nx = c.variant == FFDDP_FORCE_FEEDBACK ? 21 : 14;
  k.dt = c.dt;
  k.inner_state_reg = c.variant == FFDDP_CLASSICAL ? 1 : c.use_inner_state_reg;
  k.inner_tau_reg = c.variant == FFDDP_CLASSICAL ? 1 : c.use_inner_tau_reg;
  k.w_post = c.w_posture;
  k.w_v = c.w_v;
  for (int i = 0; i < 7; ++i) k.vdw[i] = c.v_damp_weights[i];
  // q soft limits (_make_q_soft_limit_cost, crocoddyl_classical.py:487-519)
  k.has_qsoft = c.w_q_soft_limits > 0.0;
  k.w_qs = c.w_q_soft_limits;
  const double inf = __builtin_inf();
  const double m = c.q_soft_limit_margin > 0.0 ? c.q_soft_limit_margin : 0.0;
  for (int i = 0; i < 7; ++i) {
    const double lo = c.q_lower[i], hi = c.q_upper[i];
    const double qref = 0.5 * (lo + hi);
    double lbs = lo + m, ubs = hi - m;
    if (lbs > ubs) {
      const double mid = 0.5 * (lo + hi);
      lbs = mid - 1e-3;
      ubs = mid + 1e-3;
    }
    k.qs_xref[i] = qref;
    k.qs_lb[i] = lbs - qref;
    k.qs_ub[i] = ubs - qref;
    k.qs_xref[7 + i] = 0.0;
    k.qs_lb[7 + i] = -inf;
    k.qs_ub[7 + i] = inf;
  }
  k.w_ori = c.w_ee_ori;
  for (int i = 0; i < 3; ++i) k.ori_w[i] = c.ori_weights[i];
  k.w_wd = c.w_wdamp;
  for (int i = 0; i < 3; ++i) k.wd_w[i] = c.w_wdamp_weights[i];
  k.w_ee_pos = c.w_ee_pos;
  k.ee_pos_w[0] = 1.0;
  k.ee_pos_w[1] = 1.0;
  k.ee_pos_w[2] = 2.5;
  k.w_tp = c.w_tangent_pos;
  k.w_tv = c.w_tangent_vel;
  k.has_pz = c.w_plane_z > 0.0;
  k.w_pz = c.w_plane_z;
  k.has_vz = c.w_vz > 0.0;
  k.w_vz = c.w_vz;
  for (int i = 0; i < 9; ++i) k.Rdes[i] = c.R_des[i];
  k.has_uni = c.w_unilateral > 0.0;
  k.w_uni = c.w_unilateral;
  if (c.nc == 1) {
    k.uni_lb[0] = c.friction_margin;
    k.uni_ub[0] = inf;
  } else {
    k.uni_lb[0] = k.uni_lb[1] = -inf;
    k.uni_lb[2] = c.friction_margin;
    k.uni_ub[0] = k.uni_ub[1] = k.uni_ub[2] = inf;
  }
  // friction cone (nc = 3 only, crocoddyl_classical.py:678): crocoddyl::FrictionCone
  // with R = I, nf = 4, inner_appr = false: facet rows (mu_nsurf +- t_i)^T with
  // t_i = (cos th_i, sin th_i, 0), th_i = i pi / 2, bounds (-inf, 0]; the
  // normal row e_z with bounds [0, inf); the finite bounds moved inwards by
  // friction_margin (_make_friction_barrier_activation, :891-903)
  k.has_fc = (c.nc == 3 && c.w_friction_cone > 0.0) ? 1 : 0;
  k.w_fc = c.w_friction_cone;
  {
    const double eps = c.friction_margin > 0.0 ? c.friction_margin : 0.0;
    const double theta = 2.0 * M_PI / 4.0;
    for (int i = 0; i < 2; ++i) {
      const double ti = theta * (double)i, ct = std::cos(ti), st = std::sin(ti);
      const double rp[3] = {ct, st, -c.mu}, rm[3] = {-ct, -st, -c.mu};
      for (int e = 0; e < 3; ++e) {
        k.fc_A[2 * i][e] = rp[e];
        k.fc_A[2 * i + 1][e] = rm[e];
      }
      k.fc_lb[2 * i] = k.fc_lb[2 * i + 1] = -inf;
      k.fc_ub[2 * i] = k.fc_ub[2 * i + 1] = 0.0 - eps;
    }
    k.fc_A[4][0] = 0.0;
    k.fc_A[4][1] = 0.0;
    k.fc_A[4][2] = 1.0;
    k.fc_lb[4] = 0.0 + eps;
    k.fc_ub[4] = inf;
  }
  k.has_fn = c.w_fn > 0.0;
  k.w_fn = c.w_fn;
  if (c.nc == 1) {
    k.fn_w[0] = 1.0;
    k.fn_ref[0] = c.fn_des;
  } else {
    k.fn_w[0] = k.fn_w[1] = 0.0;
    k.fn_w[2] = 1.0;
    k.fn_ref[0] = k.fn_ref[1] = 0.0;
    k.fn_ref[2] = c.fn_des;
  }
  k.w_tau = c.w_tau;
  k.has_tsoft = c.w_tau_soft_limits > 0.0;
  k.w_ts = c.w_tau_soft_limits;
  double mn = c.tau_limits[0];
  for (int i = 1; i < 7; ++i) mn = c.tau_limits[i] < mn ? c.tau_limits[i] : mn;
  double mg = c.tau_soft_limit_margin > 0.0 ? c.tau_soft_limit_margin : 0.0;
  mg = mg < mn - 1.0e-6 ? mg : mn - 1.0e-6;
  for (int i = 0; i < 7; ++i) {
    k.ts_lb[i] = -c.tau_limits[i] + mg;
    k.ts_ub[i] = c.tau_limits[i] - mg;
    k.u_lb[i] = -c.tau_limits[i];
    k.u_ub[i] = c.tau_limits[i];
  }
  k.Kp = c.contact_gains[0];
  k.Kd = c.contact_gains[1];
  k.eps = c.contact_inv_damping;
  k.z_press = c.z_press;
  // force feedback (_AugmentedLPFActionModel.__init__, :170-188)
  double al = c.ff_alpha;
  al = al < 0.0 ? 0.0 : (al > 0.999999 ? 0.999999 : al);
  k.alpha = al;
  k.beta = 1.0 - al;
  k.w_w = c.w_w > 0.0 ? c.w_w : 0.0;
  k.w_ws = c.w_w_soft_limits > 0.0 ? c.w_w_soft_limits : 0.0;
  const double wm = c.tau_soft_limit_margin > 0.0 ? c.tau_soft_limit_margin : 0.0;
  for (int i = 0; i < 7; ++i) {
    const double l = c.tau_limits[i] - wm;
    k.ws_lim[i] = l > 1.0e-9 ? l : 1.0e-9;
  }
  k.w_y = c.w_y > 0.0 ? c.w_y : 0.0;
  for (int i = 0; i < 21; ++i) k.Wy2[i] = c.y_weights[i] * c.y_weights[i];
  // solver constants (SolverBoxFDDP / SolverFDDP / BoxQP defaults)
  k.th_stop = c.use_box ? 5e-5 : 1e-9;
  k.th_grad = 1e-12;
  k.th_acceptstep = 0.1;
  k.th_acceptnegstep = 2.0;
  k.th_stepdec = 0.5;
  k.th_stepinc = 0.01;
  k.reg_min = 1e-9;
  k.reg_max = 1e9;
  k.reg_inc = 10.0;
  k.reg_dec = 10.0;
  k.neg_rule = FFDDP_NEGSTEP_CROCODDYL;
  for (int i = 0; i < NTRIALS; ++i) k.alphas[i] = 1.0 / (double)(1 << i);
  k.qp_maxiter = 100;
  k.qp_th_acceptstep = 0.1;
  k.qp_th_grad = 1e-5;
  k.qp_reg = 0.0;
}

}  // namespace ffddp
