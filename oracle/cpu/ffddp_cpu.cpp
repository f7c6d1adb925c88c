// ORACLE-SIDE CPU BASELINE — test / benchmark infrastructure only.  Never
// linked or loaded by the product (franka-force-feedback-mpc_amd/); only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
//
// A scalar C++ BoxFDDP over the same OCP, one instance per OpenMP thread on
// the host cores (SURVEY.md §8(d) "CPU baseline" item 1).  It stands in for the
// reference's CPU path — crocoddyl.SolverBoxFDDP(problem).solve(xs_init,
// us_init, maxiter, False) at src/mpc/crocoddyl_classical.py:367, 442-445 and
// src/mpc/crocoddyl_force_feedback.py:605 — which cannot run here (Crocoddyl /
// Pinocchio absent).
//
//  * Per-node math: the product's host/device node models compiled for the
//    host (ffddp_node.hpp: node_primal = calc, node_tangent_state_an /
//    node_tangent_control = the closed-form calcDiff directions, node_calc =
//    the line-search calc), Gauss-Newton assembly as k_node does it.
//  * Solver: a straight restatement of Crocoddyl 2.x SolverFDDP::solve /
//    SolverDDP::backwardPass / SolverBoxFDDP::computeGains / BoxQP::solve
//    (SURVEY.md Appendix B), dense Fx / Fu products as in oracle/fddp.py,
//    sequential line search over alpha = 2^-n (no concurrent trials).
// Cross-checked against the numpy oracle by tests/test_cpu_baseline.py.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../franka-force-feedback-mpc_amd/csrc/ffddp_consts.hpp"

using namespace ffddp;

namespace {

constexpr int NXMAX = 21;

inline bool bad(double v) { return std::isnan(v) || std::isinf(v) || v >= 1e30; }

// phase / unit hooks for tools/flops/flop_count.cpp (the fp64 operation
// count of this scalar solver per node stage, backward node and trial node);
// no-ops in the baseline build
#ifndef FFDDP_CPU_PHASE_SCOPE
#define FFDDP_CPU_PHASE_SCOPE(p)
#endif
#ifndef FFDDP_CPU_UNIT
#define FFDDP_CPU_UNIT(p) ((void)0)
#endif

// crocoddyl::BoxQP::solve (projected Newton, oracle/fddp.py:boxqp): the free
// sub-problem is solved on the full 7x7 matrix with clamped rows/columns
// replaced by identity rows; refactored whenever the free set changes.
// Returns false on an LLT failure.  L: masked factor of the final free set.
bool boxqp(const DevConsts& C, const double* H, const double* q, const double* lb, const double* ub, double* x,
           double* L, bool* clamped) {
  for (int i = 0; i < NU; ++i) x[i] = std::max(std::min(x[i], ub[i]), lb[i]);
  bool have = false;
  double xs_f[NU] = {0, 0, 0, 0, 0, 0, 0};
  for (int it = 0; it < C.qp_maxiter; ++it) {
    double g[NU];
    for (int i = 0; i < NU; ++i) {
      double acc = q[i];
      for (int j = 0; j < NU; ++j) acc += H[i * NU + j] * x[j];
      g[i] = acc;
    }
    bool changed = !have;
    for (int j = 0; j < NU; ++j) {
      const bool c = (x[j] == lb[j] && g[j] > 0.0) || (x[j] == ub[j] && g[j] < 0.0);
      changed |= (c != clamped[j]);
      clamped[j] = c;
    }
    if (changed) {
      for (int i = 0; i < NU; ++i)
        for (int j = 0; j <= i; ++j)
          L[tri(i, j)] = (!clamped[i] && !clamped[j]) ? H[i * NU + j] + (i == j ? C.qp_reg : 0.0) : (i == j ? 1.0 : 0.0);
      if (!chol_packed<NU>(L)) return false;
      have = true;
      for (int i = 0; i < NU; ++i) {
        double acc = -q[i];
        for (int j = 0; j < NU; ++j)
          if (clamped[j]) acc -= H[i * NU + j] * x[j];
        xs_f[i] = clamped[i] ? 0.0 : acc;
      }
      chol_solve<NU>(L, xs_f);
    }
    double dx[NU], dmax = 0.0;
    for (int i = 0; i < NU; ++i) {
      dx[i] = clamped[i] ? 0.0 : xs_f[i] - x[i];
      dmax = std::max(dmax, std::fabs(dx[i]));
    }
    if (dmax < C.qp_th_grad) break;
    double fold;
    {
      double a1 = 0.0, a2 = 0.0;
      for (int i = 0; i < NU; ++i) {
        double acc = 0.0;
        for (int j = 0; j < NU; ++j) acc += H[i * NU + j] * x[j];
        a1 += x[i] * acc;
        a2 += q[i] * x[i];
      }
      fold = 0.5 * a1 + a2;
    }
    for (int ia = 0; ia < NTRIALS; ++ia) {
      const double al = C.alphas[ia];
      double xn[NU];
      for (int i = 0; i < NU; ++i) xn[i] = std::max(std::min(x[i] + al * dx[i], ub[i]), lb[i]);
      double a1 = 0.0, a2 = 0.0, gd = 0.0;
      for (int i = 0; i < NU; ++i) {
        double acc = 0.0;
        for (int j = 0; j < NU; ++j) acc += H[i * NU + j] * xn[j];
        a1 += xn[i] * acc;
        a2 += q[i] * xn[i];
        gd += g[i] * (x[i] - xn[i]);
      }
      if (fold - (0.5 * a1 + a2) > C.qp_th_acceptstep * gd) {
        for (int i = 0; i < NU; ++i) x[i] = xn[i];
        break;
      }
    }
  }
  return true;
}

// One instance's problem data and solver state (one per OpenMP thread).
struct Inst {
  const DevConsts* C = nullptr;
  int N = 0, nx = 0, rec = 0, nc = 1;
  bool ff = false, surf = false;
  const double *x0 = nullptr, *nref = nullptr, *iref = nullptr;
  std::vector<double> xs, us, K, k, fs, w, recs, xs_try, us_try, Vxx, Vx, Qu, Quu;
  double cost = 0.0, preg = 0.0, dg = 0.0, dq = 0.0, stop = 0.0;
  bool feas = false;
  int n_iters = 0, n_trials = 0, n_retries = 0, n_backward = 0, n_calc = 0, n_forward = 0;
  int n_neg = 0, n_neg_acc = 0;  // trials judged / accepted by the ascent-direction branch (dVexp < 0)

  void init(const DevConsts& c) {
    C = &c;
    N = c.N;
    nx = c.nx;
    ff = c.variant == FFDDP_FORCE_FEEDBACK;
    nc = c.nc;
    rec = rec_size(nx);
    xs.assign((size_t)(N + 1) * nx, 0.0);
    us.assign((size_t)N * NU, 0.0);
    K.assign((size_t)N * NU * nx, 0.0);
    k.assign((size_t)N * NU, 0.0);
    fs.assign((size_t)(N + 1) * nx, 0.0);
    w.assign((size_t)(N + 1) * nx, 0.0);
    recs.assign((size_t)(N + 1) * rec, 0.0);
    xs_try = xs;
    us_try = us;
    Vxx.assign((size_t)(N + 1) * nx * nx, 0.0);
    Vx.assign((size_t)(N + 1) * nx, 0.0);
    Qu.assign((size_t)N * NU, 0.0);
    Quu.assign((size_t)N * NU * NU, 0.0);
  }
};

// calc + calcDiff of node t at (xs, us) into its record (A | Lxx | Lxu | Luu |
// Lx | Lu | cost | lam), as k_primal_g8 + k_node compute it; returns the node
// cost (IAM scaling and FF augmentation included).
template <int NC, bool FF>
double node_diff(const DevConsts& C, Inst& I, int t, double* r, double* xnext) {
  FFDDP_CPU_UNIT(1);
  const int N = I.N;
  constexpr int nx = FF ? 21 : 14;
  constexpr int nc = NC;
  const bool terminal = t == N;
  const int mode = !terminal ? MODE_RUNNING : (FF ? MODE_TERMINAL_U : MODE_TERMINAL_X);
  const bool surf = I.surf;
  const double* y = I.xs.data() + (size_t)t * nx;
  const double* ref = I.nref + (size_t)t * 6;
  const double* xreg = I.iref;
  const double* uin = FF ? (y + 14) : (terminal ? nullptr : I.us.data() + (size_t)t * NU);
  Primal P;
  node_primal<NC>(C, mode, surf, y, uin, ref, xreg, xreg + 14, P);
  for (int i = 0; i < 14; ++i) xnext[i] = P.xnext[i];
  double acc[NQ];
  for (int i = 0; i < NQ; ++i) acc[i] = (mode == MODE_TERMINAL_X) ? 0.0 : P.a[i];
  double lk[LK_ALLOC];
  rb_links(C.rb, y, y + NQ, acc, lk);
  const bool need_u = mode != MODE_TERMINAL_X;
  double da[14][NQ], dlam[14][3], col[14][NDENSE_MAX], dau[NU][NQ], dlamu[NU][3], colu[NU][FFDDP_MAX_NC];
  for (int j = 0; j < 14; ++j) node_tangent_state_an<NC>(C, mode, surf, lk, P, j, da[j], dlam[j], col[j]);
  for (int kk = 0; kk < NU; ++kk) {
    if (need_u) node_tangent_control<NC>(C, surf, P, kk, dau[kk], dlamu[kk]);
    for (int s = 0; s < FFDDP_MAX_NC; ++s) colu[kk][s] = (need_u && surf && s < nc) ? dlamu[kk][s] : 0.0;
  }
  // Gauss-Newton over the dense residual rows; force block with the friction
  // cone's off-diagonal couplings
  auto fq = [&](const double* a, const double* b) {
    double s = 0.0;
    for (int q = 0; q < nc; ++q) s += a[q] * P.D[12 + q] * b[q];
    if (NC == 3)
      s += P.Dfo[0] * (a[1] * b[0] + a[0] * b[1]) + P.Dfo[1] * (a[2] * b[0] + a[0] * b[2]) +
           P.Dfo[2] * (a[2] * b[1] + a[1] * b[2]);
    return s;
  };
  const double sc = (mode != MODE_TERMINAL_X) ? C.dt : 1.0;
  const double* yref = I.x0;
  std::memset(r, 0, sizeof(double) * I.rec);
  double* Lxx = r + rec_off_Lxx(nx);
  for (int j = 0; j < 14; ++j) {
    if (need_u)
      for (int i = 0; i < NQ; ++i) r[rec_off_A() + j * NQ + i] = da[j][i];
    for (int i = 0; i < 14; ++i) {
      double a = 0.0;
      for (int q = 0; q < 12; ++q) a += col[i][q] * P.D[q] * col[j][q];
      a += fq(col[i] + 12, col[j] + 12);
      if (i == j) a += P.Dx[j];
      a *= sc;
      if (FF && i == j) a += C.w_y * C.Wy2[j];
      Lxx[i * nx + j] = a;
    }
    double lx = 0.0;
    for (int q = 0; q < 12 + nc; ++q) lx += col[j][q] * P.g[q];
    lx = (lx + P.gx[j]) * sc;
    if (FF) lx += C.w_y * C.Wy2[j] * (y[j] - yref[j]);
    r[rec_off_Lx(nx) + j] = lx;
    if (need_u)
      for (int kk = 0; kk < NU; ++kk) {
        const double a = fq(col[j] + 12, colu[kk]) * sc;
        if (FF)
          Lxx[(14 + kk) * nx + j] = a;
        else
          r[rec_off_Lxu(nx) + j * NU + kk] = a;
      }
  }
  if (need_u) {
    for (int kk = 0; kk < NU; ++kk) {
      for (int i = 0; i < NQ; ++i) r[rec_off_A() + (14 + kk) * NQ + i] = dau[kk][i];
      double luu[NU];
      for (int m = 0; m < NU; ++m) {
        double a = fq(colu[m], colu[kk]);
        if (m == kk) a += P.Du[kk];
        luu[m] = a * sc;
      }
      double lu = 0.0;
      for (int q = 0; q < nc; ++q) lu += colu[kk][q] * P.g[12 + q];
      lu = (lu + P.gu[kk]) * sc;
      if (!FF) {
        for (int m = 0; m < NU; ++m) r[rec_off_Luu(nx) + m * NU + kk] = luu[m];
        r[rec_off_Lu(nx) + kk] = lu;
      } else {
        for (int i = 0; i < 14; ++i) Lxx[i * nx + 14 + kk] = fq(col[i] + 12, colu[kk]) * sc;
        for (int m = 0; m < NU; ++m) Lxx[(14 + m) * nx + 14 + kk] = luu[m] + (m == kk ? C.w_y * C.Wy2[14 + kk] : 0.0);
        r[rec_off_Lx(nx) + 14 + kk] = lu + C.w_y * C.Wy2[14 + kk] * (y[14 + kk] - yref[14 + kk]);
        // _AugmentedLPFActionModel control terms: Lu = w_w w + w_s g_soft, Luu diagonal, Lxu = 0
        const double wk = terminal ? 0.0 : I.us[(size_t)t * NU + kk];
        const double ov = std::fabs(wk) - C.ws_lim[kk];
        const bool act = ov > 0.0;
        const double gs = act ? ov * (wk > 0.0 ? 1.0 : (wk < 0.0 ? -1.0 : 0.0)) : 0.0;
        r[rec_off_Lu(nx) + kk] = C.w_w * wk + C.w_ws * gs;
        for (int m = 0; m < NU; ++m) r[rec_off_Luu(nx) + m * NU + kk] = (m == kk) ? (C.w_w + C.w_ws * (act ? 1.0 : 0.0)) : 0.0;
      }
    }
  }
  // node cost
  double c = FF ? C.dt * P.cost : (terminal ? P.cost : C.dt * P.cost);
  if (FF) {
    if (C.w_y > 0.0) {
      double a = 0.0;
      for (int i = 0; i < 21; ++i) {
        const double d = y[i] - yref[i];
        a += C.Wy2[i] * d * d;
      }
      c += 0.5 * C.w_y * a;
    }
    if (!terminal) {
      const double* ww = I.us.data() + (size_t)t * NU;
      if (C.w_w > 0.0) {
        double a = 0.0;
        for (int i = 0; i < NU; ++i) a += ww[i] * ww[i];
        c += 0.5 * C.w_w * a;
      }
      if (C.w_ws > 0.0) {
        double a = 0.0;
        for (int i = 0; i < NU; ++i) {
          const double o = std::max(std::fabs(ww[i]) - C.ws_lim[i], 0.0);
          a += o * o;
        }
        c += C.w_ws * (0.5 * a);
      }
    }
    if (!terminal) {
      const double* ww = I.us.data() + (size_t)t * NU;
      for (int i = 0; i < NU; ++i) xnext[14 + i] = C.alpha * y[14 + i] + C.beta * ww[i];
    }
  }
  r[rec_off_cost(nx)] = c;
  for (int q = 0; q < 3; ++q) r[rec_off_lam(nx) + q] = (mode == MODE_TERMINAL_X) ? 0.0 : P.lam[q];
  return c;
}

// ShootingProblem::calcDiff + the FDDP gaps (SolverFDDP::calcDiff)
template <int NC, bool FF>
void calc_diff(const DevConsts& C, Inst& I) {
  FFDDP_CPU_PHASE_SCOPE(1);
  const int N = I.N, nx = I.nx;
  double c = 0.0;
  for (int t = 0; t <= N; ++t) {
    double xn[NXMAX];
    c += node_diff<NC, FF>(C, I, t, I.recs.data() + (size_t)t * I.rec, xn);
    if (t < N) {
      double* f = I.fs.data() + (size_t)(t + 1) * nx;
      const double* yn = I.xs.data() + (size_t)(t + 1) * nx;
      for (int i = 0; i < nx; ++i) f[i] = I.feas ? 0.0 : xn[i] - yn[i];
    }
  }
  for (int i = 0; i < nx; ++i) I.fs[i] = I.feas ? 0.0 : I.x0[i] - I.xs[i];
  I.cost = c;
  I.n_calc += 1;
}

// dense Fx (nx x nx), Fu (nx x 7) of node t from its record (Euler structure)
void dynamics_jacobians(const DevConsts& C, const Inst& I, const double* r, double* Fx, double* Fu) {
  const int nx = I.nx;
  const bool ff = I.ff;
  const double dt = C.dt;
  const double* A = r + rec_off_A();
  for (int i = 0; i < nx; ++i) {
    for (int j = 0; j < nx; ++j) {
      double v = (i == j) ? 1.0 : 0.0;
      if (i < 14 && j < (ff ? 21 : 14)) {
        v += (i < 7 ? dt * dt : dt) * A[j * NQ + (i % 7)];
        if (i < 7 && j == i + 7) v += dt;
      }
      if (ff && i >= 14) v = (i == j) ? C.alpha : 0.0;
      Fx[i * nx + j] = v;
    }
    for (int kk = 0; kk < NU; ++kk)
      Fu[i * NU + kk] = !ff ? (i < 7 ? dt * dt : dt) * A[(14 + kk) * NQ + (i % 7)] : ((i >= 14 && i - 14 == kk) ? C.beta : 0.0);
  }
}

// SolverDDP::backwardPass + SolverBoxFDDP::computeGains; false = backward failure
bool backward(const DevConsts& C, Inst& I) {
  FFDDP_CPU_PHASE_SCOPE(2);
  const int N = I.N, nx = I.nx;
  const double preg = I.preg;
  const bool use_qp = C.use_box && I.feas;
  double* VxxN = I.Vxx.data() + (size_t)N * nx * nx;
  double* VxN = I.Vx.data() + (size_t)N * nx;
  const double* rT = I.recs.data() + (size_t)N * I.rec;
  double dg = 0.0, dq = 0.0, stop = 0.0;
  for (int i = 0; i < nx; ++i)
    for (int j = 0; j < nx; ++j) VxxN[i * nx + j] = rT[rec_off_Lxx(nx) + i * nx + j] + (i == j ? preg : 0.0);
  for (int i = 0; i < nx; ++i) {
    double vfs = 0.0;
    for (int j = 0; j < nx; ++j) vfs += VxxN[i * nx + j] * I.fs[(size_t)N * nx + j];
    I.w[(size_t)N * nx + i] = I.feas ? 0.0 : vfs;
    VxN[i] = rT[rec_off_Lx(nx) + i] + (I.feas ? 0.0 : vfs);
  }
  if (!I.feas)
    for (int i = 0; i < nx; ++i) {
      dg -= VxN[i] * I.fs[(size_t)N * nx + i];
      dq += I.fs[(size_t)N * nx + i] * I.w[(size_t)N * nx + i];
    }
  double Fx[NXMAX * NXMAX], Fu[NXMAX * NU], FxTV[NXMAX * NXMAX], FuTV[NU * NXMAX];
  double Qxx[NXMAX * NXMAX], Qxu[NXMAX * NU], Qx[NXMAX];
  for (int t = N - 1; t >= 0; --t) {
    FFDDP_CPU_UNIT(2);
    const double* r = I.recs.data() + (size_t)t * I.rec;
    const double* Vp = I.Vxx.data() + (size_t)(t + 1) * nx * nx;
    const double* vp = I.Vx.data() + (size_t)(t + 1) * nx;
    dynamics_jacobians(C, I, r, Fx, Fu);
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < nx; ++j) {
        double a = 0.0;
        for (int m = 0; m < nx; ++m) a += Fx[m * nx + i] * Vp[m * nx + j];
        FxTV[i * nx + j] = a;
      }
    for (int c = 0; c < NU; ++c)
      for (int j = 0; j < nx; ++j) {
        double a = 0.0;
        for (int m = 0; m < nx; ++m) a += Fu[m * NU + c] * Vp[m * nx + j];
        FuTV[c * nx + j] = a;
      }
    double* Qu = I.Qu.data() + (size_t)t * NU;
    double* Quu = I.Quu.data() + (size_t)t * NU * NU;
    for (int i = 0; i < nx; ++i) {
      double a = r[rec_off_Lx(nx) + i];
      for (int m = 0; m < nx; ++m) a += Fx[m * nx + i] * vp[m];
      Qx[i] = a;
      for (int j = 0; j < nx; ++j) {
        double b = r[rec_off_Lxx(nx) + i * nx + j];
        for (int m = 0; m < nx; ++m) b += FxTV[i * nx + m] * Fx[m * nx + j];
        Qxx[i * nx + j] = b;
      }
      for (int c = 0; c < NU; ++c) {
        double b = r[rec_off_Lxu(nx) + i * NU + c];
        for (int m = 0; m < nx; ++m) b += FxTV[i * nx + m] * Fu[m * NU + c];
        Qxu[i * NU + c] = b;
      }
    }
    for (int c = 0; c < NU; ++c) {
      double a = r[rec_off_Lu(nx) + c];
      for (int m = 0; m < nx; ++m) a += Fu[m * NU + c] * vp[m];
      Qu[c] = a;
      for (int e = 0; e < NU; ++e) {
        double b = r[rec_off_Luu(nx) + c * NU + e];
        for (int m = 0; m < nx; ++m) b += FuTV[c * nx + m] * Fu[m * NU + e];
        Quu[c * NU + e] = b + (c == e ? preg : 0.0);
      }
    }
    double* Kt = I.K.data() + (size_t)t * NU * nx;
    double* kt = I.k.data() + (size_t)t * NU;
    double L[28];
    bool cl[NU] = {false, false, false, false, false, false, false};
    if (!use_qp) {
      for (int i = 0; i < NU; ++i)
        for (int j = 0; j <= i; ++j) L[tri(i, j)] = Quu[i * NU + j];
      if (!chol_packed<NU>(L)) return false;
      double kk[NU];
      for (int c = 0; c < NU; ++c) kk[c] = Qu[c];
      chol_solve<NU>(L, kk);
      for (int c = 0; c < NU; ++c) kt[c] = kk[c];
    } else {
      double lb[NU], ub[NU], x[NU];
      for (int i = 0; i < NU; ++i) {
        lb[i] = C.u_lb[i] - I.us[(size_t)t * NU + i];
        ub[i] = C.u_ub[i] - I.us[(size_t)t * NU + i];
        x[i] = kt[i];
      }
      if (!boxqp(C, Quu, Qu, lb, ub, x, L, cl)) return false;
      for (int i = 0; i < NU; ++i) {
        kt[i] = -x[i];
        if (cl[i]) Qu[i] = 0.0;  // BoxFDDP: clamped Qu entries are zeroed
      }
    }
    // K = Quu_ff^-1 Qxu_f^T (masked factor; clamped rows zero)
    for (int j = 0; j < nx; ++j) {
      double colv[NU];
      for (int c = 0; c < NU; ++c) colv[c] = cl[c] ? 0.0 : Qxu[j * NU + c];
      chol_solve<NU>(L, colv);
      for (int c = 0; c < NU; ++c) Kt[c * nx + j] = colv[c];
    }
    double* V = I.Vxx.data() + (size_t)t * nx * nx;
    double* v = I.Vx.data() + (size_t)t * nx;
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j <= i; ++j) {
        double a1 = Qxx[i * nx + j], a2 = Qxx[j * nx + i];
        for (int c = 0; c < NU; ++c) {
          a1 -= Qxu[i * NU + c] * Kt[c * nx + j];
          a2 -= Qxu[j * NU + c] * Kt[c * nx + i];
        }
        const double val = 0.5 * (a1 + a2) + (i == j ? preg : 0.0);
        V[i * nx + j] = val;
        V[j * nx + i] = val;
      }
    bool nanv = false;
    for (int i = 0; i < nx; ++i) {
      double a = Qx[i];
      for (int c = 0; c < NU; ++c) a -= Kt[c * nx + i] * Qu[c];
      double vfs = 0.0;
      for (int j = 0; j < nx; ++j) vfs += V[i * nx + j] * I.fs[(size_t)t * nx + j];
      I.w[(size_t)t * nx + i] = I.feas ? 0.0 : vfs;
      if (!I.feas) a += vfs;
      v[i] = a;
      nanv |= bad(std::fabs(a));
      for (int j = 0; j < nx; ++j) nanv |= bad(std::fabs(V[i * nx + j]));
    }
    if (nanv) return false;
    // expected-improvement terms (SolverFDDP::updateExpectedImprovement)
    for (int c = 0; c < NU; ++c) {
      double quk = 0.0;
      for (int m = 0; m < NU; ++m) quk += Quu[c * NU + m] * kt[m];
      dg += Qu[c] * kt[c];
      dq -= kt[c] * quk;
      stop += Qu[c] * Qu[c];
    }
    if (!I.feas)
      for (int i = 0; i < nx; ++i) {
        dg -= v[i] * I.fs[(size_t)t * nx + i];
        dq += I.fs[(size_t)t * nx + i] * I.w[(size_t)t * nx + i];
      }
  }
  I.dg = dg;
  I.dq = dq;
  I.stop = stop;
  return true;
}

// SolverBoxFDDP::forwardPass(alpha) into (xs_try, us_try); returns the cost
// or NaN when raiseIfNaN would throw; *dv = the trial's gap term of the
// expected improvement
template <int NC, bool FF>
double forward(const DevConsts& C, Inst& I, double alpha, double* dv) {
  FFDDP_CPU_PHASE_SCOPE(3);
  const int N = I.N, nx = I.nx;
  const bool gap = !(I.feas || alpha == 1.0);
  double xh[NXMAX];
  for (int i = 0; i < nx; ++i) xh[i] = I.x0[i];
  double cost = 0.0, dvv = 0.0;
  Primal P;
  for (int t = 0; t <= N; ++t) {
    FFDDP_CPU_UNIT(3);
    const double* xs_t = I.xs.data() + (size_t)t * nx;
    const double* fs_t = I.fs.data() + (size_t)t * nx;
    double* xt = I.xs_try.data() + (size_t)t * nx;
    for (int i = 0; i < nx; ++i) xt[i] = gap ? xh[i] + fs_t[i] * (alpha - 1.0) : xh[i];
    if (!I.feas) {
      const double* w_t = I.w.data() + (size_t)t * nx;
      double a = 0.0;
      for (int i = 0; i < nx; ++i) a += w_t[i] * (xs_t[i] - xt[i]);
      dvv -= a;
    }
    const double* ref = I.nref + (size_t)t * 6;
    double c;
    if (t < N) {
      double* ut = I.us_try.data() + (size_t)t * NU;
      const double* us_t = I.us.data() + (size_t)t * NU;
      const double* K_t = I.K.data() + (size_t)t * NU * nx;
      const double* k_t = I.k.data() + (size_t)t * NU;
      for (int m = 0; m < NU; ++m) {
        double a = us_t[m] - k_t[m] * alpha;
        for (int i = 0; i < nx; ++i) a -= K_t[m * nx + i] * (xt[i] - xs_t[i]);
        if (C.use_box) a = std::min(std::max(a, C.u_lb[m]), C.u_ub[m]);
        ut[m] = a;
      }
      node_calc<NC, FF>(C, false, I.surf, xt, ut, ref, I.iref, I.iref + 14, I.x0, P, xh, c);
      cost += c;
      bool xb = false;
      for (int i = 0; i < nx; ++i) xb |= bad(std::fabs(xh[i]));
      if (bad(cost) || xb) return std::nan("");
    } else {
      double yn[NXMAX];
      node_calc<NC, FF>(C, true, I.surf, xt, nullptr, ref, I.iref, I.iref + 14, I.x0, P, yn, c);
      cost += c;
      if (bad(cost)) return std::nan("");
    }
  }
  *dv = dvv;
  return cost;
}

// SolverFDDP::solve(xs_init, us_init, maxiter, is_feasible) for one instance
template <int NC, bool FF>
bool solve_one(const DevConsts& C, Inst& I, int maxiter, int& iter_out) {
  I.preg = C.reg_min;
  bool was_feasible = false, recalc = true;
  std::fill(I.k.begin(), I.k.end(), 0.0);
  std::fill(I.K.begin(), I.K.end(), 0.0);
  for (int it = 0; it < maxiter; ++it) {
    iter_out = it;
    for (;;) {
      if (recalc) calc_diff<NC, FF>(C, I);
      I.n_backward += 1;
      if (backward(C, I)) break;
      recalc = false;
      I.n_retries += 1;
      I.preg = std::min(I.preg * C.reg_inc, C.reg_max);
      if (I.preg == C.reg_max) return false;
    }
    I.n_iters += 1;
    I.n_forward += 1;
    double steplength = C.alphas[0];
    for (int a = 0; a < NTRIALS; ++a) {
      steplength = C.alphas[a];
      I.n_trials += 1;
      double dv = 0.0;
      const double cost_try = forward<NC, FF>(C, I, steplength, &dv);
      if (std::isnan(cost_try)) continue;
      const double dvv = I.feas ? 0.0 : dv;
      const double dV = I.cost - cost_try;
      const double d0 = I.dg + dvv, d1 = I.dq - 2.0 * dvv;
      const double dVexp = steplength * (d0 + 0.5 * steplength * d1);
      const bool ok = dVexp >= 0 ? (std::fabs(d0) < C.th_grad || dV > C.th_acceptstep * dVexp)
                                 : (!I.feas && (C.neg_rule == FFDDP_NEGSTEP_CROCODDYL ? dV < C.th_acceptnegstep * dVexp
                                                                                       : dV > C.th_acceptnegstep * dVexp));
      if (dVexp < 0) {
        I.n_neg += 1;
        I.n_neg_acc += ok ? 1 : 0;
      }
      if (ok) {
        was_feasible = I.feas;
        I.xs.swap(I.xs_try);
        I.us.swap(I.us_try);
        I.feas = was_feasible || steplength == 1.0;
        I.cost = cost_try;
        recalc = true;
        break;
      }
    }
    if (steplength > C.th_stepdec) I.preg = std::max(I.preg / C.reg_dec, C.reg_min);
    if (steplength <= C.th_stepinc) {
      I.preg = std::min(I.preg * C.reg_inc, C.reg_max);
      if (I.preg == C.reg_max) return false;
    }
    if (was_feasible && I.stop < C.th_stop) return true;
  }
  iter_out = maxiter;
  return false;
}

template <int NC, bool FF>
int solve_batch_t(const DevConsts& C, int B, const double* x0, const double* nref, const double* iref,
                  const uint8_t* surface, const double* xs_init, const double* us_init, int maxiter,
                  int is_feasible, double* xs, double* us, double* K, double* cost, int32_t* iters, uint8_t* ok,
                  int32_t* stats, int nthreads) {
  const int N = C.N, nx = C.nx;
  if (nthreads < 1) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
  {
    Inst I;
    I.init(C);
#pragma omp for schedule(dynamic, 1)
    for (int b = 0; b < B; ++b) {
      I.x0 = x0 + (size_t)b * nx;
      I.nref = nref + (size_t)b * (N + 1) * 6;
      I.iref = iref + (size_t)b * 21;
      I.surf = surface[b] != 0;
      I.feas = is_feasible != 0;
      std::copy(xs_init + (size_t)b * (N + 1) * nx, xs_init + (size_t)(b + 1) * (N + 1) * nx, I.xs.begin());
      std::copy(us_init + (size_t)b * N * NU, us_init + (size_t)(b + 1) * N * NU, I.us.begin());
      I.n_iters = I.n_trials = I.n_retries = I.n_backward = I.n_calc = I.n_forward = 0;
      I.n_neg = I.n_neg_acc = 0;
      I.cost = 0.0;
      int it = 0;
      const bool res = solve_one<NC, FF>(C, I, maxiter, it);
      std::copy(I.xs.begin(), I.xs.end(), xs + (size_t)b * (N + 1) * nx);
      std::copy(I.us.begin(), I.us.end(), us + (size_t)b * N * NU);
      std::copy(I.K.begin(), I.K.end(), K + (size_t)b * N * NU * nx);
      cost[b] = I.cost;
      iters[b] = it;
      ok[b] = res ? 1 : 0;
      if (stats) {
        int32_t* s = stats + (size_t)b * FFDDP_NSTATS;
        s[0] = I.n_iters;
        s[1] = I.n_trials;
        s[2] = I.n_retries;
        s[3] = I.n_backward;
        s[4] = I.n_calc;
        s[5] = I.n_forward;
        s[6] = I.n_trials;
        s[7] = 0;
        s[8] = I.n_neg;
        s[9] = I.n_neg_acc;
      }
    }
  }
  return 0;
}

}  // namespace

extern "C" {

// Same arguments and outputs as ffddp_solve_batch (include/ffddp.h) on host
// arrays, plus the solver properties (ffddp_solver_params, NULL = defaults)
// and the OpenMP thread count (<= 0: all the process may use).
int ffddp_cpu_solve_batch(const ffddp_robot* robot, const ffddp_ocp_config* cfg, int B, const double* x0,
                          const double* node_ref, const double* inst_ref, const uint8_t* surface,
                          const double* xs_init, const double* us_init, int maxiter, int is_feasible, double* xs,
                          double* us, double* K, double* cost, int32_t* iters, uint8_t* ok, int32_t* stats,
                          const ffddp_solver_params* sp, int nthreads) {
  if (!robot || !cfg || B < 0 || maxiter < 0) return FFDDP_E_INVALID;
  if (cfg->nc != 1 && cfg->nc != 3) return FFDDP_E_INVALID;
  if (B == 0) return 0;
  DevConsts C;
  fill_consts(*robot, *cfg, C);
  if (sp) {
    C.th_stop = sp->th_stop;
    C.th_grad = sp->th_grad;
    C.th_acceptstep = sp->th_acceptstep;
    C.th_acceptnegstep = sp->th_acceptnegstep;
    C.th_stepdec = sp->th_stepdec;
    C.th_stepinc = sp->th_stepinc;
    C.reg_min = sp->reg_min;
    C.reg_max = sp->reg_max;
    C.reg_inc = sp->reg_incfactor;
    C.reg_dec = sp->reg_decfactor;
    C.neg_rule = sp->neg_step_rule;
  }
  const bool ff = cfg->variant == FFDDP_FORCE_FEEDBACK;
#define FFDDP_CPU(NC_, FF_) \
  solve_batch_t<NC_, FF_>(C, B, x0, node_ref, inst_ref, surface, xs_init, us_init, maxiter, is_feasible, xs, us, K, cost, iters, ok, stats, nthreads)
  if (cfg->nc == 1) return ff ? FFDDP_CPU(1, true) : FFDDP_CPU(1, false);
  return ff ? FFDDP_CPU(3, true) : FFDDP_CPU(3, false);
#undef FFDDP_CPU
}

int ffddp_cpu_max_threads(void) { return omp_get_max_threads(); }

}  // extern "C"
