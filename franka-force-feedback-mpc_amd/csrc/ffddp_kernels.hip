// ffddp_kernels.hip — batched (Box)FDDP on MI355X (gfx950), fp64.
//
// One solve() of crocoddyl::SolverBoxFDDP (reference call sites
// crocoddyl_classical.py:367 / crocoddyl_force_feedback.py:605) for B
// independent OCP instances, as a fixed sequence of kernels per FDDP
// iteration; all per-instance control flow (regularisation, line-search
// acceptance, feasibility, stopping) lives on the device, masked per instance:
//
//   k_node      calc + calcDiff of every (instance, node), 16-lane group per
//               node: lanes 0..7 run the calc (joint lanes + EE lane, log-depth
//               scans: dynamics, costs, gaps) into the group's LDS, then lane j
//               computes state direction j in closed form (Jacobian column j)
//               and the Gauss-Newton Hessians are assembled across the group.
//   k_backward_w  Riccati backward pass, one wavefront per instance, blocks in
//               LDS; Cholesky (infeasible iterations) or BoxQP gains;
//               regularisation retries inside the kernel.
//   k_forward_g8  line search: one 8-lane group per (instance, step length) —
//               the trials of SolverFDDP::solve evaluated concurrently (the
//               first accepted one is the sequential answer).
//   k_accept    acceptance test / regularisation / stopping (SolverFDDP::solve),
//               one lane per instance; the accepted trial stays in place (the
//               next k_node reads it and writes it into xs / us; k_commit at
//               the end of the solve for the rest).
#include <hip/hip_runtime.h>
#include <sched.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "ffddp_consts.hpp"
#include "ffddp_group.hpp"
#include "ffddp_plant.hpp"
#include "ffddp_primal_g8.hpp"
#include "ffddp_rollout.hpp"

using namespace ffddp;

namespace {

constexpr int NODE_GROUP = 16;
#ifndef NODE_BLOCK
#define NODE_BLOCK 64
#endif
constexpr int NODE_GPB = NODE_BLOCK / NODE_GROUP;
#ifndef NODE_WAVES
#define NODE_WAVES 2
#endif
#ifndef QC_UNROLL
#define QC_UNROLL 1
#endif
#ifndef QC_FF_LATE
#define QC_FF_LATE 0  // phase C unroll of FF's latency variant (0: full; FF B=1024 +1.4 % over 1 since the LDS diet)
#endif
// BW_PF_LATE: when k_backward_w issues the loads of the next node's record:
// at the top of the node (0), or after phase D with the record staged into
// LDS at the end of the node (S.R is dead after phase C), so the prefetch
// registers are not live across the gains (1: FF only, 2: both variants)
#ifndef BW_PF_LATE
#define BW_PF_LATE 0
#endif
// backward LDS diet (round 5): BW_DIET_UNION puts Y with the factors and M
// with K in one slot each (FF only, BwSlots), BW_DIET_SLOTS stages the
// per-lane inputs in n-entry arrays (lane l writes slot l mod n) instead of
// 64-entry ones
#ifndef BW_DIET_UNION
#define BW_DIET_UNION 1
#endif
#ifndef BW_DIET_SLOTS
#define BW_DIET_SLOTS 1
#endif
#ifndef BW_WAVES
#define BW_WAVES 1
#endif

struct InstState {
  double preg, cost, dg, dq, stop;
  double ffeas;  // max |fs| of the last calcDiff (the trace's ||ffeas||)
  int is_feasible, was_feasible, done, ok, iter, recalc, accepted, bw_ok;
  int n_iters, n_trials, n_retries, n_backward, n_calc, n_forward;
  int n_eval1, n_eval2;  // line-search trials evaluated by the first / second pass
  int n_neg, n_neg_acc;  // trials judged / accepted by the ascent-direction branch (dVexp < 0)
};

struct Dev {
  int B, N, nx, rec;
  double* rec_buf;   // [B][N+1][rec]
  double* fs;        // [B][N+1][nx]
  double* xs;        // [B][N+1][nx]
  double* us;        // [B][N][7]
  double* K;         // [B][N][7][nx]
  double* k;         // [B][N][7]
  double* w;         // [B][N+1][nx]   Vxx_t fs_t
  double* xs_try;    // [B][T][N+1][nx]
  double* us_try;    // [B][T][N][7]
  double* trial;     // [B][T][2]  cost_try, dv
  int* trial_fail;   // [B][T]
  InstState* st;     // [B]
  int* alist;        // [2][B]  active-instance lists (slice-local indices), double-buffered over iterations
  int* acnt;         // [4]     their lengths; [2 + p]: an instance of the iteration that built list p
                     //         needed more step lengths than the host's first pass (first_width)
  double* trace;     // [B][trace_it][FFDDP_TRACE_W] per-iteration records (CallbackVerbose), or null
  int trace_it;
};

// Active-instance compaction.  Iteration it reads list (it & 1): the
// instances not yet done, packed at the front, so the blocks / groups of the
// per-iteration kernels that carry work are the first ones of the grid and
// the rest exit at once.  Without it a late iteration's few active
// instances are scattered over the whole grid, and a grid larger than one
// wave per SIMD (the 1-wave/SIMD line search with 4 trials) ran its active
// waves in two dispatch rounds.  k_accept appends the instances that
// continue to the other list; k_backward_w zeroes that list's length first.
// marks accumulator registers a0..a39 used, so the kernel's register
// allocation (and its SIMD occupancy) includes them
#define RESERVE_AGPR40() asm volatile("" ::: "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39")

// a global-memory pointer (address space 1): stays one after an opaque asm
template <class T> using gptr = __attribute__((address_space(1))) T*;

struct ActiveList {
  const int* list;
  int n;
};
__device__ __forceinline__ ActiveList active_list(const Dev& d, int cur) {
  return ActiveList{d.alist + (long)cur * d.B, d.acnt[cur]};
}

// XCD-aware block order.  The hardware hands consecutive workgroups to the 8
// XCDs round-robin, each XCD with its own L2: an instance's node groups (or
// line-search trials) spread over several blocks would pull its shared lines
// (node references, the iterate, K, the instance state, partly written gap
// lines) into several L2s.  Remap so that each XCD processes one contiguous
// range of the n blocks that carry work; blocks >= n keep their index.
constexpr int N_XCD = 8;
__device__ __forceinline__ long xcd_block(long b, long n) {
  if (b >= n) return b;
  const long q = n / N_XCD, r = n % N_XCD;
  const long x = b % N_XCD, i = b / N_XCD;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// ---------------------------------------------------------------------------
// init
// ---------------------------------------------------------------------------
// xs_init / us_init may be d.xs / d.us (warm start in place, ffddp.h): not
// __restrict__; each element is read and written by the same thread
__global__ void k_init(const DevConsts* __restrict__ Cg, Dev d, const double* xs_init, const double* us_init,
                       int is_feasible) {
  const DevConsts& C = *Cg;
  const int N = C.N, nx = C.nx;
  const long nX = (long)d.B * (N + 1) * nx;
  const long nU = (long)d.B * N * NU;
  const long nK = (long)d.B * N * NU * nx;
  const long nT = d.trace ? (long)d.B * d.trace_it * FFDDP_TRACE_W : 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nK || i < nT; i += (long)gridDim.x * blockDim.x) {
    if (i < nT) d.trace[i] = __builtin_nan("");
    if (i >= nK) continue;
    if (i < nX) d.xs[i] = xs_init[i];
    if (i < nU) {
      d.us[i] = us_init[i];
      d.k[i] = 0.0;
    }
    d.K[i] = 0.0;
    if (i < d.B) {
      d.alist[i] = (int)i;
      if (i == 0) {
        d.acnt[0] = d.B;
        d.acnt[1] = 0;
        d.acnt[2] = 0;
        d.acnt[3] = 0;
      }
      InstState s;
      s.preg = C.reg_min;
      s.cost = 0.0;
      s.dg = s.dq = 0.0;
      s.stop = __builtin_nan("");
      s.is_feasible = is_feasible;
      s.was_feasible = 0;
      s.done = 0;
      s.ok = 0;
      s.iter = 0;
      s.recalc = 1;
      s.accepted = -1;
      s.bw_ok = 0;
      s.n_iters = s.n_trials = s.n_retries = s.n_backward = s.n_calc = s.n_forward = 0;
      s.n_eval1 = s.n_eval2 = 0;
      s.n_neg = s.n_neg_acc = 0;
      s.ffeas = 0.0;
      d.st[i] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// calc + calcDiff of all nodes
// ---------------------------------------------------------------------------
// Per 16-lane group.  The link record is dead once the tangents are in
// registers, so the residual-Jacobian columns reuse its space (a barrier
// separates the last read of lk from the first write of col): 18.3 KB per
// 64-lane block instead of 25 KB, i.e. 8 blocks per CU (the VGPR limit)
// instead of 6 (the LDS limit).
struct NodeGroupShared {
  Primal P;
  union {
    double lk[LK_ALLOC];
    double col[14][NDENSE_MAX];  // residual-Jacobian columns, state directions
  };
  double colu[7][FFDDP_MAX_NC];  // force rows, inner-control directions
};
struct NodeShared {
  NodeGroupShared g[NODE_GPB];
};

// The calc of one node on an 8-lane group (lanes = joints + EE): dynamics,
// costs with their Gauss-Newton weights, gaps; Primal and link record to P /
// lk (the node group's LDS in k_node).
template <int NC, bool FF>
__device__ __forceinline__ void primal_group(const DevConsts& C, const Dev& d, const double* __restrict__ x0,
                                             const double* __restrict__ node_ref, const double* __restrict__ inst_ref,
                                             const uint8_t* __restrict__ surface, int b, int t, Primal* P,
                                             double* lk, const double* __restrict__ xsrc,
                                             const double* __restrict__ usrc) {
  const int N = C.N;
  constexpr int nx = FF ? 21 : 14;
  const int li = g8_lane();
  const bool J = li < NQ;
  const int ji = J ? li : 0;
  const bool surf = surface[b] != 0;
  const bool terminal = t == N;
  const int mode = !terminal ? MODE_RUNNING : (FF ? MODE_TERMINAL_U : MODE_TERMINAL_X);
  const double* y = xsrc + (long)t * nx;
  const double* ref = node_ref + ((long)b * (N + 1) + t) * 6;
  const double* xreg = inst_ref + (long)b * 21;
  const double* uin = FF ? (y + 14) : (terminal ? nullptr : usrc + (long)t * NU);
  const double q = y[ji], v = y[7 + ji];
  const double u = (uin != nullptr) ? uin[ji] : 0.0;
  // setCandidate: the accepted line-search trial becomes (xs, us) here, node
  // by node, instead of a whole-trajectory copy on the iteration's chain.
  // Classical: stored at the end of the calc from registers; issued here,
  // the stores sat in front of the vmcnt(0) wait of every later load (the
  // per-lane cost constants in node_primal_g8, the gaps' next state).  FF
  // (at its register limit: the late stores spill) stores here.
  const bool commit = J && xsrc != d.xs + (long)b * (N + 1) * nx;
  double cu = 0.0;
  if (commit) {
    if (FF) {
#pragma unroll
      for (int k = 0; k < 3; ++k) d.xs[((long)b * (N + 1) + t) * nx + 7 * k + li] = y[7 * k + li];
      if (!terminal) d.us[((long)b * N + t) * NU + li] = usrc[(long)t * NU + li];
    } else if (!terminal) {
      cu = usrc[(long)t * NU + li];
    }
  }
  double lam[3];
  const double pc = node_primal_g8<NC>(C, mode, surf, q, v, u, xreg[ji], xreg[7 + ji], xreg[14 + ji], ref,
                                       P, lk, lam);
  double* rec = d.rec_buf + ((long)b * (N + 1) + t) * d.rec;
  // node cost (IAM scaling, FF augmentation terms): per-lane shares summed over the group
  double c = FF ? C.dt * pc : (terminal ? pc : C.dt * pc);
  if (FF) {
    double part = 0.0;
    if (J) {
      if (C.w_y > 0.0) {
        double a_ = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const double dd = y[7 * k + li] - x0[(long)b * nx + 7 * k + li];
          a_ += C.Wy2[7 * k + li] * dd * dd;
        }
        part += 0.5 * C.w_y * a_;
      }
      if (!terminal) {
        const double ww = usrc[(long)t * NU + li];
        if (C.w_w > 0.0) part += 0.5 * C.w_w * (ww * ww);
        if (C.w_ws > 0.0) {
          const double ov = fabs(ww) - C.ws_lim[li];
          const double o = ov > 0.0 ? ov : 0.0;
          part += C.w_ws * (0.5 * (o * o));
        }
      }
    }
    c += g8_sum(part);
  }
  if (li == 0) {
    rec[rec_off_cost(nx)] = c;
#pragma unroll
    for (int r = 0; r < 3; ++r) rec[rec_off_lam(nx) + r] = (mode == MODE_TERMINAL_X) ? 0.0 : lam[r];
  }
  // gaps fs[t+1] = xnext_t - xs[t+1] ; fs[0] = x0 - xs[0]  (zero once feasible)
  const bool feas = d.st[b].is_feasible != 0;
  if (J) {
    if (!terminal) {
      double* f = d.fs + ((long)b * (N + 1) + t + 1) * nx;
      const double* yn = xsrc + (long)(t + 1) * nx;
      const double dt = C.dt;
      const double a = P->a[li];  // this lane's own store
      const double qn = (mode == MODE_TERMINAL_X) ? q : q + (v * dt + a * dt * dt);
      const double vn = (mode == MODE_TERMINAL_X) ? v : v + a * dt;
      f[li] = feas ? 0.0 : qn - yn[li];
      f[7 + li] = feas ? 0.0 : vn - yn[7 + li];
      if (FF) f[14 + li] = feas ? 0.0 : (C.alpha * y[14 + li] + C.beta * usrc[(long)t * NU + li]) - yn[14 + li];
    }
    if (t == 0) {
      double* f = d.fs + (long)b * (N + 1) * nx;
#pragma unroll
      for (int k = 0; k < (FF ? 3 : 2); ++k) f[7 * k + li] = feas ? 0.0 : x0[(long)b * nx + 7 * k + li] - y[7 * k + li];
    }
  }
  if (!FF && commit) {
    double* xr = d.xs + ((long)b * (N + 1) + t) * nx;
    xr[li] = q;
    xr[7 + li] = v;
    if (!terminal) d.us[((long)b * N + t) * NU + li] = cu;
  }
}

// a^T H b over the contact-force block of the Gauss-Newton Hessian: diagonal
// Dd plus (nc = 3) the friction cone's off-diagonal couplings Do
template <int NC>
__device__ __forceinline__ double fquad(const double* a, const double* Dd, const double* Do, const double* b) {
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < NC; ++r) acc += a[r] * Dd[r] * b[r];
  if (NC == 3)
    acc += Do[0] * (a[1] * b[0] + a[0] * b[1]) + Do[1] * (a[2] * b[0] + a[0] * b[2]) +
           Do[2] * (a[2] * b[1] + a[1] * b[2]);
  return acc;
}

// calc + calcDiff tangents + Gauss-Newton assembly: 16-lane group per node.
// The group's lanes 0..7 first run the node's calc (primal_group) into the
// group's LDS, so the Primal / link records (~4 KB per node) never round-trip
// through HBM: a separate calc kernel writing them and this one reading them
// back was 129 + 366 us per launch at B=4096; fused, 255 us.
template <int NC, bool FF>
__global__ __launch_bounds__(NODE_BLOCK) __attribute__((amdgpu_waves_per_eu(NODE_WAVES))) void k_node(const DevConsts* __restrict__ Cg, Dev d,
                                                      const double* __restrict__ x0,
                                                      const double* __restrict__ node_ref,
                                                      const double* __restrict__ inst_ref,
                                                      const uint8_t* __restrict__ surface, int force_all, int cur) {
  const DevConsts& C = *Cg;
  const int N = C.N;
  constexpr int nx = FF ? 21 : 14;
  constexpr int nc = NC;
  __shared__ NodeShared S;
  const int grp = threadIdx.x / NODE_GROUP, lane = threadIdx.x % NODE_GROUP;
  const int n_work = force_all ? d.B : d.acnt[cur];  // instances with nodes to evaluate
  const long blk = xcd_block(blockIdx.x, ((long)n_work * (N + 1) + NODE_GPB - 1) / NODE_GPB);
  const long gnode = blk * NODE_GPB + grp;
  const int slot = (int)(gnode / (N + 1)), t = (int)(gnode % (N + 1));
  int b = slot;
  bool active = slot < d.B;
  if (active && !force_all) {
    const ActiveList al = active_list(d, cur);
    active = slot < al.n;
    b = active ? al.list[slot] : 0;
    if (active) active = (d.st[b].done == 0) && (d.st[b].recalc != 0);
  }
  const long node = (long)b * (N + 1) + t;
  const bool surf = active ? surface[b] != 0 : false;
  const bool terminal = t == N;
  constexpr bool ff = FF;
  const int mode = !terminal ? MODE_RUNNING : (ff ? MODE_TERMINAL_U : MODE_TERMINAL_X);
  // current iterate: the trial the last line search accepted (not yet copied
  // into xs / us: primal_group does that for its node), else xs / us
  const long perX = (long)(N + 1) * nx, perU = (long)N * NU;
  const int acc = active ? d.st[b].accepted : -1;
  const double* xsrc = acc >= 0 ? d.xs_try + ((long)b * NTRIALS + acc) * perX : d.xs + (long)b * perX;
  const double* usrc = acc >= 0 ? d.us_try + ((long)b * NTRIALS + acc) * perU : d.us + (long)b * perU;
  const double* y = xsrc + (long)t * nx;
  const double* ref = node_ref + ((long)b * (N + 1) + t) * 6;
  NodeGroupShared& G = S.g[grp];
  Primal& P = G.P;
  if (active && lane < G8) primal_group<NC, FF>(C, d, x0, node_ref, inst_ref, surface, b, t, &P, G.lk, xsrc, usrc);
  __syncthreads();
  const bool need_u = mode != MODE_TERMINAL_X;
  // control directions first, their results stored at once (neither touches
  // lk), so they are not live across the state tangent: no scratch spill at
  // 2 waves/SIMD
  if (active && lane < 7 && need_u) {
    double dau[NQ], dlamu[3];
    node_tangent_control<NC>(C, surf, P, lane, dau, dlamu);
    double* rec = d.rec_buf + ((long)b * (N + 1) + t) * d.rec;
    for (int i = 0; i < NQ; ++i) rec[rec_off_A() + (14 + lane) * NQ + i] = dau[i];
    for (int r = 0; r < nc; ++r) G.colu[lane][r] = (surf ? dlamu[r] : 0.0);
  }
  double da[NQ], dlam[3], col[NDENSE_MAX], r1[NQ], dh[3];
  if (active && lane < 14) node_tangent_state_links<NC>(C, mode, surf, G.lk, P, lane, r1, dh, col);
  __syncthreads();  // every lane's reads of lk are done before col overwrites it
  // the column's rows 0..11 go to LDS before the contact solves (which read
  // only P), so they are not live across them: no scratch spill at 2 waves/SIMD
  if (active && lane < 14) {
    for (int r = 0; r < 12; ++r) G.col[lane][r] = col[r];
    node_tangent_state_contact<NC>(mode, surf, P, r1, dh, da, dlam, col);
    for (int r = 12; r < 12 + nc; ++r) G.col[lane][r] = col[r];
  }
  __syncthreads();
  if (active) {
    double* rec = d.rec_buf + ((long)b * (N + 1) + t) * d.rec;
    const int nd = 12 + nc;
    const bool scale = mode != MODE_TERMINAL_X;
    const double sc = scale ? C.dt : 1.0;
    const double* D = P.D;
    const double* g = P.g;
    // FF's y-cost weights of this lane's components, loaded once up front:
    // at each use the scalar w_y and the lane's Wy2 entry were loaded again
    // and waited for with vmcnt(0), i.e. behind every record store in flight
    // (FF k_node 109 -> 104 us at B = 1024; the compiler contracts some of
    // the products differently, so FF solves move by <= 2e-9, classical
    // ones are bit-identical)
    double wy = 0.0, wy2j = 0.0, wy2u = 0.0;
    if (ff) {
      wy = C.w_y;
      wy2j = C.Wy2[lane < 14 ? lane : 0];
      wy2u = C.Wy2[14 + (lane < 7 ? lane : 0)];
      asm volatile("" : "+s"(wy), "+v"(wy2j), "+v"(wy2u));
    }
    if (lane < 14) {
      const int j = lane;
      // dynamics Jacobian columns
      if (need_u)
        for (int i = 0; i < NQ; ++i) rec[rec_off_A() + j * NQ + i] = da[i];
      // Lxx_in column j (rows 0..13)
      double* Lxx = rec + rec_off_Lxx(nx);
      for (int i = 0; i < 14; ++i) {
        double acc = 0.0;
        for (int r = 0; r < 12; ++r) acc += G.col[i][r] * D[r] * col[r];
        acc += fquad<NC>(&G.col[i][12], D + 12, P.Dfo, col + 12);
        if (i == j) acc += P.Dx[j];
        acc *= sc;
        if (ff && i == j) acc += wy * wy2j;
        Lxx[i * nx + j] = acc;
      }
      // Lx_in[j]
      double lx = 0.0;
      for (int r = 0; r < nd; ++r) lx += col[r] * g[r];
      lx = (lx + P.gx[j]) * sc;
      if (ff) lx += wy * wy2j * (y[j] - x0[(long)b * nx + j]);
      rec[rec_off_Lx(nx) + j] = lx;
      // Lxu_in row j (force rows only): classical -> Lxu row j; FF -> Lxx_aug[14+k][j]
      if (need_u) {
        for (int kk = 0; kk < NU; ++kk) {
          double acc = 0.0;
          acc = fquad<NC>(col + 12, D + 12, P.Dfo, G.colu[kk]);
          acc *= sc;
          if (ff)
            Lxx[(14 + kk) * nx + j] = acc;
          else
            rec[rec_off_Lxu(nx) + j * NU + kk] = acc;
        }
      }
    }
    if (lane < 7 && need_u) {
      const int kk = lane;
      // Luu_in column kk
      double luu[7];
      for (int m = 0; m < NU; ++m) {
        double acc = 0.0;
        acc = fquad<NC>(G.colu[m], D + 12, P.Dfo, G.colu[kk]);
        if (m == kk) acc += P.Du[kk];
        luu[m] = acc * sc;
      }
      double lu = 0.0;
      for (int r = 0; r < nc; ++r) lu += G.colu[kk][r] * g[12 + r];
      lu = (lu + P.gu[kk]) * sc;
      if (!ff) {
        for (int m = 0; m < NU; ++m) rec[rec_off_Luu(nx) + m * NU + kk] = luu[m];
        rec[rec_off_Lu(nx) + kk] = lu;
      } else {
        double* Lxx = rec + rec_off_Lxx(nx);
        // Lxx_aug column 14+kk: rows 0..13 = Lxu_in[:, kk], rows 14..20 = Luu_in[:, kk] + w_y Wy2
        for (int i = 0; i < 14; ++i) {
          double acc = 0.0;
          acc = fquad<NC>(&G.col[i][12], D + 12, P.Dfo, G.colu[kk]);
          Lxx[i * nx + 14 + kk] = acc * sc;
        }
        for (int m = 0; m < NU; ++m)
          Lxx[(14 + m) * nx + 14 + kk] = luu[m] + (m == kk ? wy * wy2u : 0.0);
        rec[rec_off_Lx(nx) + 14 + kk] = lu + wy * wy2u * (y[14 + kk] - x0[(long)b * nx + 14 + kk]);
        // augmented control terms: Lu = w_w w + w_s g_soft ; Luu = diag ; Lxu = 0
        double wk = 0.0;
        if (!terminal) wk = usrc[(long)t * NU + kk];
        const double ov = fabs(wk) - C.ws_lim[kk];
        const bool act = ov > 0.0;
        const double gs = act ? ov * (wk > 0.0 ? 1.0 : (wk < 0.0 ? -1.0 : 0.0)) : 0.0;
        rec[rec_off_Lu(nx) + kk] = C.w_w * wk + C.w_ws * gs;
        for (int m = 0; m < NU; ++m)
          rec[rec_off_Luu(nx) + m * NU + kk] = (m == kk) ? (C.w_w + C.w_ws * (act ? 1.0 : 0.0)) : 0.0;
        for (int i = 0; i < nx; ++i) rec[rec_off_Lxu(nx) + i * NU + kk] = 0.0;
      }
    }
    if (!need_u && lane < 7) {
      // classical terminal: no control blocks (zero them for the calcDiff export)
      for (int i = 0; i < NQ; ++i) rec[rec_off_A() + (14 + lane) * NQ + i] = 0.0;
    }
  }
}


__device__ __forceinline__ bool bad(double v) { return isnan(v) || isinf(v) || v >= 1e30; }


// sum over the 64 lanes, wave-uniform result: DPP butterflies inside each
// 16-lane row (quad swaps, half-row and row mirrors), then the four row sums
// by readlane -- no ds_bpermute round trips on the backward pass's chain
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp64<0x141>(v);  // row_half_mirror
  v += dpp64<0x140>(v);  // row_mirror
  const double r0 = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 0),
                                     __builtin_amdgcn_readlane(__double2loint(v), 0));
  const double r1 = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 16),
                                     __builtin_amdgcn_readlane(__double2loint(v), 16));
  const double r2 = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 32),
                                     __builtin_amdgcn_readlane(__double2loint(v), 32));
  const double r3 = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 48),
                                     __builtin_amdgcn_readlane(__double2loint(v), 48));
  return (r0 + r1) + (r2 + r3);
}

// max over the 64 lanes (values >= 0), wave-uniform result
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp64<0xB1>(v));
  v = fmax(v, dpp64<0x4E>(v));
  v = fmax(v, dpp64<0x141>(v));
  v = fmax(v, dpp64<0x140>(v));
  double m = v;
#pragma unroll
  for (int r = 16; r < 64; r += 16)
    m = fmax(m, __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), r),
                                 __builtin_amdgcn_readlane(__double2loint(v), r)));
  return fmax(m, __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 0),
                                  __builtin_amdgcn_readlane(__double2loint(v), 0)));
}

// ---------------------------------------------------------------------------
// backward pass, one wavefront per instance (k_backward_w)
//
// The Riccati recursion of one instance is a chain of 30 small dense steps;
// what bounds it is latency, not flops.  One wave (64 lanes) owns one
// instance and spreads each step's algebra over all lanes:
//   [Fx Fu] = I~ + D A^        (Euler structure: I~ sparse, D = [dt^2 I; dt I],
//                               A^ = node acceleration Jacobian, 7 x (nx+nu))
//   Q = L + I~'V I~ + M A^ + (M A^)',   M = I~'(V D) + 1/2 A^'(D'V D)
// so the full Q (x and u blocks) is one symmetric rank-7 update plus sparse
// terms; every lane computes a few lower-triangle entries.  The node record
// for t-1 is prefetched into registers while node t is processed (LDS-only
// fences between phases, so the prefetch stays in flight), and with no
// per-lane arrays beyond that the kernel fits several waves per SIMD, so
// instances hide each other's latency.  Gains (LLT / BoxQP on 7x7) stay on
// lane 0.
// ---------------------------------------------------------------------------
constexpr int rec_words(int nx) { return ((147 + nx * nx + nx * 7 + 49 + nx + 7 + 1) + 3 + 15) & ~15; }

__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Y (D' V D) lives in phases A-B, the factors L (packed masked Cholesky
// factor, reciprocal diagonal) and L1 (k_backward_w2: wave 1's factor of the
// full set) in D-E; M in B-C, K in D/E-G (k_backward_w2: G runs beside the
// next node's A, still before its B).  U: one slot each for Y / {L, L1} and
// M / K.  It saves FF's backward 1.5 KB of LDS (8 blocks per CU, with the
// rest of the diet), but the aliasing costs the classical pass at B = 4096
// (522k-526k vs 546k-548k solves/s without it), so only FF takes it.
template <bool U, int NM, int NK> struct BwSlots {
  double Y[NU * NU], L[28], L1[28], M[NM], K[NK];
};
template <int NM, int NK> struct BwSlots<true, NM, NK> {
  union {
    double Y[NU * NU];
    struct {
      double L[28];
      double L1[28];
    };
  };
  union {
    double M[NM];
    double K[NK];
  };
};

template <bool FF> struct BwW {
  static constexpr int NX = FF ? 21 : 14;
  static constexpr int ND = NX + NU;
  static constexpr int REC = rec_words(NX);
  // Q's distinct blocks, contiguous so that phase C stores an entry through
  // one flat index: Qxx (full, mirrored) | Qxu (row-major, NX x 7) | H =
  // Quu + preg I (full, mirrored); Qux and the Quu copy of the full ND x ND
  // matrix are never read (round 5: FF 25.7 -> 19.8 KB per wave, 8 blocks
  // per CU instead of 6)
  static constexpr int QXU = NX * NX, QH = NX * NX + NX * NU, NQQ = NX * NX + NX * NU + NU * NU;
  double R[(REC + 63) / 64 * 64];  // staged node record (A | Lxx | Lxu | Luu | Lx | Lu | cost | lam), padded
  double V[NX * NX];  // V_xx' on entry to a node, V_xx on exit
  double QQ[NQQ];
  double W[NX * NU];  // V D
  // Y lives in phases A-B, the factors in D-E: one slot
  BwSlots<FF && BW_DIET_UNION, ND * NU, NU * NX> sl;  // Y, L, L1, M, K
  int spec;           // k_backward_w2: wave 1's K (and LLT k) from L1 are valid
  double Vx[NX], Qv[ND], kk[NU], z[NU];
  // staged per node by every lane without lane guards: lane l writes slot
  // l mod n, which the lanes load from the matching index (duplicate writers
  // store the same value)
  double fs[BW_DIET_SLOTS ? NX : 64], kp[BW_DIET_SLOTS ? NU : 64], uu[BW_DIET_SLOTS ? NU : 64];
  double ulb[BW_DIET_SLOTS ? NU : 64], uub[BW_DIET_SLOTS ? NU : 64];
  double fsb[2][BW_DIET_SLOTS ? NX : 64];  // k_backward_w2: node t's gap in slot t & 1 (staged before node t+1's phase G reads its own)
  int flag;
  int badw[2];  // k_backward_w2: per-wave NaN flags of phases F / G
#ifdef BW_PAD_CL
  double pad[FF ? 1 : BW_PAD_CL];  // development: classical LDS footprint back to the round-4 size
#endif
};

// Phase C's entry for flat index e of a pass over the lower triangle (NQE
// entries, the last pass starting at `last`): a lane past the last entry
// takes an entry of that same pass, so its duplicate store is computed by the
// same instruction from the same operands as the owner's (identical bits in
// any unrolling or contraction), with no address select and no spare slot
__device__ __forceinline__ int spare_entry(int e, int nqe, int last) {
  return e < nqe ? e : last + (e - last) % (nqe - last);
}
// phase C's packed entry (r >= c): r, c and the two flat BwW::QQ indices its
// value is stored at (Qxx mirrored; Qux stored once as Qxu[c][r - NX]; Quu
// mirrored into H)
template <int NX> __device__ __forceinline__ unsigned q_entry(int r, int c) {
  // fields: r, c 5 bits each, i1, i2 11 bits each
  static_assert(NX + NU <= 32 && (NX + NU) * (NX + NU) <= 2048, "q_entry packing");
  unsigned i1, i2;
  if (r < NX) {
    i1 = r * NX + c;
    i2 = c * NX + r;
  } else if (c < NX) {
    i1 = i2 = NX * NX + c * NU + (r - NX);
  } else {
    i1 = NX * NX + NX * NU + (r - NX) * NU + (c - NX);
    i2 = NX * NX + NX * NU + (c - NX) * NU + (r - NX);
  }
  return ((unsigned)r << 27) | ((unsigned)c << 22) | (i1 << 11) | i2;
}

// nonzeros of column c of I~ (the Euler identity part of [Fx Fu]):
// returns the count and fills (row, coef) pairs.
template <bool FF> __device__ __forceinline__ int itilde(int c, double dt, double alpha, double beta, int (&row)[2],
                                                         double (&cf)[2]) {
  if (c < 7) {
    row[0] = c;
    cf[0] = 1.0;
    return 1;
  }
  if (c < 14) {
    row[0] = c;
    cf[0] = 1.0;
    row[1] = c - 7;
    cf[1] = dt;
    return 2;
  }
  if (!FF) return 0;  // classical u columns: Fu = D A_u only
  if (c < 21) {
    row[0] = c;
    cf[0] = alpha;
    return 1;
  }
  row[0] = c - 7;
  cf[0] = beta;
  return 1;
}

// branch-free form of itilde: two (row, coef) terms, coef 0 where absent (row kept in range)
template <bool FF>
__device__ __forceinline__ void itilde2(int c, double dt, double alpha, double beta, int& r0, double& a0, int& r1,
                                        double& a1) {
  const bool lo = c < 14;
  a0 = lo ? 1.0 : (FF ? (c < 21 ? alpha : beta) : 0.0);
  r0 = lo ? c : (FF ? (c < 21 ? c : c - 7) : 0);
  const bool vel = c >= 7 && c < 14;
  a1 = vel ? dt : 0.0;
  r1 = vel ? c - 7 : 0;
}

// A^[m][c] = d a_m / d dir_c (record rows 0..20; FF w-columns 21..27 are zero)
template <bool FF> __device__ __forceinline__ double ahat(const double* Ar, int m, int c) {
  return (FF && c >= 21) ? 0.0 : Ar[c * 7 + m];
}

// lower-triangle index e -> (r, c), r >= c
__device__ __forceinline__ void tri_rc(int e, int& r, int& c) {
  int rr = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  while ((rr + 1) * (rr + 2) / 2 <= e) ++rr;
  while (rr * (rr + 1) / 2 > e) --rr;
  r = rr;
  c = e - rr * (rr + 1) / 2;
}

// ---- 7x7 algebra with one row / variable per lane (lanes 0..6), uniform control flow ----
// lane k's value to every lane of its 16-lane row (DPP row_newbcast: one
// v_mov_b64_dpp, no SGPR round trip).  The 7x7 algebra below lives on lanes
// 0..6 of row 0; the other rows compute on their own (unused) lanes.
// k is a constant after unrolling: the switch folds away
__device__ __forceinline__ double rowb(double v, int k) {
  switch (k) {
    case 0: return g8_rowb<0>(v);
    case 1: return g8_rowb<1>(v);
    case 2: return g8_rowb<2>(v);
    case 3: return g8_rowb<3>(v);
    case 4: return g8_rowb<4>(v);
    case 5: return g8_rowb<5>(v);
    default: return g8_rowb<6>(v);
  }
}

// In-place LLT of the SPD matrix whose row i is held by lane i: on exit
// a[j] (j < i) = L_ij and a[i] = 1 / L_ii.  Returns false (uniformly) if a
// pivot is not positive.  The pivot test is one ballot after the
// factorisation, not a branch per pivot: past a bad pivot the values are
// garbage (NaN) but unused, and a good factorisation takes the same
// operations either way.  Every product-sum is an explicit fma (and the
// reciprocal square root's Newton steps too), so the larger basic block
// cannot change how the compiler contracts them: every backward variant and
// BoxQP's refactorisations round alike (wave 1's speculative factor in
// k_backward_w2 must equal BoxQP's for an empty clamped set, bit for bit).
__device__ __forceinline__ bool chol_rows(double (&a)[NU], int lane) {
  bool bad = false;
#pragma unroll
  for (int k = 0; k < NU; ++k) {
    double d = a[k];
#pragma unroll
    for (int m = 0; m < k; ++m) d = __builtin_fma(-a[m], a[m], d);
    const double dk = rowb(d, k);
    bad = bad || !(dk > 0.0);  // dk is uniform across the row
    double il = __builtin_amdgcn_rsq(dk);
    const double h = 0.5 * dk;
    il = il * __builtin_fma(-(h * il), il, 1.5);
    il = il * __builtin_fma(-(h * il), il, 1.5);
    double s = a[k];
#pragma unroll
    for (int m = 0; m < k; ++m) s = __builtin_fma(-a[m], rowb(a[m], k), s);
    a[k] = (lane == k) ? il : ((lane > k) ? s * il : a[k]);
  }
  return !(__ballot(bad) & 1ull);  // lane 0 holds row 0's pivots
}

// solve L L^T x = r with L held as rows (chol_rows layout); r / result per lane
__device__ __forceinline__ double chol_solve_rows(const double (&Lr)[NU], double r, int lane) {
  double y[NU];
#pragma unroll
  for (int k = 0; k < NU; ++k) {
    double s = r;
#pragma unroll
    for (int m = 0; m < k; ++m) s -= Lr[m] * y[m];
    y[k] = rowb(s * Lr[k], k);
  }
  double x[NU];
#pragma unroll
  for (int k = NU - 1; k >= 0; --k) {
    double s = y[k];
#pragma unroll
    for (int m = k + 1; m < NU; ++m) s -= rowb(Lr[k], m) * x[m];
    x[k] = s * rowb(Lr[k], k);
  }
  double out = 0.0;
#pragma unroll
  for (int k = 0; k < NU; ++k) out = (lane == k) ? x[k] : out;
  return out;
}

// phase E's factor without the LDS round trip: the lower triangle of the
// chol_rows factor (rows on lanes 0..6) in tri layout in every lane of DPP
// row 0 (lanes 0..15: the classical pass's K columns and k), by row_newbcast.
// chol_solve then reads the same values it would read from the LDS copy.
constexpr bool e_from_regs(int nx) { return nx + 1 <= 16; }
__device__ __forceinline__ void rows_to_tri(const double (&Lr)[NU], double (&Lt)[NU * (NU + 1) / 2]) {
#pragma unroll
  for (int i = 0; i < NU; ++i)
#pragma unroll
    for (int k = 0; k <= i; ++k) Lt[tri(i, k)] = rowb(Lr[k], i);
}

// a branch on lane 0's value of a condition (lane 0 holds the 8-lane sums /
// maxima like every lane of its group): a ballot bit, no readlane round trip
__device__ __forceinline__ bool lane0(bool c) { return (__ballot(c) & 1ull) != 0; }
// max over lanes 0..7 of |v| below th, as one ballot instead of max8's three
// DPP steps: the same decision (v_max_f64 skips a NaN operand and a NaN lane
// fails `>= th` alike; lane 7 holds 0 in every BoxQP vector, so the maximum
// is never taken over NaN lanes only)
__device__ __forceinline__ bool all8_below(double av, double th) { return (__ballot(av >= th) & 0x7Full) == 0; }

// crocoddyl::BoxQP::solve with variable i on lane i: projected Newton on the
// free set, refactored when it changes, Armijo line search over the same
// alphas.  hrow = row i of H; x in = warm start, out = solution; Lr = rows of
// the masked factor of the final free set; clmask = final clamped set.  The
// scalar products (objective values, directional derivative) and the step
// norm are lane-local terms summed / maxed by DPP over the 8 lanes; only the
// vectors a mat-vec needs (x, the trial point) are broadcast.
__device__ __forceinline__ bool boxqp_lanes(const DevConsts& C, const double (&hrow)[NU], double q, double lb,
                                            double ub, double& x, double (&Lr)[NU], int& clmask, int lane,
                                            unsigned long long* pq = nullptr) {
  (void)pq;  // FFDDP_PHASE_PROF builds: the split of this QP's time (BQ_*)
  BQ_T0();
  x = fmax(fmin(x, ub), lb);
  bool have = false, cl = false;
  double xsf = 0.0;
#pragma unroll 1
  for (int it = 0; it < C.qp_maxiter; ++it) {
    double xb[NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) xb[j] = rowb(x, j);
    double hx = 0.0;
#pragma unroll
    for (int j = 0; j < NU; ++j) hx += hrow[j] * xb[j];
    const double g = q + hx;
    // the objective at x: needed only if this iteration steps, but computed
    // here it overlaps the factorisation and solve instead of following them
    // (a cross-lane sum cannot move across the convergence branch by itself)
    const double fold = g8_sum(0.5 * x * hx + q * x);
    const bool c = (x == lb && g > 0.0) || (x == ub && g < 0.0);
    const bool changed = !have || ((__ballot(c != cl) & 0x7Full) != 0);
    cl = c;
    BQ_CNT(6);
    BQ_ACC(0);
    if (changed) {
      const int m = (int)(__ballot(cl) & 0x7Full);
#pragma unroll
      for (int j = 0; j < NU; ++j) {
        const bool cj = (m >> j) & 1;
        Lr[j] = (!cl && !cj) ? hrow[j] + (lane == j ? C.qp_reg : 0.0) : (lane == j ? 1.0 : 0.0);
      }
      if (!chol_rows(Lr, lane)) return false;
      BQ_CNT(7);
      BQ_ACC(1);
      have = true;
      double r = -q;
#pragma unroll
      for (int j = 0; j < NU; ++j)
        if ((m >> j) & 1) r -= hrow[j] * xb[j];
      xsf = chol_solve_rows(Lr, cl ? 0.0 : r, lane);
      clmask = m;
      BQ_ACC(2);
    }
    const double dx = cl ? 0.0 : xsf - x;
    if (all8_below(fabs(dx), C.qp_th_grad)) {
      BQ_ACC(3);
      break;
    }
    BQ_ACC(3);
    bool moved = false;
#pragma unroll 1
    for (int ia = 0; ia < NTRIALS; ++ia) {
      const double al = C.alphas[ia];
      const double xn = fmax(fmin(x + al * dx, ub), lb);
      double hxn = 0.0;
#pragma unroll
      for (int j = 0; j < NU; ++j) hxn += hrow[j] * rowb(xn, j);
      const double fnew = g8_sum(0.5 * xn * hxn + q * xn);
      const double gd = g8_sum(g * (x - xn));
      if (lane0(fold - fnew > C.qp_th_acceptstep * gd)) {
        x = xn;
        moved = true;
        break;
      }
    }
    // No step length accepted: x is unchanged, so every remaining iteration
    // recomputes the same gradient, clamped set and direction and rejects the
    // same trials (BoxQP::solve runs them to maxiter).  Stopping here returns
    // exactly what the remaining iterations would.  On the random-x0 workload
    // ~1 QP in 3700 stalls this way (numpy oracle, tests/golden/
    // make_boxqp_stagnation.py), and its ~90 repeated iterations (10 trials
    // each) set the backward launch's tail.
    BQ_ACC(4);
    if (!moved) break;
    // The next iteration's convergence test without its mat-vec: with no
    // control clamped now and none at a bound after the step, that
    // iteration's clamped set is empty again (no refactor, same xsf) and its
    // step is dx = xsf - x, so when that is below th_grad it stops right
    // there with this x.  (Otherwise it runs as usual.)
    if (!(__ballot(cl || x == lb || x == ub) & 0x7Full) && all8_below(fabs(xsf - x), C.qp_th_grad)) {
      BQ_ACC(5);
      break;
    }
    BQ_ACC(5);
  }
  return true;
}

// LATE: the variant for the latency-bound iterations (few instances left):
// phase C fully unrolled (classical), 1 wave/SIMD register budget.  Both variants are
// launched every iteration; the device-side active count picks the one that
// works (late_max: the most active instances the LATE variant takes, so its
// waves fit one per SIMD), the other one's blocks exit at once.
template <bool FF, bool LATE = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LATE ? 1 : (FF ? 2 : BW_WAVES)))) void k_backward_w(
    const DevConsts* __restrict__ Cg, Dev d, int iter, int cur, int late_max, int w2_max) {
  using S_t = BwW<FF>;
  constexpr int NX = S_t::NX, ND = S_t::ND, REC = S_t::REC, QXU = S_t::QXU, QH = S_t::QH;
  constexpr int NPF = (REC + 63) / 64;  // prefetch registers per lane
  constexpr bool PF_LATE = BW_PF_LATE == 2 || (BW_PF_LATE == 1 && FF);
  const DevConsts& C = *Cg;
  const int N = C.N;
  const int l = threadIdx.x;
  if (blockIdx.x == 0 && l == 0) d.acnt[cur ^ 1] = d.acnt[2 + (cur ^ 1)] = 0;  // the list k_accept builds
  const ActiveList al = active_list(d, cur);
  // active-count ranges: (late_max, B] this variant, (w2_max, late_max] LATE,
  // [1, w2_max] the two-wave k_backward_w2
  if ((int)blockIdx.x >= al.n || (LATE ? (al.n > late_max || al.n <= w2_max) : al.n <= late_max)) return;
  // one instance per block: the index (and every address derived from it) in SGPRs
  const int b = __builtin_amdgcn_readfirstlane(al.list[blockIdx.x]);
  InstState* st = d.st + b;
  if (st->done) return;
  // LATE runs a slice's latency-bound tail: its wave should have its SIMD to
  // itself.  FF's pass fits 254 VGPRs, which would let another slice's
  // k_node wave (253) share the SIMD (FF B = 1024: backward 306 -> 330 us
  // per launch); 40 reserved AGPRs keep the allocation above 256
  if (LATE && FF) RESERVE_AGPR40();
#ifdef FFDDP_PHASE_PROF
  const bool pp_on = (b == 0);
#endif
  PP_INIT();
  __shared__ S_t S;
  const bool feas = st->is_feasible != 0;
  const bool use_qp = C.use_box && feas;
  const double dt = C.dt, dt2 = C.dt * C.dt, alpha = C.alpha, beta = C.beta;
  const double* recb = d.rec_buf + (long)b * (N + 1) * REC;
  // this instance's slices of the state arrays (uniform bases, 32-bit lane
  // offsets in the node loop)
  const double* fs_i = d.fs + (long)b * (N + 1) * NX;
  const double* k_i = d.k + (long)b * N * NU;
  const double* us_i = d.us + (long)b * N * NU;
  double* K_i = d.K + (long)b * N * NU * NX;
  double* kw_i = d.k + (long)b * N * NU;
  double* w_i = d.w + (long)b * (N + 1) * NX;
  if (st->recalc) {
    double c = 0.0;
    for (int t = l; t <= N; t += 64) c += recb[(long)t * REC + rec_off_cost(NX)];
    c = wave_sum(c);
    if (l == 0) {
      st->cost = c;
      st->n_calc += 1;
    }
  }
  double preg = st->preg;
  int retries = 0;
  bool fail_inst = false;
  double dg = 0.0, dq = 0.0, stop = 0.0, ffl = 0.0;
  S.ulb[BW_DIET_SLOTS ? l % NU : l] = C.u_lb[l % NU];
  S.uub[BW_DIET_SLOTS ? l % NU : l] = C.u_ub[l % NU];
  // this lane's lower-triangle entries of Q (phase C) and V (phase F), fixed for the whole pass
  constexpr int NQE = ND * (ND + 1) / 2, NQL = (NQE + 63) / 64;
  // phase C unroll: full in the latency variants (FF's 7 passes move into
  // AGPRs, but since the LDS diet that is 1.4 % faster at B=1024)
  constexpr int QC_N = LATE ? (FF ? (QC_FF_LATE ? QC_FF_LATE : NQL) : NQL) : QC_UNROLL;
  constexpr int NVE = NX * (NX + 1) / 2, NVL = (NVE + 63) / 64;
  unsigned qrc[NQL];
  int vij[NVL];
#pragma unroll
  for (int k = 0; k < NQL; ++k) {
    int r = 0, c = 0;
    tri_rc(spare_entry(l + 64 * k, NQE, 64 * (NQL - 1)), r, c);
    qrc[k] = q_entry<NX>(r, c);
  }
#pragma unroll
  for (int k = 0; k < NVL; ++k) {
    int i = 0, j = 0;
    if (l + 64 * k < NVE) tri_rc(l + 64 * k, i, j);
    vij[k] = (i << 8) | j;
  }
  for (;;) {
    dg = dq = stop = ffl = 0.0;
    bool failed = false;
    // the bases, opaque per pass: the addresses of the terminal node's
    // inputs and of the first prefetch are then formed in each pass instead
    // of being hoisted out of the retry loop and held across it (FF: 15 of
    // them spilled, classical 8 more VGPRs)
    gptr<const double> rbase = (gptr<const double>)recb, fsb = (gptr<const double>)fs_i,
                       kb = (gptr<const double>)k_i, usb = (gptr<const double>)us_i;
    gptr<double> wb = (gptr<double>)w_i;
    asm volatile("" : "+s"(rbase), "+s"(fsb), "+s"(kb), "+s"(usb), "+s"(wb));
    // ---- terminal node: Vxx = Lxx_N + preg I ; Vx = Lx_N (+ Vxx fs_N) ----
    {
      gptr<const double> rT = rbase + (long)N * REC;
      for (int e = l; e < NX * NX; e += 64) {
        const int i = e / NX, j = e % NX;
        S.V[e] = rT[rec_off_Lxx(NX) + e] + (i == j ? preg : 0.0);
      }
      S.fs[BW_DIET_SLOTS ? l % NX : l] = fsb[N * NX + l % NX];
    }
    lds_sync();
    // Prefetch of the next node's inputs: unconditional loads from clamped
    // addresses and unguarded LDS stores, so the code stays straight-line and
    // the compiler can wait on exactly these loads (a guarded store makes it
    // wait vmcnt(0), i.e. also on the previous node's K / k / w stores).
    const int lx = l % NX, lu = l % NU;  // every lane loads and stages slot l mod n
    const int sx = BW_DIET_SLOTS ? lx : l, su = BW_DIET_SLOTS ? lu : l;
    double pf[NPF];
    {
      gptr<const double> r1 = rbase + (long)(N - 1) * REC;
#pragma unroll
      for (int k = 0; k < NPF; ++k) pf[k] = r1[(l + 64 * k < REC) ? l + 64 * k : REC - 1];
    }
    double pfs = fsb[(N - 1) * NX + lx];
    double pkp = kb[(N - 1) * NU + lu];
    double pus = usb[(N - 1) * NU + lu];
    {
      double cdg = 0.0, cdq = 0.0;
      if (l < NX) {
        gptr<const double> rT = rbase + (long)N * REC;
        double vfs = 0.0;
        for (int i = 0; i < NX; ++i) vfs += S.V[i * NX + l] * S.fs[i];
        const double fj = S.fs[l];
        ffl = fabs(fj);
        const double vx = rT[rec_off_Lx(NX) + l] + (feas ? 0.0 : vfs);
        if (!feas) {
          wb[N * NX + l] = vfs;
          cdg = -vx * fj;
          cdq = fj * vfs;
        }
        S.Vx[l] = vx;
      }
      dg += cdg;  // lane-local; summed over the wave after the node loop
      dq += cdq;
    }
    lds_sync();
    if (PF_LATE) {
#pragma unroll
      for (int k = 0; k < NPF; ++k) S.R[l + 64 * k] = pf[k];  // record N-1; the node loop stages the rest
    }
    for (int t = N - 1; t >= 0; --t) {
      // ---- stage record t (prefetched) ; start loading record t-1 ----
      if (!PF_LATE) {
#pragma unroll
        for (int k = 0; k < NPF; ++k) S.R[l + 64 * k] = pf[k];
      }
      S.fs[sx] = pfs;
      S.kp[su] = pkp;
      S.uu[su] = pus;
      {
        const int tn = t > 0 ? t - 1 : 0;
        if (!PF_LATE) {
#pragma unroll
          for (int k = 0; k < NPF; ++k) pf[k] = recb[(unsigned)(tn * REC + ((l + 64 * k < REC) ? l + 64 * k : REC - 1))];
        }
        pfs = fs_i[(unsigned)(tn * NX + lx)];
        pkp = k_i[(unsigned)(tn * NU + lu)];
        pus = us_i[(unsigned)(tn * NU + lu)];
      }
      // no barrier here: phase A reads only V / Vx, and its closing barrier
      // publishes the staged record and gap before phase B reads them
      PP(0);
      const double* Ar = S.R + rec_off_A();
      // ---- phase A: W = V D (NX x 7), Y = D' V D (7 x 7), z = D' Vx ----
#pragma unroll
      for (int k = 0; k < (NX * NU + 63) / 64; ++k) {
        const int e = l + 64 * k;
        if (e < NX * NU) {
          const int i = e / NU, m = e - (e / NU) * NU;
          S.W[e] = dt2 * S.V[i * NX + m] + dt * S.V[i * NX + 7 + m];
        }
      }
      if (l < NU * NU) {
        const int m = l / NU, n = l - (l / NU) * NU;
        const double wq = dt2 * S.V[m * NX + n] + dt * S.V[m * NX + 7 + n];
        const double wv = dt2 * S.V[(7 + m) * NX + n] + dt * S.V[(7 + m) * NX + 7 + n];
        S.sl.Y[l] = dt2 * wq + dt * wv;
      }
      if (l < NU) S.z[l] = dt2 * S.Vx[l] + dt * S.Vx[7 + l];
      lds_sync();
      PP(1);
      // ---- phase B: row c = l of M = I~'W + 1/2 A^'Y ; Qv[c] = [Lx; Lu] + I~'Vx + A^'z ----
      if (l < ND) {
        const int c = l;
        int r0, r1;
        double a0, a1;
        itilde2<FF>(c, dt, alpha, beta, r0, a0, r1, a1);
        const double ac = (FF && c >= 21) ? 0.0 : 1.0;
        const int cc = (FF && c >= 21) ? 0 : c;
        double Acol[NU];
#pragma unroll
        for (int n = 0; n < NU; ++n) Acol[n] = ac * Ar[cc * 7 + n];
#pragma unroll
        for (int m = 0; m < NU; ++m) {
          double h = 0.0;
#pragma unroll
          for (int n = 0; n < NU; ++n) h += Acol[n] * S.sl.Y[n * NU + m];
          S.sl.M[c * NU + m] = (a0 * S.W[r0 * NU + m] + a1 * S.W[r1 * NU + m]) + 0.5 * h;
        }
        double qv = (c < NX) ? S.R[rec_off_Lx(NX) + c] : S.R[rec_off_Lu(NX) + c - NX];
        qv += a0 * S.Vx[r0] + a1 * S.Vx[r1];
#pragma unroll
        for (int m = 0; m < NU; ++m) qv += Acol[m] * S.z[m];
        S.Qv[c] = qv;
      }
      lds_sync();
      PP(2);
      // ---- phase C: Q lower triangle (mirrored), entries fixed per lane ----
#pragma unroll QC_N
      for (int k = 0; k < NQL; ++k) {
        // no range guard: a lane past the last entry recomputes an entry of
        // the same (last) pass (spare_entry), so the passes need no divergent
        // branch and can interleave
        {
          const int r = (qrc[k] >> 27) & 31, c = (qrc[k] >> 22) & 31;
          double lv;
          if (r < NX)
            lv = S.R[rec_off_Lxx(NX) + r * NX + c];
          else if (c < NX)
            lv = S.R[rec_off_Lxu(NX) + c * NU + (r - NX)];
          else
            lv = S.R[rec_off_Luu(NX) + (r - NX) * NU + (c - NX)];
          int rr0, rr1, cr0, cr1;
          double ra0, ra1, ca0, ca1;
          itilde2<FF>(r, dt, alpha, beta, rr0, ra0, rr1, ra1);
          itilde2<FF>(c, dt, alpha, beta, cr0, ca0, cr1, ca1);
          const double g = ra0 * (ca0 * S.V[rr0 * NX + cr0] + ca1 * S.V[rr0 * NX + cr1]) +
                           ra1 * (ca0 * S.V[rr1 * NX + cr0] + ca1 * S.V[rr1 * NX + cr1]);
          const double sr = (FF && r >= 21) ? 0.0 : 1.0, sc = (FF && c >= 21) ? 0.0 : 1.0;
          const int ir = (FF && r >= 21) ? 0 : r, ic = (FF && c >= 21) ? 0 : c;
          double h1 = 0.0, h2 = 0.0;
#pragma unroll
          for (int m = 0; m < NU; ++m) {
            h1 += S.sl.M[r * NU + m] * Ar[ic * 7 + m];
            h2 += S.sl.M[c * NU + m] * Ar[ir * 7 + m];
          }
          double v = lv + g + (sc * h1 + sr * h2);
          if (r == c && r >= NX) v += preg;
          S.QQ[(qrc[k] >> 11) & 2047] = v;
          S.QQ[qrc[k] & 2047] = v;
        }
      }
      lds_sync();
      PP(3);
      // ---- phase D: gains (Eigen::LLT or BoxQP), row / variable i on lane i ----
      int clm = 0;  // the final clamped set (uniform: phase E runs on this wave)
      constexpr bool EREG = e_from_regs(NX);
      double Lr[NU];  // the factor (EREG: read by phase E from these registers)
      {
        double hrow[NU];
#pragma unroll
        for (int j = 0; j < NU; ++j) hrow[j] = (l < NU) ? S.QQ[QH + l * NU + j] : (l == j ? 1.0 : 0.0);
        bool ok;
        if (!use_qp) {
#pragma unroll
          for (int j = 0; j < NU; ++j) Lr[j] = hrow[j];
          ok = chol_rows(Lr, l);
        } else {
          const bool v = l < NU;
          const double q = v ? S.Qv[NX + l] : 0.0;
          const double lb = v ? S.ulb[l % NU] - S.uu[l % NU] : 0.0;
          const double ub = v ? S.uub[l % NU] - S.uu[l % NU] : 0.0;
          double x = v ? S.kp[l % NU] : 0.0;
          ok = boxqp_lanes(C, hrow, q, lb, ub, x, Lr, clm, l);
          if (ok && v) {
            const bool c = (clm >> l) & 1;
            S.kk[l] = -x;
            if (c) S.Qv[NX + l] = 0.0;  // BoxFDDP: clamped Qu entries are zeroed
          }
        }
        if (!ok) {
          failed = true;
          break;
        }
        if (!EREG && l < NU)
#pragma unroll
          for (int j = 0; j < NU; ++j)
            if (j <= l) S.sl.L[tri(l, j)] = Lr[j];
      }
      lds_sync();
      PP(4);
      if (PF_LATE) {  // the next node's record (S.R is dead after phase C)
        const int tn = t > 0 ? t - 1 : 0;
#pragma unroll
        for (int k = 0; k < NPF; ++k) pf[k] = recb[(unsigned)(tn * REC + ((l + 64 * k < REC) ? l + 64 * k : REC - 1))];
      }
      // ---- phase E: K columns (and k for LLT) ----
      if (l < NX || (!use_qp && l == NX)) {
        double col[NU];
        if (l < NX) {
#pragma unroll
          for (int c = 0; c < NU; ++c) col[c] = ((clm >> c) & 1) ? 0.0 : S.QQ[QXU + l * NU + c];
        } else {
#pragma unroll
          for (int c = 0; c < NU; ++c) col[c] = S.Qv[NX + c];
        }
        if (EREG) {
          double Lt[NU * (NU + 1) / 2];
          rows_to_tri(Lr, Lt);
          chol_solve<NU>(Lt, col);
        } else {
          chol_solve<NU>(S.sl.L, col);
        }
        if (l < NX) {
#pragma unroll
          for (int c = 0; c < NU; ++c) {
            S.sl.K[c * NX + l] = col[c];
            K_i[(unsigned)((t * NU + c) * NX + l)] = col[c];
          }
        } else {
#pragma unroll
          for (int c = 0; c < NU; ++c) S.kk[c] = col[c];
        }
      }
      lds_sync();
      PP(5);
      // ---- phase F: Vxx = sym(Qxx - Qxu K) + preg I (lower triangle, mirrored) ----
      int badv = 0;
#pragma unroll 1
      for (int k = 0; k < NVL; ++k) {
        if (l + 64 * k >= NVE) continue;
        const int i = vij[k] >> 8, j = vij[k] & 255;
        double a1 = 0.0, a2 = 0.0;
#pragma unroll
        for (int c = 0; c < NU; ++c) {
          a1 += S.QQ[QXU + i * NU + c] * S.sl.K[c * NX + j];
          a2 += S.QQ[QXU + j * NU + c] * S.sl.K[c * NX + i];
        }
        const double v = S.QQ[i * NX + j] - 0.5 * (a1 + a2) + (i == j ? preg : 0.0);
        S.V[i * NX + j] = v;
        S.V[j * NX + i] = v;
        badv |= bad(fabs(v)) ? 1 : 0;
      }
      lds_sync();
      PP(6);
      // ---- phase G: Vx, gap terms, expected improvement, k ----
      double cdg = 0.0, cdq = 0.0, cst = 0.0;
      if (l < NX) {
        // V fs (the gap term) only while infeasible: a feasible pass never
        // reads it (uniform branch; FF computes it always: the branch costs
        // its throughput pass a 12 B spill)
        double vfs = 0.0;
        if (FF || !feas) {
#pragma unroll
          for (int i = 0; i < NX; ++i) vfs += S.V[i * NX + l] * S.fs[i];
        }
        double vx = S.Qv[l];
#pragma unroll
        for (int c = 0; c < NU; ++c) vx -= S.sl.K[c * NX + l] * S.Qv[NX + c];
        if (!feas) vx += vfs;
        badv |= bad(fabs(vx)) ? 1 : 0;
        ffl = fmax(ffl, fabs(S.fs[l]));
        if (!feas) {
          w_i[(unsigned)(t * NX + l)] = vfs;
          cdg -= vx * S.fs[l];
          cdq += S.fs[l] * vfs;
        }
        if (l < NU) {
          double quk = 0.0;
#pragma unroll
          for (int m = 0; m < NU; ++m) quk += S.QQ[QH + l * NU + m] * S.kk[m];
          const double qu = S.Qv[NX + l], kl = S.kk[l];
          cdg += qu * kl;
          cdq -= kl * quk;
          cst += qu * qu;
          kw_i[(unsigned)(t * NU + l)] = kl;
        }
        S.Vx[l] = vx;  // old Vx is dead after phase B
      }
      badv = __any(badv);
      if (badv) {
        failed = true;
        break;
      }
      dg += cdg;
      dq += cdq;
      stop += cst;
      if (PF_LATE) {
#pragma unroll
        for (int k = 0; k < NPF; ++k) S.R[l + 64 * k] = pf[k];
      }
      lds_sync();
      PP(7);
    }
    // ---- retry bookkeeping (SolverFDDP::solve: increaseRegularization) ----
    if (!failed) {
      // expected-improvement terms: lane-local sums over the nodes, reduced
      // once here instead of three wave reductions per node
      dg = wave_sum(dg);
      dq = wave_sum(dq);
      stop = wave_sum(stop);
      ffl = wave_max(ffl);
      break;
    }
    retries++;
    preg = fmin(preg * C.reg_inc, C.reg_max);
    if (preg == C.reg_max) {
      fail_inst = true;
      break;
    }
    lds_sync();
  }
  PP_FLUSH();
  if (l == 0) {
    st->preg = preg;
    st->n_retries += retries;
    // the trial k_node read in place has been written into (xs, us): no
    // later kernel may take it for the current iterate (k_commit)
    st->accepted = -1;
    if (fail_inst) {
      st->bw_ok = 0;
      st->iter = iter;
      st->done = 1;
      st->ok = 0;
      st->n_backward += retries;
    } else {
      st->dg = dg;
      st->dq = dq;
      st->stop = stop;
      st->ffeas = ffl;
      st->bw_ok = 1;
      st->n_backward += retries + 1;
      st->n_iters += 1;
    }
  }
}

// ---------------------------------------------------------------------------
// k_backward_w2: the backward pass on TWO wavefronts per instance, for slices
// whose active instances fit two waves per SIMD-pair (the latency-bound
// end of a solve and small per-GPU batches).  Same per-entry arithmetic as
// k_backward_w (bit-identical results), spread over 128 lanes:
//   A, B, C, F  the entry-parallel phases on both waves (half the passes),
//   D           gains on wave 0 (rows on lanes 0..6) while wave 1 stages the
//               next node's record into LDS (S.R is dead after phase C) and
//               issues the prefetch of the one after,
//   E, G        wave 0 (one column / state component per lane, as before).
// ---------------------------------------------------------------------------
// WPE: waves per SIMD the register budget allows.  1 (296 registers) for
// small slices, where the pass is the solve's chain; 2 (256, some spilled)
// in the tails of large slices, where a block that needs two whole SIMDs
// waits for the other slices' kernels to drain them: at 2 its waves share a
// SIMD with one of theirs (B = 4096: +2 % over the one-wave LATE variant
// there).  Same arithmetic either way.
template <bool FF, int WPE = 1>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(WPE))) void k_backward_w2(
    const DevConsts* __restrict__ Cg, Dev d, int iter, int cur, int w2_max) {
  using S_t = BwW<FF>;
  constexpr int NX = S_t::NX, ND = S_t::ND, REC = S_t::REC, QXU = S_t::QXU, QH = S_t::QH;
  constexpr int NPF = (REC + 63) / 64;  // prefetch registers per lane of wave 1
  const DevConsts& C = *Cg;
  const int N = C.N;
  const int tid = threadIdx.x;
  const int wv = tid >> 6, l = tid & 63;
  if (blockIdx.x == 0 && tid == 0) d.acnt[cur ^ 1] = d.acnt[2 + (cur ^ 1)] = 0;  // the list k_accept builds
  const ActiveList al = active_list(d, cur);
  if ((int)blockIdx.x >= al.n || al.n > w2_max) return;
  // one instance per block: the index (and every address derived from it) in SGPRs
  const int b = __builtin_amdgcn_readfirstlane(al.list[blockIdx.x]);
  InstState* st = d.st + b;
  if (st->done) return;
#ifdef FFDDP_PHASE_PROF
  const bool pp_on = (b == 0) && tid == 0;
  unsigned long long dwave = 0;
#endif
  PP_INIT();
  __shared__ S_t S;
  const bool feas = st->is_feasible != 0;
  const bool use_qp = C.use_box && feas;
  const double dt = C.dt, dt2 = C.dt * C.dt, alpha = C.alpha, beta = C.beta;
  const double* recb = d.rec_buf + (long)b * (N + 1) * REC;
  // this instance's slices of the state arrays (uniform bases, 32-bit lane
  // offsets in the node loop)
  const double* fs_i = d.fs + (long)b * (N + 1) * NX;
  const double* k_i = d.k + (long)b * N * NU;
  const double* us_i = d.us + (long)b * N * NU;
  double* K_i = d.K + (long)b * N * NU * NX;
  double* kw_i = d.k + (long)b * N * NU;
  double* w_i = d.w + (long)b * (N + 1) * NX;
  if (st->recalc && wv == 0) {
    double c = 0.0;
    for (int t = l; t <= N; t += 64) c += recb[(long)t * REC + rec_off_cost(NX)];
    c = wave_sum(c);
    if (l == 0) {
      st->cost = c;
      st->n_calc += 1;
    }
  }
  double preg = st->preg;
  int retries = 0;
  bool fail_inst = false;
  double dg = 0.0, dq = 0.0, stop = 0.0, ffl = 0.0;
  if (wv == 0) {
    S.ulb[BW_DIET_SLOTS ? l % NU : l] = C.u_lb[l % NU];
    S.uub[BW_DIET_SLOTS ? l % NU : l] = C.u_ub[l % NU];
  }
  // this lane's lower-triangle entries of Q (phase C) and V (phase F) over 128 lanes
  constexpr int NQE = ND * (ND + 1) / 2, NQL = (NQE + 127) / 128;
  constexpr int NVE = NX * (NX + 1) / 2, NVL = (NVE + 127) / 128;
  unsigned qrc[NQL];
  int vij[NVL];
#pragma unroll
  for (int k = 0; k < NQL; ++k) {
    int r = 0, c = 0;
    tri_rc(spare_entry(tid + 128 * k, NQE, 128 * (NQL - 1)), r, c);
    qrc[k] = q_entry<NX>(r, c);
  }
#pragma unroll
  for (int k = 0; k < NVL; ++k) {
    int i = 0, j = 0;
    if (tid + 128 * k < NVE) tri_rc(tid + 128 * k, i, j);
    vij[k] = (i << 8) | j;
  }
  const int lx = l % NX, lu = l % NU;  // every lane loads and stages slot l mod n
  const int sx = BW_DIET_SLOTS ? lx : l, su = BW_DIET_SLOTS ? lu : l;
  for (;;) {
    dg = dq = stop = ffl = 0.0;
    bool failed = false;
    // the bases, opaque per pass (k_backward_w)
    gptr<const double> rbase = (gptr<const double>)recb, fsb = (gptr<const double>)fs_i,
                       kb = (gptr<const double>)k_i, usb = (gptr<const double>)us_i;
    gptr<double> wb = (gptr<double>)w_i;
    asm volatile("" : "+s"(rbase), "+s"(fsb), "+s"(kb), "+s"(usb), "+s"(wb));
    // ---- terminal node: Vxx = Lxx_N + preg I ; Vx = Lx_N (+ Vxx fs_N) ----
    {
      gptr<const double> rT = rbase + (long)N * REC;
      for (int e = tid; e < NX * NX; e += 128) {
        const int i = e / NX, j = e % NX;
        S.V[e] = rT[rec_off_Lxx(NX) + e] + (i == j ? preg : 0.0);
      }
      if (wv == 0) S.fs[sx] = fsb[N * NX + lx];
    }
    // wave 1: record N-1 into LDS now, the prefetch of record N-2 in flight
    double pf[NPF];
    if (wv == 1) {
      gptr<const double> r1 = rbase + (long)(N - 1) * REC;
#pragma unroll
      for (int k = 0; k < NPF; ++k) pf[k] = r1[(l + 64 * k < REC) ? l + 64 * k : REC - 1];
#pragma unroll
      for (int k = 0; k < NPF; ++k) S.R[l + 64 * k] = pf[k];
      gptr<const double> r2 = rbase + (long)(N > 1 ? N - 2 : 0) * REC;
#pragma unroll
      for (int k = 0; k < NPF; ++k) pf[k] = r2[(l + 64 * k < REC) ? l + 64 * k : REC - 1];
    }
    lds_sync();
    double pfs = 0.0, pkp = 0.0, pus = 0.0;
    if (wv == 0) {
      pfs = fsb[(N - 1) * NX + lx];
      pkp = kb[(N - 1) * NU + lu];
      pus = usb[(N - 1) * NU + lu];
      double cdg = 0.0, cdq = 0.0;
      if (l < NX) {
        gptr<const double> rT = rbase + (long)N * REC;
        double vfs = 0.0;
        for (int i = 0; i < NX; ++i) vfs += S.V[i * NX + l] * S.fs[i];
        const double fj = S.fs[l];
        ffl = fabs(fj);
        const double vx = rT[rec_off_Lx(NX) + l] + (feas ? 0.0 : vfs);
        if (!feas) {
          wb[N * NX + l] = vfs;
          cdg = -vx * fj;
          cdq = fj * vfs;
        }
        S.Vx[l] = vx;
      }
      dg += cdg;
      dq += cdq;
    }
    lds_sync();
    // ---- phase G of node tg: Vx, gap terms, expected improvement, k (wave 0) ----
    int badf = 0;  // wave 0's non-finite V entries of phase F, reported with its phase G
    auto phase_g = [&](int tg) {
      double cdg = 0.0, cdq = 0.0, cst = 0.0;
      int badv = badf;
      if (l < NX) {
        double vfs = 0.0;
        const double* fsg = S.fsb[tg & 1];
        if (FF || !feas) {  // the gap term only while infeasible (uniform branch)
#pragma unroll
          for (int i = 0; i < NX; ++i) vfs += S.V[i * NX + l] * fsg[i];
        }
        double vx = S.Qv[l];
#pragma unroll
        for (int c = 0; c < NU; ++c) vx -= S.sl.K[c * NX + l] * S.Qv[NX + c];
        if (!feas) vx += vfs;
        badv |= bad(fabs(vx)) ? 1 : 0;
        ffl = fmax(ffl, fabs(fsg[l]));
        if (!feas) {
          w_i[(unsigned)(tg * NX + l)] = vfs;
          cdg -= vx * fsg[l];
          cdq += fsg[l] * vfs;
        }
        if (l < NU) {
          double quk = 0.0;
#pragma unroll
          for (int m = 0; m < NU; ++m) quk += S.QQ[QH + l * NU + m] * S.kk[m];
          const double qu = S.Qv[NX + l], kl = S.kk[l];
          cdg += qu * kl;
          cdq -= kl * quk;
          cst += qu * qu;
          kw_i[(unsigned)(tg * NU + l)] = kl;
        }
        S.Vx[l] = vx;  // old Vx is dead after phase B
      }
      badv = __any(badv);
      if (l == 0) S.badw[0] = badv;
      // (a failed node aborts the pass, which restarts with dg / dq / stop reset)
      dg += cdg;
      dq += cdq;
      stop += cst;
    };
    for (int t = N - 1; t >= 0; --t) {
      // ---- wave 0: phase G of node t+1 beside this node's phase A (one
      // barrier less per node), then this node's gap / warm start / control
      // (record t is in LDS) ----
      if (wv == 0) {
        // staging first: its wait for the loads prefetched one node ago
        // would otherwise also wait for phase G's global stores (w, k) just
        // issued (vmcnt counts loads and stores in issue order, and the
        // lane-guarded stores leave the compiler only vmcnt(0)); staged
        // here, the stores have a whole node to complete before the next wait
        S.fsb[t & 1][sx] = pfs;
        S.kp[su] = pkp;
        S.uu[su] = pus;
        const int tn = t > 0 ? t - 1 : 0;
        pfs = fs_i[(unsigned)(tn * NX + lx)];
        pkp = k_i[(unsigned)(tn * NU + lu)];
        pus = us_i[(unsigned)(tn * NU + lu)];
        PP(8);  // (profiling build: wave 0's staging apart from its phase G)
        if (t < N - 1) {
          phase_g(t + 1);
          // z below reads Vx entries other lanes of this wave just wrote
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        }
      }
      PP(0);
      const double* Ar = S.R + rec_off_A();
      // ---- phase A: W = V D (NX x 7), Y = D' V D (7 x 7), z = D' Vx ----
      for (int e = tid; e < NX * NU; e += 128) {
        const int i = e / NU, m = e - (e / NU) * NU;
        S.W[e] = dt2 * S.V[i * NX + m] + dt * S.V[i * NX + 7 + m];
      }
      if (tid >= 128 - NU * NU) {
        const int e = tid - (128 - NU * NU);
        const int m = e / NU, n = e - (e / NU) * NU;
        const double wq = dt2 * S.V[m * NX + n] + dt * S.V[m * NX + 7 + n];
        const double wv_ = dt2 * S.V[(7 + m) * NX + n] + dt * S.V[(7 + m) * NX + 7 + n];
        S.sl.Y[e] = dt2 * wq + dt * wv_;
      }
      if (tid < NU) S.z[tid] = dt2 * S.Vx[tid] + dt * S.Vx[7 + tid];
      lds_sync();
      PP(1);
      // node t+1's phase F / G flags: read now, tested after phase B (whose
      // results a failed pass discards), so the LDS round trip is not on the
      // node's chain
      const int badprev = t < N - 1 ? (S.badw[0] | S.badw[1]) : 0;
      // ---- phase B: row c of M = I~'W + 1/2 A^'Y (columns m split over the
      // two waves) ; Qv[c] = [Lx; Lu] + I~'Vx + A^'z (wave 1) ----
      if (l < ND) {
        const int c = l;
        int r0, r1;
        double a0, a1;
        itilde2<FF>(c, dt, alpha, beta, r0, a0, r1, a1);
        const double ac = (FF && c >= 21) ? 0.0 : 1.0;
        const int cc = (FF && c >= 21) ? 0 : c;
        double Acol[NU];
#pragma unroll
        for (int n = 0; n < NU; ++n) Acol[n] = ac * Ar[cc * 7 + n];
        // columns [M0, M1) with compile-time bounds, so their independent
        // 7-term chains interleave (a runtime column range kept each column in
        // a basic block of its own: one LDS round trip and one dependent
        // chain after another)
        auto mcols = [&](auto m0c, auto m1c) {
          constexpr int M0 = decltype(m0c)::value, M1 = decltype(m1c)::value;
          double h[M1 - M0];
#pragma unroll
          for (int m = M0; m < M1; ++m) {
            h[m - M0] = 0.0;
#pragma unroll
            for (int n = 0; n < NU; ++n) h[m - M0] += Acol[n] * S.sl.Y[n * NU + m];
          }
#pragma unroll
          for (int m = M0; m < M1; ++m)
            S.sl.M[c * NU + m] = (a0 * S.W[r0 * NU + m] + a1 * S.W[r1 * NU + m]) + 0.5 * h[m - M0];
        };
        if (wv == 0)
          mcols(std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{});
        else
          mcols(std::integral_constant<int, 4>{}, std::integral_constant<int, NU>{});
        if (wv == 1) {
          double qv = (c < NX) ? S.R[rec_off_Lx(NX) + c] : S.R[rec_off_Lu(NX) + c - NX];
          qv += a0 * S.Vx[r0] + a1 * S.Vx[r1];
#pragma unroll
          for (int m = 0; m < NU; ++m) qv += Acol[m] * S.z[m];
          S.Qv[c] = qv;
        }
      }
      lds_sync();
      if (badprev) {
        failed = true;
        break;
      }
      PP(2);
      // ---- phase C: Q lower triangle (mirrored), entries over 128 lanes ----
#pragma unroll
      for (int k = 0; k < NQL; ++k) {
        // no range guard: a lane past the last entry recomputes an entry of
        // the same (last) pass (spare_entry), so the passes need no divergent
        // branch and can interleave
        {
          const int r = (qrc[k] >> 27) & 31, c = (qrc[k] >> 22) & 31;
          double lv;
          if (r < NX)
            lv = S.R[rec_off_Lxx(NX) + r * NX + c];
          else if (c < NX)
            lv = S.R[rec_off_Lxu(NX) + c * NU + (r - NX)];
          else
            lv = S.R[rec_off_Luu(NX) + (r - NX) * NU + (c - NX)];
          int rr0, rr1, cr0, cr1;
          double ra0, ra1, ca0, ca1;
          itilde2<FF>(r, dt, alpha, beta, rr0, ra0, rr1, ra1);
          itilde2<FF>(c, dt, alpha, beta, cr0, ca0, cr1, ca1);
          const double g = ra0 * (ca0 * S.V[rr0 * NX + cr0] + ca1 * S.V[rr0 * NX + cr1]) +
                           ra1 * (ca0 * S.V[rr1 * NX + cr0] + ca1 * S.V[rr1 * NX + cr1]);
          const double sr = (FF && r >= 21) ? 0.0 : 1.0, sc = (FF && c >= 21) ? 0.0 : 1.0;
          const int ir = (FF && r >= 21) ? 0 : r, ic = (FF && c >= 21) ? 0 : c;
          double h1 = 0.0, h2 = 0.0;
#pragma unroll
          for (int m = 0; m < NU; ++m) {
            h1 += S.sl.M[r * NU + m] * Ar[ic * 7 + m];
            h2 += S.sl.M[c * NU + m] * Ar[ir * 7 + m];
          }
          double v = lv + g + (sc * h1 + sr * h2);
          if (r == c && r >= NX) v += preg;
          S.QQ[(qrc[k] >> 11) & 2047] = v;
          S.QQ[qrc[k] & 2047] = v;
        }
      }
      lds_sync();
      PP(3);
#ifdef FFDDP_PHASE_PROF
      const unsigned long long dwt0 = __builtin_readcyclecounter();
#endif
      // ---- phase D: gains on wave 0 (rows on lanes 0..6); wave 1 stages the
      // next node's record (S.R is not read after phase C) ----
      constexpr bool EREG = e_from_regs(NX);
      double Lr0[NU];  // wave 0's factor (EREG: read by phase E from these registers)
      if (wv == 0) {
        double hrow[NU];
        double (&Lr)[NU] = Lr0;
#pragma unroll
        for (int j = 0; j < NU; ++j) hrow[j] = (l < NU) ? S.QQ[QH + l * NU + j] : (l == j ? 1.0 : 0.0);
        bool ok;
        int clm = 0;
        if (!use_qp) {
#pragma unroll
          for (int j = 0; j < NU; ++j) Lr[j] = hrow[j];
          ok = chol_rows(Lr, l);
        } else {
          const bool v = l < NU;
          const double q = v ? S.Qv[NX + l] : 0.0;
          const double lb = v ? S.ulb[l % NU] - S.uu[l % NU] : 0.0;
          const double ub = v ? S.uub[l % NU] - S.uu[l % NU] : 0.0;
          double x = v ? S.kp[l % NU] : 0.0;
#ifdef FFDDP_PHASE_PROF
          unsigned long long bq[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          ok = boxqp_lanes(C, hrow, q, lb, ub, x, Lr, clm, l, b == 0 ? bq : nullptr);
          if (b == 0 && l == 0)
            for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&g_pp[32 + k_], bq[k_]);
#else
          ok = boxqp_lanes(C, hrow, q, lb, ub, x, Lr, clm, l);
#endif
          if (ok && v) {
            const bool c = (clm >> l) & 1;
            S.kk[l] = -x;
            if (c) S.Qv[NX + l] = 0.0;  // BoxFDDP: clamped Qu entries are zeroed
          }
        }
        if (!EREG && ok && l < NU)
#pragma unroll
          for (int j = 0; j < NU; ++j)
            if (j <= l) S.sl.L[tri(l, j)] = Lr[j];
        // ok, and the final clamped set above it (one LDS word for the tests below)
        if (l == 0) S.flag = ok ? 1 | (clm << 1) : 0;
      } else {
        if (t > 0) {
#pragma unroll
          for (int k = 0; k < NPF; ++k) S.R[l + 64 * k] = pf[k];
          const int tn = t > 1 ? t - 2 : 0;
#pragma unroll
          for (int k = 0; k < NPF; ++k) pf[k] = recb[(unsigned)(tn * REC + ((l + 64 * k < REC) ? l + 64 * k : REC - 1))];
        }
        // Speculative gains on wave 1: the factor of the full set (Quu, or
        // Quu + qp_reg I as BoxQP factors an empty clamped set: the same
        // operations, so the same bits) and phase E's K columns (and the LLT
        // k) from it, while wave 0 runs the gains.  Used when the final
        // clamped set is empty (always for LLT); otherwise phase E runs.
        double hrow[NU], Lr[NU];
#pragma unroll
        for (int j = 0; j < NU; ++j) hrow[j] = (l < NU) ? S.QQ[QH + l * NU + j] : (l == j ? 1.0 : 0.0);
#pragma unroll
        for (int j = 0; j < NU; ++j) Lr[j] = use_qp ? hrow[j] + (l == j ? C.qp_reg : 0.0) : hrow[j];
        const bool ok1 = chol_rows(Lr, l);
        if (ok1) {
          if (l < NU)
#pragma unroll
            for (int j = 0; j < NU; ++j)
              if (j <= l) S.sl.L1[tri(l, j)] = Lr[j];
          // lanes of this wave read the rows the others just wrote: LDS
          // accesses of one wave complete in order; the fence keeps the
          // compiler from moving the reads above the writes
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
          if (l < NX || (!use_qp && l == NX)) {
            double col[NU];
            if (l < NX) {
#pragma unroll
              for (int c = 0; c < NU; ++c) col[c] = S.QQ[QXU + l * NU + c];
            } else {
#pragma unroll
              for (int c = 0; c < NU; ++c) col[c] = S.Qv[NX + c];
            }
            chol_solve<NU>(S.sl.L1, col);
            if (l < NX) {
              double* Kt = K_i + (unsigned)(t * NU * NX);
#pragma unroll
              for (int c = 0; c < NU; ++c) {
                S.sl.K[c * NX + l] = col[c];
                Kt[c * NX + l] = col[c];
              }
            } else {
#pragma unroll
              for (int c = 0; c < NU; ++c) S.kk[c] = col[c];
            }
          }
        }
        if (l == 0) S.spec = ok1 ? 1 : 0;
      }
#ifdef FFDDP_PHASE_PROF
      // development: each wave's own phase-D time (instance 0) into g_pp[28 + wave]
      if (b == 0 && l == 0) dwave += __builtin_readcyclecounter() - dwt0;
#endif
      lds_sync();
      PP(4);
      const int dflag = S.flag;
      if (dflag == 0) {
        failed = true;
        break;
      }
      // wave 1's gains stand unless BoxQP clamped a control
      const bool spec_ok = S.spec != 0 && (dflag >> 1) == 0;
      // ---- phase E: K columns (and k for LLT), wave 0 ----
      if (!spec_ok && wv == 0 && (l < NX || (!use_qp && l == NX))) {
        double col[NU];
        if (l < NX) {
#pragma unroll
          for (int c = 0; c < NU; ++c) col[c] = ((dflag >> (1 + c)) & 1) ? 0.0 : S.QQ[QXU + l * NU + c];
        } else {
#pragma unroll
          for (int c = 0; c < NU; ++c) col[c] = S.Qv[NX + c];
        }
        if (EREG) {
          double Lt[NU * (NU + 1) / 2];
          rows_to_tri(Lr0, Lt);
          chol_solve<NU>(Lt, col);
        } else {
          chol_solve<NU>(S.sl.L, col);
        }
        if (l < NX) {
          double* Kt = K_i + (unsigned)(t * NU * NX);
#pragma unroll
          for (int c = 0; c < NU; ++c) {
            S.sl.K[c * NX + l] = col[c];
            Kt[c * NX + l] = col[c];
          }
        } else {
#pragma unroll
          for (int c = 0; c < NU; ++c) S.kk[c] = col[c];
        }
      }
      if (!spec_ok) lds_sync();  // (uniform: read from LDS)
      PP(5);
      // ---- phase F: Vxx = sym(Qxx - Qxu K) + preg I, entries over 128 lanes ----
      int badv = 0;
#pragma unroll
      for (int k = 0; k < NVL; ++k) {
        if (tid + 128 * k >= NVE) continue;
        const int i = vij[k] >> 8, j = vij[k] & 255;
        double a1 = 0.0, a2 = 0.0;
#pragma unroll
        for (int c = 0; c < NU; ++c) {
          a1 += S.QQ[QXU + i * NU + c] * S.sl.K[c * NX + j];
          a2 += S.QQ[QXU + j * NU + c] * S.sl.K[c * NX + i];
        }
        const double v = S.QQ[i * NX + j] - 0.5 * (a1 + a2) + (i == j ? preg : 0.0);
        S.V[i * NX + j] = v;
        S.V[j * NX + i] = v;
        badv |= bad(fabs(v)) ? 1 : 0;
      }
      if (wv == 1) {
        badv = __any(badv);
        if (l == 0) S.badw[1] = badv;
      } else {
        badf = badv;
      }
      lds_sync();
      PP(6);
    }
    if (!failed) {
      if (wv == 0) phase_g(0);
      lds_sync();
      PP(7);
      if (S.badw[0] | S.badw[1]) failed = true;
    }
    // ---- retry bookkeeping (SolverFDDP::solve: increaseRegularization) ----
    if (!failed) {
      if (wv == 0) {
        dg = wave_sum(dg);
        dq = wave_sum(dq);
        stop = wave_sum(stop);
        ffl = wave_max(ffl);
      }
      break;
    }
    retries++;
    preg = fmin(preg * C.reg_inc, C.reg_max);
    if (preg == C.reg_max) {
      fail_inst = true;
      break;
    }
    lds_sync();
  }
  PP_FLUSH();
#ifdef FFDDP_PHASE_PROF
  if (b == 0 && l == 0) atomicAdd(&g_pp[28 + wv], dwave);
#endif
  if (tid == 0) {
    st->preg = preg;
    st->n_retries += retries;
    st->accepted = -1;
    if (fail_inst) {
      st->bw_ok = 0;
      st->iter = iter;
      st->done = 1;
      st->ok = 0;
      st->n_backward += retries;
    } else {
      st->dg = dg;
      st->dq = dq;
      st->stop = stop;
      st->ffeas = ffl;
      st->bw_ok = 1;
      st->n_backward += retries + 1;
      st->n_iters += 1;
    }
  }
}

// ---------------------------------------------------------------------------
// line search with an 8-lane group per (instance, step length): the rollout
// of one trial is still sequential over the nodes, but each node calc runs
// joint-parallel (node_calc_g8), which shortens the dependent chain that
// bounds this kernel.  Lane i < 7 carries joint i of x (q_i, v_i, FF tau_i).
// ---------------------------------------------------------------------------
// SolverFDDP::solve acceptance of trial tr (tryStep + expectedImprovement)
// for an instance in state s; dV / dVexp / d1 of the trial out (trace)
// the line search's results of instance b, trials 0..n-1, loaded at once
// (n is NTRIALS or the first pass's width): the acceptance loop below exits
// at the first accepted trial, and with the loads inside it every trial
// cost a dependent global-memory round trip
struct TrialRes {
  double cost[NTRIALS], dv[NTRIALS];
  bool fail[NTRIALS];
};
__device__ __forceinline__ void load_trials(const Dev& d, int b, int n, TrialRes& T) {
  const double* tb = d.trial + (long)b * NTRIALS * 2;
  const int* fb = d.trial_fail + (long)b * NTRIALS;
#pragma unroll
  for (int tr = 0; tr < NTRIALS; ++tr) {
    const bool in = tr < n;
    T.cost[tr] = in ? tb[2 * tr] : 0.0;
    T.dv[tr] = in ? tb[2 * tr + 1] : 0.0;
    T.fail[tr] = in ? fb[tr] != 0 : true;
  }
}

__device__ __forceinline__ bool trial_accepted(const DevConsts& C, const InstState& s, const TrialRes& T, int tr,
                                               double* o_dV = nullptr, double* o_dVexp = nullptr,
                                               double* o_d1 = nullptr) {
  if (T.fail[tr]) return false;
  const double a = C.alphas[tr];
  const double cost_try = T.cost[tr];
  const double dv = s.is_feasible ? 0.0 : T.dv[tr];
  const double dV = s.cost - cost_try;
  const double d0 = s.dg + dv, d1 = s.dq - 2.0 * dv;
  const double dVexp = a * (d0 + 0.5 * a * d1);
  if (o_dV) {
    *o_dV = dV;
    *o_dVexp = dVexp;
    *o_d1 = d1;
  }
  if (dVexp >= 0) return fabs(d0) < C.th_grad || dV > C.th_acceptstep * dVexp;
  // ascent direction (closing the gaps may raise the cost): only while
  // infeasible.  Crocoddyl's comparator is dV < th_acceptnegstep dVexp; the
  // alternative accepts a rise of at most th_acceptnegstep x the predicted
  // one (include/ffddp.h FFDDP_NEGSTEP_*)
  if (s.is_feasible) return false;
  return C.neg_rule == FFDDP_NEGSTEP_CROCODDYL ? dV < C.th_acceptnegstep * dVexp
                                               : dV > C.th_acceptnegstep * dVexp;
}

// Width of the line search's first pass, decided on the device: every step
// length at once while the slice's active instances fit the threshold
// wide_max and the previous iteration had an instance that needed more than
// the host's width n1 (then the second pass, a whole extra rollout on the
// iteration's chain, would likely run again), else n1.  The first pass, the
// second pass and k_accept read the same two values.  Which trials run in
// which pass changes no result (each trial is evaluated alone).
__device__ __forceinline__ int first_width(int n1, const Dev& d, int cur, int wide_max) {
  return (d.acnt[cur] <= wide_max && d.acnt[2 + cur] != 0) ? NTRIALS : n1;
}

// one wave per SIMD: the register budget holds the next node's K row,
// prefetched one node ahead (a 2-waves/SIMD variant without the prefetch
// measured slower in every iteration).
// ROW (ffddp_rollout.hpp): one trial group per 16-lane DPP row (latency
// layout) instead of two (throughput layout).  Both instantiations are
// launched for a pass whose layout the host cannot know; each reads the
// slice's active count and returns at once unless it is the chosen one:
// ROW while the pass's trial groups fit row_max (one wave per SIMD share at
// four groups per wave).  The two give the same bits, so the choice never
// makes a result depend on the batch.  The node loop is written with
// explicit fma under fp contract(off) for that reason.
__device__ __forceinline__ int ls_row_bcast0(int v) {  // lane 0 of the row into every lane of it
  return __builtin_amdgcn_update_dpp(v, v, 0x150, 0xf, 0xf, false);
}
#pragma clang fp contract(off)
#ifndef FW_WPE
#define FW_WPE 1  // waves per SIMD of the two-groups-per-row layout's register budget
#endif
template <int NC, bool FF, bool ROW>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ROW ? 1 : FW_WPE))) void k_forward_g8(const DevConsts* __restrict__ Cg, Dev d,
                                                   const double* __restrict__ x0,
                                                   const double* __restrict__ node_ref,
                                                   const double* __restrict__ inst_ref,
                                                   const uint8_t* __restrict__ surface, int tr0, int ntr,
                                                   int only_more, int cur, int wide_max, int row_max) {
  const DevConsts& C = *Cg;
  const int N = C.N;
  constexpr int nx = FF ? 21 : 14;
  constexpr int GL = ROW ? 16 : G8;  // lanes per trial group slot
  // host: first pass (0, n1), second pass (n1, NTRIALS - n1); the device may
  // widen the first pass to all step lengths (first_width)
  {
    const int n1 = first_width(only_more ? tr0 : ntr, d, cur, wide_max);
    tr0 = only_more ? n1 : 0;
    ntr = only_more ? NTRIALS - n1 : n1;
    if (ntr == 0) return;
    // the layout of this pass (same decision in both instantiations)
    if (((long)d.acnt[cur] * ntr <= (long)row_max) != ROW) return;
  }
  const long blk = xcd_block(blockIdx.x, ((long)d.acnt[cur] * ntr * GL + 63) / 64);
  const long gid = (blk * (long)blockDim.x + threadIdx.x) / GL;
  const int li = g8_lane();
  const bool J = li < NQ;
  const int ji = J ? li : 0;
  const bool real = !ROW || (threadIdx.x & 8) == 0;  // ROW: lanes 8..15 of a row are the phantom group
  const bool Js = J && real;                          // stores
  const int slot = (int)(gid / ntr), tr = tr0 + (int)(gid % ntr);
  __shared__ LaneK LKs[ROW ? 16 : G8];
  lane_consts_fill(C, LKs, (int)threadIdx.x);
  if (ROW) lane_consts_fill_phantom(C, LKs, (int)threadIdx.x);
  __syncthreads();
  const LaneK& K = LKs[ROW ? (threadIdx.x & 15) : li];
  const unsigned fl = ls_flags(C);
  const ActiveList al = active_list(d, cur);
  if (slot >= al.n) return;
  const int b = al.list[slot];
  const InstState* st = d.st + b;
  if (st->done) return;
  if (only_more) {
    // second pass of the line search: only instances none of whose first
    // tr0 trials was accepted (the first pass's results are complete: same stream)
    const InstState sv = *st;
    TrialRes T;
    load_trials(d, b, tr0, T);
    bool any = false;
    // constant trip count: T stays in registers (a runtime bound indexes
    // it dynamically, i.e. through scratch memory)
#pragma unroll
    for (int t2 = 0; t2 < NTRIALS; ++t2) any = any || (t2 < tr0 && trial_accepted(C, sv, T, t2));
    if (any) return;
  }
#ifdef FFDDP_PHASE_PROF
  const bool pp_on = (b == 0 && tr == 0);
#endif
  PP_INIT();
  const double alpha = C.alphas[tr];
  const bool feas = st->is_feasible != 0;
  const bool gap = !(feas || alpha == 1.0);
  const bool surf = surface[b] != 0;
  const double* xreg = inst_ref + (long)b * 21;
  const double xq = xreg[ji], xv = xreg[7 + ji], tref = xreg[14 + ji];
  // FF: y reference (= y0) of this lane's joint, loaded once
  double yq = 0.0, yv = 0.0, yt = 0.0;
  if (FF) {
    yq = x0[(long)b * nx + ji];
    yv = x0[(long)b * nx + 7 + ji];
    yt = x0[(long)b * nx + 14 + ji];
  }
  // predicted state (lane-local joint components)
  double hq = J ? x0[(long)b * nx + ji] : 0.0;
  double hv = J ? x0[(long)b * nx + 7 + ji] : 0.0;
  double ht = (FF && J) ? x0[(long)b * nx + 14 + ji] : 0.0;
  double cost = 0.0, dvp = 0.0;
  bool fail = false, fail_l = false;
  double* xtr = d.xs_try + ((long)b * NTRIALS + tr) * (N + 1) * nx;
  double* utr = d.us_try + ((long)b * NTRIALS + tr) * N * NU;
  // node inputs of the rollout, prefetched one node ahead (joint lane ji)
  constexpr int NCX = FF ? 3 : 2;  // state components per joint lane
  double pxs[3] = {0, 0, 0}, pfs[3] = {0, 0, 0}, pw[3] = {0, 0, 0}, pK[21], pus = 0.0, pk = 0.0, pref[6];
  auto fetch = [&](int t) {
    const long nb = (long)b * (N + 1) + t;
#pragma unroll
    for (int c = 0; c < 6; ++c) pref[c] = node_ref[nb * 6 + c];
#pragma unroll
    for (int c = 0; c < NCX; ++c) {
      pxs[c] = J ? d.xs[nb * nx + 7 * c + ji] : 0.0;
      pfs[c] = (J && gap) ? d.fs[nb * nx + 7 * c + ji] : 0.0;
      pw[c] = (J && !feas) ? d.w[nb * nx + 7 * c + ji] : 0.0;
    }
    if (t < N) {
      const long ub = (long)b * N + t;
      pus = J ? d.us[ub * NU + ji] : 0.0;
      pk = J ? d.k[ub * NU + ji] : 0.0;
      const double* K_t = d.K + ub * NU * nx + (long)ji * nx;
#pragma unroll
      for (int m = 0; m < nx; ++m) pK[m] = J ? K_t[m] : 0.0;
    }
  };
  fetch(0);
  for (int t = 0; t <= N; ++t) {
    double xq_t = hq, xv_t = hv, xt_t = ht;
    const double sq = pxs[0], sv = pxs[1], stt = pxs[2];
    if (gap) {
      xq_t = fma(pfs[0], alpha - 1.0, hq);
      xv_t = fma(pfs[1], alpha - 1.0, hv);
      if (FF) xt_t = fma(pfs[2], alpha - 1.0, ht);
    }
    if (!feas) {
      dvp = fma(-pw[0], sq - xq_t, dvp);
      dvp = fma(-pw[1], sv - xv_t, dvp);
      if (FF) dvp = fma(-pw[2], stt - xt_t, dvp);
    }
    if (Js) {
      xtr[(long)t * nx + ji] = xq_t;
      xtr[(long)t * nx + 7 + ji] = xv_t;
      if (FF) xtr[(long)t * nx + 14 + ji] = xt_t;
    }
    double ref[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) ref[c] = pref[c];
    if (t < N) {
      // u_i = us_i - alpha k_i - K_i (x - xs)  (crocoddyl order: x components q, v, tau)
      double u = 0.0;
      {
        double acc = fma(-pk, alpha, pus);
        const double dq = xq_t - sq, dv = xv_t - sv, dtt = xt_t - stt;
#pragma unroll
        for (int m = 0; m < NQ; ++m) {
          const double dqm = ls_get<ROW>(dq, m), dvm = ls_get<ROW>(dv, m);
          acc = fma(-pK[m], dqm, acc);
          acc = fma(-pK[7 + m], dvm, acc);
          if (FF) acc = fma(-pK[14 + m], ls_get<ROW>(dtt, m), acc);
        }
        if (fl & RF_BOX) acc = fmin(fmax(acc, K.ulb), K.uub);
        u = acc;
        if (Js) utr[(long)t * NU + ji] = u;
      }
      fetch(t + 1);
      double qn, vn, cp, lam[3];
      const double uin = FF ? xt_t : u;
      PP(8);
      ls_node_calc<NC, ROW>(C, fl, K, MODE_RUNNING, surf, xq_t, xv_t, uin, xq, xv, tref, ref, qn, vn, cp, lam
#ifdef FFDDP_PHASE_PROF
                            , pp_acc, pp_last
#endif
      );
      double c = C.dt * cp;
      double tn = 0.0;
      if (FF) {
        tn = fma(C.beta, u, C.alpha * xt_t);
        if (J) {
          const double e1 = xq_t - yq, e2 = xv_t - yv, e3 = xt_t - yt;
          c = fma(0.5 * C.w_y, fma(K.wy2t * e3, e3, fma(K.wy2v * e2, e2, (K.wy2q * e1) * e1)), c);
          c = fma(0.5 * C.w_w, u * u, c);
          const double ov = fabs(u) - K.wslim;
          const double oo = ov > 0.0 ? ov : 0.0;
          c = fma(C.w_ws, 0.5 * (oo * oo), c);
        }
      }
      cost += g8_sum(c);
      // a non-finite or huge state or cost fails the trial (forwardPass's
      // raiseIfNaN); the test is lane-local here and reduced once after the
      // last node, so no cross-lane reduction or branch sits on each node's
      // chain.  A failed trial's remaining nodes run on garbage whose results
      // nothing reads (its cost and trajectory are never accepted), and a bad
      // cost stays bad to the end
      fail_l = fail_l || (J && (bad(fabs(qn)) || bad(fabs(vn)) || (FF && bad(fabs(tn)))));
      hq = qn;
      hv = vn;
      ht = tn;
    } else {
      double qn, vn, cp, lam[3];
      const int mode = FF ? MODE_TERMINAL_U : MODE_TERMINAL_X;
      PP(8);
      ls_node_calc<NC, ROW>(C, fl, K, mode, surf, xq_t, xv_t, FF ? xt_t : 0.0, xq, xv, tref, ref, qn, vn, cp, lam
#ifdef FFDDP_PHASE_PROF
                            , pp_acc, pp_last
#endif
      );
      double c = FF ? C.dt * cp : cp;
      if (FF && J) {
        const double e1 = xq_t - yq, e2 = xv_t - yv, e3 = xt_t - yt;
        c = fma(0.5 * C.w_y, fma(K.wy2t * e3, e3, fma(K.wy2v * e2, e2, (K.wy2q * e1) * e1)), c);
      }
      cost += g8_sum(c);
    }
  }
  {
    int f = (bad(cost) || g8_or(fail_l ? 1 : 0)) ? 1 : 0;
    if (ROW) f = ls_row_bcast0(f);  // the phantom group follows the real one
    fail = f != 0;
  }
  PP(9);
  PP_FLUSH_AT(16);
  const double dv = g8_sum(dvp);
  if (li == 0 && real) {
    d.trial[((long)b * NTRIALS + tr) * 2 + 0] = cost;
    d.trial[((long)b * NTRIALS + tr) * 2 + 1] = dv;
    d.trial_fail[(long)b * NTRIALS + tr] = fail ? 1 : 0;
  }
}
#pragma clang fp contract(fast)

// ---------------------------------------------------------------------------
// acceptance / regularisation / stopping: one lane per instance
// ---------------------------------------------------------------------------
// SolverFDDP::solve after the line search for instance b: first accepted step
// length, regularisation update, stopping test.  Returns the accepted trial
// (-1: none, or the instance is done).
__device__ int accept_instance(const DevConsts& C, Dev& d, int b, int iter, int n1) {
  InstState s = d.st[b];
  TrialRes T;  // issued with the state load (unused for a done instance)
  load_trials(d, b, NTRIALS, T);
  if (s.done) {
    d.st[b].accepted = -1;
    return -1;
  }
  s.iter = iter;
  int acc = -1;
  double steplength = C.alphas[NTRIALS - 1];
  int tried = NTRIALS;
  // dV, dVexp, d1 of the accepted (else the last finite) trial, for the trace
  double tdV = __builtin_nan(""), tdVexp = __builtin_nan(""), td1 = __builtin_nan("");
  for (int tr = 0; tr < NTRIALS; ++tr) {
    const double a = C.alphas[tr];
    const double cost_try = T.cost[tr];
    double e0 = tdV, e1 = tdVexp, e2 = td1;
    const bool okt = trial_accepted(C, s, T, tr, &e0, &e1, &e2);
    tdV = e0;
    tdVexp = e1;
    td1 = e2;
    if (!T.fail[tr] && e1 < 0) {
      s.n_neg += 1;
      s.n_neg_acc += okt ? 1 : 0;
    }
    if (okt) {
      acc = tr;
      steplength = a;
      tried = tr + 1;
      s.was_feasible = s.is_feasible;
      s.is_feasible = (s.was_feasible || a == 1.0) ? 1 : 0;
      s.cost = cost_try;
      s.recalc = 1;
      break;
    }
  }
  if (acc < 0) s.recalc = 0;  // (xs, us) unchanged: node data stays valid
  // step lengths the line-search kernels evaluated (first pass: n1; second
  // pass: the rest, only when none of the first n1 was accepted)
  s.n_eval1 += n1;
  const bool second = n1 < NTRIALS && (acc < 0 || acc >= n1);  // the second pass evaluated this instance
  if (second) s.n_eval2 += NTRIALS - n1;
  s.n_trials += tried;
  s.n_forward += second ? 2 : 1;  // line-search launches that processed it
  s.accepted = acc;
  if (steplength > C.th_stepdec) s.preg = fmax(s.preg / C.reg_dec, C.reg_min);
  if (steplength <= C.th_stepinc) {
    s.preg = fmin(s.preg * C.reg_inc, C.reg_max);
    if (s.preg == C.reg_max) {
      s.done = 1;
      s.ok = 0;
    }
  }
  // CallbackVerbose record of this iteration (before the stopping test, as
  // the callbacks run in SolverFDDP::solve; none when preg reached reg_max)
  if (d.trace && iter < d.trace_it && !s.done) {
    double* r = d.trace + ((long)b * d.trace_it + iter) * FFDDP_TRACE_W;
    r[0] = (double)iter;
    r[1] = s.cost;
    r[2] = s.stop;
    r[3] = -td1;
    r[4] = s.preg;
    r[5] = s.preg;
    r[6] = steplength;
    r[7] = s.ffeas;
    r[8] = tdV;
    r[9] = tdVexp;
  }
  if (!s.done && s.was_feasible && s.stop < C.th_stop) {
    s.done = 1;
    s.ok = 1;
  }
  d.st[b] = s;
  return acc;
}

// acceptance / regularisation / stopping, one lane per instance; the
// continuing instances are appended to the next active list with one atomic
// per wave.  The accepted trial is not copied here: the next iteration's
// k_node reads it in place and writes it into (xs, us) node by node, and
// k_commit does it for the instances no further k_node visits.
__global__ __launch_bounds__(64) void k_accept(const DevConsts* __restrict__ Cg, Dev d, int iter, int n1, int cur,
                                               int wide_max) {
  const DevConsts& C = *Cg;
  const ActiveList al = active_list(d, cur);
  const int n1h = n1;
  n1 = first_width(n1, d, cur, wide_max);
  if ((int)blockIdx.x * 64 >= al.n) return;
  const int slot = (int)blockIdx.x * 64 + (int)threadIdx.x;
  const bool has = slot < al.n;
  const int b = has ? al.list[slot] : 0;
  bool cont = false;
  int acc = -1;
  if (has) {
    acc = accept_instance(C, d, b, iter, n1);
    cont = d.st[b].done == 0;
  }
  // a continuing instance needed more step lengths than the host's first pass:
  // the next iteration's first pass may take them all (first_width)
  if (cont && (acc < 0 || acc >= n1h)) d.acnt[2 + (cur ^ 1)] = 1;
  const unsigned long long m = __ballot(cont);
  int base = 0;
  if (threadIdx.x == 0 && m != 0ull) base = atomicAdd(d.acnt + (cur ^ 1), __popcll(m));
  base = __builtin_amdgcn_readfirstlane(base);
  if (cont) d.alist[(long)(cur ^ 1) * d.B + base + __popcll(m & ((1ull << threadIdx.x) - 1ull))] = b;
}

// end of solve: the accepted trial of every instance whose last iteration
// accepted one and that no k_node visited since becomes (xs, us); 16 lanes
// per instance, a chunk's loads all in flight before its stores
constexpr int COMMIT_IPB = 4;
__global__ __launch_bounds__(64) void k_commit(const DevConsts* __restrict__ Cg, Dev d) {
  const DevConsts& C = *Cg;
  const int q = threadIdx.x / 16, l = threadIdx.x % 16;
  const int b = (int)blockIdx.x * COMMIT_IPB + q;
  if (b >= d.B) return;
  const int acc = d.st[b].accepted;
  if (acc < 0) return;
  const int N = C.N, nx = C.nx;
  const long perX = (long)(N + 1) * nx, perU = (long)N * NU;
  const double* sx = d.xs_try + ((long)b * NTRIALS + acc) * perX;
  const double* su = d.us_try + ((long)b * NTRIALS + acc) * perU;
  double* dx = d.xs + (long)b * perX;
  double* du = d.us + (long)b * perU;
  constexpr int CH = 16;
  for (long base = l; base < perX + perU; base += 16 * CH) {
    double v[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const long i = base + 16 * u;
      v[u] = i < perX ? sx[i] : (i < perX + perU ? su[i - perX] : 0.0);
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const long i = base + 16 * u;
      if (i < perX)
        dx[i] = v[u];
      else if (i < perX + perU)
        du[i - perX] = v[u];
    }
  }
}

// solution read-back helpers: iter/ok, contact force at knots 0 and 1
template <int NC, bool FF>
__global__ __launch_bounds__(64) void k_finalize(const DevConsts* __restrict__ Cg, Dev d, int maxiter, const double* __restrict__ x0,
                           const double* __restrict__ node_ref, const double* __restrict__ inst_ref,
                           const uint8_t* __restrict__ surface, double* cost, int32_t* iters, uint8_t* ok,
                           double* fn_pred, int32_t* stats) {
  const DevConsts& C = *Cg;
  const int N = C.N;
  constexpr int nx = FF ? 21 : 14;
  const long gid = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int b = (int)(gid / 2), knot = (int)(gid % 2);
  if (b >= d.B) return;
  const InstState s = d.st[b];
  if (knot == 0) {
    cost[b] = s.cost;
    iters[b] = s.done ? s.iter : maxiter;
    ok[b] = (s.done && s.ok) ? 1 : 0;
    if (stats) {
      stats[(long)b * FFDDP_NSTATS + 0] = s.n_iters;
      stats[(long)b * FFDDP_NSTATS + 1] = s.n_trials;
      stats[(long)b * FFDDP_NSTATS + 2] = s.n_retries;
      stats[(long)b * FFDDP_NSTATS + 3] = s.n_backward;
      stats[(long)b * FFDDP_NSTATS + 4] = s.n_calc;
      stats[(long)b * FFDDP_NSTATS + 5] = s.n_forward;
      stats[(long)b * FFDDP_NSTATS + 6] = s.n_eval1;
      stats[(long)b * FFDDP_NSTATS + 7] = s.n_eval2;
      stats[(long)b * FFDDP_NSTATS + 8] = s.n_neg;
      stats[(long)b * FFDDP_NSTATS + 9] = s.n_neg_acc;
    }
  }
  if (fn_pred == nullptr) return;
  const int t = knot < N ? knot : N - 1;
  if (!surface[b]) {
    fn_pred[(long)b * 2 + knot] = __builtin_nan("");
    return;
  }
  const double* y = d.xs + ((long)b * (N + 1) + t) * nx;
  const double* u = d.us + ((long)b * N + t) * NU;
  const double* ref = node_ref + ((long)b * (N + 1) + t) * 6;
  const double* xreg = inst_ref + (long)b * 21;
  Primal P;
  double yn[21], c;
  node_calc<NC, FF>(C, false, true, y, u, ref, xreg, xreg + 14, x0 + (long)b * nx, P, yn, c);
  fn_pred[(long)b * 2 + knot] = (NC == 1) ? P.lam[0] : P.lam[2];
}

// closed-loop plant stand-in: one thread per instance (ffddp_plant.hpp)
__global__ __launch_bounds__(64) void k_plant(const ffddp_robot* __restrict__ rb, const ffddp_plant_params* __restrict__ pp,
                                              int B, double* __restrict__ q, double* __restrict__ v,
                                              const double* __restrict__ tau, const double* __restrict__ plane,
                                              int integrate, double* __restrict__ obs, int32_t* __restrict__ fail) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double qb[NQ], vb[NQ], tb[NQ], ob[PO_WORDS];
  for (int i = 0; i < NQ; ++i) {
    qb[i] = q[(long)b * NQ + i];
    vb[i] = v[(long)b * NQ + i];
    tb[i] = tau[(long)b * NQ + i];
  }
  const double* pl = plane + (long)b * 6;
  const bool ok = plant_step(*rb, *pp, qb, vb, tb, pl, pl + 3, integrate, ob);
  for (int i = 0; i < NQ; ++i) {
    q[(long)b * NQ + i] = qb[i];
    v[(long)b * NQ + i] = vb[i];
  }
  for (int e = 0; e < PO_WORDS; ++e) obs[(long)b * PO_WORDS + e] = ob[e];
  if (fail) fail[b] = ok ? 0 : 1;
}

__global__ __launch_bounds__(64) void k_gravity(const ffddp_robot* __restrict__ rb, int B, const double* __restrict__ q,
                          double* __restrict__ tau) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  gravity_torque(*rb, q + (long)b * NQ, tau + (long)b * NQ);
}

// ---------------------------------------------------------------------------
// Problem builder (ffddp_build_problem_dev): one thread per (instance, knot).
// make_approach_then_circle (trajectories.py:8-93) + the benchmark hold
// (run_classical.py:256-264), MuJoCo -> Pinocchio (crocoddyl_classical.py:
// 250-258, R_MJ_FROM_PIN = diag(-1,-1,1)), references (:447-466).
// ---------------------------------------------------------------------------
struct TaskTraj {
  double center[3], radius, omega, z_contact, t_approach, t_pre, t_hold;
  double p_start[3], p_pre[3], p_cs[3];
};

__device__ __forceinline__ double smoothstep01(double s) {
  s = fmin(fmax(s, 0.0), 1.0);
  return s * s * (3.0 - 2.0 * s);
}

__device__ __forceinline__ double dsmoothstep01(double s) {
  s = fmin(fmax(s, 0.0), 1.0);
  return 6.0 * s * (1.0 - s);
}

// base(t) -> (p, v, surface) in the MuJoCo world
__device__ bool task_base(const TaskTraj& T, double t, double p[3], double v[3]) {
  const double* p0;
  const double* p1;
  double tau, dur;
  if (T.t_pre > 0.0 && t < T.t_pre) {
    p0 = T.p_start; p1 = T.p_pre; tau = t; dur = T.t_pre;
  } else if (t < T.t_pre + T.t_approach) {
    p0 = T.t_pre > 0.0 ? T.p_pre : T.p_start; p1 = T.p_cs; tau = t - T.t_pre; dur = T.t_approach;
  } else {
    const double th = T.omega * (t - (T.t_pre + T.t_approach));
    double sn, cs;
    sincos(th, &sn, &cs);
    p[0] = T.center[0] + T.radius * cs;
    p[1] = T.center[1] + T.radius * sn;
    p[2] = T.z_contact;
    v[0] = -T.radius * T.omega * sn;
    v[1] = T.radius * T.omega * cs;
    v[2] = 0.0;
    return true;
  }
  const double sl = tau / dur, s = smoothstep01(sl), dsdt = dsmoothstep01(sl) / dur;
  for (int i = 0; i < 3; ++i) {
    p[i] = (1.0 - s) * p0[i] + s * p1[i];
    v[i] = dsdt * (p1[i] - p0[i]);
  }
  return false;
}

__device__ bool task_eval(const TaskTraj& T, double t, double p[3], double v[3]) {
  const bool surf = task_base(T, t, p, v);
  const double tc = T.t_pre + T.t_approach;
  if (surf && t < tc + T.t_hold) {
    double vh[3];
    task_base(T, tc, p, vh);
    v[0] = v[1] = v[2] = 0.0;
  }
  return surf;
}

__global__ __launch_bounds__(64) void k_build(const ffddp_robot* __restrict__ rb, TaskTraj T, ffddp_task task, int B,
                                              int N, int nx, double dt, const double* __restrict__ t0,
                                              const double* __restrict__ x0, double* __restrict__ node_ref,
                                              double* __restrict__ inst_ref, uint8_t* __restrict__ surface) {
  const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long)B * (N + 1)) return;
  const int b = (int)(g / (N + 1)), k = (int)(g - (long)b * (N + 1));
  double p[3], v[3];
  task_eval(T, t0[b] + k * dt, p, v);
  double* o = node_ref + g * 6;
  o[0] = -p[0] - task.p_site_minus_frame[0];
  o[1] = -p[1] - task.p_site_minus_frame[1];
  o[2] = p[2] - task.p_site_minus_frame[2];
  o[3] = -v[0];
  o[4] = -v[1];
  o[5] = v[2];
  if (k != 0) return;
  double pp[3], vv[3];
  surface[b] = task_eval(T, t0[b], pp, vv) ? 1 : 0;
  const double* xb = x0 + (long)b * nx;
  double* ir = inst_ref + (long)b * 21;
  for (int i = 0; i < 7; ++i) {
    ir[i] = task.posture_mode ? task.q_nom[i] : xb[i];
    ir[7 + i] = task.posture_mode ? 0.0 : xb[7 + i];
  }
  if (task.torque_mode == 2) {
    for (int i = 0; i < 7; ++i) ir[14 + i] = 0.0;
  } else {
    gravity_torque(*rb, task.torque_mode == 1 ? task.q_nom : xb, ir + 14);
  }
}

}  // namespace

// ===========================================================================
// host side
// ===========================================================================
// copies of the host entry point, issued per slice by launch_solve_t: inputs
// host -> device before the slice's first kernel, outputs device -> host
// after its last; `done[k]` is recorded on slice k's stream after them
struct HostIO {
  struct In {
    void* dev;
    const void* host;
    size_t per_inst;
  } in[6];
  struct Out {
    void* host;
    const void* dev;
    size_t per_inst;
  } out[5];
  int n_in = 0, n_out = 0;
  hipEvent_t* done = nullptr;
  // filled by launch_solve_t: the slices [b0[k], b0[k] + bk[k])
  int ns = 0;
  int b0[8] = {0}, bk[8] = {0};
  // optional: called before slice k's input copies are enqueued (the host
  // stages that slice's pageable inputs); with it the slices are enqueued
  // one after the other instead of iteration by iteration
  std::function<int(int)> stage;
  // optional: xs / us / K are not copied down by launch_solve_t and done[k]
  // is not recorded there (the caller enqueues both later on ss[k], from the
  // slice's device buffers dxs / dus / dK)
  bool defer_out = false;
  hipStream_t ss[8] = {};
  const double *dxs[8] = {}, *dus[8] = {}, *dK[8] = {};
};

// Host memcpy / zero-fill pool of the host entry point: persistent threads
// (FFDDP_COPY_THREADS, default the CPUs this process may use, at most 16)
// that split a list of jobs into 1 MiB pieces with the calling thread.
struct CopyJob {
  void* dst;
  const void* src;  // nullptr: zero-fill dst (first touch of fresh output pages)
  size_t n;
};
class CopyPool {
 public:
  explicit CopyPool(int nthreads) {
    // no exception may cross the C ABI: with fewer threads than asked (or
    // none) the calling thread does the rest of the copies
    try {
      for (int i = 1; i < nthreads; ++i) th_.emplace_back([this] { worker(); });
    } catch (...) {
    }
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  int threads() const { return (int)th_.size() + 1; }
  void run(const std::vector<CopyJob>& jobs) {
    constexpr size_t kPiece = size_t(1) << 20;
    std::vector<CopyJob> pieces;
    size_t tot = 0;
    for (const CopyJob& j : jobs) {
      for (size_t o = 0; o < j.n; o += kPiece)
        pieces.push_back(CopyJob{(char*)j.dst + o, j.src ? (const char*)j.src + o : nullptr, std::min(kPiece, j.n - o)});
      tot += j.n;
    }
    if (pieces.empty()) return;
    if (th_.empty() || tot < 4 * kPiece) {  // small: the calling thread alone
      for (const CopyJob& c : pieces) exec(c);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      work_ = &pieces;
      next_.store(0);
      left_ = pieces.size();
      ++gen_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return left_ == 0; });
    work_ = nullptr;
  }

 private:
  static void exec(const CopyJob& c) {
    if (c.src)
      std::memcpy(c.dst, c.src, c.n);
    else
      std::memset(c.dst, 0, c.n);
  }
  void drain() {
    size_t did = 0;
    const std::vector<CopyJob>* w = work_;
    for (size_t i = next_++; i < w->size(); i = next_++) {
      exec((*w)[i]);
      ++did;
    }
    if (did) {
      std::lock_guard<std::mutex> lk(mu_);
      left_ -= did;
      if (left_ == 0) done_cv_.notify_all();
    }
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || (gen_ != seen && work_ != nullptr); });
        if (stop_) return;
        seen = gen_;
      }
      drain();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::vector<CopyJob>* work_ = nullptr;
  std::atomic<size_t> next_{0};
  size_t left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct ffddp_handle {
  int device = 0;
  int max_batch = 0;
  DevConsts hc{};
  DevConsts* dc = nullptr;
  ffddp_robot* drb = nullptr;
  Dev d{};
  // staging for host-pointer API
  double *in_x0 = nullptr, *in_nref = nullptr, *in_iref = nullptr, *in_xs = nullptr, *in_us = nullptr;
  uint8_t* in_surf = nullptr;
  double *out_xs = nullptr, *out_us = nullptr, *out_K = nullptr, *out_cost = nullptr, *out_fn = nullptr;
  int32_t *out_iters = nullptr, *out_stats = nullptr;
  uint8_t* out_ok = nullptr;
  std::string err;
  // host entry point: page-locked staging (inputs + outputs, max_batch)
  // and the per-slice completion events
  char* stage = nullptr;
  size_t stage_bytes = 0;
  std::vector<hipEvent_t> hdone;
  CopyPool* pool = nullptr;  // host copies of the host entry point (first host solve)
  // per-iteration trace (ffddp_trace_enable)
  double* trace = nullptr;
  int trace_it = 0;
  // live solve plans (their graphs captured this handle's workspace and
  // trace pointer): ffddp_trace_enable refuses while any is alive and
  // ffddp_destroy invalidates them; last_done marks the end of the last
  // solve_batch[_dev] call, which ffddp_plan_run waits for on the device
  std::vector<ffddp_plan*> plans;
  hipEvent_t last_done = nullptr;
  bool last_done_set = false;
  // sub-batch streams: the batch is split into nstreams slices solved on their
  // own HIP streams, so latency-bound phases of one slice overlap with the
  // throughput-bound phases of another (FFDDP_STREAMS, default 4: three
  // created streams plus the caller's stream, the 4 hardware queues a process
  // gets; FFDDP_CALLER_SLICE=0 puts every slice on a created stream)
  int nstreams = 4;
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> sev;  // fork + per-stream join events
  std::vector<hipEvent_t> stg;  // start-stagger events (FFDDP_STAGGER)
  bool caller_slice = true;  // FFDDP_CALLER_SLICE
  // FFDDP_STAGGER: 0 off, 1 slice k's first node stage after slice k-1's,
  // 2 after its init; -1 (default) picks per solve: 1 when the slices exceed
  // one wave per SIMD share (throughput-bound first iterations: B=4096
  // +2.3 %, B=2048 +4 % over 2), else 0 (latency-bound: the stagger only
  // delays the last slice, B=512/1024 +1.2 % over 1)
  int stagger = -1;
  int fw_first = 4;  // trials evaluated before the fallback pass (FFDDP_FW_FIRST)
  // first-pass trial counts of the first iterations (FFDDP_FW_SCHED="2,2,2,2"):
  // while every instance is active the line search is throughput-bound, so a
  // 2-trial first pass (alpha 1, 1/2 cover ~90 % of the instances) halves its
  // work and the second pass, needed there anyway, covers the rest; once most
  // instances are done the pass is latency-bound and 4 trials in one pass win
  std::vector<int> fw_sched{2, 2, 2, 2};
  int bw_late_max = -1;  // active instances up to which a slice's backward pass uses the latency variant
                         // (FFDDP_BW_LATE_MAX; -1: SIMDs / slices)
  int bw_w2_max = -1;    // ... and the two-wave variant (FFDDP_BW_W2_MAX; -1: SIMDs / (2 slices); 0: never)
  int n_simd = 1024;     // SIMDs of the device (4 per CU)
  bool fw_fill = true;   // widen the first line-search pass to fill the SIMDs (FFDDP_FW_FILL=0: off)
  // horizon from which an 8-wide first pass takes all ten (FFDDP_FW_LONG;
  // 0: never, the default since round 5: C5 tracking 64.0k-64.8k -> 65.7k-66.1k,
  // random x0 29.3k -> 28.9k; round 3 measured +4.5 % for it)
  int fw_long = 0;
  int fw_wide_max = -1;  // active instances per slice up to which the first pass takes every step length
                         // (decided on the device; FFDDP_FW_WIDE_MAX; -1: SIMDs / slices; 0: never)
  int ls_row_max = -1;   // trial groups of a line-search pass up to which it runs one group per DPP row
                         // (decided on the device; FFDDP_LS_ROW_MAX; -1: 4 SIMDs / slices, one wave
                         // per SIMD share; 0: never)
  // optional per-kernel timing
  bool prof = false;
  int prof_mask = 0;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<int> ev_class;  // class per event pair
  double prof_ms[FFDDP_NKERNELS] = {0};
  int64_t prof_n[FFDDP_NKERNELS] = {0};
};

namespace {

bool stream_pool_acquire(int device, int n, std::vector<hipStream_t>& out);
void stream_pool_release(int device, int n);


int fail(ffddp_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  return code;
}

#define HIPCHK(h, expr)                                                                    \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(h, FFDDP_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));  \
  } while (0)

template <class T> int dalloc(ffddp_handle* h, T** p, size_t n) {
  if (hipMalloc((void**)p, n * sizeof(T) + 64) != hipSuccess) {
    *p = nullptr;
    return fail(h, FFDDP_E_OOM, "hipMalloc failed");
  }
  return 0;
}

void free_all(ffddp_handle* h) {
  void* ps[] = {h->dc, h->drb, h->d.alist, h->d.acnt, h->d.rec_buf, h->d.fs, h->d.xs, h->d.us, h->d.K, h->d.k, h->d.w, h->d.xs_try,
                h->d.us_try, h->d.trial, h->d.trial_fail, h->d.st, h->in_x0, h->in_nref, h->in_iref, h->in_xs,
                h->in_us, h->in_surf, h->out_xs, h->out_us, h->out_K, h->out_cost, h->out_fn, h->out_iters,
                h->out_stats, h->out_ok};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (h->trace) (void)hipFree(h->trace);
  if (h->stage) (void)hipHostFree(h->stage);
}

// event pair around a launch (only when profiling is enabled)
struct ProfScope {
  ffddp_handle* h;
  hipStream_t s;
  bool on;
  ProfScope(ffddp_handle* h_, hipStream_t s_, int cls) : h(h_), s(s_), on(h_->prof && ((h_->prof_mask >> cls) & 1)) {
    if (!on) return;
    if (h->ev_used + 2 > h->ev_pool.size()) {
      for (int i = 0; i < 256; ++i) {
        hipEvent_t e;
        (void)hipEventCreate(&e);
        h->ev_pool.push_back(e);
      }
    }
    h->ev_class.push_back(cls);
    (void)hipEventRecord(h->ev_pool[h->ev_used], s);
  }
  ~ProfScope() {
    if (!on) return;
    (void)hipEventRecord(h->ev_pool[h->ev_used + 1], s);
    h->ev_used += 2;
  }
};

// profiling classes: one kernel per class (KC_COMMIT: the end-of-solve k_commit)
enum { KC_INIT = 0, KC_NODE, KC_BACKWARD, KC_FORWARD, KC_ACCEPT, KC_COMMIT, KC_FINALIZE, KC_FORWARD2 };

// the per-instance slice [b0, b0 + Bk) of the handle workspace
Dev dev_slice(const Dev& d0, int b0, int Bk, int k) {
  Dev d = d0;
  const long N = d0.N, nx = d0.nx;
  d.B = Bk;
  d.rec_buf += (long)b0 * (N + 1) * d0.rec;
  d.fs += (long)b0 * (N + 1) * nx;
  d.xs += (long)b0 * (N + 1) * nx;
  d.us += (long)b0 * N * NU;
  d.K += (long)b0 * N * NU * nx;
  d.k += (long)b0 * N * NU;
  d.w += (long)b0 * (N + 1) * nx;
  d.xs_try += (long)b0 * NTRIALS * (N + 1) * nx;
  d.us_try += (long)b0 * NTRIALS * N * NU;
  d.trial += (long)b0 * NTRIALS * 2;
  d.trial_fail += (long)b0 * NTRIALS;
  d.st += b0;
  d.alist += 2L * b0;
  d.acnt += 4 * k;
  if (d.trace) d.trace += (long)b0 * d0.trace_it * FFDDP_TRACE_W;
  return d;
}

template <int NC, bool FF>
int launch_solve_t(ffddp_handle* h, int B, const double* x0, const double* nref, const double* iref,
                 const uint8_t* surf, const double* xs_init, const double* us_init, int maxiter, int is_feasible,
                 double* xs, double* us, double* K, double* cost, int32_t* iters, uint8_t* ok, double* fn_pred,
                 int32_t* stats, hipStream_t s, HostIO* io) {
  const int N = h->hc.N, nx = h->hc.nx;
  int S = h->nstreams;
  if (B < 64 * S) S = 1;
  if (S > 1) {
    // the streams normally come with the handle (ffddp_create); the fork /
    // join and stagger events on first use
    if ((int)h->streams.size() < S && !stream_pool_acquire(h->device, S, h->streams))
      return fail(h, FFDDP_E_DEVICE, "hipStreamCreate failed");
    while ((int)h->sev.size() < S + 1) {
      hipEvent_t e;
      HIPCHK(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      h->sev.push_back(e);
    }
    while ((int)h->stg.size() < S) {
      hipEvent_t e;
      HIPCHK(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      h->stg.push_back(e);
    }
  }
  const int Bs = (B + S - 1) / S;
  const int stagger = S == 1 ? 0 : (h->stagger >= 0 ? h->stagger : (Bs > h->n_simd / S ? 1 : 0));
  struct Slice {
    Dev d;
    hipStream_t s;
    int b0, B;
  };
  Slice sl[8];
  // device entry point: the solve iterates in the caller's xs / us / K
  // (same [B][N+1][nx] / [B][N][7] / [B][N][7][nx] layout as the handle's
  // buffers), so no copy of the solution follows the last kernel; the host
  // entry point keeps the handle's buffers (its outputs are host memory)
  Dev dbase = h->d;
  if (!io) {
    dbase.xs = xs;
    dbase.us = us;
    dbase.K = K;
  }
  for (int k = 0; k < S; ++k) {
    sl[k].b0 = k * Bs;
    sl[k].B = (B - sl[k].b0) < Bs ? (B - sl[k].b0) : Bs;
    sl[k].d = dev_slice(dbase, sl[k].b0, sl[k].B, k);
    // FFDDP_CALLER_SLICE: the last slice runs on the caller's stream (its
    // hardware queue is otherwise idle during the solve)
    sl[k].s = (S > 1 && !(h->caller_slice && k == S - 1)) ? h->streams[k] : s;
  }
  if (S > 1) {
    HIPCHK(h, hipEventRecord(h->sev[0], s));
    for (int k = 0; k < S; ++k)
      if (sl[k].s != s) HIPCHK(h, hipStreamWaitEvent(sl[k].s, h->sev[0], 0));
  }
  const long nxl = nx, N1 = N + 1;
  if (io) {
    io->ns = S;
    for (int k = 0; k < S; ++k) {
      io->b0[k] = sl[k].b0;
      io->bk[k] = sl[k].B;
    }
  }
  // host entry point: slice k's inputs go up on its own stream, so its
  // copies overlap the other slices' kernels
  auto enqueue_in = [&](int k) -> int {
    for (int i = 0; i < io->n_in; ++i) {
      const size_t o = (size_t)sl[k].b0 * io->in[i].per_inst;
      HIPCHK(h, hipMemcpyAsync((char*)io->in[i].dev + o, (const char*)io->in[i].host + o,
                               (size_t)sl[k].B * io->in[i].per_inst, hipMemcpyHostToDevice, sl[k].s));
    }
    return 0;
  };
  auto enqueue_init = [&](int k) {
    ProfScope p(h, sl[k].s, KC_INIT);
    const long b0 = sl[k].b0;
    hipLaunchKernelGGL(k_init, dim3(1024), dim3(256), 0, sl[k].s, h->dc, sl[k].d, xs_init + b0 * N1 * nxl,
                       us_init + b0 * (long)N * NU, is_feasible);
  };
  // one FDDP iteration of slice k: node stage, backward pass, line search, step decision
  auto enqueue_iter = [&](int k, int it) -> int {
    const Dev& d = sl[k].d;
    const hipStream_t ss = sl[k].s;
    const int Bk = sl[k].B;
    const long b0 = sl[k].b0;
    const double* x0k = x0 + b0 * nxl;
    const double* nrefk = nref + b0 * N1 * 6;
    const double* irefk = iref + b0 * 21;
    const uint8_t* surfk = surf + b0;
    const long nodes = (long)Bk * (N + 1);
    // optional start stagger: slice k's first node stage waits for slice
    // k-1's, so the throughput-bound node stages do not all collide
    if (it == 0 && k > 0 && stagger) HIPCHK(h, hipStreamWaitEvent(ss, h->stg[k - 1], 0));
    if (it == 0 && stagger == 2 && k + 1 < S) HIPCHK(h, hipEventRecord(h->stg[k], ss));
    {
      ProfScope p(h, ss, KC_NODE);
      hipLaunchKernelGGL((k_node<NC, FF>), dim3((int)((nodes + NODE_GPB - 1) / NODE_GPB)), dim3(NODE_BLOCK), 0, ss,
                         h->dc, d, x0k, nrefk, irefk, surfk, 0, it & 1);
    }
    if (it == 0 && stagger == 1 && k + 1 < S) HIPCHK(h, hipEventRecord(h->stg[k], ss));
    {
      ProfScope p(h, ss, KC_BACKWARD);
      const int lmax = h->bw_late_max >= 0 ? h->bw_late_max : h->n_simd / S;
      // two-wave variant: for slices no larger than one wave per SIMD share
      // (small per-GPU batches, where the whole solve is latency-bound) at
      // one wave per SIMD; in the tails of large slices (active count up to
      // lmax) at two waves per SIMD, so its blocks need not wait for the
      // other slices' kernels to free whole SIMDs (the one-wave kernel there:
      // B = 4096 -1.7 %; this one +2 % over LATE).  FF's
      // two-wave pass spills too much at two waves per SIMD: LATE there.
      const bool small = Bk <= h->n_simd / S;
      const int w2auto = small ? h->n_simd / (2 * S) : (FF ? 0 : lmax);
      const int w2max = std::min(lmax, h->bw_w2_max >= 0 ? h->bw_w2_max : w2auto);
      if (lmax < Bk)
        hipLaunchKernelGGL((k_backward_w<FF>), dim3(Bk), dim3(64), 0, ss, h->dc, d, it, it & 1, lmax, w2max);
      if (lmax > w2max && w2max < Bk)
        hipLaunchKernelGGL((k_backward_w<FF, true>), dim3(lmax < Bk ? lmax : Bk), dim3(64), 0, ss, h->dc, d, it, it & 1,
                           lmax, w2max);
      if (w2max > 0) {
        const dim3 g2(w2max < Bk ? w2max : Bk);
        if constexpr (!FF) {
          if (!small) {
            hipLaunchKernelGGL((k_backward_w2<FF, 2>), g2, dim3(128), 0, ss, h->dc, d, it, it & 1, w2max);
          } else {
            hipLaunchKernelGGL((k_backward_w2<FF, 1>), g2, dim3(128), 0, ss, h->dc, d, it, it & 1, w2max);
          }
        } else {
          hipLaunchKernelGGL((k_backward_w2<FF, 1>), g2, dim3(128), 0, ss, h->dc, d, it, it & 1, w2max);
        }
      }
    }
    int n1 = NTRIALS;
    {
      // first pass: trials 0..n1-1, per-iteration schedule (fw_sched) then
      // fw_first; the second pass evaluates the rest for the instances that
      // accepted none of them
      n1 = it < (int)h->fw_sched.size() ? h->fw_sched[it] : h->fw_first;
      // a small batch leaves SIMDs idle: evaluate as many step lengths in
      // the first pass as one wave per SIMD holds (8 groups per wave), so
      // the second pass (a whole extra rollout on the chain) is rarely needed
      if (h->fw_fill) n1 = std::max(n1, std::min(NTRIALS, 8 * h->n_simd / std::max(B, 1)));
      // long horizons (FFDDP_FW_LONG, off by default): a second pass is a
      // rollout ~N node-calcs long, so once the first pass is 8 wide it
      // could take all ten (N=100 point3d, B=1024: +4.5 % in round 3; on
      // the round-5 kernels -2.3 % in the tracking regime, +1.4 % random)
      if (h->fw_fill && h->fw_long > 0 && N >= h->fw_long && n1 >= 8) n1 = NTRIALS;
      // device-side widening of the first pass: while a slice's active
      // instances fit one wave per SIMD share at every step length, all ten
      // run at once (random x0 at B=1024: the second pass ran in every
      // iteration)
      const int wide = h->fw_wide_max >= 0 ? h->fw_wide_max : h->n_simd / S;
      const long g1 = std::max((long)Bk * n1, (long)std::min(Bk, wide) * NTRIALS);  // first-pass groups
      // layout of each pass (ffddp_rollout.hpp): one trial group per DPP
      // row while the pass's groups fit row_max, two otherwise, decided on
      // the device from the active count.  Only slices that fit one wave
      // per SIMD share take the row layout at all: a large slice's late
      // passes would gain it, but launching both layouts every pass (the
      // unchosen one exits at once) cost more than that at B = 4096
      // (507.9k vs 512.4k solves/s).  When every possible
      // pass of the slice fits, only the row layout is launched.
      const int row_max = (h->ls_row_max >= 0 ? h->ls_row_max : 4 * h->n_simd / S) *
                          (h->ls_row_max < 0 && Bk > h->n_simd / S ? 0 : 1);
      const bool row_only = row_max > 0 && (long)Bk * NTRIALS <= (long)row_max;
      auto fw = [&](int tr0, int ntr, int more) {
        const long groups = more ? (long)Bk * ntr : g1;
        if (!row_only) {
          const dim3 grid((unsigned)((groups * G8 + 63) / 64));
          hipLaunchKernelGGL((k_forward_g8<NC, FF, false>), grid, dim3(64), 0, ss, h->dc, d, x0k, nrefk, irefk,
                             surfk, tr0, ntr, more, it & 1, wide, row_max);
        }
        if (row_max > 0) {
          const long rg = std::min(groups, (long)row_max);  // the row layout runs only when they fit
          const dim3 grid((unsigned)((rg * 16 + 63) / 64));
          hipLaunchKernelGGL((k_forward_g8<NC, FF, true>), grid, dim3(64), 0, ss, h->dc, d, x0k, nrefk, irefk,
                             surfk, tr0, ntr, more, it & 1, wide, row_max);
        }
      };
      {
        ProfScope p(h, ss, KC_FORWARD);
        fw(0, n1, 0);
      }
      if (n1 < NTRIALS) {
        ProfScope p(h, ss, KC_FORWARD2);
        fw(n1, NTRIALS - n1, 1);
      }
    }
    {
      ProfScope p(h, ss, KC_ACCEPT);
      hipLaunchKernelGGL(k_accept, dim3((Bk + 63) / 64), dim3(64), 0, ss, h->dc, d, it, n1, it & 1,
                         h->fw_wide_max >= 0 ? h->fw_wide_max : h->n_simd / S);
    }
    return 0;
  };
  const size_t bxs = (size_t)(N + 1) * nx * sizeof(double);
  const size_t bus = (size_t)N * NU * sizeof(double);
  const size_t bks = (size_t)N * NU * nx * sizeof(double);
  // the end of slice k's solve: accepted trials committed, results, and
  // (host entry point) its outputs down and its completion event
  auto enqueue_tail = [&](int k) -> int {
    const Dev& d = sl[k].d;
    const hipStream_t ss = sl[k].s;
    const long b0 = sl[k].b0;
    const int Bk = sl[k].B;
    {
      ProfScope p(h, ss, KC_COMMIT);
      hipLaunchKernelGGL(k_commit, dim3((Bk + COMMIT_IPB - 1) / COMMIT_IPB), dim3(64), 0, ss, h->dc, d);
    }
    {
      ProfScope p(h, ss, KC_FINALIZE);
      hipLaunchKernelGGL((k_finalize<NC, FF>), dim3((2 * Bk + 63) / 64), dim3(64), 0, ss, h->dc, d, maxiter,
                         x0 + b0 * nxl, nref + b0 * N1 * 6, iref + b0 * 21, surf + b0, cost + b0, iters + b0, ok + b0,
                         fn_pred ? fn_pred + 2 * b0 : nullptr, stats ? stats + b0 * FFDDP_NSTATS : nullptr);
    }
    // host entry point: page-locked host memory, the slice's results go
    // down as soon as it finishes (the device entry point solved in place)
    if (io) {
      io->ss[k] = ss;
      io->dxs[k] = d.xs;
      io->dus[k] = d.us;
      io->dK[k] = d.K;
      if (!io->defer_out) {
        HIPCHK(h, hipMemcpyAsync(xs + b0 * N1 * nxl, d.xs, bxs * Bk, hipMemcpyDefault, ss));
        HIPCHK(h, hipMemcpyAsync(us + b0 * (long)N * NU, d.us, bus * Bk, hipMemcpyDefault, ss));
        HIPCHK(h, hipMemcpyAsync(K + b0 * (long)N * NU * nx, d.K, bks * Bk, hipMemcpyDefault, ss));
      }
      for (int i = 0; i < io->n_out; ++i) {
        const size_t o = (size_t)b0 * io->out[i].per_inst;
        HIPCHK(h, hipMemcpyAsync((char*)io->out[i].host + o, (const char*)io->out[i].dev + o,
                                 (size_t)Bk * io->out[i].per_inst, hipMemcpyDeviceToHost, ss));
      }
      if (!io->defer_out) HIPCHK(h, hipEventRecord(io->done[k], ss));
    }
    return 0;
  };
  if (io && io->stage) {
    // host entry point with pageable inputs: slice by slice, the host stages
    // slice k's inputs into page-locked memory and enqueues its whole solve
    // before staging slice k+1, so the staging of the later slices overlaps
    // the earlier slices' copies and kernels
    for (int k = 0; k < S; ++k) {
      if (const int rc = io->stage(k)) return rc;
      if (const int rc = enqueue_in(k)) return rc;
      enqueue_init(k);
      for (int it = 0; it < maxiter; ++it)
        if (const int rc = enqueue_iter(k, it)) return rc;
      if (const int rc = enqueue_tail(k)) return rc;
    }
  } else {
    // iteration-major across the slices (the device entry point and solve
    // plans; the host entry point with page-locked inputs)
    if (io)
      for (int k = 0; k < S; ++k)
        if (const int rc = enqueue_in(k)) return rc;
    for (int k = 0; k < S; ++k) enqueue_init(k);
    for (int it = 0; it < maxiter; ++it)
      for (int k = 0; k < S; ++k)
        if (const int rc = enqueue_iter(k, it)) return rc;
    for (int k = 0; k < S; ++k)
      if (const int rc = enqueue_tail(k)) return rc;
  }
  if (hipGetLastError() != hipSuccess) return fail(h, FFDDP_E_DEVICE, "kernel launch failed");
  if (S > 1) {
    for (int k = 0; k < S; ++k) {
      if (sl[k].s == s) continue;
      HIPCHK(h, hipEventRecord(h->sev[1 + k], sl[k].s));
      HIPCHK(h, hipStreamWaitEvent(s, h->sev[1 + k], 0));
    }
  }
  return 0;
}

int launch_solve(ffddp_handle* h, int B, const double* x0, const double* nref, const double* iref,
                 const uint8_t* surf, const double* xs_init, const double* us_init, int maxiter, int is_feasible,
                 double* xs, double* us, double* K, double* cost, int32_t* iters, uint8_t* ok, double* fn_pred,
                 int32_t* stats, hipStream_t s, HostIO* io = nullptr) {
  const bool ff = h->hc.variant == FFDDP_FORCE_FEEDBACK;
  const int nc = h->hc.nc;
#define FFDDP_LS(NC_, FF_) \
  launch_solve_t<NC_, FF_>(h, B, x0, nref, iref, surf, xs_init, us_init, maxiter, is_feasible, xs, us, K, cost, iters, ok, fn_pred, stats, s, io)
  if (nc == 1) return ff ? FFDDP_LS(1, true) : FFDDP_LS(1, false);
  return ff ? FFDDP_LS(3, true) : FFDDP_LS(3, false);
#undef FFDDP_LS
}

template <int NC, bool FF>
void launch_node(ffddp_handle* h, Dev d, int B, hipStream_t s, int force_all) {
  const long nodes = (long)B * (h->hc.N + 1);
  hipLaunchKernelGGL((k_node<NC, FF>), dim3((int)((nodes + NODE_GPB - 1) / NODE_GPB)), dim3(NODE_BLOCK), 0, s, h->dc,
                     d, h->in_x0, h->in_nref, h->in_iref, h->in_surf, force_all, 0);
}

// Slice streams shared by every handle of the process on a device: a
// process gets 4 hardware queues (GPU_MAX_HW_QUEUES), and every stream
// beyond them shares a queue with another, serialising two slices (a second
// handle's own 3 streams took a B = 4096 host-entry solve from 11.4 to
// 15.4 ms).  Handles are not thread-safe anyway; two handles used from one
// thread just queue their slices on the same streams.  Ref-counted: the last
// release destroys them.
struct StreamPool {
  std::vector<hipStream_t> s;
  int refs = 0;
};
std::mutex g_pool_mu;
StreamPool g_pool[64];

bool stream_pool_acquire(int device, int n, std::vector<hipStream_t>& out) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  StreamPool& p = g_pool[device & 63];
  while ((int)p.s.size() < n) {
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return false;
    p.s.push_back(st);
  }
  const int had = (int)out.size();
  out.assign(p.s.begin(), p.s.begin() + n);
  p.refs += n - had;
  return true;
}

void stream_pool_release(int device, int n) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  StreamPool& p = g_pool[device & 63];
  p.refs -= n;
  if (p.refs <= 0) {
    for (hipStream_t st : p.s) (void)hipStreamDestroy(st);
    p.s.clear();
    p.refs = 0;
  }
}

// page-locked (hipHostMalloc'd / registered) host memory?
bool host_pinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// the host-copy pool's size: FFDDP_COPY_THREADS, else the CPUs this process
// may run on (the GPU box grants 16 per GPU), at most 16
int copy_threads() {
  if (const char* e = std::getenv("FFDDP_COPY_THREADS")) {
    const int v = std::atoi(e);
    return v < 1 ? 1 : (v > 64 ? 64 : v);
  }
  cpu_set_t cs;
  int n = 8;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
  return n < 1 ? 1 : (n > 16 ? 16 : n);
}

bool valid_cfg(const ffddp_ocp_config& c) {
  return (c.variant == FFDDP_CLASSICAL || c.variant == FFDDP_FORCE_FEEDBACK) && c.horizon >= 1 &&
         c.horizon <= 4096 && (c.nc == 1 || c.nc == 3) && c.dt > 0.0;
}

}  // namespace

extern "C" {

int ffddp_create(const ffddp_robot* robot, const ffddp_ocp_config* cfg, int device, int max_batch,
                 ffddp_handle** out) {
  if (!robot || !cfg || !out || max_batch < 1) return FFDDP_E_INVALID;
  *out = nullptr;
  if (!valid_cfg(*cfg)) return FFDDP_E_INVALID;
  ffddp_handle* h = new (std::nothrow) ffddp_handle();
  if (!h) return FFDDP_E_OOM;
  h->device = device;
  h->max_batch = max_batch;
  fill_consts(*robot, *cfg, h->hc);
  if (hipSetDevice(device) != hipSuccess) {
    delete h;
    return FFDDP_E_DEVICE;
  }
  const long B = max_batch, N = cfg->horizon, nx = h->hc.nx;
  Dev& d = h->d;
  d.N = (int)N;
  d.nx = (int)nx;
  d.rec = rec_size((int)nx);
  if (d.rec != rec_words((int)nx)) {
    delete h;
    return FFDDP_E_INVALID;
  }
  {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0)
      h->n_simd = 4 * cu;
    const char* ns = std::getenv("FFDDP_STREAMS");
    if (ns) {
      const int v = std::atoi(ns);
      h->nstreams = v < 1 ? 1 : (v > 8 ? 8 : v);
    }
    if (const char* bl = std::getenv("FFDDP_BW_LATE_MAX")) h->bw_late_max = std::atoi(bl);
    if (const char* bw2 = std::getenv("FFDDP_BW_W2_MAX")) h->bw_w2_max = std::atoi(bw2);
    if (const char* ff = std::getenv("FFDDP_FW_FILL")) h->fw_fill = std::atoi(ff) != 0;
    if (const char* fl = std::getenv("FFDDP_FW_LONG")) h->fw_long = std::atoi(fl);
    if (const char* fwm = std::getenv("FFDDP_FW_WIDE_MAX")) h->fw_wide_max = std::atoi(fwm);
    if (const char* lrm = std::getenv("FFDDP_LS_ROW_MAX")) h->ls_row_max = std::atoi(lrm);
    if (const char* fsch = std::getenv("FFDDP_FW_SCHED")) {
      h->fw_sched.clear();
      for (const char* p = fsch; *p;) {
        const int v = std::atoi(p);
        h->fw_sched.push_back(v < 1 ? 1 : (v > NTRIALS ? NTRIALS : v));
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
      }
    }
    if (const char* sg = std::getenv("FFDDP_STAGGER")) h->stagger = std::atoi(sg);
    if (const char* cs = std::getenv("FFDDP_CALLER_SLICE")) h->caller_slice = std::atoi(cs) != 0;
    const char* f1 = std::getenv("FFDDP_FW_FIRST");
    if (f1) {
      const int v = std::atoi(f1);
      h->fw_first = v < 1 ? 1 : (v > NTRIALS ? NTRIALS : v);
    }
  }
  // the slice streams now, not at the first solve: a process's first
  // streams get hardware queues of their own (GPU_MAX_HW_QUEUES, 4), and a
  // communicator created before them (RCCL's streams) would leave the
  // slices sharing queues
  if (h->nstreams > 1 && !stream_pool_acquire(h->device, h->nstreams, h->streams)) {
    delete h;
    return FFDDP_E_DEVICE;
  }
  int rc = 0;
  rc |= dalloc(h, &h->dc, 1);
  rc |= dalloc(h, &h->drb, 1);
  rc |= dalloc(h, &d.rec_buf, (size_t)B * (N + 1) * d.rec);
  rc |= dalloc(h, &d.fs, (size_t)B * (N + 1) * nx);
  rc |= dalloc(h, &d.xs, (size_t)B * (N + 1) * nx);
  rc |= dalloc(h, &d.us, (size_t)B * N * NU);
  rc |= dalloc(h, &d.K, (size_t)B * N * NU * nx);
  rc |= dalloc(h, &d.k, (size_t)B * N * NU);
  rc |= dalloc(h, &d.w, (size_t)B * (N + 1) * nx);
  rc |= dalloc(h, &d.xs_try, (size_t)B * NTRIALS * (N + 1) * nx);
  rc |= dalloc(h, &d.us_try, (size_t)B * NTRIALS * N * NU);
  rc |= dalloc(h, &d.trial, (size_t)B * NTRIALS * 2);
  rc |= dalloc(h, &d.trial_fail, (size_t)B * NTRIALS);
  rc |= dalloc(h, &d.st, (size_t)B);
  rc |= dalloc(h, &d.alist, (size_t)B * 2);
  rc |= dalloc(h, &d.acnt, (size_t)4 * 8);
  rc |= dalloc(h, &h->in_x0, (size_t)B * nx);
  rc |= dalloc(h, &h->in_nref, (size_t)B * (N + 1) * 6);
  rc |= dalloc(h, &h->in_iref, (size_t)B * 21);
  rc |= dalloc(h, &h->in_xs, (size_t)B * (N + 1) * nx);
  rc |= dalloc(h, &h->in_us, (size_t)B * N * NU);
  rc |= dalloc(h, &h->in_surf, (size_t)B);
  rc |= dalloc(h, &h->out_xs, (size_t)B * (N + 1) * nx);
  rc |= dalloc(h, &h->out_us, (size_t)B * N * NU);
  rc |= dalloc(h, &h->out_K, (size_t)B * N * NU * nx);
  rc |= dalloc(h, &h->out_cost, (size_t)B);
  rc |= dalloc(h, &h->out_fn, (size_t)B * 2);
  rc |= dalloc(h, &h->out_iters, (size_t)B);
  rc |= dalloc(h, &h->out_stats, (size_t)B * FFDDP_NSTATS);
  rc |= dalloc(h, &h->out_ok, (size_t)B);
  if (rc) {
    if (!h->streams.empty()) stream_pool_release(h->device, (int)h->streams.size());
    free_all(h);
    delete h;
    return FFDDP_E_OOM;
  }
  if (hipMemcpy(h->dc, &h->hc, sizeof(DevConsts), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->drb, robot, sizeof(ffddp_robot), hipMemcpyHostToDevice) != hipSuccess) {
    if (!h->streams.empty()) stream_pool_release(h->device, (int)h->streams.size());
    free_all(h);
    delete h;
    return FFDDP_E_DEVICE;
  }
  *out = h;
  return 0;
}

#ifdef FFDDP_PHASE_PROF
extern "C" int ffddp_debug_phase_read(unsigned long long* out, int n, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ffddp::g_pp), sizeof(unsigned long long) * (n < 48 ? n : 48)) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[48] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(ffddp::g_pp), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

int ffddp_profile_enable(ffddp_handle* h, int classes) {
  if (!h) return FFDDP_E_INVALID;
  h->prof_mask = classes & FFDDP_PROFILE_ALL;
  h->prof = h->prof_mask != 0;
  return 0;
}

int ffddp_profile_read(ffddp_handle* h, double* ms, int64_t* launches, int reset) {
  if (!h) return FFDDP_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  for (size_t i = 0; i < h->ev_class.size(); ++i) {
    hipEvent_t a = h->ev_pool[2 * i], b = h->ev_pool[2 * i + 1];
    HIPCHK(h, hipEventSynchronize(b));
    float t = 0.f;
    HIPCHK(h, hipEventElapsedTime(&t, a, b));
    h->prof_ms[h->ev_class[i]] += t;
    h->prof_n[h->ev_class[i]] += 1;
  }
  h->ev_class.clear();
  h->ev_used = 0;
  for (int k = 0; k < FFDDP_NKERNELS; ++k) {
    if (ms) ms[k] = h->prof_ms[k];
    if (launches) launches[k] = h->prof_n[k];
    if (reset) {
      h->prof_ms[k] = 0.0;
      h->prof_n[k] = 0;
    }
  }
  return 0;
}

static void plan_invalidate(ffddp_plan* p);

void ffddp_destroy(ffddp_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  for (ffddp_plan* p : h->plans) plan_invalidate(p);
  h->plans.clear();
  if (h->last_done) (void)hipEventDestroy(h->last_done);
  for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->sev) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->stg) (void)hipEventDestroy(e);
  if (!h->streams.empty()) stream_pool_release(h->device, (int)h->streams.size());
  for (hipEvent_t e : h->hdone) (void)hipEventDestroy(e);
  delete h->pool;
  free_all(h);
  delete h;
}

const char* ffddp_last_error(const ffddp_handle* h) { return h ? h->err.c_str() : "null handle"; }

// the end of the solve just enqueued on stream s (every slice has joined s),
// for ffddp_plan_run to wait on
static int mark_solve_done(ffddp_handle* h, hipStream_t s) {
  if (!h->last_done) HIPCHK(h, hipEventCreateWithFlags(&h->last_done, hipEventDisableTiming));
  HIPCHK(h, hipEventRecord(h->last_done, s));
  h->last_done_set = true;
  return 0;
}

int ffddp_solve_batch_dev(ffddp_handle* h, int B, const double* x0, const double* node_ref, const double* inst_ref,
                          const uint8_t* surface, const double* xs_init, const double* us_init, int maxiter,
                          int is_feasible, double* xs, double* us, double* K, double* cost, int32_t* iters,
                          uint8_t* ok, double* fn_pred, int32_t* stats, void* stream) {
  if (!h) return FFDDP_E_INVALID;
  if (B < 0 || maxiter < 0) return fail(h, FFDDP_E_INVALID, "negative B or maxiter");
  if (B > h->max_batch) return fail(h, FFDDP_E_CAPACITY, "B exceeds max_batch");
  if (B == 0) return 0;
  if (!x0 || !node_ref || !inst_ref || !surface || !xs_init || !us_init || !xs || !us || !K || !cost || !iters || !ok)
    return fail(h, FFDDP_E_INVALID, "null pointer");
  HIPCHK(h, hipSetDevice(h->device));
  // the handle's workspace is shared by every solve: a solve enqueued on
  // another (possibly non-blocking) stream must finish before this one starts
  if (h->last_done_set) HIPCHK(h, hipStreamWaitEvent((hipStream_t)stream, h->last_done, 0));
  const int rc = launch_solve(h, B, x0, node_ref, inst_ref, surface, xs_init, us_init, maxiter, is_feasible, xs, us,
                              K, cost, iters, ok, fn_pred, stats, (hipStream_t)stream);
  if (rc) return rc;
  return mark_solve_done(h, (hipStream_t)stream);
}

// error exit of the host entry point after its first asynchronous copy: the
// slice streams may still be copying from the staging buffer or the caller's
// page-locked arrays, or into them; wait for all of them before returning
static int drain_host_solve(ffddp_handle* h, int rc) {
  for (hipStream_t st : h->streams) (void)hipStreamSynchronize(st);
  (void)hipStreamSynchronize(nullptr);
  (void)hipGetLastError();
  return rc;
}

int ffddp_solve_batch(ffddp_handle* h, int B, const double* x0, const double* node_ref, const double* inst_ref,
                      const uint8_t* surface, const double* xs_init, const double* us_init, int maxiter,
                      int is_feasible, double* xs, double* us, double* K, double* cost, int32_t* iters, uint8_t* ok,
                      double* fn_pred, int32_t* stats) {
  if (!h) return FFDDP_E_INVALID;
  if (B < 0 || maxiter < 0) return fail(h, FFDDP_E_INVALID, "negative B or maxiter");
  if (B > h->max_batch) return fail(h, FFDDP_E_CAPACITY, "B exceeds max_batch");
  if (B == 0) return 0;
  if (!x0 || !node_ref || !inst_ref || !surface || !xs_init || !us_init || !xs || !us || !K || !cost || !iters || !ok)
    return fail(h, FFDDP_E_INVALID, "null pointer");
  HIPCHK(h, hipSetDevice(h->device));
  const size_t N = (size_t)h->hc.N, nx = (size_t)h->hc.nx;
  // per-instance bytes: inputs x0, node_ref, inst_ref, surface, xs_init, us_init;
  // outputs xs, us, K, cost, iters, ok, fn_pred, stats
  const size_t per[14] = {nx * 8, (N + 1) * 6 * 8, 21 * 8, 1, (N + 1) * nx * 8, N * NU * 8,
                          (N + 1) * nx * 8, N * NU * 8, N * NU * nx * 8, 8, 4, 1, 16, FFDDP_NSTATS * 4};
  size_t off[14], tot = 0;
  for (int i = 0; i < 14; ++i) {
    off[i] = tot;
    tot += ((per[i] * (size_t)h->max_batch + 255) / 256) * 256;
  }
  if (!h->stage) {
    if (hipHostMalloc((void**)&h->stage, tot, hipHostMallocDefault) != hipSuccess) {
      h->stage = nullptr;
      (void)hipGetLastError();
      return fail(h, FFDDP_E_OOM, "hipHostMalloc (staging) failed");
    }
    h->stage_bytes = tot;
  }
  while (h->hdone.size() < 8) {
    hipEvent_t e;
    HIPCHK(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    h->hdone.push_back(e);
  }
  if (!h->pool) {
    try {
      h->pool = new CopyPool(copy_threads());
    } catch (...) {
      h->pool = nullptr;
    }
  }
  if (!h->pool) return fail(h, FFDDP_E_OOM, "copy pool");
  CopyPool& pool = *h->pool;
  HostIO io;
  io.done = h->hdone.data();
  const bool tm = std::getenv("FFDDP_HOSTIO_TIMING") != nullptr;
  auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = tm ? now() : 0.0;
  // inputs: page-locked caller memory goes up directly, pageable memory
  // through the staging buffer, slice by slice: the host stages slice k and
  // enqueues its whole solve, then stages slice k+1 while slice k runs
  const void* uin[6] = {x0, node_ref, inst_ref, surface, xs_init, us_init};
  void* din[6] = {h->in_x0, h->in_nref, h->in_iref, h->in_surf, h->in_xs, h->in_us};
  bool stin[6];
  bool any_in = false;
  for (int i = 0; i < 6; ++i) {
    stin[i] = !host_pinned(uin[i]);
    any_in |= stin[i];
    io.in[io.n_in++] = HostIO::In{din[i], stin[i] ? (const void*)(h->stage + off[i]) : uin[i], per[i]};
  }
  // FFDDP_HOSTIO_REGISTER=1: page-lock the pageable xs / us / K for the call
  // (see below) instead of draining them through the staging buffer
  {
    const char* r = std::getenv("FFDDP_HOSTIO_REGISTER");
    io.defer_out = r && std::atoi(r) != 0 && (!host_pinned(xs) || !host_pinned(us) || !host_pinned(K));
  }
  double tst[8] = {0};
  if (any_in)
    io.stage = [&](int k) {
      std::vector<CopyJob> jobs;
      for (int i = 0; i < 6; ++i)
        if (stin[i]) {
          const size_t o = (size_t)io.b0[k] * per[i];
          jobs.push_back(CopyJob{h->stage + off[i] + o, (const char*)uin[i] + o, (size_t)io.bk[k] * per[i]});
        }
      pool.run(jobs);
      if (tm) tst[k] = now();
      return 0;
    };
  // outputs: slice by slice into page-locked caller memory, else into the
  // staging buffer and from there into the caller's arrays as each slice ends
  void* uout[8] = {xs, us, K, cost, iters, ok, fn_pred, stats};
  void* hout[8];
  bool staged[8];
  for (int i = 0; i < 8; ++i) {
    staged[i] = uout[i] != nullptr && !host_pinned(uout[i]);
    hout[i] = uout[i] == nullptr ? nullptr : (staged[i] ? (void*)(h->stage + off[6 + i]) : uout[i]);
  }
  const void* dsmall[5] = {h->out_cost, h->out_iters, h->out_ok, h->out_fn, h->out_stats};
  for (int i = 0; i < 5; ++i)
    if (hout[3 + i]) io.out[io.n_out++] = HostIO::Out{hout[3 + i], dsmall[i], per[9 + i]};
  // the caller slice runs on the null stream: a created stream of its own
  // would be a fifth stream on the process's 4 hardware queues and share one
  // with a slice (measured: 15.3 vs 11.6 ms per B = 4096 solve)
  hipStream_t cs = nullptr;
  // after an asynchronous device-entry solve still running on a caller
  // stream (possibly non-blocking): this solve reuses its workspace
  if (h->last_done_set) {
    const hipError_t e = hipStreamWaitEvent(cs, h->last_done, 0);
    if (e != hipSuccess) return fail(h, FFDDP_E_DEVICE, std::string("hipStreamWaitEvent: ") + hipGetErrorString(e));
  }
  int rc = launch_solve(h, B, h->in_x0, h->in_nref, h->in_iref, h->in_surf, h->in_xs, h->in_us, maxiter, is_feasible,
                        (double*)hout[0], (double*)hout[1], (double*)hout[2], h->out_cost, h->out_iters, h->out_ok,
                        h->out_fn, h->out_stats, cs, &io);
  if (rc) return drain_host_solve(h, rc);
  const double t2 = tm ? now() : 0.0;
  // while the device solves: the first touch of the caller's pageable output
  // arrays (fresh numpy arrays are unmapped pages; faulting them in during
  // the drain below would sit on the solve's tail), by the same threads
  {
    std::vector<CopyJob> jobs;
    for (int i = 0; i < 8; ++i)
      if (staged[i]) jobs.push_back(CopyJob{uout[i], nullptr, (size_t)B * per[6 + i]});
    pool.run(jobs);
  }
  // register mode: the (now resident) pageable xs / us / K are page-locked
  // for this call and copied into by DMA directly, slice by slice (no host
  // copy after the solve); an array the runtime will not register goes
  // through the staging buffer as usual
  struct Registered {
    void* p[3] = {nullptr, nullptr, nullptr};
    ~Registered() {
      for (void* q : p)
        if (q) (void)hipHostUnregister(q);
    }
  } regd;
  if (io.defer_out) {
    for (int i = 0; i < 3; ++i) {
      if (!staged[i]) continue;
      if (hipHostRegister(uout[i], (size_t)B * per[6 + i], hipHostRegisterDefault) == hipSuccess) {
        regd.p[i] = uout[i];
        staged[i] = false;  // DMA straight into the caller's array
        hout[i] = uout[i];
      } else {
        (void)hipGetLastError();
      }
    }
    for (int k = 0; k < io.ns; ++k) {
      const size_t b0 = (size_t)io.b0[k], bk = (size_t)io.bk[k];
      const double* dsrc[3] = {io.dxs[k], io.dus[k], io.dK[k]};
      for (int i = 0; i < 3; ++i) {
        const hipError_t e = hipMemcpyAsync((char*)hout[i] + b0 * per[6 + i], dsrc[i], bk * per[6 + i],
                                            hipMemcpyDefault, io.ss[k]);
        if (e != hipSuccess)
          return drain_host_solve(h, fail(h, FFDDP_E_DEVICE, std::string("hipMemcpyAsync: ") + hipGetErrorString(e)));
      }
      const hipError_t e = hipEventRecord(io.done[k], io.ss[k]);
      if (e != hipSuccess)
        return drain_host_solve(h, fail(h, FFDDP_E_DEVICE, std::string("hipEventRecord: ") + hipGetErrorString(e)));
    }
  }
  const double t3 = tm ? now() : 0.0;
  // drain the slices in the order they finish
  double tw[8] = {0}, tc[8] = {0};
  bool drained[8] = {false};
  for (int left = io.ns; left > 0;) {
    int k = -1;
    for (int j = 0; j < io.ns && k < 0; ++j) {
      if (drained[j]) continue;
      const hipError_t e = hipEventQuery(io.done[j]);
      if (e == hipSuccess) k = j;
      else if (e != hipErrorNotReady)
        return drain_host_solve(h, fail(h, FFDDP_E_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(e)));
    }
    if (k < 0) {
      std::this_thread::yield();
      continue;
    }
    if (tm) tw[k] = now();
    std::vector<CopyJob> jobs;
    for (int i = 0; i < 8; ++i) {
      if (!staged[i]) continue;
      const size_t o = (size_t)io.b0[k] * per[6 + i];
      jobs.push_back(CopyJob{(char*)uout[i] + o, (const char*)hout[i] + o, (size_t)io.bk[k] * per[6 + i]});
    }
    pool.run(jobs);
    if (tm) tc[k] = now();
    drained[k] = true;
    --left;
  }
  {
    const hipError_t e = hipStreamSynchronize(cs);
    if (e != hipSuccess)
      return drain_host_solve(h, fail(h, FFDDP_E_DEVICE, std::string("hipStreamSynchronize: ") + hipGetErrorString(e)));
  }
  if (tm) {
    std::fprintf(stderr, "[ffddp host io] %d copy threads | enqueue+stage-in %.2f ms", pool.threads(), t2 - t0);
    for (int k = 0; k < io.ns; ++k) std::fprintf(stderr, " (slice %d staged +%.2f)", k, tst[k] - t0);
    std::fprintf(stderr, " | output first touch done +%.2f", t3 - t0);
    for (int k = 0; k < io.ns; ++k) std::fprintf(stderr, " | slice %d done +%.2f copied +%.2f", k, tw[k] - t0, tc[k] - t0);
    std::fprintf(stderr, " | total %.2f ms\n", now() - t0);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// solve plans: the whole host-array solve of a fixed batch captured once as a
// HIP graph (one input copy, every kernel, one output copy) and replayed per
// call -- the receding-horizon loop's one solve per control tick
// ---------------------------------------------------------------------------
struct ffddp_plan {
  ffddp_handle* h = nullptr;  // null once the handle is destroyed (plan_invalidate)
  int device = 0;
  int B = 0;
  hipStream_t s = nullptr;
  hipGraphExec_t ge = nullptr;
  char *hin = nullptr, *hout = nullptr;  // page-locked, packed
  char *din = nullptr, *dout = nullptr;  // device, same layouts
  size_t in_bytes = 0, out_bytes = 0;
};

namespace {
// packed layouts: 8-byte fields first, then int32, then bytes; each field
// starts on a 256-byte boundary
struct PlanLayout {
  size_t x0, nref, iref, xs_init, us_init, surf, in_bytes;
  size_t xs, us, K, cost, fn, iters, stats, ok, out_bytes;
};
static PlanLayout plan_layout(int B, int N, int nx) {
  PlanLayout L{};
  size_t o = 0;
  auto put = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  const size_t b = (size_t)B, n = (size_t)N, x = (size_t)nx;
  L.x0 = put(b * x * 8);
  L.nref = put(b * (n + 1) * 6 * 8);
  L.iref = put(b * 21 * 8);
  L.xs_init = put(b * (n + 1) * x * 8);
  L.us_init = put(b * n * NU * 8);
  L.surf = put(b);
  L.in_bytes = o;
  o = 0;
  L.xs = put(b * (n + 1) * x * 8);
  L.us = put(b * n * NU * 8);
  L.K = put(b * n * NU * x * 8);
  L.cost = put(b * 8);
  L.fn = put(b * 2 * 8);
  L.iters = put(b * 4);
  L.stats = put(b * FFDDP_NSTATS * 4);
  L.ok = put(b);
  L.out_bytes = o;
  return L;
}

static void plan_free(ffddp_plan* p) {
  if (p->ge) (void)hipGraphExecDestroy(p->ge);
  if (p->s) (void)hipStreamDestroy(p->s);
  if (p->din) (void)hipFree(p->din);
  if (p->dout) (void)hipFree(p->dout);
  if (p->hin) (void)hipHostFree(p->hin);
  if (p->hout) (void)hipHostFree(p->hout);
  delete p;
}
}  // namespace

int ffddp_plan_create(ffddp_handle* h, int B, int maxiter, int is_feasible, ffddp_plan** out, ffddp_plan_io* io) {
  if (!h) return FFDDP_E_INVALID;
  if (!out || !io) return fail(h, FFDDP_E_INVALID, "null pointer");
  *out = nullptr;
  if (B < 1 || maxiter < 0) return fail(h, FFDDP_E_INVALID, "plan needs B >= 1 and maxiter >= 0");
  if (B > h->max_batch) return fail(h, FFDDP_E_CAPACITY, "B exceeds max_batch");
  HIPCHK(h, hipSetDevice(h->device));
  const int N = h->hc.N, nx = h->hc.nx;
  const PlanLayout L = plan_layout(B, N, nx);
  ffddp_plan* p = new (std::nothrow) ffddp_plan();
  if (!p) return fail(h, FFDDP_E_OOM, "plan allocation failed");
  p->h = h;
  p->device = h->device;
  p->B = B;
  p->in_bytes = L.in_bytes;
  p->out_bytes = L.out_bytes;
  if (hipHostMalloc((void**)&p->hin, L.in_bytes, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&p->hout, L.out_bytes, hipHostMallocDefault) != hipSuccess ||
      hipMalloc((void**)&p->din, L.in_bytes) != hipSuccess || hipMalloc((void**)&p->dout, L.out_bytes) != hipSuccess) {
    (void)hipGetLastError();
    plan_free(p);
    return fail(h, FFDDP_E_OOM, "plan buffers");
  }
  std::memset(p->hin, 0, L.in_bytes);
  std::memset(p->hout, 0, L.out_bytes);
  if (hipStreamCreateWithFlags(&p->s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    plan_free(p);
    return fail(h, FFDDP_E_DEVICE, "hipStreamCreate (plan)");
  }
  // capture: inputs up, the device entry point's launch sequence iterating in
  // the plan's own output region, outputs down.  Per-kernel timing events are
  // not captured (profiling is off while capturing).
  const bool prof = h->prof;
  h->prof = false;
  char* di = p->din;
  char* dq = p->dout;
  int rc = 0;
  hipError_t e = hipStreamBeginCapture(p->s, hipStreamCaptureModeThreadLocal);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(p->din, p->hin, L.in_bytes, hipMemcpyHostToDevice, p->s);
    if (e == hipSuccess)
      rc = launch_solve(h, B, (const double*)(di + L.x0), (const double*)(di + L.nref), (const double*)(di + L.iref),
                        (const uint8_t*)(di + L.surf), (const double*)(di + L.xs_init),
                        (const double*)(di + L.us_init), maxiter, is_feasible, (double*)(dq + L.xs),
                        (double*)(dq + L.us), (double*)(dq + L.K), (double*)(dq + L.cost), (int32_t*)(dq + L.iters),
                        (uint8_t*)(dq + L.ok), (double*)(dq + L.fn), (int32_t*)(dq + L.stats), p->s);
    if (e == hipSuccess && rc == 0) e = hipMemcpyAsync(p->hout, p->dout, L.out_bytes, hipMemcpyDeviceToHost, p->s);
    hipGraph_t g = nullptr;
    const hipError_t e2 = hipStreamEndCapture(p->s, &g);
    if (e == hipSuccess) e = e2;
    if (e == hipSuccess && rc == 0) e = hipGraphInstantiate(&p->ge, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
  }
  h->prof = prof;
  if (rc == 0 && e != hipSuccess) rc = fail(h, FFDDP_E_DEVICE, std::string("plan capture: ") + hipGetErrorString(e));
  if (rc) {
    (void)hipGetLastError();
    plan_free(p);
    return rc;
  }
  char* hi = p->hin;
  char* ho = p->hout;
  io->x0 = (double*)(hi + L.x0);
  io->node_ref = (double*)(hi + L.nref);
  io->inst_ref = (double*)(hi + L.iref);
  io->surface = (uint8_t*)(hi + L.surf);
  io->xs_init = (double*)(hi + L.xs_init);
  io->us_init = (double*)(hi + L.us_init);
  io->xs = (const double*)(ho + L.xs);
  io->us = (const double*)(ho + L.us);
  io->K = (const double*)(ho + L.K);
  io->cost = (const double*)(ho + L.cost);
  io->iters = (const int32_t*)(ho + L.iters);
  io->ok = (const uint8_t*)(ho + L.ok);
  io->fn_pred = (const double*)(ho + L.fn);
  io->stats = (const int32_t*)(ho + L.stats);
  h->plans.push_back(p);
  *out = p;
  return 0;
}

int ffddp_plan_run(ffddp_plan* p) {
  if (!p || !p->h || !p->ge) return FFDDP_E_INVALID;  // null, or its handle was destroyed
  ffddp_handle* h = p->h;
  HIPCHK(h, hipSetDevice(h->device));
  // the graph works in the handle's workspace: after a solve still running
  // on another stream (solve_batch_dev is asynchronous), never beside it
  if (h->last_done_set) HIPCHK(h, hipStreamWaitEvent(p->s, h->last_done, 0));
  HIPCHK(h, hipGraphLaunch(p->ge, p->s));
  HIPCHK(h, hipStreamSynchronize(p->s));
  return 0;
}

// the handle is going away: drop the graph (it references the handle's
// workspace); the page-locked io arrays and the device buffers stay until
// ffddp_plan_destroy
static void plan_invalidate(ffddp_plan* p) {
  (void)hipStreamSynchronize(p->s);
  if (p->ge) (void)hipGraphExecDestroy(p->ge);
  p->ge = nullptr;
  p->h = nullptr;
}

void ffddp_plan_destroy(ffddp_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  (void)hipStreamSynchronize(p->s);
  if (p->h) {
    std::vector<ffddp_plan*>& v = p->h->plans;
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i] == p) {
        v.erase(v.begin() + (long)i);
        break;
      }
  }
  plan_free(p);
}

int ffddp_host_alloc(size_t bytes, void** p) {
  if (!p) return FFDDP_E_INVALID;
  *p = nullptr;
  if (hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
    *p = nullptr;
    (void)hipGetLastError();
    return FFDDP_E_OOM;
  }
  return 0;
}

int ffddp_host_free(void* p) {
  if (!p) return 0;
  return hipHostFree(p) == hipSuccess ? 0 : FFDDP_E_DEVICE;
}

int ffddp_get_solver_params(const ffddp_handle* h, ffddp_solver_params* p) {
  if (!h || !p) return FFDDP_E_INVALID;
  const DevConsts& c = h->hc;
  *p = ffddp_solver_params{};
  p->th_stop = c.th_stop;
  p->th_grad = c.th_grad;
  p->th_acceptstep = c.th_acceptstep;
  p->th_acceptnegstep = c.th_acceptnegstep;
  p->th_stepdec = c.th_stepdec;
  p->th_stepinc = c.th_stepinc;
  p->reg_min = c.reg_min;
  p->reg_max = c.reg_max;
  p->reg_incfactor = c.reg_inc;
  p->reg_decfactor = c.reg_dec;
  p->neg_step_rule = c.neg_rule;
  return 0;
}

int ffddp_set_solver_params(ffddp_handle* h, const ffddp_solver_params* p) {
  if (!h || !p) return FFDDP_E_INVALID;
  const double v[10] = {p->th_stop, p->th_grad, p->th_acceptstep, p->th_acceptnegstep, p->th_stepdec,
                        p->th_stepinc, p->reg_min, p->reg_max, p->reg_incfactor, p->reg_decfactor};
  for (double x : v)
    if (!std::isfinite(x) || x < 0.0) return fail(h, FFDDP_E_INVALID, "solver parameters must be finite and >= 0");
  if (!(p->reg_min > 0.0) || p->reg_max < p->reg_min || !(p->reg_incfactor > 1.0) || !(p->reg_decfactor > 1.0))
    return fail(h, FFDDP_E_INVALID, "need 0 < reg_min <= reg_max and reg factors > 1");
  if (p->neg_step_rule != FFDDP_NEGSTEP_CROCODDYL && p->neg_step_rule != FFDDP_NEGSTEP_BOUNDED_RISE)
    return fail(h, FFDDP_E_INVALID, "neg_step_rule must be FFDDP_NEGSTEP_CROCODDYL or FFDDP_NEGSTEP_BOUNDED_RISE");
  DevConsts c = h->hc;
  c.th_stop = p->th_stop;
  c.th_grad = p->th_grad;
  c.th_acceptstep = p->th_acceptstep;
  c.th_acceptnegstep = p->th_acceptnegstep;
  c.th_stepdec = p->th_stepdec;
  c.th_stepinc = p->th_stepinc;
  c.reg_min = p->reg_min;
  c.reg_max = p->reg_max;
  c.reg_inc = p->reg_incfactor;
  c.reg_dec = p->reg_decfactor;
  c.neg_rule = p->neg_step_rule;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipDeviceSynchronize());  // no solve in flight reads the constants while they change
  HIPCHK(h, hipMemcpy(h->dc, &c, sizeof(DevConsts), hipMemcpyHostToDevice));
  h->hc = c;
  return 0;
}

int ffddp_trace_enable(ffddp_handle* h, int max_iters) {
  if (!h || max_iters < 0) return FFDDP_E_INVALID;
  // a live plan's graph writes the trace buffer it captured (or none)
  if (!h->plans.empty())
    return fail(h, FFDDP_E_INVALID, "solve plans of this handle are alive: destroy them before ffddp_trace_enable");
  HIPCHK(h, hipSetDevice(h->device));
  if (h->trace) {
    HIPCHK(h, hipDeviceSynchronize());
    (void)hipFree(h->trace);
  }
  h->trace = nullptr;
  h->trace_it = 0;
  h->d.trace = nullptr;
  h->d.trace_it = 0;
  if (max_iters == 0) return 0;
  if (int rc = dalloc(h, &h->trace, (size_t)h->max_batch * max_iters * FFDDP_TRACE_W)) return rc;
  h->trace_it = max_iters;
  h->d.trace = h->trace;
  h->d.trace_it = max_iters;
  return 0;
}

int ffddp_trace_read(ffddp_handle* h, int B, double* out) {
  if (!h || !out || B < 0 || B > h->max_batch) return FFDDP_E_INVALID;
  if (!h->trace) return fail(h, FFDDP_E_INVALID, "trace not enabled (ffddp_trace_enable)");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipDeviceSynchronize());  // diagnostic read: every stream's solve has finished
  HIPCHK(h, hipMemcpy(out, h->trace, (size_t)B * h->trace_it * FFDDP_TRACE_W * 8, hipMemcpyDeviceToHost));
  return 0;
}

int ffddp_calc_diff(ffddp_handle* h, int B, const double* x0, const double* node_ref, const double* inst_ref,
                    const uint8_t* surface, const double* xs, const double* us, double* Fx, double* Fu, double* Lx,
                    double* Lu, double* Lxx, double* Lxu, double* Luu, double* cost, double* xnext, double* lam) {
  if (!h) return FFDDP_E_INVALID;
  if (B < 1 || B > h->max_batch) return fail(h, FFDDP_E_CAPACITY, "bad B");
  HIPCHK(h, hipSetDevice(h->device));
  const int N = h->hc.N, nx = h->hc.nx, R = h->d.rec;
  const bool ff = h->hc.variant == FFDDP_FORCE_FEEDBACK;
  Dev d = h->d;
  d.B = B;
  HIPCHK(h, hipMemcpy(h->in_x0, x0, (size_t)B * nx * 8, hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->in_nref, node_ref, (size_t)B * (N + 1) * 6 * 8, hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->in_iref, inst_ref, (size_t)B * 21 * 8, hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->in_surf, surface, (size_t)B, hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->in_xs, xs, (size_t)B * (N + 1) * nx * 8, hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(h->in_us, us, (size_t)B * N * NU * 8, hipMemcpyHostToDevice));
  // node kernel reads (xs, us) from the solver state: initialise it from the inputs
  hipLaunchKernelGGL(k_init, dim3(1024), dim3(256), 0, nullptr, h->dc, d, h->in_xs, h->in_us, 0);
  if (h->hc.nc == 1)
    ff ? launch_node<1, true>(h, d, B, nullptr, 1) : launch_node<1, false>(h, d, B, nullptr, 1);
  else
    ff ? launch_node<3, true>(h, d, B, nullptr, 1) : launch_node<3, false>(h, d, B, nullptr, 1);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipDeviceSynchronize());
  std::vector<double> rec((size_t)B * (N + 1) * R), fsv((size_t)B * (N + 1) * nx);
  HIPCHK(h, hipMemcpy(rec.data(), d.rec_buf, rec.size() * 8, hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemcpy(fsv.data(), d.fs, fsv.size() * 8, hipMemcpyDeviceToHost));
  const double dt = h->hc.dt;
  for (int b = 0; b < B; ++b) {
    for (int t = 0; t <= N; ++t) {
      const double* r = rec.data() + ((size_t)b * (N + 1) + t) * R;
      const size_t nt = (size_t)b * (N + 1) + t;
      for (int i = 0; i < nx; ++i) Lx[nt * nx + i] = r[rec_off_Lx(nx) + i];
      for (int e = 0; e < nx * nx; ++e) Lxx[nt * nx * nx + e] = r[rec_off_Lxx(nx) + e];
      cost[nt] = r[rec_off_cost(nx)];
      for (int c = 0; c < 3; ++c) lam[nt * 3 + c] = r[rec_off_lam(nx) + c];
      if (t == N) continue;
      const size_t rt = (size_t)b * N + t;
      const double* A = r + rec_off_A();
      for (int i = 0; i < NU; ++i) Lu[rt * NU + i] = r[rec_off_Lu(nx) + i];
      for (int e = 0; e < nx * NU; ++e) Lxu[rt * nx * NU + e] = r[rec_off_Lxu(nx) + e];
      for (int e = 0; e < NU * NU; ++e) Luu[rt * NU * NU + e] = r[rec_off_Luu(nx) + e];
      for (int i = 0; i < nx; ++i) {
        for (int j = 0; j < nx; ++j) {
          double v = (i == j) ? 1.0 : 0.0;
          if (i < 14 && j < (ff ? 21 : 14)) {
            v += (i < 7 ? dt * dt : dt) * A[j * NQ + (i % 7)];
            if (i < 7 && j == i + 7) v += dt;
          }
          if (ff && i >= 14) v = (i == j) ? h->hc.alpha : 0.0;
          Fx[rt * nx * nx + i * nx + j] = v;
        }
        for (int kk = 0; kk < NU; ++kk) {
          double v;
          if (!ff)
            v = (i < 7 ? dt * dt : dt) * A[(14 + kk) * NQ + (i % 7)];
          else
            v = (i >= 14 && i - 14 == kk) ? h->hc.beta : 0.0;
          Fu[rt * nx * NU + i * NU + kk] = v;
        }
      }
      // xnext = xs[t+1] + fs[t+1]  (fs computed with is_feasible = 0)
      for (int i = 0; i < nx; ++i)
        xnext[rt * nx + i] = xs[((size_t)b * (N + 1) + t + 1) * nx + i] + fsv[((size_t)b * (N + 1) + t + 1) * nx + i];
    }
  }
  return 0;
}

int ffddp_frame_placement(const ffddp_robot* robot, const double* q, double* R, double* p) {
  if (!robot || !q || !R || !p) return FFDDP_E_INVALID;
  RBOut<double> o;
  const double zero[NQ] = {0, 0, 0, 0, 0, 0, 0};
  rb_pass<double, false, false>(*robot, q, zero, zero, nullptr, o, nullptr);
  for (int i = 0; i < 9; ++i) R[i] = o.Ree.m[i];
  p[0] = o.pee.x;
  p[1] = o.pee.y;
  p[2] = o.pee.z;
  return 0;
}

int ffddp_gravity_torque(const ffddp_robot* robot, int B, const double* q, double* tau) {
  if (!robot || !q || !tau || B < 0) return FFDDP_E_INVALID;
  for (int b = 0; b < B; ++b) gravity_torque(*robot, q + (size_t)b * NQ, tau + (size_t)b * NQ);
  return 0;
}

int ffddp_gravity_torque_dev(ffddp_handle* h, int B, const double* q, double* tau, void* stream) {
  if (!h || B < 0) return FFDDP_E_INVALID;
  if (B == 0) return 0;
  HIPCHK(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(k_gravity, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, h->drb, B, q, tau);
  HIPCHK(h, hipGetLastError());
  return 0;
}

int ffddp_build_problem_dev(ffddp_handle* h, int B, const ffddp_task* task, const double* t0, const double* x0,
                            double* node_ref, double* inst_ref, uint8_t* surface, void* stream) {
  if (!h || !task || B < 0) return FFDDP_E_INVALID;
  if (B == 0) return 0;
  if (!t0 || !x0 || !node_ref || !inst_ref || !surface) return FFDDP_E_INVALID;
  if (task->posture_mode < 0 || task->posture_mode > 1 || task->torque_mode < 0 || task->torque_mode > 2) {
    h->err = "ffddp_build_problem_dev: posture_mode must be 0/1 and torque_mode 0/1/2";
    return FFDDP_E_INVALID;
  }
  // make_approach_then_circle's closure constants (trajectories.py:36-60)
  TaskTraj T{};
  for (int i = 0; i < 3; ++i) T.center[i] = task->center[i];
  T.radius = task->radius;
  T.omega = task->omega;
  T.z_contact = task->z_contact;
  T.t_approach = std::max(task->t_approach, 1.0e-6);
  T.t_pre = std::max(task->t_pre, 0.0);
  T.t_hold = task->t_hold;
  for (int i = 0; i < 3; ++i) T.p_cs[i] = task->center[i];
  T.p_cs[0] += task->radius;
  T.p_cs[2] = task->z_contact;
  for (int i = 0; i < 3; ++i) T.p_start[i] = task->has_ee_start ? task->ee_start[i] : T.p_cs[i];
  if (!task->has_ee_start) T.p_start[2] += 0.08;
  const double z_pre = task->has_z_pre ? task->z_pre : std::max(task->z_contact + 0.05, T.p_start[2]);
  for (int i = 0; i < 3; ++i) T.p_pre[i] = T.p_cs[i];
  T.p_pre[2] = z_pre;
  const int N = h->hc.N;
  const long n = (long)B * (N + 1);
  HIPCHK(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(k_build, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream, h->drb, T, *task, B, N,
                     h->hc.nx, h->hc.dt, t0, x0, node_ref, inst_ref, surface);
  HIPCHK(h, hipGetLastError());
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// plant stand-in
// ---------------------------------------------------------------------------
struct ffddp_plant {
  int device = 0, max_batch = 0;
  ffddp_robot* drb = nullptr;
  ffddp_plant_params* dpp = nullptr;
  double *q = nullptr, *v = nullptr, *tau = nullptr, *plane = nullptr, *obs = nullptr;
  int32_t* fail = nullptr;
};

extern "C" {

int ffddp_plant_create(const ffddp_robot* robot, const ffddp_plant_params* p, int device, int max_batch,
                       ffddp_plant** out) {
  static_assert(PO_WORDS == FFDDP_PLANT_OBS, "plant observation layout");
  if (!robot || !p || !out || max_batch < 1 || p->timestep <= 0.0 || p->n_substeps < 1) return FFDDP_E_INVALID;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return FFDDP_E_DEVICE;
  ffddp_plant* h = new (std::nothrow) ffddp_plant();
  if (!h) return FFDDP_E_OOM;
  h->device = device;
  h->max_batch = max_batch;
  const size_t B = (size_t)max_batch;
  bool bad_alloc = hipMalloc((void**)&h->drb, sizeof(ffddp_robot)) != hipSuccess;
  bad_alloc |= hipMalloc((void**)&h->dpp, sizeof(ffddp_plant_params)) != hipSuccess;
  bad_alloc |= hipMalloc((void**)&h->q, B * NQ * 8) != hipSuccess;
  bad_alloc |= hipMalloc((void**)&h->v, B * NQ * 8) != hipSuccess;
  bad_alloc |= hipMalloc((void**)&h->tau, B * NQ * 8) != hipSuccess;
  bad_alloc |= hipMalloc((void**)&h->plane, B * 6 * 8) != hipSuccess;
  bad_alloc |= hipMalloc((void**)&h->obs, B * PO_WORDS * 8) != hipSuccess;
  bad_alloc |= hipMalloc((void**)&h->fail, B * 4) != hipSuccess;
  if (bad_alloc || hipMemcpy(h->drb, robot, sizeof(ffddp_robot), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->dpp, p, sizeof(ffddp_plant_params), hipMemcpyHostToDevice) != hipSuccess) {
    ffddp_plant_destroy(h);
    return bad_alloc ? FFDDP_E_OOM : FFDDP_E_DEVICE;
  }
  *out = h;
  return 0;
}

void ffddp_plant_destroy(ffddp_plant* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  void* ps[] = {h->drb, h->dpp, h->q, h->v, h->tau, h->plane, h->obs, h->fail};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  delete h;
}

int ffddp_plant_step_dev(ffddp_plant* h, int B, double* q, double* v, const double* tau, const double* plane,
                         int integrate, double* obs, int32_t* fail, void* stream) {
  if (!h || B < 0 || B > h->max_batch) return FFDDP_E_INVALID;
  if (B == 0) return 0;
  if (!q || !v || !tau || !plane || !obs) return FFDDP_E_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return FFDDP_E_DEVICE;
  hipLaunchKernelGGL(k_plant, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, h->drb, h->dpp, B, q, v, tau,
                     plane, integrate, obs, fail);
  return hipGetLastError() == hipSuccess ? 0 : FFDDP_E_DEVICE;
}

int ffddp_plant_step(ffddp_plant* h, int B, double* q, double* v, const double* tau, const double* plane,
                     int integrate, double* obs) {
  if (!h || B < 0 || B > h->max_batch) return FFDDP_E_INVALID;
  if (B == 0) return 0;
  if (!q || !v || !tau || !plane || !obs) return FFDDP_E_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return FFDDP_E_DEVICE;
  const size_t n7 = (size_t)B * NQ * 8;
  if (hipMemcpy(h->q, q, n7, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->v, v, n7, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->tau, tau, n7, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->plane, plane, (size_t)B * 6 * 8, hipMemcpyHostToDevice) != hipSuccess)
    return FFDDP_E_DEVICE;
  int rc = ffddp_plant_step_dev(h, B, h->q, h->v, h->tau, h->plane, integrate, h->obs, h->fail, nullptr);
  if (rc) return rc;
  std::vector<int32_t> fl((size_t)B);
  if (hipMemcpy(q, h->q, n7, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(v, h->v, n7, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(obs, h->obs, (size_t)B * PO_WORDS * 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(fl.data(), h->fail, (size_t)B * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return FFDDP_E_DEVICE;
  for (int b = 0; b < B; ++b)
    if (fl[b]) return FFDDP_E_INVALID;
  return 0;
}

}  // extern "C"
