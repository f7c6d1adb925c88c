/*
 * ffddp.h — C-ABI of the MI355X-native batched (Box)FDDP solver.
 *
 * Drop-in boundary for the reference's hot path
 *     ok = solver.solve(xs_init, us_init, max_iters, False)
 * at src/mpc/crocoddyl_classical.py:367 (ClassicalCrocoddylMPC) and
 * src/mpc/crocoddyl_force_feedback.py:605 (ForceFeedbackCrocoddylMPC), where
 * `solver` is crocoddyl.SolverBoxFDDP(problem) (crocoddyl_classical.py:442-445)
 * over the ShootingProblem built by _build_problem (:521-556 / FF :776-836).
 * The reference binds Crocoddyl through boost-python; this library is bound
 * through ctypes (ffddp._abi) and through a pybind11 module over the same
 * entry points (csrc/ffddp_pybind.cpp).  Plain pointers
 * and sizes only.
 *
 * Conventions
 *   - fp64 everywhere; all matrices row-major.
 *   - One handle = one OCP definition (robot + weights + horizon + variant),
 *     bound to one HIP device.  A handle is not thread-safe.  Handles on the
 *     same device share one pool of slice streams (and the null stream), so
 *     solves of two handles driven from two threads are correct but
 *     serialise on the GPU rather than overlap.
 *   - Return 0 on success or a negative FFDDP_E* code for API / launch / OOM
 *     errors.  Per-instance numerical failure is reported in ok[b] = 0 (the
 *     cost may be NaN), exactly like Crocoddyl's solve() returning False.
 *   - No C++ exception crosses this boundary.
 */
#ifndef FFDDP_H_
#define FFDDP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FFDDP_NQ 7      /* Panda arm joints (fingers locked, crocoddyl_classical.py:189-197) */
#define FFDDP_NU 7      /* ActuationModelFull: nu = nv (:147) */
#define FFDDP_MAX_NC 3  /* ContactModel1D (nc=1) or ContactModel3D (nc=3) */
#define FFDDP_NSTATS 10 /* per-instance counters returned by the solve */
#define FFDDP_NKERNELS 8 /* kernel classes reported by ffddp_profile_read */

enum {
  FFDDP_OK = 0,
  FFDDP_E_INVALID = -1,  /* bad argument (sizes, null pointers, config) */
  FFDDP_E_DEVICE = -2,   /* HIP runtime / launch error */
  FFDDP_E_OOM = -3,      /* device allocation failed */
  FFDDP_E_CAPACITY = -4  /* B larger than the handle's max_batch */
};

enum { FFDDP_CLASSICAL = 0, FFDDP_FORCE_FEEDBACK = 1 };

/* Rigid-body model of the 7-DoF arm: revolute-z joints in a serial chain.
 * Replaces example_robot_data.load("panda") + pin.buildReducedModel
 * (crocoddyl_classical.py:137-145, 189-197). */
typedef struct ffddp_robot {
  double joint_R[FFDDP_NQ][9]; /* placement of joint i in its parent (rotation) */
  double joint_p[FFDDP_NQ][3]; /* placement of joint i in its parent (translation) */
  double mass[FFDDP_NQ];
  double com[FFDDP_NQ][3];     /* COM in the link frame */
  double inertia[FFDDP_NQ][9]; /* rotational inertia about the COM, link frame */
  double ee_R[9];              /* EE frame ("panda_link8") in link 7 */
  double ee_p[3];
  double gravity[3];           /* world gravity, (0,0,-9.81) */
} ffddp_robot;

/* OCP definition: every field the reference's _build_problem/_make_dam reads
 * from ClassicalMPCConfig / ForceFeedbackMPCConfig
 * (crocoddyl_classical.py:12-110, 521-728; crocoddyl_force_feedback.py:12-146,
 * 149-290, 776-1009).  Costs with weight 0 are not added (as in the reference). */
typedef struct ffddp_ocp_config {
  int32_t variant;      /* FFDDP_CLASSICAL (nx=14) or FFDDP_FORCE_FEEDBACK (nx=21) */
  int32_t horizon;      /* N running nodes + 1 terminal node */
  int32_t nc;           /* 1 = ContactModel1D normal_1d, 3 = ContactModel3D point3d */
  int32_t use_box;      /* 1 = SolverBoxFDDP (default), 0 = SolverFDDP */
  double dt;            /* dt_ocp */
  double z_press;
  double w_ee_pos, w_ee_ori;
  double ori_weights[3];
  double w_posture, w_v;
  double v_damp_weights[7];
  double w_tau, w_tau_soft_limits, tau_soft_limit_margin;
  double w_q_soft_limits, q_soft_limit_margin;
  double q_lower[7], q_upper[7];
  double w_tangent_pos, w_tangent_vel, w_plane_z, w_vz;
  double w_unilateral, friction_margin, w_fn, fn_des;
  double w_wdamp;
  double w_wdamp_weights[3];
  double contact_gains[2];   /* Baumgarte [Kp, Kd] */
  double contact_inv_damping;/* JMinvJt_damping */
  double tau_limits[7];      /* u_lb = -tau_limits, u_ub = +tau_limits */
  double R_des[9];           /* FrameRotation reference, Pinocchio world */
  /* force-feedback augmentation (_AugmentedLPFActionModel) */
  double ff_alpha;           /* tau_{k+1} = alpha tau_k + (1-alpha) w_k */
  double w_w, w_w_soft_limits, w_y;
  double y_weights[21];
  int32_t use_inner_state_reg, use_inner_tau_reg;
  /* friction cone, built only for nc = 3 (crocoddyl_classical.py:678-687; FF
   * crocoddyl_force_feedback.py:959-966): ResidualModelContactFrictionCone over
   * crocoddyl.FrictionCone(I, mu, nf = 4, inner = False)
   * (crocoddyl_classical.py:999-1018, crocoddyl_force_feedback.py:1428-1447)
   * with a QuadraticBarrier narrowed by friction_margin (:891-903), weight
   * w_friction_cone */
  double w_friction_cone, mu;
} ffddp_ocp_config;

/* Task description for the device-side problem builder:
 * the approach-then-circle EE reference of src/tasks/trajectories.py:8-93
 * with the benchmark runner's contact-onset hold (run_classical.py:221-264),
 * the MuJoCo->Pinocchio target mapping (crocoddyl_classical.py:250-258) and
 * the posture / torque reference modes (crocoddyl_classical.py:447-466). */
typedef struct ffddp_task {
  double center[3];   /* circle centre, MuJoCo world (z = contact height) */
  double radius, omega, z_contact, t_approach, t_pre;
  double z_pre;       /* used when has_z_pre, else max(z_contact + 0.05, ee_start z) */
  double t_hold;      /* benchmark hold at contact onset (0.2 s; 0 = none) */
  double ee_start[3]; /* used when has_ee_start, else contact start + (0, 0, 0.08) */
  int32_t has_ee_start, has_z_pre;
  double p_site_minus_frame[3]; /* _calibrate_site_position_offset (Pinocchio frame) */
  double q_nom[7];
  int32_t posture_mode; /* 0: x_reg_ref = x0[:14]; 1: [q_nom, 0] */
  int32_t torque_mode;  /* 0: gravity(x0 q); 1: gravity(q_nom); 2: zero */
} ffddp_task;

typedef struct ffddp_handle ffddp_handle;

/* crocoddyl.SolverBoxFDDP(problem) / setProblem (crocoddyl_classical.py:350-361):
 * allocates device workspace for up to max_batch instances. */
int ffddp_create(const ffddp_robot* robot, const ffddp_ocp_config* cfg, int device,
                 int max_batch, ffddp_handle** out);
void ffddp_destroy(ffddp_handle* h);
const char* ffddp_last_error(const ffddp_handle* h);

/* Batched solver.solve(xs_init, us_init, maxiter, is_feasible)
 * (crocoddyl_classical.py:365-388, crocoddyl_force_feedback.py:603-628).
 * Host pointers, row-major:
 *   x0       [B][nx]           problem.x0 (FF: y0 = [q, v, tau_hat])
 *   node_ref [B][N+1][6]       p_ref, v_ref per node, Pinocchio world (:526-546)
 *   inst_ref [B][21]           x_reg_ref (14), tau_ref (7)           (:523-524)
 *   surface  [B]               0 free-space DAM, 1 contact DAM       (:533, 614)
 *   xs_init  [B][N+1][nx], us_init [B][N][7]                         (:365)
 * Outputs (solver.xs, solver.us, solver.K, solver.cost, solver.iter, ok):
 *   xs [B][N+1][nx], us [B][N][7], K [B][N][7][nx], cost [B], iters [B], ok [B]
 *   fn_pred [B][2]   contact lambda_normal at knots 0 and 1 of the solution
 *                    (crocoddyl_classical.py:905-942, FF :1219-1299; NaN if free)
 *   stats  [B][FFDDP_NSTATS]  (optional, may be NULL) per instance:
 *                    [0] FDDP iterations with a successful backward pass,
 *                    [1] line-search trials a sequential solver executes,
 *                    [2] regularisation retries of the backward pass,
 *                    [3] backward passes run, [4] calcDiff evaluations,
 *                    [5] line-search kernel launches that processed the
 *                    instance (first pass + second pass when it ran),
 *                    [6] / [7] step lengths evaluated by the first / second
 *                    line-search pass — for the roofline byte count
 *                    (SURVEY.md §8(d)),
 *                    [8] / [9] line-search trials judged / accepted by the
 *                    ascent-direction branch (dVexp < 0, see
 *                    ffddp_solver_params.neg_step_rule). */
int ffddp_solve_batch(ffddp_handle* h, int B, const double* x0, const double* node_ref,
                      const double* inst_ref, const uint8_t* surface, const double* xs_init,
                      const double* us_init, int maxiter, int is_feasible, double* xs, double* us,
                      double* K, double* cost, int32_t* iters, uint8_t* ok, double* fn_pred,
                      int32_t* stats);

/* Same with DEVICE pointers (inputs resident in HBM) on `stream` (hipStream_t,
 * NULL = default stream).  Asynchronous: the caller synchronises the stream.
 * xs / us / K are the solver's working storage during the solve (it iterates
 * in them; no copy follows the last kernel): they must not overlap the other
 * inputs, except xs_init == xs and us_init == us (warm start in place). */
int ffddp_solve_batch_dev(ffddp_handle* h, int B, const double* x0, const double* node_ref,
                          const double* inst_ref, const uint8_t* surface, const double* xs_init,
                          const double* us_init, int maxiter, int is_feasible, double* xs,
                          double* us, double* K, double* cost, int32_t* iters, uint8_t* ok,
                          double* fn_pred, int32_t* stats, void* stream);

/* Solve plan for a receding-horizon loop: one solve of a fixed batch per
 * control tick (crocoddyl_classical.py:367 called every tick at
 * run_classical.py:412).  ffddp_plan_create captures the whole host-array
 * solve once as a HIP graph -- one copy of the packed inputs up, every kernel
 * of maxiter iterations, one copy of the packed outputs down -- and
 * ffddp_plan_run replays it and waits: one graph launch per tick instead of
 * ~50 kernel launches and 14 copies.  The plan owns page-locked input and
 * output arrays (the ffddp_solve_batch arguments, same layouts), returned in
 * *io: refill the inputs in place before each run, read the outputs after it
 * (overwritten by the next run).  Results equal ffddp_solve_batch's bit for
 * bit.  The solver properties (ffddp_set_solver_params) apply to later runs;
 * tracing and per-kernel timing are fixed at creation (timing off):
 * ffddp_trace_enable returns FFDDP_E_INVALID while a plan of the handle is
 * alive.  A plan uses its handle's workspace.  ffddp_plan_run first waits (on
 * the device) for the handle's last solve_batch[_dev] call to finish, on
 * whatever stream it ran; do not run a plan from a second host thread while
 * another solve of the same handle is being enqueued.  ffddp_destroy
 * invalidates the handle's live plans: their ffddp_plan_run then returns
 * FFDDP_E_INVALID, and ffddp_plan_destroy still frees them (their io arrays
 * stay valid until then). */
typedef struct ffddp_plan ffddp_plan;
typedef struct ffddp_plan_io {
  double* x0;        /* [B][nx]        inputs, written by the caller */
  double* node_ref;  /* [B][N+1][6] */
  double* inst_ref;  /* [B][21] */
  uint8_t* surface;  /* [B] */
  double* xs_init;   /* [B][N+1][nx] */
  double* us_init;   /* [B][N][7] */
  const double* xs;  /* [B][N+1][nx]  outputs of the last run */
  const double* us;  /* [B][N][7] */
  const double* K;   /* [B][N][7][nx] */
  const double* cost;
  const int32_t* iters;
  const uint8_t* ok;
  const double* fn_pred; /* [B][2] */
  const int32_t* stats;  /* [B][FFDDP_NSTATS] */
} ffddp_plan_io;
int ffddp_plan_create(ffddp_handle* h, int B, int maxiter, int is_feasible, ffddp_plan** out, ffddp_plan_io* io);
int ffddp_plan_run(ffddp_plan* p);
void ffddp_plan_destroy(ffddp_plan* p);

/* problem.calcDiff(xs, us) on the device (ShootingProblem::calcDiff; used by
 * parity tests of the per-node models).  Host pointers.  Outputs per node in
 * Crocoddyl layout (running nodes t < N, terminal node t = N):
 *   Fx [B][N][nx][nx], Fu [B][N][nx][7], Lx [B][N+1][nx], Lu [B][N][7],
 *   Lxx [B][N+1][nx][nx], Lxu [B][N][nx][7], Luu [B][N][7][7],
 *   cost [B][N+1], xnext [B][N][nx], lam [B][N+1][3] (contact force, 0 if free). */
int ffddp_calc_diff(ffddp_handle* h, int B, const double* x0, const double* node_ref,
                    const double* inst_ref, const uint8_t* surface, const double* xs,
                    const double* us, double* Fx, double* Fu, double* Lx, double* Lu, double* Lxx,
                    double* Lxu, double* Luu, double* cost, double* xnext, double* lam);

/* Host-side setup helpers (CPU, same model code): frame placement of the EE
 * (pin.forwardKinematics + updateFramePlacements, crocoddyl_classical.py:199-225)
 * and gravity torque rnea(q, 0, 0) (_gravity_torque, :447-451) for B configurations. */
int ffddp_frame_placement(const ffddp_robot* robot, const double* q, double* R, double* p);
int ffddp_gravity_torque(const ffddp_robot* robot, int B, const double* q, double* tau);

/* Solver properties of crocoddyl.SolverBoxFDDP / SolverFDDP (the attributes
 * the reference leaves at their defaults: th_stop, th_grad, th_acceptstep,
 * th_acceptnegstep, th_stepdec, th_stepinc, reg_min/reg_max/reg_incfactor/
 * reg_decfactor; crocoddyl_classical.py:442-445 constructs the solver and
 * sets none of them).  neg_step_rule selects the comparator of the
 * ascent-direction acceptance (dVexp < 0, only while infeasible,
 * SolverFDDP::solve):
 *   FFDDP_NEGSTEP_CROCODDYL     accept iff dV < th_acceptnegstep * dVexp
 *                               (Crocoddyl's source; default)
 *   FFDDP_NEGSTEP_BOUNDED_RISE  accept iff dV > th_acceptnegstep * dVexp
 *                               (a rise of at most th_acceptnegstep x the
 *                               predicted one; accepts the exact LQR step)
 * Values set here apply to the following solves of the handle. */
enum { FFDDP_NEGSTEP_CROCODDYL = 0, FFDDP_NEGSTEP_BOUNDED_RISE = 1 };
typedef struct ffddp_solver_params {
  double th_stop;          /* SolverBoxFDDP 5e-5, SolverFDDP 1e-9 */
  double th_grad;          /* 1e-12 */
  double th_acceptstep;    /* 0.1 */
  double th_acceptnegstep; /* 2.0 */
  double th_stepdec;       /* 0.5 */
  double th_stepinc;       /* 0.01 */
  double reg_min, reg_max; /* 1e-9, 1e9 */
  double reg_incfactor, reg_decfactor; /* 10, 10 */
  int32_t neg_step_rule;   /* FFDDP_NEGSTEP_* */
  int32_t reserved;
} ffddp_solver_params;
int ffddp_get_solver_params(const ffddp_handle* h, ffddp_solver_params* p);
int ffddp_set_solver_params(ffddp_handle* h, const ffddp_solver_params* p);

/* Per-iteration solver trace: what crocoddyl.CallbackVerbose prints at the end
 * of every iteration (solver.setCallbacks([crocoddyl.CallbackVerbose()]),
 * crocoddyl_classical.py:352-353, 360-361; FF :588-599).  ffddp_trace_enable
 * (h, max_iters) keeps a record per instance and iteration for the next solves
 * (0 = off); ffddp_trace_read copies the last solve's records for its B
 * instances to out [B][max_iters][FFDDP_TRACE_W] (host pointer):
 *   [0] iter, [1] cost, [2] stop = sum ||Qu||^2, [3] grad = -d1 of the last
 *   tried step length, [4] preg, [5] dreg (= preg), [6] step length (the
 *   accepted one, else the smallest tried), [7] ||ffeas|| = max |fs| of the
 *   iteration's calcDiff, [8] dV, [9] dV_exp of that step length.
 * Iterations an instance did not reach (stopped earlier, failed backward
 * pass) hold NaN rows. */
#define FFDDP_TRACE_W 10
int ffddp_trace_enable(ffddp_handle* h, int max_iters);
int ffddp_trace_read(ffddp_handle* h, int B, double* out);

/* Page-locked host memory for the host-pointer entry points: arrays passed to
 * ffddp_solve_batch that live in such memory are copied by DMA on the slice
 * streams, overlapping the other slices' kernels; pageable arrays go through
 * the handle's own page-locked staging buffers. */
int ffddp_host_alloc(size_t bytes, void** p);
int ffddp_host_free(void* p);

/* Optional per-kernel device timing (HIP events recorded around every launch
 * on the launch stream), one kernel per class.  Classes, in order: init,
 * node (calc + calcDiff tangents + Gauss-Newton, one fused kernel), backward,
 * forward (line search, first pass), accept (acceptance test, regularisation,
 * stopping; no copy: the next node kernel reads the accepted trial in place),
 * commit (end of solve: accepted trials no node kernel consumed become
 * xs / us), finalize, forward2 (line search, second pass).
 * `classes` is a bit mask over those classes (bit i = class i; 0 = off,
 * FFDDP_PROFILE_ALL = every class).  Timing only the kernel of interest keeps
 * the event overhead out of the other launches.
 * ffddp_profile_read synchronises the recorded events and returns, per class,
 * the summed milliseconds and launch counts since the last reset. */
#define FFDDP_PROFILE_ALL 0xFF
int ffddp_profile_enable(ffddp_handle* h, int classes);
int ffddp_profile_read(ffddp_handle* h, double* ms, int64_t* launches, int reset);

/* Batched gravity torque on the device (tau_ref for B instances), device pointers. */
int ffddp_gravity_torque_dev(ffddp_handle* h, int B, const double* q, double* tau, void* stream);

/* Device-side problem builder: what _build_problem (crocoddyl_classical.py:
 * 521-556; FF :776-836) feeds the action models, for B instances at once,
 * as the solver's input arrays.  Instance b solves from time t0[b] and state
 * x0[b] (nx): knot k samples the task at t0 + k dt_ocp (k = 0..N) and maps
 * it to the Pinocchio frame; surface[b] = the task's contact flag at t0
 * (phase_source "trajectory"); inst_ref = posture and torque references.
 * Device pointers: t0[B], x0[B][nx] -> node_ref[B][N+1][6],
 * inst_ref[B][21], surface[B]. */
int ffddp_build_problem_dev(ffddp_handle* h, int B, const ffddp_task* task, const double* t0, const double* x0,
                            double* node_ref, double* inst_ref, uint8_t* surface, void* stream);

/* ---------------------------------------------------------------------------
 * Closed-loop plant stand-in: the MuJoCo plant of the
 * reference's closed loop, FrankaMujocoSim.step() in torque mode
 * (src/sim/franka_sim.py:144-169) on assets/scenes/panda_table_scene.xml:
 * arm (+ joint armature / damping, panda_robot.xml:9), tool sphere at the
 * ee_site (:189-199) against the table_contact plane (condim 1, soft
 * constraint solref/solimp), implicitfast integration, n_substeps physics
 * steps per control step.  Observation record: FFDDP_PLANT_OBS words per
 * instance (q, dq, qfrc_bias, qfrc_constraint, site pos/vel/rot, contact force,
 * site Jacobian), see ffddp_plant.hpp.  Parity with MuJoCo is unpinned.
 * ------------------------------------------------------------------------- */
#define FFDDP_PLANT_OBS 69
typedef struct ffddp_plant_params {
  double timestep;      /* model.opt.timestep (benchmark protocol: 0.001) */
  int32_t n_substeps;   /* physics steps per control step (5) */
  double armature[7], damping[7];
  double r_tool;        /* ee_collision sphere radius (0.03) */
  double margin;        /* contact margin (0.001) */
  double solref[2];     /* (timeconst, dampratio), MuJoCo default (0.02, 1) */
  double solimp[5];     /* MuJoCo default (0.9, 0.95, 0.001, 0.5, 2) */
  double site_R[2];     /* cos, sin of the tool-body yaw (135 deg) */
} ffddp_plant_params;

typedef struct ffddp_plant ffddp_plant;
int ffddp_plant_create(const ffddp_robot* robot, const ffddp_plant_params* p, int device, int max_batch,
                       ffddp_plant** out);
void ffddp_plant_destroy(ffddp_plant* h);
/* One control step of B plants (integrate = 0: forward only, like mj_forward).
 * Host pointers: q, v [B][7] (in/out), tau [B][7] applied torque, plane [B][6]
 * = table normal (3) and a point on the plane (3), MuJoCo world; obs
 * [B][FFDDP_PLANT_OBS].  Returns FFDDP_E_INVALID on a non-SPD mass matrix. */
int ffddp_plant_step(ffddp_plant* h, int B, double* q, double* v, const double* tau, const double* plane,
                     int integrate, double* obs);
/* Same on device pointers, asynchronous on `stream` (per-instance failure flags in fail[B], may be NULL). */
int ffddp_plant_step_dev(ffddp_plant* h, int B, double* q, double* v, const double* tau, const double* plane,
                         int integrate, double* obs, int32_t* fail, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FFDDP_H_ */
