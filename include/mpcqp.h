/*
 * mpcqp.h -- C-ABI of the MI355X batched bicycle-MPC QP solver (libmpcqp.so).
 *
 * Drop-in boundary for the reference's MPC hot path (CagriCatik/RRT-MPC):
 *
 *   reference call                                         replaced by
 *   -----------------------------------------------------  -----------------------------
 *   src/control/mpc_controller.py:17-30  MPCParameters      mpcqp_params (+ solver settings
 *                                                          of mpc_controller.py:121-131)
 *   src/control/mpc_controller.py:59-70  unwrap + N x       mpcqp_build   (HIP kernel K1)
 *   src/control/vehicle_model.py:24-45   linearize()
 *   src/control/mpc_controller.py:53-117 cvxpy assembly +   mpcqp_solve   (HIP kernel K2)
 *   src/control/mpc_controller.py:119-132 OSQP solve
 *   src/control/mpc_controller.py:133-141 status / return   status[] codes below
 *
 * The reference binds this path from Python; the ctypes binding lives in
 * rrt-mpc_amd/mpcqp/_lib.py and INTEGRATION.md shows the reference-side stub.
 *
 * Conventions
 *  - All numeric I/O is IEEE float64, row-major, contiguous, caller-owned DEVICE
 *    memory (e.g. torch.cuda tensors); the library never frees caller buffers.
 *  - Calls are asynchronous on the given hipStream_t (NULL = default stream).
 *  - Return value: 0 on success, a negative MPCQP_E_* code otherwise; no C++
 *    exception crosses the ABI.  mpcqp_last_error() describes the last failure
 *    of the calling thread.
 *  - Re-entrant across distinct workspaces; NOT thread-safe on one workspace.
 *  - One workspace is bound to one device; use one process per GPU.
 */
#ifndef MPCQP_H
#define MPCQP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCQP_ABI_VERSION 9

/* error codes (function return values) */
#define MPCQP_OK 0
#define MPCQP_E_ARG (-1)         /* bad pointer / size / parameter */
#define MPCQP_E_HORIZON (-2)     /* horizon outside [1, MPCQP_MAX_HORIZON] */
#define MPCQP_E_BATCH (-3)       /* B > max_batch of the workspace */
#define MPCQP_E_HIP (-4)         /* HIP runtime / launch error */
#define MPCQP_E_STATE (-5)       /* mpcqp_solve before mpcqp_build of the same B */
#define MPCQP_E_DEVICE (-6)      /* the device reported a fault at a stream synchronisation (sticky:
                                    an earlier kernel faulted; the device context is unusable) */

#define MPCQP_MAX_HORIZON 1024   /* per-QP workspace 16 (2N)^2 bytes: 67 MB at N = 1024 */
#define MPCQP_WIDE_MIN_HORIZON 33 /* N <= 32: one wave per QP (2N <= 64 variables on the lanes, the KKT
                                     inverse in registers); N >= 33: one workgroup per QP */
#define MPCQP_MID_MAX_HORIZON 64  /* 33 <= N <= 64 (fast mode): 2-4 x 1-2 waves per QP, the KKT inverse's
                                     rows split in column parts over their registers; beyond, and in
                                     reproducible mode, 256 threads restating the C code */

/* per-QP status codes (mirror OSQP's; mpc_controller.py:137 accepts 1 and 2).
 * Where the meaning differs from OSQP's: OSQP reports "solved" whenever ADMM met eps_abs/eps_rel and
 * records a failed polish separately (info.status_polish = -1, the ADMM iterate returned).  This
 * library reports that case as MPCQP_SOLVED_INACCURATE (2), the ADMM iterate returned as OSQP does,
 * so MPCQP_SOLVED (1) always means the polished exact optimum.  The reference accepts both codes
 * (mpc_controller.py:137), so its loop behaves the same; a batch consumer counting OSQP "solved"
 * should count 1 and 2 when ADMM converged (iters[1] > 0 marks that a polish ran). */
#define MPCQP_SOLVED 1            /* polish converged: exact optimum (active set reproduces itself) */
#define MPCQP_SOLVED_INACCURATE 2 /* ADMM met eps_abs/eps_rel but polish did not converge (OSQP: solved,
                                     status_polish -1), or max_iter reached within 10x the tolerances
                                     (OSQP: solved_inaccurate) */
#define MPCQP_MAX_ITER_REACHED (-2)
#define MPCQP_NUMERICAL_ERROR (-10) /* non-finite data or non-positive pivot */

/* active[] codes per soft row */
#define MPCQP_ROW_INACTIVE 0
#define MPCQP_ROW_LOWER 1         /* row value below its lower bound (slack > 0) */
#define MPCQP_ROW_UPPER 2         /* row value above its upper bound (slack > 0) */

/* solve methods */
#define MPCQP_METHOD_ADMM 0       /* OSQP algorithm: Ruiz scaling, ADMM, adaptive rho, polish */
#define MPCQP_METHOD_NEWTON 1     /* polish iteration only (semismooth Newton from the unconstrained optimum) */

/*
 * Parameter block.  Mirrors MPCParameters (mpc_controller.py:17-30) and the
 * OSQP settings of mpc_controller.py:121-131.  Matrices are row-major.
 */
typedef struct mpcqp_params {
  int32_t horizon;            /* N */
  int32_t method;             /* MPCQP_METHOD_* */
  double wheelbase_px;        /* L (config.py:79-81: wheelbase_m / map_resolution) */
  double dt;
  double q[16];               /* Q   (4x4) stage state weight, quad_form without 1/2 */
  double r[4];                /* R   (2x2) input weight */
  double q_terminal[16];      /* Q_N (4x4) */
  double u_bounds[4];         /* {a_lo, a_hi, delta_lo, delta_hi} */
  double v_bounds[2];         /* {v_lo, v_hi} */
  double du_bounds[4];        /* {da_lo, da_hi, ddelta_lo, ddelta_hi} */
  double slack_velocity;      /* w_v  (default 1e3) */
  double slack_input;         /* w_u  (default 5e2) */
  double slack_rate;          /* w_du (default 5e2) */
  /* solver settings */
  double rho;                 /* 0.1 */
  double sigma;               /* 1e-6 (OSQP default) */
  double alpha;               /* 1.6 */
  double eps_abs;             /* 1e-3 */
  double eps_rel;             /* 1e-3 */
  double adaptive_rho_tolerance; /* 5 (OSQP default) */
  int32_t max_iter;           /* 60000 */
  int32_t check_termination;  /* 25 (OSQP default) */
  int32_t scaling;            /* Ruiz iterations: 1 in this build's Python defaults (OSQP's default 10;
                                 one pass halves the ADMM iterations on these QPs) */
  int32_t adaptive_rho;       /* 1 */
  int32_t adaptive_rho_interval; /* 25 (deterministic; OSQP's default is timing based) */
  int32_t polish;             /* 1 */
  int32_t polish_max_iter;    /* 100 */
  int32_t debug_state;        /* 1: also write the per-QP solver state buffer (mpcqp_state_buffer; tests) */
  int32_t polish_from;        /* 75 (Python default): from this ADMM iteration on, every termination check also tries the
                                 polish (capped at polish_attempt_max_iter); a polish that reaches a
                                 self-consistent active set is the exact optimum and ends the solve as
                                 solved, a failed attempt resumes ADMM.  0: polish only after ADMM stops */
  int32_t polish_attempt_max_iter; /* 30 */
  double polish_near;         /* 3: also attempt the polish from iteration 2*check_termination on when
                                 both residuals are within this factor of their tolerances; 0 off */
  int32_t reproducible;       /* 0: one wave per QP for N < MPCQP_WIDE_MIN_HORIZON (fast; its wave-tree
                                 reductions round differently from the C restatement).  1: every
                                 horizon runs the workgroup-per-QP kernel, which is oracle/mpcqp_cpu.c
                                 parallelised without changing a floating-point operation: solutions,
                                 statuses and every iteration counter bit-identical to the C code given
                                 the same LTV model.  Fixed at mpcqp_create (it sizes the workspace). */
} mpcqp_params;

typedef struct mpcqp_ws mpcqp_ws;

/* ABI version (MPCQP_ABI_VERSION). */
int mpcqp_version(void);

/* Build id of this library: a hash of its sources and compile flags (__graft_entry__.source_hash),
 * compiled in by build(), which rebuilds whenever the sources' hash differs from it.  32 hex digits. */
const char* mpcqp_build_id(void);

/* Thread-local description of the last error ("" if none). */
const char* mpcqp_last_error(void);

/* Number of soft rows per QP: 5N+1 (v rows 0..N, input rows, rate rows). */
int mpcqp_num_rows(int horizon);

/* Workspace of capacity max_batch QPs on HIP device `device`.
 * Replaces the per-call cvxpy Problem construction (mpc_controller.py:53-119). */
int mpcqp_create(const mpcqp_params* p, int max_batch, int device, mpcqp_ws** ws);

/* Replace the parameter block (same horizon), e.g. for the relaxation retry of
 * control_stage.py:45-55.  Stream-ordered with respect to later launches.  Invalidates the last
 * mpcqp_build: the next mpcqp_solve returns MPCQP_E_STATE until mpcqp_build runs again, so a
 * build is always solved with the parameters it was made with. */
int mpcqp_set_params(mpcqp_ws* ws, const mpcqp_params* p);

void mpcqp_destroy(mpcqp_ws* ws);

/*
 * K1: window -> LTV model.  Per QP: np.unwrap of the reference yaw
 * (mpc_controller.py:59-60, numpy semantics) and the N Jacobians of
 * linearize() at ref[max(k-1,0)], u=0 (mpc_controller.py:65-70,108;
 * vehicle_model.py:24-45).  Inputs (device):
 *   x0     B x 4
 *   ref    B x (N+1) x 4     [x, y, yaw, v] per row, as ref_traj of solve()
 *   u_prev B x 2             (NULL = zeros, mpc_controller.py:48-49)
 * For N < MPCQP_WIDE_MIN_HORIZON (and debug_state off) this step is FUSED into the kernel of
 * the next mpcqp_solve, which reads x0 / ref / u_prev itself: the buffers must stay valid and
 * unchanged until that solve has run (stream order).  mpcqp_build then enqueues nothing.
 */
int mpcqp_build(mpcqp_ws* ws, int B, const double* x0, const double* ref, const double* u_prev,
                void* stream);

/*
 * K2: condense + (ADMM + polish | Newton) for the B QPs of the last build.
 * Outputs (device, any may be NULL except status):
 *   u0     B x 2             U[:,0]  (mpc_controller.py:141)
 *   X      B x 4 x (N+1)     predicted states, X[:,0] = x0
 *   U      B x 2 x N         inputs
 *   status B                 MPCQP_SOLVED / ... per QP
 *   iters  B x 4             {ADMM iterations, polish iterations, KKT factorizations,
 *                             line-search trials}
 *   active B x (5N+1)        MPCQP_ROW_* per soft row at the returned solution
 */
int mpcqp_solve(mpcqp_ws* ws, int B, double* u0, double* X, double* U, int32_t* status,
                int32_t* iters, uint8_t* active, void* stream);

/*
 * B = 1 low-latency path (ABI 7): the sequential closed loop of TrajectoryTracker.track solves one QP
 * per step (control_stage.py:100-129), where host overhead, not the kernel, decides the step time.
 * The workspace owns two blocks of pinned, device-mapped, coherent host memory and a private
 * non-blocking stream, allocated by the first mpcqp_stage:
 *   in   doubles: x0[4] | ref[(N+1) x 4] | u_prev[2]          (the caller writes them in place)
 *   out  bytes at offsets[0..5]: u0 (2 f64) | X (4 x (N+1) f64) | U (2 x N f64) | status (i32) |
 *        iters (4 i32) | active (5N+1 u8)                     (the kernels write them in place)
 * mpcqp_solve_staged runs mpcqp_build + mpcqp_solve for the one QP in the `in` block on that stream
 * and waits for it: one launch, no copy commands, one synchronisation.  The outputs are then in the
 * `out` block.  MPCQP_E_DEVICE when a fault surfaces at the synchronisation.
 * Replaces the per-call cvxpy build + OSQP solve of MPCController.solve (mpc_controller.py:53-141). */
int mpcqp_stage(mpcqp_ws* ws, double** in, void** out, int32_t offsets[6]);
int mpcqp_solve_staged(mpcqp_ws* ws);
/* The same contract without a launch per call: the first call starts one resident wave on the
 * workspace's stream that solves the staged QP each time this function raises a request in a
 * mailbox of mapped host memory, and publishes completion there (the call spins on it).  The wave
 * leaves after 2 ms without a request, at mpcqp_set_params and at mpcqp_destroy; the next call
 * starts it again.  One server is resident per device while its workspaces are used from one thread:
 * a request on another workspace of the same device first stops the live one (a switch costs one stop
 * and one launch).  Distinct workspaces may be served from distinct threads at the same time: each call
 * holds its own workspace's lock, and a workspace busy in a call on another thread keeps its wave (two
 * resident waves until one goes idle) instead of being stopped.  The workspace's stream has the
 * device's highest priority, so its hardware queue is not one that default-priority streams (torch's)
 * share.  While a wave is resident, a device-wide synchronisation (hipDeviceSynchronize) waits for it
 * to go idle.  A request unanswered for 30 s returns MPCQP_E_DEVICE and the workspace refuses later
 * B = 1 requests; it has told its wave to leave, and mpcqp_destroy of that workspace waits until the
 * wave has left (it may still be queued).  Horizons without the one-wave kernel (N > 32, reproducible,
 * debug builds) run mpcqp_solve_staged.  Not thread-safe per workspace (the closed loop is sequential). */
int mpcqp_solve_served(mpcqp_ws* ws);

/* Two QPs per wave for horizons N <= 15 (2N <= 30 variables: a one-wave QP leaves half its lanes on
 * padding): lanes 0-31 and 32-63 of a wave solve two QPs of the batch (mpcqp_solve with the model
 * built in the solve) or two vehicles of the fused loop (mpcqp_fleet_loop, mpcqp_swarm_loop), with
 * the results of the one-QP-per-wave kernel bit for bit.  MPCQP_PAIR_AUTO (the default) pairs once
 * a launch has more QPs than the device has wave slots (8 per CU); ON / OFF force it.  Ignored where
 * the one-wave kernel does not run (N > 15, reproducible, debug_state).  No counterpart in the
 * reference (OSQP solves one QP per call). */
#define MPCQP_PAIR_OFF 0
#define MPCQP_PAIR_ON 1
#define MPCQP_PAIR_AUTO 2
int mpcqp_set_pairing(mpcqp_ws* ws, int mode);

/*
 * Closed-loop fleet: V vehicles tracking their own references, one MPC step each per call
 * (SURVEY.md §8f row 1).  Replaces, per vehicle, one iteration of the loop body of
 * TrajectoryTracker.track (src/pipeline/control_stage.py:100-150):
 *   window gather + tail padding (:101-105), _solve_with_relaxation (:33-56, :107-110),
 *   plant f_discrete (:127, vehicle_model.py:11-21), u_prev (:129), path_idx advance
 *   (:141-145), goal test (:147-150).
 * Every pointer is caller-owned DEVICE memory; the per-vehicle loop state lives on the
 * device between calls, so a run of steps needs no host round trip.
 */
#define MPCQP_FLEET_RUNNING 0
#define MPCQP_FLEET_GOAL 1        /* hypot(state - goal) < 8 after a step (control_stage.py:147) */
#define MPCQP_FLEET_ABORTED 2     /* unsolved after relaxation (control_stage.py:108-110) */
#define MPCQP_FLEET_OUT_OF_STEPS 3 /* steps == max_steps (sim_steps) */
#define MPCQP_FLEET_REPLAN_RUNNING 4 /* transient inside mpcqp_swarm_step: off track, being replanned */
#define MPCQP_FLEET_REPLAN_ABORTED 5 /* transient inside mpcqp_swarm_step: aborted, being replanned */

typedef struct mpcqp_fleet {
  int32_t vehicles;          /* V (<= max_batch of both workspaces) */
  int32_t ref_stride;        /* rows per vehicle in ref_global */
  int32_t max_steps;         /* sim_steps: rows per vehicle in trace / u_trace */
  int32_t reserved;
  const double* ref_global;  /* V x ref_stride x 4: build_reference() output, rows >= ref_len unused */
  const int32_t* ref_len;    /* V: valid rows, >= 1 */
  const double* goal;        /* V x 2 */
  double* state;             /* V x 4 (in/out) */
  double* u_prev;            /* V x 2 (in/out) */
  int32_t* path_idx;         /* V (in/out) */
  int32_t* phase;            /* V (in/out): MPCQP_FLEET_* */
  int32_t* steps;            /* V (in/out): closed-loop steps taken = rows written to trace */
  uint8_t* mask;             /* 2 x V scratch: solve-this-QP masks (nominal, relaxed) */
  int32_t* status;           /* 2 x V out: status of the nominal / relaxed solve of the last step */
  double* u0;                /* 2 x V x 2 out: u0 of the nominal / relaxed solve of the last step */
  double* X;                 /* V x 4 x (N+1) out: prediction of the accepted solve (nullable) */
  double* trace;             /* V x max_steps x 4: state after each step, TrackingResult.states (nullable) */
  double* u_trace;           /* V x max_steps x 2: applied input of each step (nullable) */
} mpcqp_fleet;

/* One closed-loop step for every RUNNING vehicle.  The device validates each RUNNING vehicle's
 * loop state before any indexed access: ref_len outside [1, ref_stride] or path_idx < 0 ->
 * MPCQP_FLEET_ABORTED, steps outside [0, max_steps) -> MPCQP_FLEET_OUT_OF_STEPS.  `nominal` holds the base parameters,
 * `relaxed` the retry parameters of control_stage.py:45-55 (du_bounds widened by
 * (5, 0.05); the reference speed column is scaled by 0.6 on the device); both have the
 * same horizon and max_batch >= V.  Vehicles not RUNNING are skipped (their waves exit). */
int mpcqp_fleet_step(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, void* stream);

/* `steps` calls of mpcqp_fleet_step.  use_graph != 0 captures one step in a hipGraph on an
 * internal stream (ordered after / before `stream` by events) and replays it `steps` times. */
int mpcqp_fleet_run(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, int steps, int use_graph,
                    void* stream);

/* `steps` steps of every RUNNING vehicle in ONE kernel launch (ABI 6): each vehicle's wave loops
 * over its steps with no kernel boundary and no host round trip -- the same operations as
 * mpcqp_fleet_run, so every output buffer (state, u_prev, path_idx, phase, steps, trace, u_trace,
 * X, and status / u0 of each vehicle's last step) equals mpcqp_fleet_run's bit for bit (the mask
 * scratch keeps each vehicle's last-step masks).  The loop does not write debug state.  Vehicles leave
 * the loop at the goal, on abort or out of steps, so one call with steps = max_steps runs every
 * vehicle to its end.  Horizons N <= 32 in fast mode without debug_state run the fused kernel;
 * other parameter blocks (mid / long horizons, reproducible or debug_state) are executed by
 * mpcqp_fleet_run's graph path. */
int mpcqp_fleet_loop(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, int steps, void* stream);

/*
 * Batched build_reference: src/control/ref_builder.py:10-22 with
 * src/common/geometry.py:9-45 (resample_polyline, heading_from_path, curvature_slowdown) for
 * V polylines at once, one wave per polyline.  Inputs (device):
 *   pts       P_total x 2      the polylines' points, concatenated
 *   path_off  V + 1            polyline v = pts[path_off[v] .. path_off[v+1])
 *   max_points                 >= every polyline's point count (LDS staging; at most 6144)
 * Outputs (device):
 *   ref       V x ref_stride x 4   rows [x, y, yaw, v] (the reference's xref, tail-padded)
 *   ref_len   V                    rows written (>= horizon + 1; 0 for an empty polyline),
 *                                  -(rows needed) when that exceeds ref_stride (nothing written),
 *                                  MPCQP_REF_BAD_PATH when a polyline has more than max_points
 * x and y follow numpy bit for bit given the same arc lengths; hypot and atan2 are the
 * device's (within an ulp of the host libm), see tests/test_gpu_refbuild.py. */
#define MPCQP_REF_BAD_PATH (-2147483647 - 1)
int mpcqp_build_reference(int V, const double* pts, const int32_t* path_off, int max_points, double desired_speed,
                          int horizon, double dt, int ref_stride, double* ref, int32_t* ref_len, void* stream);

/*
 * Batched RRT* tree growth: RRTStarPlanner.plan's loop
 * (src/planning/rrt_star.py:201-248, helpers :320-383) for V planning problems on one
 * occupancy grid, one workgroup per problem.  The random samples (_sample, :320-325) replay
 * each problem's numpy stream exactly, from one of:
 *   samples    V x max_iterations x 2   drawn on the host, or NULL to draw on the device from
 *   rng_state  V x 4 uint64             numpy.random.default_rng(seed).bit_generator.state:
 *                                       {state lo, state hi, inc lo, inc hi} (PCG64)
 * Inputs (device):
 *   occupancy  height x width uint8, row-major, 1 = free (the inflated grid), at least 2 x 2
 *   start_goal V x 4          {start_x, start_y, goal_x, goal_y}
 * Outputs (device):
 *   nodes      V x (max_iterations + 2) x 4   {x, y, cost, parent (-1 = root)} per tree node
 *   count      V                   tree nodes (goal node included when reached)
 *   meta       V x 2               {iterations run, goal index or -1}
 */
typedef struct mpcqp_rrt_params {
  double step;            /* PlannerParameters.step (step_size, default 3) */
  double goal_radius;     /* 10 */
  double rewire_radius;   /* 20 */
  double collision_step;  /* rrt_collision_step, 0.75 */
  double goal_sample_rate; /* 0.1 (device sampling) */
  int32_t max_iterations; /* <= 5000 (LDS holds the tree) */
  int32_t width;          /* occupancy.shape[1] */
  int32_t height;         /* occupancy.shape[0] */
  int32_t reserved;
} mpcqp_rrt_params;

int mpcqp_rrt_plan(const mpcqp_rrt_params* p, int V, const uint8_t* occupancy, const double* start_goal,
                   const double* samples, const uint64_t* rng_state, double* nodes, int32_t* count, int32_t* meta,
                   void* stream);

/*
 * The planner's elementary functions over n device values, as the RRT* kernels evaluate them
 * (csrc/mpcqp_math.h) -- exposed so tests can hold them to the host's bit for bit:
 *   op 0  out0 = math.hypot(a, b) as CPython computes it (rrt_star.py:319, :362-363)
 *   op 1  _steer (rrt_star.py:307-311): out0 = atan2(a, b) (a = dy, b = dx), out1 = cos(out0),
 *         out2 = sin(out0), each correctly rounded (glibc's agree on ~99.9 % of arguments)
 */
int mpcqp_plan_math(int op, int n, const double* a, const double* b, double* out0, double* out1, double* out2,
                    void* stream);

/*
 * Path extraction + shortcut pruning for the trees mpcqp_rrt_plan grew (replaces the host
 * post-processing of src/planning/rrt_star.py:245-262 and _shortcut_prune :376-389; the
 * Catmull-Rom smoothing :264-283 stays with the caller).  Same params, occupancy and
 * nodes/count/meta as mpcqp_rrt_plan; prune = params.prune_path.
 * Outputs (device), M = max_iterations + 2:
 *   raw        V x M x 2   root -> goal node coordinates (raw_path)
 *   raw_len    V           0 when the tree has no goal node
 *   pruned     V x M x 2   the shortcut-pruned path (= raw when prune == 0 or raw_len <= 2)
 *   pruned_len V
 */
int mpcqp_rrt_paths(const mpcqp_rrt_params* p, int V, int prune, const uint8_t* occupancy, const double* nodes,
                    const int32_t* count, const int32_t* meta, double* raw, int32_t* raw_len, double* pruned,
                    int32_t* pruned_len, void* stream);

/*
 * Centripetal Catmull-Rom smoothing (src/planning/rrt_star.py:104-159 with _dedupe_consecutive
 * :93-101, applied at :264-283) of V paths on the device, one wave each: path v = in[v * in_stride
 * .. + in_len[v]) points (x, y), out[v * out_stride ..] and out_len[v] points (-1: more than
 * out_stride points, or more than 4096 after deduplication).  The knot powers |d|^alpha are the
 * device's (sqrt for alpha = 0.5), within an ulp of the host libm's.
 */
int mpcqp_catmull_rom(int V, const double* in, const int32_t* in_len, int in_stride, int samples, double alpha,
                      double dedupe_tol, double* out, int32_t* out_len, int out_stride, void* stream);

/*
 * The config-5 swarm: one mpcqp_fleet_step plus, in the same step and on
 * the device, the replan trigger of the reference's roadmap (README.md:146-148) and the
 * replanning: a RUNNING vehicle farther than replan_distance from ref_global[path_idx] after its
 * step, or a vehicle the step ABORTED, with replans left (replans[v] < max_replans), is planned
 * again from where it stands to its goal -- RRT* (mpcqp_rrt_plan with the PCG64 state
 * rng_table[v][replans[v]]), path extraction + pruning, Catmull-Rom, build_reference -- and when
 * that yields a reference it continues on it from path_idx 0 (pose, speed and u_prev carry over);
 * otherwise it keeps its reference (or stays ABORTED).  Each attempt uses one replan.
 * The swarm WRITES the fleet's ref_global / ref_len rows of replanned vehicles.
 * Every pointer is caller-owned device memory; M = rrt.max_iterations + 2, S = fleet ref_stride.
 */
typedef struct mpcqp_swarm {
  mpcqp_rrt_params rrt;      /* planner parameters and grid size */
  const uint8_t* occupancy;  /* rrt.height x rrt.width, 1 = free (the inflated grid) */
  int32_t prune;             /* PlannerParameters.prune_path */
  int32_t spline_samples;    /* PlannerParameters.spline_samples (<= 1: no smoothing) */
  double spline_alpha;       /* 0.5 */
  double dedupe_tol;         /* 1e-9 */
  double desired_speed;      /* build_reference speed (px/s) */
  double dt;                 /* build_reference dt */
  int32_t horizon;           /* build_reference horizon (tail padding to horizon + 1 rows) */
  int32_t max_replans;       /* replans per vehicle (0: the plain fleet step) */
  double replan_distance;    /* off-track trigger in px (<= 0: only aborted vehicles replan) */
  int32_t path_cap;          /* smoothed-path capacity per vehicle (points) */
  int32_t reserved;
  const uint64_t* rng_table; /* V x max_replans x 4: PCG64 states {state lo, hi, inc lo, hi} */
  int32_t* replans;          /* V in/out: replans used (set >= max_replans to never replan) */
  int32_t* replan_step;      /* V x max_replans out (nullable): steps[v] at each replan, -steps-1 if it failed */
  /* scratch */
  double* start_goal;        /* V x 4 */
  double* nodes;             /* V x M x 4 */
  int32_t* count;            /* V */
  int32_t* meta;             /* V x 2 */
  double* raw;               /* V x M x 2 */
  int32_t* raw_len;          /* V */
  double* pruned;            /* V x M x 2 */
  int32_t* pruned_len;       /* V */
  double* smooth;            /* V x path_cap x 2 */
  int32_t* smooth_len;       /* V */
  double* new_ref;           /* V x S x 4 */
  int32_t* new_len;          /* V */
} mpcqp_swarm;

/* One closed-loop step of every RUNNING vehicle (mpcqp_fleet_step) + trigger + replanning. */
int mpcqp_swarm_step(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, const mpcqp_swarm* s, void* stream);

/* `steps` swarm steps; use_graph != 0 replays one captured step as a hipGraph (no host round trip). */
int mpcqp_swarm_run(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, const mpcqp_swarm* s, int steps,
                    int use_graph, void* stream);

/* The whole swarm run (every vehicle to its goal, abort or max_steps) as max_replans + 1 launches of
 * the fused fleet loop (mpcqp_fleet_loop) with the replan trigger inside -- a vehicle leaves its loop
 * when the trigger fires -- and the replanning kernels between them (ABI 6).  The same operations per
 * vehicle as mpcqp_swarm_run to the end, so every fleet and swarm output buffer equals it bit for bit.
 * Parameter blocks without the fused kernel run mpcqp_swarm_run(max_steps, graph). */
int mpcqp_swarm_loop(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, const mpcqp_swarm* s, void* stream);

/*
 * Occupancy inflation: src/maps/inflate.py:18-51 (the fallback
 * dilation the reference uses without OpenCV) for B grids of height x width uint8
 * (1 = free, 0 = obstacle): out = 0 within the disk dx^2 + dy^2 <= r^2 of an obstacle.
 * radius_px <= 0 copies.  Device pointers, out != occupancy.
 */
int mpcqp_inflate(int B, int height, int width, int radius_px, const uint8_t* occupancy, uint8_t* out, void* stream);

/* Workspace device buffers (for tests / inspection), layouts documented in DESIGN.md:
 *   model: K1 output, B x mpcqp_model_stride(N) doubles
 *   state: scaled QP + ADMM iterate (K2a/K2b output), B x mpcqp_state_stride(N) doubles
 * Both are allocated (max_batch QPs) at the first call that writes them: mpcqp_create for the
 * long-horizon kernels, else an mpcqp_build with debug_state = 1 (model and state) or the stepped
 * fleet (model).  The fused one-wave solve uses neither; NULL until then.  A first use inside a
 * stream capture returns MPCQP_E_STATE (allocation cannot be captured): run it once uncaptured. */
const double* mpcqp_model_buffer(const mpcqp_ws* ws);
int mpcqp_model_stride(int horizon);
const double* mpcqp_state_buffer(const mpcqp_ws* ws);
int mpcqp_state_stride(int horizon);
/* Per-QP doubles of this workspace's state buffer (its kernel: mpcqp_params.reproducible). */
int mpcqp_ws_state_stride(const mpcqp_ws* ws);

/* Test hook: applies the kernels' 64-lane wavefront primitives (DPP prefix/suffix scans,
 * reductions, lane shifts) to in[64] -> out[10 x 64] on the device. */
int mpcqp_debug_wave_ops(const double* in, double* out, void* stream);

/* Test hook for the B = 1 server's failure paths: mode 1 refuses the next server launch
 * (MPCQP_E_HIP), mode 2 makes the live wave leave without telling the host (the next request finds it
 * gone and relaunches it), mode 3 returns 1 while a server is believed resident, else 0. */
int mpcqp_debug_serve_fault(mpcqp_ws* ws, int mode);

/* Diagnostic builds only (-DMPCQP_STAMPS; the measured library returns MPCQP_E_ARG):
 * per-phase s_memtime cycle sums over all waves since the last reset. */
int mpcqp_debug_stamps(unsigned long long* out32, int reset);

#ifdef __cplusplus
}
#endif

#endif /* MPCQP_H */
