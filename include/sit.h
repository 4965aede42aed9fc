/*
 * sit.h — C ABI of the MI355X-native ship-in-transit (SIT) environment step.
 *
 * This is the drop-in boundary for the one hot path of AndreasKing-Goks/sac-maritime-ast:
 * the two-ship `MultiShipRLEnv` (RLEnv/MSRL_Env.py:37-450, completed by
 * RLEnv/MSRL_env_ex.py:450-980) stepping the ship-in-transit simulator
 * (the simulators/ship_in_transit package).  One handle holds N independent two-ship
 * environments ("envs"): ship type 0 is the ship under test, type 1 the obstacle
 * ship whose route the AST sampler perturbs with intermediate waypoints (IWs).
 *
 * Conventions
 *  - Plain C types only; no HIP/torch types cross the boundary.  `stream` is a
 *    hipStream_t passed as void* (NULL = default stream).
 *  - "real" below means float32 when the handle was created with SIT_F32 and
 *    float64 with SIT_F64.  Every per-step array argument is a DEVICE pointer
 *    owned by the caller; setup calls (sit_load_*) take HOST pointers.
 *  - Every entry point returns SIT_OK (0) or a negative SIT_E_* code; the message
 *    is available from sit_last_error().  No exception crosses the ABI.
 *  - Calls are stream-ordered and asynchronous.  A handle must not be used from two
 *    host threads at once; independent handles (one per GPU/stream) are independent.
 *
 * Reference interface each entry point replaces (file:line in the reference):
 *   sit_create / sit_load_*   MultiShipRLEnv.__init__ + ShipAssets    MSRL_Env.py:25-116,
 *                             ShipModelAST/ShipMachineryModel/controllers constructors
 *                             (ship_model.py:563-574, ship_engine.py:298-353,
 *                              controllers.py:114-136, 253-296), PolygonObstacle obstacle.py:98-124
 *   sit_reset                 MultiShipRLEnv.reset                    MSRL_Env.py:147-188
 *   sit_init_step             MultiShipRLEnv.init_step                MSRL_Env.py:190-217
 *   sit_step                  MultiShipRLEnv.step                     MSRL_Env.py:404-442
 *                             (+ reward_function                      MSRL_env_ex.py:906-980)
 *   sit_rollout               K x step with the driver loop of test_beds/main_ast.py:310-412
 *                             (the consumer ast_core/samplers/intermediate_waypoint_sampler.py
 *                              is empty in the reference; the synthetic sampler is SURVEY §8(d))
 *   sit_get_state/set_state   (no reference counterpart: SoA export/import for teacher-forced
 *                              parity and checkpointing)
 */
#ifndef SIT_H
#define SIT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIT_ABI_VERSION 1

/* ---- return codes ---------------------------------------------------------------- */
#define SIT_OK 0
#define SIT_E_INVALID (-1)   /* bad argument (null pointer, out-of-range size, ...) */
#define SIT_E_HIP (-2)       /* a HIP runtime call failed */
#define SIT_E_NOMEM (-3)     /* device allocation failed */
#define SIT_E_STATE (-4)     /* call out of order (e.g. stepping before routes are loaded) */

/* ---- precision of a handle -------------------------------------------------------- */
#define SIT_F32 32
#define SIT_F64 64

/* ---- hybrid shaft generator state (ship_engine.py:32-76) --------------------------- */
#define SIT_SG_MOTOR 0 /* 'MOTOR' (PTI)  */
#define SIT_SG_GEN 1   /* 'GEN'   (PTO)  */
#define SIT_SG_OFF 2   /* anything else  */

/* ---- machinery model (sit_params.machinery_model) ---------------------------------- */
#define SIT_MACH_SHAFT 0      /* ShipMachineryModel: shaft speed ODE, thrust = k D^4 w|w| (ship_engine.py:298-395) */
#define SIT_MACH_SIMPLIFIED 1 /* SimplifiedMachineryModel: first-order thrust-force lag (ship_engine.py:398-433)
                               * with ThrottleFromSpeedSetPointSimplifiedPropulsion (controllers.py:154-172);
                               * the shaft_speed state holds the thrust force [N], see sit_params */

/* ---- status bitmask: one bit per reference status string, in the order the
 *      reference concatenates them (MSRL_env_ex.py:755-803, 830-874, 897-899) ------- */
#define SIT_ST_TEST_ENDPOINT (1u << 0)   /* "|Test ship reaches endpoint|"             */
#define SIT_ST_TEST_HORIZON (1u << 1)    /* "|Test ship hits map horizon|"             */
#define SIT_ST_TEST_TERRAIN (1u << 2)    /* "|Test ship collides with the terrain|"    */
#define SIT_ST_TEST_MECHANICAL (1u << 3) /* "|Test ship mechanical failure|"           */
#define SIT_ST_TEST_NAVIGATION (1u << 4) /* "|Test ship navigation failure|"           */
#define SIT_ST_TEST_BLACKOUT (1u << 5)   /* "|Test ship blackout failure|"             */
#define SIT_ST_OBS_ENDPOINT (1u << 6)    /* "|Obstacle ship reaches endpoint|"         */
#define SIT_ST_OBS_HORIZON (1u << 7)     /* "|Obstacle ship hits map horizon|"         */
#define SIT_ST_OBS_TERRAIN (1u << 8)     /* "|Obstacle ship collides with the terrain|"*/
#define SIT_ST_OBS_IW_TERMINAL (1u << 9) /* "|Obstacle ship IW sampled in terminal state|" */
#define SIT_ST_OBS_NAVIGATION (1u << 10) /* "|Obstacle ship navigation failure|"       */
#define SIT_ST_COLLISION (1u << 11)      /* "|Ship collision|"                         */
#define SIT_ST_TEST_DONE (1u << 12)      /* test ship terminal  (else "|Test ship not in terminal state|")     */
#define SIT_ST_OBS_DONE (1u << 13)       /* obstacle ship terminal (else "|Obstacle ship not in terminal state|") */
#define SIT_ST_NO_STEP (1u << 30)        /* policy mode: the env waited for its action; no step taken in this row */
#define SIT_ST_ROUTE_OVERFLOW (1u << 31) /* IW insertion dropped: route table full (no reference counterpart) */

/* ---- next_state layout (MSRL_Env.py:426-437) --------------------------------------- */
#define SIT_OBS_DIM 10 /* test n,e,psi,rpm,|e_ct|,P_me[kW], obs n,e,psi,|e_ct| */
/* ---- replay transition record (memory.push, test_beds/main_ast.py:385-396) ----------
 *   [0:10] state (the observation before the step; reset()'s array at an episode start)
 *   [10] action: the SAC action of the event in [-1, 1] (the route angle a = action * pi/6; the
 *        synthetic sampler's U[-1, 1] draw or the policy's squashed action; NaN in explicit mode),
 *   [11] reward, [12:22] next_state,
 *   [22] mask (1 if the episode step reaches mask_horizon, else not done), [23] env id */
#define SIT_TRANSITION_DIM 24
/* Trajectory log rows per env and step (sit_rollout_args.log): ShipModelAST.store_simulation_data's
 * 27 keys (ship_model.py:645-684, in that order: time [s], north/east position [m], yaw angle
 * [deg], rudder angle [deg], forward/sideways speed [m/s], yaw rate [deg/sec], propeller shaft
 * speed [rpm], commanded load fraction me/hsg [-], power me [kw], available power me [kw], power
 * electrical [kw], available power electrical [kw], power [kw], propulsion power [kw], fuel
 * rate me/hsg/total [kg/s], fuel consumption me/hsg/total [kg], motor torque [Nm], thrust force
 * [kN], cross track error [m], heading error [deg] (radians, as the reference stores it)) for
 * the ship under test (rows 0-26) and the obstacle ship (rows 27-53), then the 8 per-step terms
 * whose per-episode sums are MultiShipRLEnv.reward_results (MSRL_env_ex.py:926-964): test
 * reward_e_ct, reward_near_col, total_non_terminal; obstacle reward_base, reward_e_ct,
 * reward_near_col, total_non_terminal; shared total_non_terminal (rows 54-61). */
#define SIT_LOG_KEYS 27
#define SIT_LOG_ROWS 62

/* ---- per-ship initial values for sit_load_initial ---------------------------------- */
enum {
  SIT_INIT_NORTH = 0,      /* SimulationConfiguration.initial_north_position_m           */
  SIT_INIT_EAST,           /* initial_east_position_m                                    */
  SIT_INIT_YAW,            /* initial_yaw_angle_rad                                      */
  SIT_INIT_SURGE,          /* initial_forward_speed_m_per_s                              */
  SIT_INIT_SWAY,           /* initial_sideways_speed_m_per_s                             */
  SIT_INIT_YAW_RATE,       /* initial_yaw_rate_rad_per_s                                 */
  SIT_INIT_SHAFT_SPEED,    /* initial_propeller_shaft_speed_rad_per_s (ship_model.py:567) */
  SIT_INIT_DESIRED_SPEED,  /* ShipAssets.desired_forward_speed (MSRL_Env.py:30)           */
  SIT_INIT_SHIP_SPEED_I,   /* ship-speed PI initial integral (controllers.py:122-124: 0)  */
  SIT_INIT_SHAFT_SPEED_I,  /* initial_shaft_speed_integral_error (controllers.py:119, 129) */
  SIT_INIT_NF
};

/* ---- configuration: the reference's NamedTuple fields, verbatim ------------------- */
typedef struct sit_params {
  /* ShipConfiguration (ship_model.py:20-35) */
  double dead_weight_tonnage;
  double coefficient_of_deadweight_to_displacement;
  double bunkers;
  double ballast;
  double length_of_ship;
  double width_of_ship;
  double added_mass_coefficient_in_surge;
  double added_mass_coefficient_in_sway;
  double added_mass_coefficient_in_yaw;
  double mass_over_linear_friction_coefficient_in_surge;
  double mass_over_linear_friction_coefficient_in_sway;
  double mass_over_linear_friction_coefficient_in_yaw;
  double nonlinear_friction_coefficient_in_surge;
  double nonlinear_friction_coefficient_in_sway;
  double nonlinear_friction_coefficient_in_yaw;
  /* EnvironmentConfiguration (ship_model.py:38-42) */
  double current_velocity_component_from_north;
  double current_velocity_component_from_east;
  double wind_speed;
  double wind_direction;
  /* wind model constants hard-coded in BaseShipModel (ship_model.py:123-130) */
  double rho_air;
  double front_height;
  double side_height;
  double cx;
  double cy;
  double cn;
  /* SimulationConfiguration.integration_step (ship_model.py:52) */
  double integration_step;
  /* MachinerySystemConfiguration (ship_engine.py:121-138) and the selected MachineryMode */
  double hotel_load;
  double main_engine_capacity;   /* MachineryModeParams of the operating mode */
  double electrical_capacity;
  int32_t shaft_generator_state; /* SIT_SG_* */
  int32_t machinery_model;       /* SIT_MACH_* (0 = the reference's ShipModelAST machinery)  */
  double rated_speed_main_engine_rpm;
  double linear_friction_main_engine;
  double linear_friction_hybrid_shaft_generator;
  double gear_ratio_between_main_engine_and_propeller;
  double gear_ratio_between_hybrid_shaft_generator_and_propeller;
  double propeller_inertia;
  double propeller_speed_to_torque_coefficient;
  double propeller_diameter;
  double propeller_speed_to_thrust_force_coefficient;
  double rudder_angle_to_sway_force_coefficient;
  double rudder_angle_to_yaw_force_coefficient;
  double max_rudder_angle_degrees;
  /* ThrottleControllerGains (controllers.py:16-20) */
  double kp_ship_speed;
  double ki_ship_speed;
  double kp_shaft_speed;
  double ki_shaft_speed;
  /* HeadingControllerGains (controllers.py:23-26) */
  double heading_kp;
  double heading_kd;
  double heading_ki;
  /* LosParameters (LOS_guidance.py:15-19) */
  double radius_of_acceptance;
  double lookahead_distance;
  double los_integral_gain;
  double integrator_windup_limit;
  /* env args (test_policy.py:39-42) and reward constants of MSRL_env_ex.py */
  double theta;                  /* navigation-failure coefficient (:569)      */
  int32_t sampling_frequency;    /* AB segment divisor (:125)                  */
  int32_t collision_bias;        /* 1 = reference behaviour: always on (MSRL_Env.py:98-99, 242) */
  double e_tolerance;            /* 1000 (:119)                                */
  double arrival_radius;         /* 200  (:754, :829)                          */
  double shaft_rpm_max;          /* 2000 (:557)                                */
  double minimum_ship_distance;  /* 50   (:592)                                */
  double bias_throttle_scale;    /* 0.5  (MSRL_Env.py:246)                     */
  double bias_throttle_max;      /* 1.1  (MSRL_Env.py:247)                     */
  double bias_rudder_degrees;    /* 3    (MSRL_Env.py:250)                     */
  /* specific fuel consumption a x^2 + b x + c [g/kWh] of the main engine and the diesel
   * generators (MachinerySystemConfiguration, ship_engine.py:137-138, 89-115; test_policy.py:
   * 162-163): logging only (trajectory log, fuel keys) */
  double fuel_me_a, fuel_me_b, fuel_me_c;
  double fuel_dg_a, fuel_dg_b, fuel_dg_c;
  /* SIT_MACH_SIMPLIFIED only (SimplifiedPropulsionMachinerySystemConfiguration, ship_engine.py:
   * 148-157): thrust_force_dynamic_time_constant [s].  In that mode the ship-speed PI gains
   * kp_ship_speed / ki_ship_speed are ThrottleFromSpeedSetPointSimplifiedPropulsion's kp / ki
   * (throttle saturated to [0, 1.1]), the shaft-speed PI is unused, the shaft_speed state and
   * SIT_INIT_SHAFT_SPEED hold the thrust force [N] (initial_thrust_force), and the observed shaft
   * speed is 0 (the model has no shaft, so no mechanical failure). */
  double thrust_force_dynamic_time_constant;
} sit_params;

/* Fill `p` with the configuration of test_beds/test_policy.py:94-226 (PTI mode). */
void sit_params_default(sit_params* p);
/* sizeof(sit_params) as compiled into the library (binding layout check). */
size_t sit_params_size(void);

/* ---- handle lifecycle ------------------------------------------------------------- */
typedef struct sit_handle sit_handle;

/* Create N envs on the current HIP device.  `wpt_capacity` bounds the waypoints of one
 * ship's route including start and end (IW insertions beyond it set
 * SIT_ST_ROUTE_OVERFLOW and are dropped).  `precision` is SIT_F32 or SIT_F64. */
int sit_create(const sit_params* p, int32_t n_env, int32_t wpt_capacity, int32_t precision,
               sit_handle** out);
void sit_destroy(sit_handle* h);
/* Last error message of `h`, or of the failed sit_create on this thread when h == NULL. */
const char* sit_last_error(const sit_handle* h);
int32_t sit_abi_version(void);
int32_t sit_precision(const sit_handle* h);
int32_t sit_n_env(const sit_handle* h);
/* Instantiation name of the step kernel the last sit_step / sit_rollout launch of `h` ran, e.g.
 * "k_env_steps_sync<float,kSynth,MACH=0>" (diagnostics and bench labels; "" before the first). */
const char* sit_step_kernel(const sit_handle* h);

/* ---- setup (host pointers) --------------------------------------------------------- */
/* Island map: PolygonObstacle(list_of_vertices_list) (obstacle.py:98-124).  Vertices are
 * (east, north) pairs exactly as in the reference; polygon p owns vertices
 * [vert_offsets[p], vert_offsets[p+1]).  The ring is closed implicitly. */
int sit_load_map(sit_handle* h, int32_t n_poly, const int32_t* vert_offsets,
                 const double* verts_en);
/* Routes: wpt_ne[env][ship][i][2] = (north, east) for i < n_wpt[env][ship], laid out with
 * stride wpt_capacity in i (NavigationSystem.load_waypoints, LOS_guidance.py:65-86). */
int sit_load_routes(sit_handle* h, const double* wpt_ne, const int32_t* n_wpt);
/* Construction-time values: init[env][ship][SIT_INIT_NF]. */
int sit_load_initial(sit_handle* h, const double* init);
/* Spatial-index statistics of the loaded map (diagnostics; no reference counterpart):
 * info[0] bytes of the map blob staged into LDS per step-kernel block, [1] mixed class cells
 * with a point-in-polygon record, [2] live edge entries of those records, [3] nearest-edge
 * grid and bands in use, [4] cell records in use, [5] LDS bytes per block for the map.
 * Writes min(n, 6) values. */
int sit_map_info(const sit_handle* h, int64_t* info, int32_t n);
/* The step kernel's map predicates at arbitrary points (test/diagnostic entry; the reference
 * counterparts are PolygonObstacle.obstacles_distance / Polygon.contains / is_pos_inside_obstacles,
 * obstacle.py:126-141, MSRL_env_ex.py:490-515), through the same spatial index:
 *   pts_ne real[n][2] (north, east); dist real[n] boundary distance; inside u8[n] point strictly
 *   inside a polygon; hull u8[n] any hull corner (+-l/2) inside.  Device pointers; any output may
 *   be NULL. */
int sit_probe_map(sit_handle* h, int32_t n, const void* pts_ne, void* dist, uint8_t* inside,
                  uint8_t* hull, void* stream);
/* Self-test of the IEEE float64 helpers the knife-edge decisions use (diagnostic; no reference
 * counterpart): out[i] = op(a[i], b[i]) with op 0 a / b, 1 sqrt(a), 2 a*a + b*b, 3 (a + b) - a,
 * 4 a*b + b*a (each correctly rounded per operation, as numpy's float64), 5 sin(a), 6 cos(a),
 * 7 atan2(a, b) (the device math library the float64 path uses), 8 the fused step kernel's wave
 * roles (sync_role_of) for the SIMD assignment a (base 4, digit v = SIMD of wave v) and CU ticket b,
 * packed as role of wave v in base-4 digit v, 9 / 10 sin / cos of (float)a as the float32 step takes
 * them (xsincos), 11 atan((float)a), 12 atan2((float)a, (float)b) in float32, each widened to
 * float64.  fast_tu != 0 runs the copy compiled with the float32
 * step kernels' fast-math flags.  Device pointers. */
int sit_selftest_f64(int32_t op, int32_t n, const double* a, const double* b, double* out, int32_t fast_tu,
                     void* stream);
/* Debug builds (libsit_debug.so, compiled with -DSIT_DEBUG; no reference counterpart): every table
 * index the step kernels compute is bounds-checked; a failed check sets bit i of the returned word
 * (0 route-table row, 1 next-waypoint index, 2 route length, 3 spatial-index entry or range, 4 edge
 * id, 5 class-grid word, 6 mixed-cell record or live-edge range, 7 in-kernel serving: a block's
 * published request count outside [0, 64] or its LDS past the launch's dynamic LDS, 8 in-kernel
 * serving: a served env id outside [0, n_env)), and every table read or write it guards is
 * clamped into its table (indices to a valid entry, ranges to their in-table part; the next-waypoint
 * and route-length checks guard the route-table rows of bit 0), so the launch completes without an
 * out-of-bounds access.  sit_debug_flags synchronises the device, returns the bits set since the last
 * call and clears them; release builds return 0.  sit_debug_build: 1 in a debug build. */
int sit_debug_flags(uint32_t* flags);
int32_t sit_debug_build(void);
/* Placement record of the fused two-wave step kernel (no reference counterpart): the number of
 * blocks, since the last reset, whose four waves did not sit on four different SIMDs.  Roles are a
 * permutation of D0, D1, P0, P1 for every placement (results never depend on it); the count shows
 * how often the issue-priority pairing the kernel is tuned for was not available.  Synchronises the
 * device; reset != 0 clears the count. */
int sit_role_fallbacks(uint64_t* count, int32_t reset);
/* Put every env into its construction-time state (as if freshly built).  Unlike
 * sit_reset this also re-initialises the shaft speed and all controller integrators. */
int sit_restart(sit_handle* h, void* stream);

/* ---- stepping (device pointers, stream-ordered) ------------------------------------ */
/* MultiShipRLEnv.reset for envs with env_mask[e] != 0 (NULL = all).  Keeps shaft speed and
 * all PI/PID integrator states, as the reference does.  If initial_state is not NULL it
 * receives the construction-time observation of every env, real[n_env][SIT_OBS_DIM]. */
int sit_reset(sit_handle* h, const uint8_t* env_mask, void* initial_state, void* stream);
/* MultiShipRLEnv.init_step for masked envs (NULL = all). */
int sit_init_step(sit_handle* h, const uint8_t* env_mask, void* stream);
/* MultiShipRLEnv.step for all envs.
 *   action_ne  real[n_env][2]  converted_action = intermediate waypoint (north, east)
 *   sac_update u8[n_env]       SAC_update: insert the IW into the obstacle ship's route
 *   init       u8[n_env]       init: first step of an episode (no distance accounting)
 *   next_state real[n_env][SIT_OBS_DIM], reward real[n_env], done u8[n_env], status u32[n_env]
 *   done_count int32[1] or NULL: += number of envs with done (wave ballot reduction)
 * next_state (and action_out below) must be aligned to 2 reals (SIT_E_INVALID otherwise). */
int sit_step(sit_handle* h, const void* action_ne, const uint8_t* sac_update,
             const uint8_t* init, void* next_state, void* reward, uint8_t* done,
             uint32_t* status, int32_t* done_count, void* stream);
/* MultiShipRLEnv.step with HOST arrays (the scalar drop-in, compat.MultiShipRLEnv.step; the reference
 * API is synchronous): the same step as sit_step, with the arrays above in host memory and
 *   log   real[SIT_LOG_ROWS][n_env] or NULL: the step's trajectory-log row (sit_rollout_args.log)
 *   state sit_state_bytes() bytes or NULL: the state blob after the step (sit_get_state)
 * The inputs go into the handle's pinned, coherent host staging, which the step kernel reads and
 * writes directly (no copy call); one launch, one copy of the state blob when asked, one
 * synchronisation of `stream`, then the outputs are copied to the caller's arrays.  Any output may be
 * NULL.  Returns after the step has completed. */
int sit_step_host(sit_handle* h, const void* action_ne, const uint8_t* sac_update, const uint8_t* init,
                  void* next_state, void* reward, uint8_t* done, uint32_t* status, void* log, void* state,
                  void* stream);

/* K fused steps.  With action_ne == NULL the synthetic AST sampler drives the obstacle
 * ship: a sampling event happens on the first step of an episode and
 * whenever the obstacle ship's sampling distance reaches AB_len; it draws
 * a ~ U[-pi/6, pi/6] from Philox4x32-10(key = seed, counter = (env_id, event, 0x5A4D, 0))
 * and inserts IW = (n + AB_len cos(AB_alpha + a), e + AB_len sin(AB_alpha + a)).
 * Otherwise action_ne/sac_update/init are [n_steps][n_env] explicit inputs.
 * With auto_reset != 0, an env whose step returned done is reset, init-stepped and
 * restarted at episode step 1 before its next step (test_beds/main_ast.py:310-330).
 * Output arrays are [n_steps][n_env]...; any may be NULL except that at least one of
 * next_state/reward must be given.  action_out (real[n_steps][n_env][4]) receives
 * (IW north, IW east, scoping angle a, SAC_update) of every step. */
typedef struct sit_rollout_args {
  int32_t n_steps;
  int32_t auto_reset;
  uint64_t seed;
  int64_t env_id_offset;     /* global id of env 0 (for sharding across GPUs) */
  const void* action_ne;     /* real[n_steps][n_env][2] or NULL (synthetic sampler) */
  const uint8_t* sac_update; /* u8[n_steps][n_env] (explicit mode only) */
  const uint8_t* init;       /* u8[n_steps][n_env] (explicit mode only) */
  void* next_state;          /* real[n_steps][n_env][SIT_OBS_DIM] or NULL */
  void* reward;              /* real[n_steps][n_env] or NULL */
  uint8_t* done;             /* u8[n_steps][n_env] or NULL */
  uint32_t* status;          /* u32[n_steps][n_env] or NULL */
  void* action_out;          /* real[n_steps][n_env][4] or NULL */
  int32_t* done_count;       /* int32[n_steps] or NULL: += envs done at each step */
  /* sampling-event transitions (synthetic sampler mode): one record per step whose
   * SAC_update is set, appended at transition_count (atomic); records beyond
   * transition_capacity are counted but not written */
  void* transitions;          /* real[transition_capacity][SIT_TRANSITION_DIM] or NULL, 4-real aligned */
  int32_t* transition_count;  /* int32[1] */
  int32_t transition_capacity;
  int32_t mask_horizon;       /* args.num_steps_episode (main_ast.py:71, 387); 0 = none */
  /* Policy mode (action_ne == NULL, policy_action != NULL): the actions of sampling events come
   * from a policy evaluated between launches (the SAC actor, agent.select_action mode 1,
   * main_ast.py:344-349).  At a sampling event an env consumes policy_action[e] if
   * policy_ready[e] == SIT_POLICY_READY (route angle a = policy_action[e] * pi/6, IW as in the
   * synthetic sampler); otherwise it takes no further step in this launch (its rows get status
   * SIT_ST_NO_STEP and done 0).  At the end of the launch policy_ready[e] is SIT_POLICY_WAITING
   * for every env stopped at a sampling event, SIT_POLICY_READY for an env holding an unused
   * action, else 0.
   * Admission (after the step kernel, same call, same stream; deterministic): the waiting envs
   * enter the request queue oldest request first, ties by env id, at most request_capacity of
   * them; request_age[e] counts the admission rounds env e has waited (kept by the library,
   * zero-initialised by the caller).  An env that starts waiting in launch L is admitted at the
   * latest in round L + ceil(n_env / request_capacity) - 1 (exact while ceil(n_env / request_capacity) < 16).  The
   * queue rows are in env-id order: request_env[q] = e, request_obs[q] = the observation the env
   * waits at (state field last_obs), request_noise[q] = N(0,1) from Philox4x32-10(key = seed,
   * counter = (env_id, event, 0x504F, 0)) (Box-Muller), *request_count = rows.  Which envs step
   * how many rows is therefore a function of (scenario, seed, request_capacity, n_steps, actions),
   * never of scheduling.  The caller runs the policy on the queue and writes policy_action /
   * policy_ready = SIT_POLICY_READY for the queued envs before the next launch (sit_policy_actor
   * does both).  Per-env trajectories equal those of a synchronous per-step loop. */
  const void* policy_action;  /* real[n_env] in [-1, 1] */
  int32_t* policy_ready;      /* int32[n_env]: 0, SIT_POLICY_READY or SIT_POLICY_WAITING */
  int32_t* request_env;       /* int32[request_capacity] */
  void* request_noise;        /* real[request_capacity] */
  void* request_obs;          /* real[request_capacity][SIT_OBS_DIM]: the waiting env's state */
  int32_t* request_count;     /* int32[1] */
  int32_t request_capacity;
  int64_t* env_steps;         /* int64[1] or NULL: += env-steps executed (policy mode) */
  /* Trajectory log (optional): real[n_steps][SIT_LOG_ROWS][n_env].  The obstacle ship's stop
   * path repeats its last logged row with the time updated (store_last_simulation_data), and
   * the fuel consumption accumulates over logged steps only (logging-only quantities). */
  void* log;
  int32_t* request_age;       /* int32[n_env] (policy mode): admission rounds waited, see above */
  /* In-kernel serving (policy mode, optional).  With actor_weights != NULL the launch evaluates the
   * actor itself — sit_policy_actor's network, weight layout and head, in float32, on the observation
   * each env waits at and its event's normal draw (as request_obs / request_noise above) — for every
   * env that ends the launch waiting, at the end of the same launch: policy_action[e] = its squashed
   * action, policy_ready[e] = SIT_POLICY_READY (never SIT_POLICY_WAITING), *actor_served += the envs
   * served.  No queue and no capacity: request_env/noise/obs/count/age may be NULL and
   * request_capacity is ignored.  An env stopped at a sampling event steps again from the start of the
   * next launch, and every env's rows equal those of the queued path with request_capacity = n_env
   * and sit_policy_actor, bit for bit.  (Logged launches, which run the one-wave kernel, are served
   * through the library's own queue of capacity n_env and sit_policy_actor, with the same result.) */
  const float* actor_weights;  /* float32[SIT_ACTOR_WEIGHTS] (sit_policy_actor's layout) or NULL */
  int32_t actor_deterministic; /* nonzero: x = mu (no sampling noise) */
  int64_t* actor_served;       /* int64[1] or NULL: += envs served */
} sit_rollout_args;
#define SIT_POLICY_READY 1    /* policy_ready: an action waits in policy_action[e] */
#define SIT_POLICY_WAITING 2  /* policy_ready: the env stopped at a sampling event for its action */
int sit_rollout(sit_handle* h, const sit_rollout_args* a, void* stream);
size_t sit_rollout_args_size(void);
/* Policy mode helper: the squashed Gaussian head of the actor (ast_core/distributions/normal.py:
 * 88-101, ast_core/policies/gaussian_policy.py:71-72) applied to the actor network's output and
 * scattered into the env action slots, for request rows q < *request_count:
 *   x = mu + exp(clip(log_sigma, -20, 2)) * noise[q]   (x = mu when deterministic != 0)
 *   policy_action[request_env[q]] = tanh(x); policy_ready[request_env[q]] = 1
 * head real[capacity][head_stride] holds (mu, log_sigma) in its first two columns.
 *   served   int64[1] or NULL: += min(*request_count, capacity) (the policy evaluations used, as
 *            sit_policy_actor counts them) */
int sit_policy_apply(sit_handle* h, int32_t capacity, const void* head, int32_t head_stride,
                     const void* noise, const int32_t* request_env, const int32_t* request_count,
                     int32_t deterministic, void* policy_action, int32_t* policy_ready, int64_t* served,
                     void* stream);
/* Policy mode helper, the whole actor in one kernel: the SAC-AST Gaussian policy's MLP
 * (ast_core/nn_models/mlp.py:95-148: obs[SIT_OBS_DIM] -> 256 -> ReLU -> 256 -> ReLU -> (mu, log_sigma),
 * main_ast.py:67's hidden sizes) in float32 on request rows q < min(*request_count, capacity), then the
 * head and scatter of sit_policy_apply (GaussianPolicy.get_actions, gaussian_policy.py:114-126, as
 * agent.select_action mode 1 calls it, main_ast.py:344-349).
 *   weights  float32[SIT_ACTOR_WEIGHTS]: W1 [256][SIT_OBS_DIM] (torch Linear layout), b1 [256],
 *            W2 transposed [256 in][256 out], b2 [256], W3 [2][256], b3 [2]
 *   obs      real[capacity][SIT_OBS_DIM] (the request_obs rows of sit_rollout_args)
 *   served   int64[1] or NULL: += min(*request_count, capacity)
 *   clear_count int32[1] or NULL: set to 0 (one store, no grid-wide synchronisation).  sit_rollout's
 *            admission writes *request_count itself, so the build's sampler passes NULL. */
#define SIT_ACTOR_HIDDEN 256
#define SIT_ACTOR_WEIGHTS (SIT_ACTOR_HIDDEN * SIT_OBS_DIM + SIT_ACTOR_HIDDEN + SIT_ACTOR_HIDDEN * SIT_ACTOR_HIDDEN + \
                           SIT_ACTOR_HIDDEN + 2 * SIT_ACTOR_HIDDEN + 2)
int sit_policy_actor(sit_handle* h, int32_t capacity, const float* weights, const void* obs, const void* noise,
                     const int32_t* request_env, const int32_t* request_count, int32_t deterministic,
                     void* policy_action, int32_t* policy_ready, int64_t* served, int32_t* clear_count,
                     void* stream);

/* ---- state export / import (device blob) ------------------------------------------ */
/* The dynamic state of all envs (ship states, controller integrators, route tables,
 * stop flags, counters) lives in one device blob; fields are described by
 * sit_state_field(id) for id in [0, sit_state_nfields()). */
#define SIT_DT_REAL 0
#define SIT_DT_I32 1
#define SIT_DT_U32 2
int32_t sit_state_nfields(void);
int sit_state_field(const sit_handle* h, int32_t id, const char** name, size_t* offset,
                    int32_t* dtype, int64_t* count);
int sit_state_bytes(const sit_handle* h, size_t* bytes);
int sit_get_state(sit_handle* h, void* dst, void* stream);
int sit_set_state(sit_handle* h, const void* src, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SIT_H */
