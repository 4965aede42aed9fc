// sit_kernels.hip — C ABI of the ship-in-transit env step (include/sit.h) on MI355X (gfx950).
// Kernels and host helpers: sit_impl.h.  float32 step kernels: sit_steps_f32.hip.

#include "sit_impl.h"
#include "sit_actor.h"

namespace {

#ifdef SIT_F32_TU
}  // namespace
int sit_launch_steps_f32(sit_handle* h, const void* io, void* stream);   // sit_steps_f32.hip
int sit_launch_probe_f32(sit_handle* h, int n, const void* pts_ne, void* dist, uint8_t* inside, uint8_t* hull,
                         void* stream);
int sit_launch_selftest_f32tu(int op, int n, const double* a, const double* b, double* out, void* stream);
int sit_role_fallbacks_f32tu(unsigned long long* out, int reset);
#ifdef SIT_DEBUG
int sit_debug_flags_f32tu(uint32_t* out);
#endif
namespace {
int launch_steps_f32(sit_handle* h, const StepIO<float>& io, void* stream) {
  return sit_launch_steps_f32(h, &io, stream);
}
int launch_probe_f32(sit_handle* h, int n, const void* pts, void* dist, uint8_t* inside, uint8_t* hull, void* stream) {
  return sit_launch_probe_f32(h, n, pts, dist, inside, hull, stream);
}
int launch_selftest_f32tu(int op, int n, const double* a, const double* b, double* out, void* stream) {
  return sit_launch_selftest_f32tu(op, n, a, b, out, stream);
}
#else   // single-TU build (diagnostic builds): float32 step kernels compiled here, strict fp
int launch_steps_f32(sit_handle* h, const StepIO<float>& io, void* stream) {
  return launch_steps<float>(h, io, (hipStream_t)stream);
}
int launch_probe_f32(sit_handle* h, int n, const void* pts, void* dist, uint8_t* inside, uint8_t* hull, void* stream) {
  return launch_probe<float>(h, n, pts, dist, inside, hull, (hipStream_t)stream);
}
int launch_selftest_f32tu(int op, int n, const double* a, const double* b, double* out, void* stream) {
  return launch_selftest(op, n, a, b, out, (hipStream_t)stream);
}
#endif

}  // namespace

// =======================================================================================
// C ABI
// =======================================================================================
extern "C" {

#if defined(SIT_DIAG_PATHS) || defined(SIT_DIAG_PHASES) || defined(SIT_DIAG_SYNC) || defined(SIT_DIAG_SERVE)
#ifdef SIT_DIAG_PHASES
int sit_diag_read_waves(unsigned long long* out, int n) {   // [n][4], diagnostic builds only
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (n > kDiagWaves) n = kDiagWaves;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sit_wave), sizeof(unsigned long long) * 4 * n) != hipSuccess) return -1;
  return 0;
}
#endif
int sit_diag_read(unsigned long long* out, int reset) { return diag_read_impl(out, reset); }   // diagnostic builds only
#endif

int sit_probe_map(sit_handle* h, int32_t n, const void* pts_ne, void* dist, uint8_t* inside, uint8_t* hull,
                  void* stream) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (!h->have_map) return fail(h, SIT_E_STATE, "sit_load_map has not been called");
  if (n < 0 || (n > 0 && !pts_ne)) return fail(h, SIT_E_INVALID, "need n >= 0 points");
  if (n == 0) return SIT_OK;
  if (h->precision == SIT_F64) return launch_probe<double>(h, n, pts_ne, dist, inside, hull, (hipStream_t)stream);
  return launch_probe_f32(h, n, pts_ne, dist, inside, hull, stream);
}

int sit_selftest_f64(int32_t op, int32_t n, const double* a, const double* b, double* out, int32_t fast_tu,
                     void* stream) {
  if (op < 0 || op > 12 || n < 0 || (n > 0 && (!a || !b || !out))) return SIT_E_INVALID;
  if (n == 0) return SIT_OK;
  return fast_tu ? launch_selftest_f32tu(op, n, a, b, out, stream)
                 : launch_selftest(op, n, a, b, out, (hipStream_t)stream);
}

int sit_policy_apply(sit_handle* h, int32_t capacity, const void* head, int32_t head_stride, const void* noise,
                     const int32_t* request_env, const int32_t* request_count, int32_t deterministic,
                     void* policy_action, int32_t* policy_ready, int64_t* served, void* stream) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (capacity <= 0 || !head || head_stride < 2 || !request_env || !request_count || !policy_action ||
      !policy_ready || (!deterministic && !noise))
    return fail(h, SIT_E_INVALID, "policy_apply: bad arguments");
  const int blocks = (capacity + 255) / 256;
  if (h->precision == SIT_F64)
    hipLaunchKernelGGL(k_policy_apply<double>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, capacity,
                       (const double*)head, head_stride, (const double*)noise, request_env, request_count,
                       deterministic, (double*)policy_action, policy_ready, (unsigned long long*)served, h->n_env);
  else
    hipLaunchKernelGGL(k_policy_apply<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, capacity,
                       (const float*)head, head_stride, (const float*)noise, request_env, request_count,
                       deterministic, (float*)policy_action, policy_ready, (unsigned long long*)served, h->n_env);
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

int sit_policy_actor(sit_handle* h, int32_t capacity, const float* weights, const void* obs, const void* noise,
                     const int32_t* request_env, const int32_t* request_count, int32_t deterministic,
                     void* policy_action, int32_t* policy_ready, int64_t* served, int32_t* clear_count,
                     void* stream) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (capacity <= 0 || !weights || !obs || !request_env || !request_count || !policy_action || !policy_ready ||
      (!deterministic && !noise))
    return fail(h, SIT_E_INVALID, "policy_actor: bad arguments");
  int rc = h->precision == SIT_F64
               ? launch_policy_actor<double>(h, capacity, weights, obs, noise, request_env, request_count,
                                             deterministic, policy_action, policy_ready, served, clear_count,
                                             (hipStream_t)stream)
               : launch_policy_actor<float>(h, capacity, weights, obs, noise, request_env, request_count,
                                            deterministic, policy_action, policy_ready, served, clear_count,
                                            (hipStream_t)stream);
  if (rc) return rc;
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

int sit_map_info(const sit_handle* h, int64_t* info, int32_t n) {
  if (!h || !info || n < 0) return SIT_E_INVALID;
  if (!h->have_map) return SIT_E_STATE;
  const int64_t v[6] = {(int64_t)h->map_bytes, h->n_mixed, h->n_live, h->use_index, h->use_cells,
                        (int64_t)map_lds_bytes(h)};
  for (int i = 0; i < n && i < 6; ++i) info[i] = v[i];
  return SIT_OK;
}

int32_t sit_abi_version(void) { return SIT_ABI_VERSION; }

#ifdef SIT_DEBUG
int32_t sit_debug_build(void) { return 1; }
#else
int32_t sit_debug_build(void) { return 0; }
#endif

int sit_debug_flags(uint32_t* flags) {
  if (!flags) return SIT_E_INVALID;
  *flags = 0;
#ifdef SIT_DEBUG
  int rc = debug_flags_impl(flags);
#ifdef SIT_F32_TU
  if (rc == SIT_OK) rc = sit_debug_flags_f32tu(flags);
#endif
  return rc;
#else
  return SIT_OK;
#endif
}
int sit_role_fallbacks(uint64_t* count, int32_t reset) {
  if (!count) return SIT_E_INVALID;
  unsigned long long v = 0;
  int rc = role_fallbacks_impl(&v, reset);
#ifdef SIT_F32_TU
  if (rc == SIT_OK) rc = sit_role_fallbacks_f32tu(&v, reset);
#endif
  *count = v;
  return rc;
}
size_t sit_rollout_args_size(void) { return sizeof(sit_rollout_args); }
size_t sit_params_size(void) { return sizeof(sit_params); }

void sit_params_default(sit_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  // test_beds/test_policy.py:102-124
  p->dead_weight_tonnage = 3850000;
  p->coefficient_of_deadweight_to_displacement = 0.7;
  p->bunkers = 200000;
  p->ballast = 200000;
  p->length_of_ship = 80;
  p->width_of_ship = 16;
  p->added_mass_coefficient_in_surge = 0.4;
  p->added_mass_coefficient_in_sway = 0.4;
  p->added_mass_coefficient_in_yaw = 0.4;
  p->mass_over_linear_friction_coefficient_in_surge = 130;
  p->mass_over_linear_friction_coefficient_in_sway = 18;
  p->mass_over_linear_friction_coefficient_in_yaw = 90;
  p->nonlinear_friction_coefficient_in_surge = 2400;
  p->nonlinear_friction_coefficient_in_sway = 4000;
  p->nonlinear_friction_coefficient_in_yaw = 400;
  p->current_velocity_component_from_north = -2;
  p->current_velocity_component_from_east = -2;
  p->wind_speed = 2;
  p->wind_direction = -M_PI / 4;
  // ship_model.py:123-130
  p->rho_air = 1.2; p->front_height = 8.0; p->side_height = 8.0;
  p->cx = 0.5; p->cy = 0.7; p->cn = 0.08;
  p->integration_step = 0.5;
  // test_policy.py:132-168 (PTI mode)
  p->hotel_load = 200000;
  p->main_engine_capacity = 0;
  p->electrical_capacity = 2 * 510e3;
  p->shaft_generator_state = SIT_SG_MOTOR;
  p->rated_speed_main_engine_rpm = 1000;
  p->linear_friction_main_engine = 68;
  p->linear_friction_hybrid_shaft_generator = 57;
  p->gear_ratio_between_main_engine_and_propeller = 0.6;
  p->gear_ratio_between_hybrid_shaft_generator_and_propeller = 0.6;
  p->propeller_inertia = 6000;
  p->propeller_speed_to_torque_coefficient = 7.5;
  p->propeller_diameter = 3.1;
  p->propeller_speed_to_thrust_force_coefficient = 1.7;
  p->rudder_angle_to_sway_force_coefficient = 50e3;
  p->rudder_angle_to_yaw_force_coefficient = 500e3;
  p->max_rudder_angle_degrees = 30;
  // test_policy.py:199-217
  p->kp_ship_speed = 7; p->ki_ship_speed = 0.13; p->kp_shaft_speed = 0.05; p->ki_shaft_speed = 0.005;
  p->heading_kp = 1; p->heading_kd = 90; p->heading_ki = 0.01;
  p->radius_of_acceptance = 300; p->lookahead_distance = 1000;
  p->los_integral_gain = 0.002; p->integrator_windup_limit = 4000;
  // test_policy.py:39-42; MSRL_env_ex.py:119, 557, 592, 754; MSRL_Env.py:246-250
  p->theta = 2; p->sampling_frequency = 7; p->collision_bias = 1;
  p->e_tolerance = 1000; p->arrival_radius = 200; p->shaft_rpm_max = 2000; p->minimum_ship_distance = 50;
  p->bias_throttle_scale = 0.5; p->bias_throttle_max = 1.1; p->bias_rudder_degrees = 3;
  // SpecificFuelConsumptionWartila6L26 / Baudouin6M26Dot3 (ship_engine.py:89-115), test_policy.py:162-163
  p->fuel_me_a = 128.9; p->fuel_me_b = -168.9; p->fuel_me_c = 246.8;
  p->fuel_dg_a = 108.7; p->fuel_dg_b = -289.9; p->fuel_dg_c = 324.9;
  // SIT_MACH_SIMPLIFIED only: the reference configures no SimplifiedMachineryModel (no value to
  // quote); 30 s is this library's default
  p->machinery_model = SIT_MACH_SHAFT;
  p->thrust_force_dynamic_time_constant = 30;
}

const char* sit_last_error(const sit_handle* h) { return h ? h->err.c_str() : g_create_err.c_str(); }
int32_t sit_precision(const sit_handle* h) { return h ? h->precision : 0; }
int32_t sit_n_env(const sit_handle* h) { return h ? h->n_env : 0; }
const char* sit_step_kernel(const sit_handle* h) { return h ? h->last_kernel : ""; }
int32_t sit_state_nfields(void) { return kNumFields; }

int sit_create(const sit_params* p, int32_t n_env, int32_t wpt_capacity, int32_t precision, sit_handle** out) {
  if (!p || !out) return fail(nullptr, SIT_E_INVALID, "null argument");
  *out = nullptr;
  if (n_env <= 0) return fail(nullptr, SIT_E_INVALID, "n_env must be positive (got %d)", n_env);
  if (wpt_capacity < 2 || wpt_capacity > 1024)
    return fail(nullptr, SIT_E_INVALID, "wpt_capacity must be in [2, 1024] (got %d)", wpt_capacity);
  if (precision != SIT_F32 && precision != SIT_F64)
    return fail(nullptr, SIT_E_INVALID, "precision must be SIT_F32 or SIT_F64 (got %d)", precision);
  if (p->integration_step <= 0 || p->sampling_frequency <= 0 || p->lookahead_distance <= 0)
    return fail(nullptr, SIT_E_INVALID, "integration_step, sampling_frequency and lookahead_distance must be positive");
  if (p->shaft_generator_state < SIT_SG_MOTOR || p->shaft_generator_state > SIT_SG_OFF)
    return fail(nullptr, SIT_E_INVALID, "shaft_generator_state out of range");
  if (p->machinery_model != SIT_MACH_SHAFT && p->machinery_model != SIT_MACH_SIMPLIFIED)
    return fail(nullptr, SIT_E_INVALID, "machinery_model out of range");
  if (p->machinery_model == SIT_MACH_SIMPLIFIED && !(p->thrust_force_dynamic_time_constant > 0))
    return fail(nullptr, SIT_E_INVALID, "thrust_force_dynamic_time_constant must be > 0");
  sit_handle* h = new sit_handle();
  h->precision = precision;
  h->n_env = n_env;
  h->cap = wpt_capacity;
  h->p = *p;
  // diagnostic kernel selection (read once; the launch path reads no environment)
  if (const char* sel = getenv("SIT_STEP_KERNEL")) h->kernel_classic = strcmp(sel, "classic") == 0;
  if (const char* lm = getenv("SIT_LDS_MAP")) h->lds_map_sel = (lm[0] == '0') ? 0 : (lm[0] == '1') ? 1 : -1;
  // test hook (tests/test_gpu_placement.py): the fused step kernel's waves report SIMD digit w of this
  // base-4 assignment (XOR the block index's low bits) instead of HW_ID, so shared-SIMD placements run
  if (const char* fs = getenv("SIT_TEST_FAKE_SIMDS")) h->fake_simds = 0x100 | (atoi(fs) & 0xFF);
  hipError_t e = setup_device(&h->device);
  if (e != hipSuccess) { fail(nullptr, SIT_E_HIP, "hipGetDevice: %s", hipGetErrorString(e)); delete h; return SIT_E_HIP; }
  const size_t rs = real_size(h);
  size_t off = 0;
  for (int f = 0; f < kNumFields; ++f) {
    int64_t cnt = kFields[f].extent == kShip ? 2LL * n_env
                 : kFields[f].extent == kEnv ? (int64_t)n_env
                 : kFields[f].extent == kObs ? (int64_t)SIT_OBS_DIM * n_env
                 : kFields[f].extent == kLogRow ? (int64_t)SIT_LOG_KEYS * n_env : 2LL * wpt_capacity * n_env;
    const size_t el = kFields[f].dtype == SIT_DT_REAL ? rs : 4;
    h->off[f] = off;
    h->count[f] = cnt;
    off = align256(off + (size_t)cnt * el);
  }
  h->blob_bytes = off;
  // scenario
  size_t so = 0;
  h->scen_init = so; so = align256(so + (size_t)2 * SIT_INIT_NF * n_env * rs);
  h->scen_init_lo = so; so = align256(so + (size_t)2 * SIT_INIT_NF * n_env * rs);
  h->scen_end_n = so; so = align256(so + (size_t)2 * n_env * rs);
  h->scen_end_e = so; so = align256(so + (size_t)2 * n_env * rs);
  h->scen_nw0 = so; so = align256(so + (size_t)2 * n_env * 4);
  h->scen_ab_len = so; so = align256(so + (size_t)n_env * 8);
  h->scen_ab_alpha = so; so = align256(so + (size_t)n_env * 8);
  h->scen_initial = so; so = align256(so + (size_t)n_env * SIT_OBS_DIM * rs);
  // policy-mode admission scratch (sit_actor.h): per 64-env group the age-bucket counts and the plan
  const size_t n_groups = ((size_t)n_env + kAdmitGroup - 1) / kAdmitGroup;
  h->scen_admit = so; so = align256(so + (n_groups * (kAgeBuckets + 2) + 16) * 4);
  // in-kernel serving's fallback queue (logged policy launches): capacity n_env, zero ages
  h->scen_serve = so; so = align256(so + (size_t)n_env * (3 * 4 + (SIT_OBS_DIM + 1) * rs) + 256);
  h->scen_bytes = so;
  if (setup_alloc(&h->blob, h->blob_bytes) != hipSuccess || setup_alloc(&h->scen, h->scen_bytes) != hipSuccess) {
    fail(nullptr, SIT_E_NOMEM, "hipMalloc of %zu + %zu bytes failed", h->blob_bytes, h->scen_bytes);
    sit_destroy(h);
    return SIT_E_NOMEM;
  }
  if (setup_zero(h->blob, h->blob_bytes) != hipSuccess || setup_zero(h->scen, h->scen_bytes) != hipSuccess) {
    fail(nullptr, SIT_E_HIP, "hipMemset failed");
    sit_destroy(h);
    return SIT_E_HIP;
  }
  *out = h;
  return SIT_OK;
}

void sit_destroy(sit_handle* h) {
  if (!h) return;
  if (h->blob) (void)setup_free(h->blob);
  if (h->scen) (void)setup_free(h->scen);
  if (h->map) (void)setup_free(h->map);
#ifndef SIT_HOST_MEMORY_TEST
  if (h->stage) (void)hipHostFree(h->stage);
#endif
  delete h;
}

int sit_load_map(sit_handle* h, int32_t n_poly, const int32_t* vert_offsets, const double* verts_en) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (n_poly <= 0 || n_poly > kMaxPolys || !vert_offsets || !verts_en)
    return fail(h, SIT_E_INVALID, "need 1..%d polygons with offsets and vertices", kMaxPolys);
  if (vert_offsets[0] != 0) return fail(h, SIT_E_INVALID, "vert_offsets[0] must be 0");
  for (int p = 0; p < n_poly; ++p)
    if (vert_offsets[p + 1] - vert_offsets[p] < 3) return fail(h, SIT_E_INVALID, "polygon %d has < 3 vertices", p);
  const int nv = vert_offsets[n_poly];
  if (nv > kMaxPolyVerts) return fail(h, SIT_E_INVALID, "at most %d vertices (got %d)", kMaxPolyVerts, nv);
  const size_t rs = real_size(h);
  std::vector<double> vx(nv), vy(nv), il2(nv), bbox(4 * n_poly);
  std::vector<int32_t> nxt(nv), offs(vert_offsets, vert_offsets + n_poly + 1);
  // PolygonObstacle.map_boundaries (obstacle.py:111-124): vertices are (east, north)
  h->min_e = h->min_n = INFINITY;
  h->max_e = h->max_n = -INFINITY;
  for (int p = 0; p < n_poly; ++p) {
    double bx0 = INFINITY, bx1 = -INFINITY, by0 = INFINITY, by1 = -INFINITY;
    for (int i = offs[p]; i < offs[p + 1]; ++i) {
      vx[i] = verts_en[2 * i];
      vy[i] = verts_en[2 * i + 1];
      nxt[i] = (i + 1 < offs[p + 1]) ? i + 1 : offs[p];
      bx0 = std::min(bx0, vx[i]); bx1 = std::max(bx1, vx[i]);
      by0 = std::min(by0, vy[i]); by1 = std::max(by1, vy[i]);
    }
    bbox[4 * p + 0] = bx0; bbox[4 * p + 1] = bx1; bbox[4 * p + 2] = by0; bbox[4 * p + 3] = by1;
    h->min_e = std::min(h->min_e, bx0); h->max_e = std::max(h->max_e, bx1);
    h->min_n = std::min(h->min_n, by0); h->max_n = std::max(h->max_n, by1);
  }
  std::vector<double> bxv(nv), byv(nv);
  for (int i = 0; i < nv; ++i) {
    bxv[i] = vx[nxt[i]];
    byv[i] = vy[nxt[i]];
    const double ex = bxv[i] - vx[i], ey = byv[i] - vy[i];
    const double l2 = ex * ex + ey * ey;
    il2[i] = l2 > 0 ? 1.0 / l2 : 0.0;
  }
  // ---- spatial index (see sit_device.h): conservative nearest-edge candidates per grid cell,
  //      edges per horizontal band.  Exact by construction; 1 m slack covers float rounding.
  std::vector<int> poly_of(nv);
  for (int p = 0; p < n_poly; ++p)
    for (int i = offs[p]; i < offs[p + 1]; ++i) poly_of[i] = p;
  const double ext_x = h->max_e - h->min_e, ext_y = h->max_n - h->min_n;
  const double mg = 0.1 * std::max(ext_x, ext_y) + 500.0;
  const double gx0 = h->min_e - mg, gy0 = h->min_n - mg;
  const double sx = (ext_x + 2 * mg) / kGrid, sy = (ext_y + 2 * mg) / kGrid;
  const double hd = 0.5 * std::sqrt(sx * sx + sy * sy) + 1.0;
  auto seg_dist = [&](double px, double py, int i) {
    const double ex = bxv[i] - vx[i], ey = byv[i] - vy[i], l2 = ex * ex + ey * ey;
    double t = l2 > 0 ? ((px - vx[i]) * ex + (py - vy[i]) * ey) / l2 : 0.0;
    t = std::min(1.0, std::max(0.0, t));
    return std::hypot(px - (vx[i] + t * ex), py - (vy[i] + t * ey));
  };
  // packed u16 index: [grid records (u32 per cell)][band starts (NB+1)][band entries][grid groups]
  std::vector<uint16_t> gentries, bentries;
  std::vector<uint32_t> gstart(kGrid * kGrid + 1), bstart(kBands + 1);
  std::vector<double> dcell(nv);
  std::vector<int> cand;
  constexpr int kSamples = 64;   // per cell side for the candidate refinement
  for (int j = 0; j < kGrid; ++j)
    for (int i = 0; i < kGrid; ++i) {
      const double cx = gx0 + (i + 0.5) * sx, cy = gy0 + (j + 0.5) * sy;
      double D = INFINITY;
      for (int e = 0; e < nv; ++e) { dcell[e] = seg_dist(cx, cy, e); D = std::min(D, dcell[e] + hd); }
      gstart[j * kGrid + i] = (uint32_t)gentries.size();
      const size_t first = gentries.size();
      // conservative prefilter, then the Lipschitz refinement: for every point p of the cell
      // grown by 1 m, some sample s lies within r; the nearest edge e* of p has
      // d_e*(s) <= d*(p) + r and min_f d_f(s) >= d*(p) - r, so e* is kept by
      // d_e(s) <= min_f d_f(s) + 2r + 1 m at some sample.  A dropped edge is >= 1 m farther than
      // the nearest at every point of the grown cell, so float rounding cannot make it the
      // minimum: the minimum over the list equals the full scan's.
      cand.clear();
      for (int e = 0; e < nv; ++e)
        if (dcell[e] - hd <= D + 1.0) cand.push_back(e);
      if (cand.size() > 1) {
        const double x0 = gx0 + i * sx - 1.0, y0 = gy0 + j * sy - 1.0;
        const double dx = (sx + 2.0) / kSamples, dy = (sy + 2.0) / kSamples;
        const double r2 = std::sqrt(dx * dx + dy * dy) + 1.0;   // 2r + 1 m
        std::vector<char> keep(cand.size(), 0);
        std::vector<double> dd(cand.size());
        for (int v = 0; v < kSamples; ++v)
          for (int u = 0; u < kSamples; ++u) {
            const double px = x0 + (u + 0.5) * dx, py = y0 + (v + 0.5) * dy;
            double m = INFINITY;
            for (size_t q = 0; q < cand.size(); ++q) { dd[q] = seg_dist(px, py, cand[q]); m = std::min(m, dd[q]); }
            for (size_t q = 0; q < cand.size(); ++q) keep[q] |= dd[q] <= m + r2;
          }
        size_t w = 0;
        for (size_t q = 0; q < cand.size(); ++q)
          if (keep[q]) cand[w++] = cand[q];
        cand.resize(w);
      }
      // groups of 5 u8 ids in 8 bytes (padded with the list's first id): every list of the
      // reference map fits one group (lists of 5 near some vertices would need two groups of 4)
      while (cand.size() % 5) cand.push_back(cand[0]);
      for (size_t q = 0; q < cand.size(); q += 5) {
        gentries.push_back((uint16_t)(cand[q] | (cand[q + 1] << 8)));
        gentries.push_back((uint16_t)(cand[q + 2] | (cand[q + 3] << 8)));
        gentries.push_back((uint16_t)cand[q + 4]);
        gentries.push_back(0);
      }
      (void)first;
    }
  gstart[kGrid * kGrid] = (uint32_t)gentries.size();
  const double by0 = h->min_n - 1.0, bh = (ext_y + 2.0) / kBands;
  for (int b = 0; b < kBands; ++b) {
    bstart[b] = (uint32_t)bentries.size();
    const double lo = by0 + b * bh - 1.0, hi = by0 + (b + 1) * bh + 1.0;
    for (int e = 0; e < nv; ++e)
      if (std::min(vy[e], byv[e]) <= hi && std::max(vy[e], byv[e]) >= lo) bentries.push_back((uint16_t)e);
  }
  bstart[kBands] = (uint32_t)bentries.size();
  // point-in-polygon by crossing number for class-grid cell centres (>= 1 m off every edge)
  auto inside_center = [&](double px, double py) {
    bool in = false;
    for (int p = 0; p < n_poly; ++p) {
      int cross = 0;
      for (int i = offs[p]; i < offs[p + 1]; ++i) {
        const double x1 = vx[i], y1 = vy[i], x2 = bxv[i], y2 = byv[i];
        if ((y1 > py) != (y2 > py)) {
          const double xi = x1 + (py - y1) * (x2 - x1) / (y2 - y1);
          if (xi > px) ++cross;
        }
      }
      in |= (cross & 1) != 0;
    }
    return in;
  };
  // fine 2-bit classes over the map extent + 100 m
  const double fx0 = h->min_e - 100.0, fy0 = h->min_n - 100.0;
  const double fsx = (ext_x + 200.0) / kFine, fsy = (ext_y + 200.0) / kFine;
  const double fhd = 0.5 * std::sqrt(fsx * fsx + fsy * fsy) + 1.0;
  std::vector<uint32_t> fine(kFineWords, 0);
  for (int j = 0; j < kFine; ++j)
    for (int i = 0; i < kFine; ++i) {
      const double cx = fx0 + (i + 0.5) * fsx, cy = fy0 + (j + 0.5) * fsy;
      double dmin = INFINITY;
      for (int e = 0; e < nv && dmin > fhd + 1.0; ++e) dmin = std::min(dmin, seg_dist(cx, cy, e));
      const uint32_t k = dmin > fhd + 1.0 ? (inside_center(cx, cy) ? 1u : 0u) : 2u;
      const int cell = j * kFine + i;
      fine[cell >> 4] |= k << ((cell & 15) * 2);
    }
  h->fx0 = fx0; h->fy0 = fy0; h->finvx = 1.0 / fsx; h->finvy = 1.0 / fsy;
  // point-in-polygon records of the mixed cells (see Map in sit_device.h).  An edge's GEOS
  // crossing contribution is the same for every point of cell [x0,x1]x[y0,y1] when (1 m
  // margin, far above float rounding of coordinates <= 1e5 m): it lies wholly left of the cell
  // (early return), its y-range misses the cell's rows, or it spans the rows strictly and,
  // within them, lies wholly right or wholly left of the cell (then it straddles every row and
  // its orientation against every point is that against the centre).  All other edges are live.
  std::vector<uint16_t> frank(kFineWords, 0);
  std::vector<uint32_t> crec;
  std::vector<uint8_t> clive;
  {
    int rank = 0;
    for (int w = 0; w < kFineWords; ++w) {
      frank[w] = (uint16_t)std::min(rank, 65535);
      rank += __builtin_popcount((fine[w] >> 1) & 0x55555555u);
    }
    for (int cell = 0; cell < kFine * kFine; ++cell) {
      if (((fine[cell >> 4] >> ((cell & 15) * 2)) & 3) != 2) continue;
      const int i = cell % kFine, j = cell / kFine;
      const double x0 = fx0 + i * fsx, x1 = fx0 + (i + 1) * fsx, y0 = fy0 + j * fsy, y1 = fy0 + (j + 1) * fsy;
      const double cx = 0.5 * (x0 + x1), cy = 0.5 * (y0 + y1), mgn = 1.0;
      uint32_t par = 0;
      const size_t first = clive.size();
      for (int e = 0; e < nv; ++e) {
        const double p1x = vx[e], p1y = vy[e], p2x = bxv[e], p2y = byv[e];
        const double xmax = std::max(p1x, p2x), ymin = std::min(p1y, p2y), ymax = std::max(p1y, p2y);
        if (xmax < x0 - mgn) continue;                          // left of every point: no count
        if (ymax < y0 - mgn || ymin > y1 + mgn) continue;       // never straddles a cell row
        if (ymin < y0 - mgn && ymax > y1 + mgn) {
          const double ta = (y0 - mgn - p1y) / (p2y - p1y), tb = (y1 + mgn - p1y) / (p2y - p1y);
          const double xa = p1x + ta * (p2x - p1x), xb = p1x + tb * (p2x - p1x);
          const bool right = std::min(xa, xb) > x1 + mgn && xmax > x1 + mgn;
          const bool left = std::max(xa, xb) < x0 - mgn && xmax > x1 + mgn;
          if (right || left) {
            const double det = (p1x - cx) * (p2y - cy) - (p1y - cy) * (p2x - cx);
            const int o = (det > 0) - (det < 0);
            const int oo = (p2y < p1y) ? -o : o;
            if (oo > 0) par ^= 1u << poly_of[e];
            continue;
          }
        }
        clive.push_back((uint8_t)e);
      }
      const size_t cnt = clive.size() - first;
      crec.push_back(par);
      crec.push_back((uint32_t)first | ((uint32_t)cnt << 16));
    }
  }
  const bool cells_ok = crec.size() / 2 <= 65535 && clive.size() <= 65535;
  // each cell's first group goes into its record; the further groups (lists of > 5) follow the
  // band entries
  std::vector<uint16_t> grest;
  std::vector<uint32_t> rstart(kGrid * kGrid);
  for (int c = 0; c < kGrid * kGrid; ++c) {
    rstart[c] = (uint32_t)grest.size();
    grest.insert(grest.end(), gentries.begin() + gstart[c] + 4, gentries.begin() + gstart[c + 1]);
  }
  const size_t head = (size_t)kIdxHead;
  const size_t gbase = (head + bentries.size() + 3) & ~size_t(3);   // 8-byte aligned groups
  const size_t n_idx = gbase + grest.size();
  h->use_index = (n_idx < 65535 && n_idx * 2 <= 48 * 1024) ? 1 : 0;
  h->gx0 = gx0; h->gy0 = gy0; h->ginvx = 1.0 / sx; h->ginvy = 1.0 / sy;
  h->by0 = by0; h->binv = 1.0 / bh;
  std::vector<uint16_t> idx(h->use_index ? n_idx : 4, 0);
  h->n_idx = (int64_t)idx.size();
  if (h->use_index) {
    for (int c = 0; c < kGrid * kGrid; ++c) {
      const uint16_t* f = gentries.data() + gstart[c];
      const uint32_t more = (gstart[c + 1] - gstart[c]) / 4 - 1;    // < 52: ids are u8, 5 per group
      const uint32_t y = (f[2] & 0xffu) | (more << 8) | ((uint32_t)((gbase + rstart[c]) / 4) << 16);
      idx[4 * c] = f[0];                       // ids 0, 1
      idx[4 * c + 1] = f[1];                   // ids 2, 3
      idx[4 * c + 2] = (uint16_t)(y & 0xffffu);
      idx[4 * c + 3] = (uint16_t)(y >> 16);
    }
    for (int b = 0; b <= kBands; ++b) idx[kBandBase + b] = (uint16_t)(head + bstart[b]);
    std::copy(bentries.begin(), bentries.end(), idx.begin() + head);
    std::copy(grest.begin(), grest.end(), idx.begin() + gbase);
  }
  // blob: [Edge<T>[nv]][u16 index][u32 classes] (staged into LDS) [ring offsets][bboxes] (fallback, global)
  const size_t esz = rs == 8 ? sizeof(Edge<double>) : sizeof(Edge<float>);
  size_t o = align256(nv * esz);
  h->map_idx = o; o = align256(o + idx.size() * 2);
  h->map_fine = o; o = align256(o + fine.size() * 4);
  h->use_cells = cells_ok ? 1 : 0;
  h->n_mixed = (int64_t)crec.size() / 2;
  h->n_live = (int64_t)clive.size();
  h->map_frank = o; o += (cells_ok ? frank.size() * 2 : 0); o = (o + 7) & ~size_t(7);
  h->map_crec = o; o += (cells_ok ? crec.size() * 4 : 0);
  h->map_clive = o; o = align256(o + (cells_ok ? clive.size() : 0));
  h->map_bytes = o;
  h->map_off = o; o = align256(o + (n_poly + 1) * 4);
  h->map_bbox = o; o = align256(o + 4 * n_poly * rs);
  std::vector<unsigned char> host(o, 0);
  for (int e = 0; e < nv; ++e) {
    if (rs == 8) {
      Edge<double> g{vx[e], vy[e], bxv[e], byv[e], il2[e], (uint32_t)poly_of[e]};
      std::memcpy(host.data() + e * esz, &g, sizeof(g));
    } else {
      Edge<float> g{(float)vx[e], (float)vy[e], (float)bxv[e], (float)byv[e], (float)il2[e], (uint32_t)poly_of[e]};
      std::memcpy(host.data() + e * esz, &g, sizeof(g));
    }
  }
  std::memcpy(host.data() + h->map_idx, idx.data(), idx.size() * 2);
  std::memcpy(host.data() + h->map_fine, fine.data(), fine.size() * 4);
  if (cells_ok) {
    std::memcpy(host.data() + h->map_frank, frank.data(), frank.size() * 2);
    std::memcpy(host.data() + h->map_crec, crec.data(), crec.size() * 4);
    if (!clive.empty()) std::memcpy(host.data() + h->map_clive, clive.data(), clive.size());
  }
  std::memcpy(host.data() + h->map_off, offs.data(), (n_poly + 1) * 4);
  for (size_t i = 0; i < bbox.size(); ++i) {
    if (rs == 8) reinterpret_cast<double*>(host.data() + h->map_bbox)[i] = bbox[i];
    else reinterpret_cast<float*>(host.data() + h->map_bbox)[i] = (float)bbox[i];
  }
  if (h->map) { (void)setup_free(h->map); h->map = nullptr; }
  HIP_TRY(h, setup_alloc(&h->map, o));
  HIP_TRY(h, setup_upload(h->map, host.data(), o));
  h->n_poly = n_poly;
  h->n_vert = nv;
  h->have_map = true;
  // the cached IW tests describe the previous map
  HIP_TRY(h, setup_zero(h->blob + h->off[F_IWK_FLAGS], (size_t)h->n_env * 4));
  return SIT_OK;
}

int sit_load_routes(sit_handle* h, const double* wpt_ne, const int32_t* n_wpt) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (!wpt_ne || !n_wpt) return fail(h, SIT_E_INVALID, "null route arrays");
  const int n = h->n_env, cap = h->cap;
  const size_t rs = real_size(h);
  std::vector<double> tab((size_t)2 * 2 * cap * n, 0.0), end((size_t)2 * 2 * n), ab_len(n), ab_alpha(n);
  std::vector<int32_t> nw0((size_t)2 * n);
  for (int e = 0; e < n; ++e) {
    for (int t = 0; t < 2; ++t) {
      const int nw = n_wpt[2 * e + t];
      if (nw < 2 || nw > cap) return fail(h, SIT_E_INVALID, "env %d ship %d: n_wpt %d not in [2, %d]", e, t, nw, cap);
      const double* r = wpt_ne + ((size_t)(e * 2 + t) * cap) * 2;
      for (int i = 0; i < nw - 1; ++i) {
        tab[((size_t)(0 * 2 + t) * cap + i) * n + e] = r[2 * i];
        tab[((size_t)(1 * 2 + t) * cap + i) * n + e] = r[2 * i + 1];
      }
      end[(size_t)(0 * 2 + t) * n + e] = r[2 * (nw - 1)];
      end[(size_t)(1 * 2 + t) * n + e] = r[2 * (nw - 1) + 1];
      nw0[(size_t)t * n + e] = nw;
      if (t == 1) {   // reward_function_params (MSRL_Env.py:119-128)
        const double dn = r[2 * (nw - 1)] - r[0], de = r[2 * (nw - 1) + 1] - r[1];
        ab_len[e] = std::sqrt(dn * dn + de * de) / h->p.sampling_frequency;
        ab_alpha[e] = std::atan2(de, dn);
      }
    }
  }
  auto conv = [&](const double* src, size_t cnt) {
    std::vector<unsigned char> out(cnt * rs);
    for (size_t i = 0; i < cnt; ++i) {
      if (rs == 8) reinterpret_cast<double*>(out.data())[i] = src[i];
      else reinterpret_cast<float*>(out.data())[i] = (float)src[i];
    }
    return out;
  };
  const size_t tcnt = (size_t)2 * cap * n;
  auto tn = conv(tab.data(), tcnt), te = conv(tab.data() + tcnt, tcnt);
  auto en = conv(end.data(), (size_t)2 * n), ee = conv(end.data() + (size_t)2 * n, (size_t)2 * n);
  HIP_TRY(h, setup_upload(h->blob + h->off[F_WN], tn.data(), tn.size()));
  HIP_TRY(h, setup_upload(h->blob + h->off[F_WE], te.data(), te.size()));
  HIP_TRY(h, setup_upload(h->scen + h->scen_end_n, en.data(), en.size()));
  HIP_TRY(h, setup_upload(h->scen + h->scen_end_e, ee.data(), ee.size()));
  HIP_TRY(h, setup_upload(h->scen + h->scen_nw0, nw0.data(), nw0.size() * 4));
  HIP_TRY(h, setup_upload(h->scen + h->scen_ab_len, ab_len.data(), (size_t)n * 8));
  HIP_TRY(h, setup_upload(h->scen + h->scen_ab_alpha, ab_alpha.data(), (size_t)n * 8));
  h->have_routes = true;
  return SIT_OK;
}

int sit_load_initial(sit_handle* h, const double* init) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (!init) return fail(h, SIT_E_INVALID, "null init array");
  const int n = h->n_env;
  const size_t rs = real_size(h);
  std::vector<double> sc((size_t)2 * SIT_INIT_NF * n), ist((size_t)n * SIT_OBS_DIM, 0.0);
  for (int e = 0; e < n; ++e)
    for (int t = 0; t < 2; ++t)
      for (int f = 0; f < SIT_INIT_NF; ++f)
        sc[((size_t)t * SIT_INIT_NF + f) * n + e] = init[((size_t)e * 2 + t) * SIT_INIT_NF + f];
  // construction-time observation, rounded to float32 as the reference's array (MSRL_Env.py:88-91)
  for (int e = 0; e < n; ++e) {
    const double* a = init + (size_t)e * 2 * SIT_INIT_NF;
    const double* b = a + SIT_INIT_NF;
    double* o = &ist[(size_t)e * SIT_OBS_DIM];
    o[0] = (float)a[SIT_INIT_NORTH]; o[1] = (float)a[SIT_INIT_EAST]; o[2] = (float)a[SIT_INIT_YAW];
    o[6] = (float)b[SIT_INIT_NORTH]; o[7] = (float)b[SIT_INIT_EAST]; o[8] = (float)b[SIT_INIT_YAW];
  }
  auto conv = [&](const std::vector<double>& src) {
    std::vector<unsigned char> out(src.size() * rs);
    for (size_t i = 0; i < src.size(); ++i) {
      if (rs == 8) reinterpret_cast<double*>(out.data())[i] = src[i];
      else reinterpret_cast<float*>(out.data())[i] = (float)src[i];
    }
    return out;
  };
  auto a = conv(sc), b = conv(ist);
  HIP_TRY(h, setup_upload(h->scen + h->scen_init, a.data(), a.size()));
  if (rs == 4) {   // float32: the low parts of the initial values (double-float starts, comp_add)
    std::vector<float> lo(sc.size());
    for (size_t i = 0; i < sc.size(); ++i) lo[i] = (float)(sc[i] - (double)(float)sc[i]);
    HIP_TRY(h, setup_upload(h->scen + h->scen_init_lo, lo.data(), lo.size() * 4));
  }
  HIP_TRY(h, setup_upload(h->scen + h->scen_initial, b.data(), b.size()));
  h->have_init = true;
  return SIT_OK;
}

int sit_restart(sit_handle* h, void* stream) {
  int rc = ready(h);
  if (rc) return rc;
  const int blocks = (h->n_env + 255) / 256;
  if (h->precision == SIT_F64)
    hipLaunchKernelGGL(k_restart<double>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, make_args<double>(h));
  else
    hipLaunchKernelGGL(k_restart<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, make_args<float>(h));
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

int sit_reset(sit_handle* h, const uint8_t* env_mask, void* initial_state, void* stream) {
  int rc = ready(h);
  if (rc) return rc;
  const int blocks = (h->n_env + 255) / 256;
  if (h->precision == SIT_F64)
    hipLaunchKernelGGL(k_reset<double>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, make_args<double>(h),
                       env_mask, (double*)initial_state);
  else
    hipLaunchKernelGGL(k_reset<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, make_args<float>(h),
                       env_mask, (float*)initial_state);
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

int sit_init_step(sit_handle* h, const uint8_t* env_mask, void* stream) {
  int rc = ready(h);
  if (rc) return rc;
  const int blocks = (2 * h->n_env + 255) / 256;
  if (h->precision == SIT_F64)
    hipLaunchKernelGGL(k_init_step<double>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, make_args<double>(h), env_mask);
  else
    hipLaunchKernelGGL(k_init_step<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, make_args<float>(h), env_mask);
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

// next_state and action_out rows are written with paired stores (store2)
static bool pair_aligned(const sit_handle* h, const void* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  return (a % (2 * (h->precision == SIT_F64 ? sizeof(double) : sizeof(float)))) == 0;
}

int sit_step(sit_handle* h, const void* action_ne, const uint8_t* sac_update, const uint8_t* init,
             void* next_state, void* reward, uint8_t* done, uint32_t* status, int32_t* done_count,
             void* stream) {
  int rc = ready(h);
  if (rc) return rc;
  if (!action_ne || !sac_update || !init) return fail(h, SIT_E_INVALID, "action_ne, sac_update and init are required");
  if (!next_state && !reward) return fail(h, SIT_E_INVALID, "need next_state or reward output");
  if (!pair_aligned(h, next_state)) return fail(h, SIT_E_INVALID, "next_state must be aligned to 2 reals");
  if (h->precision == SIT_F64) {
    StepIO<double> io{};
    io.n_steps = 1; io.action_ne = (const double*)action_ne; io.sac_update = sac_update; io.init = init;
    io.next_state = (double*)next_state; io.reward = (double*)reward; io.done = done; io.status = status;
    io.done_count = done_count;
    return launch_steps<double>(h, io, (hipStream_t)stream);
  }
  StepIO<float> io{};
  io.n_steps = 1; io.action_ne = (const float*)action_ne; io.sac_update = sac_update; io.init = init;
  io.next_state = (float*)next_state; io.reward = (float*)reward; io.done = done; io.status = status;
  io.done_count = done_count;
  return launch_steps_f32(h, io, stream);
}

// sit_step_host's staging: pinned, coherent host memory mapped for the device (the step kernel reads
// the inputs and writes the outputs there directly; no copy call per step)
struct StageLayout {
  size_t act, sac, init, ns, rw, dn, st, log, blob, bytes;
};
static StageLayout stage_layout(const sit_handle* h) {
  const size_t n = (size_t)h->n_env, rs = real_size(h);
  StageLayout L{};
  size_t o = 0;
  L.act = o; o = align256(o + 2 * n * rs);
  L.sac = o; o = align256(o + n);
  L.init = o; o = align256(o + n);
  L.ns = o; o = align256(o + (size_t)SIT_OBS_DIM * n * rs);
  L.rw = o; o = align256(o + n * rs);
  L.dn = o; o = align256(o + n);
  L.st = o; o = align256(o + 4 * n);
  L.log = o; o = align256(o + (size_t)SIT_LOG_ROWS * n * rs);
  L.blob = o; o = align256(o + h->blob_bytes);
  L.bytes = o;
  return L;
}

int sit_step_host(sit_handle* h, const void* action_ne, const uint8_t* sac_update, const uint8_t* init,
                  void* next_state, void* reward, uint8_t* done, uint32_t* status, void* log, void* state,
                  void* stream) {
  int rc = ready(h);
  if (rc) return rc;
  if (!action_ne || !sac_update || !init) return fail(h, SIT_E_INVALID, "action_ne, sac_update and init are required");
#ifdef SIT_HOST_MEMORY_TEST
  (void)next_state; (void)reward; (void)done; (void)status; (void)log; (void)state; (void)stream;
  return fail(h, SIT_E_STATE, "sit_step_host: no device in the host-memory test build");
#else
  const StageLayout L = stage_layout(h);
  if (!h->stage_dev) {   // allocated into locals; published only once both calls succeeded
    unsigned char* hp = nullptr;
    HIP_TRY(h, hipHostMalloc(reinterpret_cast<void**>(&hp), L.bytes, hipHostMallocMapped | hipHostMallocCoherent));
    void* dp = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&dp, hp, 0);
    if (e != hipSuccess || !dp) {
      (void)hipHostFree(hp);
      return fail(h, SIT_E_HIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
    }
    h->stage = hp;
    h->stage_dev = static_cast<unsigned char*>(dp);
  }
  const size_t n = (size_t)h->n_env, rs = real_size(h);
  std::memcpy(h->stage + L.act, action_ne, 2 * n * rs);
  std::memcpy(h->stage + L.sac, sac_update, n);
  std::memcpy(h->stage + L.init, init, n);
  unsigned char* d = h->stage_dev;
  hipStream_t s = (hipStream_t)stream;
  if (h->precision == SIT_F64) {
    StepIO<double> io{};
    io.n_steps = 1; io.action_ne = (const double*)(d + L.act); io.sac_update = d + L.sac; io.init = d + L.init;
    io.next_state = (double*)(d + L.ns); io.reward = (double*)(d + L.rw); io.done = d + L.dn;
    io.status = (uint32_t*)(d + L.st); io.log = log ? (double*)(d + L.log) : nullptr;
    rc = launch_steps<double>(h, io, s);
  } else {
    StepIO<float> io{};
    io.n_steps = 1; io.action_ne = (const float*)(d + L.act); io.sac_update = d + L.sac; io.init = d + L.init;
    io.next_state = (float*)(d + L.ns); io.reward = (float*)(d + L.rw); io.done = d + L.dn;
    io.status = (uint32_t*)(d + L.st); io.log = log ? (float*)(d + L.log) : nullptr;
    rc = launch_steps_f32(h, io, stream);
  }
  if (rc) return rc;
  if (state) HIP_TRY(h, hipMemcpyAsync(h->stage + L.blob, h->blob, h->blob_bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(h, hipStreamSynchronize(s));
  if (next_state) std::memcpy(next_state, h->stage + L.ns, (size_t)SIT_OBS_DIM * n * rs);
  if (reward) std::memcpy(reward, h->stage + L.rw, n * rs);
  if (done) std::memcpy(done, h->stage + L.dn, n);
  if (status) std::memcpy(status, h->stage + L.st, 4 * n);
  if (log) std::memcpy(log, h->stage + L.log, (size_t)SIT_LOG_ROWS * n * rs);
  if (state) std::memcpy(state, h->stage + L.blob, h->blob_bytes);
  return SIT_OK;
#endif
}

int sit_rollout(sit_handle* h, const sit_rollout_args* ra, void* stream) {
  int rc = ready(h);
  if (rc) return rc;
  if (!ra) return fail(h, SIT_E_INVALID, "null rollout args");
  if (ra->n_steps <= 0) return fail(h, SIT_E_INVALID, "n_steps must be positive");
  if (!ra->next_state && !ra->reward) return fail(h, SIT_E_INVALID, "need next_state or reward output");
  if (ra->action_ne && (!ra->sac_update || !ra->init))
    return fail(h, SIT_E_INVALID, "explicit actions need sac_update and init");
  if (ra->env_id_offset < 0) return fail(h, SIT_E_INVALID, "env_id_offset must be >= 0");
  if (!pair_aligned(h, ra->next_state) || !pair_aligned(h, ra->action_out))
    return fail(h, SIT_E_INVALID, "next_state and action_out must be aligned to 2 reals");
  if (ra->transitions && (!ra->transition_count || ra->transition_capacity <= 0))
    return fail(h, SIT_E_INVALID, "transitions need transition_count and a positive capacity");
  if (reinterpret_cast<uintptr_t>(ra->transitions) % (4 * real_size(h)) != 0)
    return fail(h, SIT_E_INVALID, "transitions must be aligned to 4 reals");
  if (ra->policy_action && ra->action_ne)
    return fail(h, SIT_E_INVALID, "policy mode and explicit actions are exclusive");
  const bool serve = ra->policy_action && ra->actor_weights;
  if (ra->actor_weights && !ra->policy_action) return fail(h, SIT_E_INVALID, "actor_weights need policy mode");
  if (serve && !ra->policy_ready) return fail(h, SIT_E_INVALID, "policy mode needs policy_ready");
  if (ra->policy_action && !serve &&
      (!ra->policy_ready || !ra->request_env || !ra->request_noise || !ra->request_obs || !ra->request_count ||
       !ra->request_age || ra->request_capacity <= 0))
    return fail(h, SIT_E_INVALID, "policy mode needs policy_ready, request_env, request_noise, "
                                  "request_obs, request_count, request_age and a positive request_capacity "
                                  "(or actor_weights: in-kernel serving)");
  auto fill = [&](auto* io, auto* tag) {
    using R = std::remove_pointer_t<decltype(tag)>;
    io->n_steps = ra->n_steps; io->auto_reset = ra->auto_reset; io->seed = ra->seed;
    io->env_id_offset = ra->env_id_offset;
    io->action_ne = (const R*)ra->action_ne; io->sac_update = ra->sac_update; io->init = ra->init;
    io->next_state = (R*)ra->next_state; io->reward = (R*)ra->reward; io->done = ra->done;
    io->status = ra->status; io->action_out = (R*)ra->action_out; io->done_count = ra->done_count;
    io->transitions = (R*)ra->transitions; io->transition_count = ra->transition_count;
    io->transition_capacity = ra->transition_capacity; io->mask_horizon = ra->mask_horizon;
    // (policy_action: the kernel reads it and, serving, writes it)
    io->policy_action = const_cast<R*>(static_cast<const R*>(ra->policy_action)); io->policy_ready = ra->policy_ready;
    io->request_age = serve ? nullptr : ra->request_age;
    io->group_counts = (ra->policy_action && !serve) ? admit_counts(h) : nullptr;
    io->env_steps = reinterpret_cast<unsigned long long*>(ra->env_steps);
    io->log = (R*)ra->log;
    io->actor_w = serve ? ra->actor_weights : nullptr;
    io->actor_det = ra->actor_deterministic;
    io->actor_served = reinterpret_cast<unsigned long long*>(ra->actor_served);
  };
  // policy mode: the step kernel, then the deterministic admission of the waiting envs into the
  // request queue (k_policy_admit, sit_actor.h) on the same stream — or, serving in the kernel, nothing;
  // a serving launch that takes the one-wave kernel (logged) is served through the library's own queue
  auto run = [&](auto* io, auto launch) -> int {
    using R = std::remove_pointer_t<decltype(io->next_state)>;
    sit_rollout_args q = *ra;
    if (serve && sync_launch_lds<R>(h, *io, nullptr, nullptr) == 0) {
      const ServeQueue sq = serve_queue(h);
      io->actor_w = nullptr;
      io->request_age = sq.age;
      io->group_counts = admit_counts(h);
      q.request_capacity = h->n_env; q.request_env = sq.env; q.request_obs = sq.obs; q.request_noise = sq.noise;
      q.request_count = sq.count; q.request_age = sq.age;
    } else if (serve) {
      return launch(*io);
    }
    int r = launch(*io);
    if (r == SIT_OK && ra->policy_action) r = launch_policy_admit<R>(h, &q, (hipStream_t)stream);
    if (r == SIT_OK && serve)
      r = launch_policy_actor<R>(h, h->n_env, ra->actor_weights, q.request_obs, q.request_noise, q.request_env,
                                 q.request_count, ra->actor_deterministic, const_cast<void*>(ra->policy_action),
                                 ra->policy_ready, ra->actor_served, nullptr, (hipStream_t)stream);
    return r;
  };
  if (h->precision == SIT_F64) {
    StepIO<double> io{};
    fill(&io, (double*)nullptr);
    rc = run(&io, [&](const StepIO<double>& x) { return launch_steps<double>(h, x, (hipStream_t)stream); });
  } else {
    StepIO<float> io{};
    fill(&io, (float*)nullptr);
    rc = run(&io, [&](const StepIO<float>& x) { return launch_steps_f32(h, x, stream); });
  }
  if (rc) return rc;
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

int sit_state_field(const sit_handle* h, int32_t id, const char** name, size_t* offset, int32_t* dtype,
                    int64_t* count) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (id < 0 || id >= kNumFields) return SIT_E_INVALID;
  if (name) *name = kFields[id].name;
  if (offset) *offset = h->off[id];
  if (dtype) *dtype = kFields[id].dtype;
  if (count) *count = h->count[id];
  return SIT_OK;
}

int sit_state_bytes(const sit_handle* h, size_t* bytes) {
  if (!h || !bytes) return fail(nullptr, SIT_E_INVALID, "null argument");
  *bytes = h->blob_bytes;
  return SIT_OK;
}

int sit_get_state(sit_handle* h, void* dst, void* stream) {
  if (!h || !dst) return fail(h, SIT_E_INVALID, "null argument");
  HIP_TRY(h, hipMemcpyAsync(dst, h->blob, h->blob_bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return SIT_OK;
}

int sit_set_state(sit_handle* h, const void* src, void* stream) {
  if (!h || !src) return fail(h, SIT_E_INVALID, "null argument");
  HIP_TRY(h, hipMemcpyAsync(h->blob, src, h->blob_bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  // the cached IW terrain tests (iw_key_*) are answers for the map of the handle that saved the blob:
  // a restored state re-tests its IW against this handle's map
  HIP_TRY(h, hipMemsetAsync(h->blob + h->off[F_IWK_FLAGS], 0, (size_t)h->n_env * 4, (hipStream_t)stream));
  return SIT_OK;
}

}  // extern "C"
