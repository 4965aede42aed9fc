// sit_device.h — device-side building blocks of the ship-in-transit env step (gfx950).
//
// Everything here is templated on the real type T (float for the SIT_F32 handle, double for
// SIT_F64).  The arithmetic follows the reference's operation order where that is free;
// where a closed form replaces a numpy construct the comment names the reference line:
//   rotation inverse / mass-matrix inverse      ship_model.py:252-255, 590-603 (closed forms)
//   wind load, gamma = -atan2(v_rw, u_rw)         ship_model.py:211-231 (trig-free identity)
//   LOS sin/cos(atan2(dy, dx))                    LOS_guidance.py:110-113 (float32: dy/L, dx/L)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sit.h"

namespace sit {

template <typename T>
constexpr bool kIsF32 = std::is_same<T, float>::value;
// diagnostic builds only (tools/ab2.sh): the float32 knife-edge re-evaluations switched off, to
// price them
#ifndef SIT_EXP_KNIFE_MASK
#define SIT_EXP_KNIFE_MASK 15     // 1 LOS clamp/windup, 2 shaft rpm, 4 arrival/collision radii, 8 containment
#endif
constexpr bool kKnifeLos = (SIT_EXP_KNIFE_MASK & 1) != 0, kKnifeRpm = (SIT_EXP_KNIFE_MASK & 2) != 0,
               kKnifeRad = (SIT_EXP_KNIFE_MASK & 4) != 0, kKnifePip = (SIT_EXP_KNIFE_MASK & 8) != 0;

// --------------------------------------------------------------------------------------
// IEEE float64 (round to nearest, no contraction, no reassociation) for knife-edge decisions.
// The float32 step kernels are compiled with device fast-math (the TU keeps
// -ffp-contract=fast-honor-pragmas so these scopes' contract(off) is honoured); add/sub/mul run in
// pragma scopes, division and square root are the correctly rounded gfx950 sequences written
// out with the div_scale/div_fmas/div_fixup and rsq builtins, which no fast-math flag rewrites.
// Inputs converted from float32 are exact, so a decision taken here is the oracle's decision on
// the same float32 state (checked bitwise against numpy: sit_selftest_f64, tests/test_gpu_parity.py).
// --------------------------------------------------------------------------------------
__device__ __forceinline__ double ieee_add(double a, double b) {
#pragma clang fp reassociate(off) contract(off)
  return a + b;
}
__device__ __forceinline__ double ieee_sub(double a, double b) {
#pragma clang fp reassociate(off) contract(off)
  return a - b;
}
__device__ __forceinline__ double ieee_mul(double a, double b) {
#pragma clang fp reassociate(off) contract(off)
  return a * b;
}
// a / b correctly rounded: the v_div_scale / v_rcp / Newton / v_div_fmas / v_div_fixup sequence
__device__ __forceinline__ double ieee_div(double a, double b) {
#pragma clang fp reassociate(off) contract(off)
  bool f_den, f_num;
  const double den = __builtin_amdgcn_div_scale(a, b, false, &f_den);
  const double num = __builtin_amdgcn_div_scale(a, b, true, &f_num);
  const double r0 = __builtin_amdgcn_rcp(den);
  const double e0 = __builtin_fma(-den, r0, 1.0);
  const double r1 = __builtin_fma(r0, e0, r0);
  const double e1 = __builtin_fma(-den, r1, 1.0);
  const double r2 = __builtin_fma(r1, e1, r1);
  const double q = num * r2;
  const double rem = __builtin_fma(-den, q, num);
  (void)f_den;
  return __builtin_amdgcn_div_fixup(__builtin_amdgcn_div_fmas(rem, r2, q, f_num), b, a);
}
// sqrt(a) correctly rounded: rsq seed, Goldschmidt / Newton steps with fma, scaled for tiny a
__device__ __forceinline__ double ieee_sqrt(double a) {
#pragma clang fp reassociate(off) contract(off)
  const bool tiny = a < 0x1.0p-767;
  const double x = tiny ? __builtin_amdgcn_ldexp(a, 256) : a;
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  g = tiny ? __builtin_amdgcn_ldexp(g, -128) : g;
  // +-0, +inf and NaN pass through unchanged (class mask: NaNs, -0, +0, +inf)
  return __builtin_amdgcn_class(x, 0x263) ? a : g;
}
// a^2 + b^2 as numpy evaluates (dn ** 2 + de ** 2): two roundings of the squares, one of the sum
__device__ __forceinline__ double ieee_sq2(double a, double b) { return ieee_add(ieee_mul(a, a), ieee_mul(b, b)); }
// x * y + z * w as numpy evaluates it (no fused multiply-add)
__device__ __forceinline__ double ieee_dot2(double x, double y, double z, double w) {
  return ieee_add(ieee_mul(x, y), ieee_mul(z, w));
}

// Debug builds (-DSIT_DEBUG, libsit_debug.so; SURVEY §5: bounds asserts in a debug kernel variant):
// every table index the step computes is checked before use.  A failed check sets its bit in
// g_dbg_flags (one word per translation unit, read and cleared by sit_debug_flags) instead of
// trapping, and the index is clamped into its table: the launch completes without touching memory
// out of bounds and the host reports which check failed.  Release builds compile the checks out.
enum DebugCheck {
  kDbgRouteIndex = 0,    // a route-table row outside [0, wpt_capacity)
  kDbgWaypoint = 1,      // the next-waypoint index k outside [1, n_wpt)
  kDbgRouteLen = 2,      // a route length outside [2, wpt_capacity]
  kDbgIndexEntry = 3,    // a grid / band entry outside the packed spatial index
  kDbgEdgeId = 4,        // an edge id >= the map's edge count
  kDbgClassWord = 5,     // a class-grid word outside the grid
  kDbgCellRecord = 6,    // a mixed-cell record or live-edge entry outside its table
  kDbgServeCount = 7,    // in-kernel serving: a published request count outside [0, 64], or the serving
                         // LDS (ServeWork, ServePub) past the launch's dynamic LDS
  kDbgServeEnv = 8,      // in-kernel serving: a published env id outside [0, n_env)
};
#ifdef SIT_DEBUG
namespace {
__device__ unsigned int g_dbg_flags;
}
__device__ __forceinline__ int dbg_clamp(int i, int n, int id) {
  if (i < 0 || i >= n) {
    atomicOr(&g_dbg_flags, 1u << id);
    return 0;
  }
  return i;
}
// a range [first, first + cnt) of a table of n entries: the count that stays inside it
__device__ __forceinline__ int dbg_span(int first, int cnt, int n, int id) {
  if (first < 0 || cnt < 0 || first + cnt > n) {
    atomicOr(&g_dbg_flags, 1u << id);
    return first < 0 || first >= n ? 0 : max(0, min(cnt, n - first));
  }
  return cnt;
}
#define SIT_DCHECK(cond, id) do { if (!(cond)) atomicOr(&::sit::g_dbg_flags, 1u << (id)); } while (0)
#define SIT_DCLAMP(i, n, id) ::sit::dbg_clamp((i), (n), (id))
#define SIT_DSPAN(first, cnt, n, id) ::sit::dbg_span((first), (cnt), (n), (id))
#else
#define SIT_DCHECK(cond, id) do { } while (0)
#define SIT_DCLAMP(i, n, id) (i)
#define SIT_DSPAN(first, cnt, n, id) (cnt)
#endif
// an edge id read from the spatial index (checked and clamped in debug builds)
#define SIT_DEDGE(m, i) SIT_DCLAMP((int)(i), (m).n_edge, kDbgEdgeId)

constexpr int kWave = 64;         // CDNA wavefront

// The role (0 D0, 1 D1, 2 P0, 3 P1) of wave w of a k_env_steps_sync block from the SIMDs its four waves
// sit on (simd[v] = HW_ID SIMD of wave v) and the block's CU ticket (tk: the second block of a CU
// mirrors): the rank of (simd[w], w) among the block's four (simd, wave) pairs, XOR mirror for tk = 1.
// Always a permutation of the four roles, whatever the placement (the pairs are distinct and totally
// ordered); equal to simd[w] (^ mirror) when the four SIMDs differ, the placement the issue
// priorities are tuned for.  (Dispatch gives no guarantee of that placement: MI355X_MICROARCH.md.)
#ifndef SIT_SIMD_ROLES
#define SIT_SIMD_ROLES 1    // fused k_env_steps_sync launches take their roles by SIMD (sit_sync.h)
#endif
#ifndef SIT_SIMD_MIRROR
#define SIT_SIMD_MIRROR 2   // the second block's roles: ^ 2 pairs (D0, P0), (D1, P1); ^ 3 pairs (D0, P1), (D1, P0)
#endif
__host__ __device__ constexpr int sync_role_of(int s0, int s1, int s2, int s3, int w, int tk, int mirror) {
  const int s[4] = {s0, s1, s2, s3};
  const int me = s[w];
  int rank = 0;
  for (int v = 0; v < 4; ++v) rank += (s[v] < me || (s[v] == me && v < w)) ? 1 : 0;
  return tk ? (rank ^ mirror) : rank;
}
// whether the four SIMDs are pairwise different (the placement the roles are tuned for)
__host__ __device__ constexpr bool sync_simds_distinct(int s0, int s1, int s2, int s3) {
  return ((1 << (s0 & 3)) | (1 << (s1 & 3)) | (1 << (s2 & 3)) | (1 << (s3 & 3))) == 0xF;
}
#ifndef SIT_ENVS_PER_BLOCK
#define SIT_ENVS_PER_BLOCK 64
#endif
// envs per step-kernel block: one wave of test ships + one wave of obstacle ships, the first
// kEnvsPerBlock lanes of each wave active
constexpr int kEnvsPerBlock = SIT_ENVS_PER_BLOCK;
#ifndef SIT_GROUPS
#define SIT_GROUPS 1
#endif
// env groups (wave pairs) per step-kernel block; the groups of a block share one LDS map copy
constexpr int kGroups = SIT_GROUPS;
#ifndef SIT_MIN_WAVES
#define SIT_MIN_WAVES 1   // step kernel: waves per SIMD the register budget must allow
#endif
constexpr int kMaxPolyVerts = 256;
constexpr int kMaxPolys = 32;

// --------------------------------------------------------------------------------------
// math overloads
// --------------------------------------------------------------------------------------
// float32 sine / cosine (the heading's every step, the IW direction): the hardware's v_sin / v_cos
// (argument scaled to revolutions; error measured and bounded by a GPU test) instead of
// the library's range-reduced polynomial: C3 +2.9 %, C5 +1.6 % in same-box A/Bs, float32 drift
// unchanged.  0: sincosf.  The float64 handle keeps the library's sin / cos.
#ifndef SIT_FAST_TRIG
#define SIT_FAST_TRIG 1
#endif
#if SIT_FAST_TRIG
// v_sin / v_cos take the angle in revolutions and only |x / 2 pi| <= 256.  The argument is scaled to
// revolutions in two parts, t = x * c_hi and its rounding error e = fma(x, c_hi, -t) + x * c_lo
// (c_hi + c_lo = 1 / 2 pi to ~2^-48), and reduced to [-0.5, 0.5] as (t - rint(t)) + e: t - rint(t) is
// exact, so the revolution carries no error of its own at any heading (the reference does not wrap
// headings, Q4).  Round to nearest, not v_fract: fract maps a small negative t to 1 - |t|, whose
// float32 grid (6e-8 rev) is far coarser than t's own.  What remains is the instructions' own error,
// measured and bounded by tests/test_gpu_parity.py::test_f32_fast_trig_accuracy (sit_selftest_f64
// ops 9-10; profiles/r06_f32_trig_accuracy.json).
__device__ __forceinline__ void xsincos(float x, float* s, float* c) {
#pragma clang fp reassociate(off) contract(off)
  constexpr float kRevHi = 0.15915493667125702f, kRevLo = 6.420638e-09f;
  const float t = x * kRevHi;
  const float e = __builtin_fmaf(x, kRevHi, -t) + x * kRevLo;
  const float rev = (t - __builtin_rintf(t)) + e;
  *s = __builtin_amdgcn_sinf(rev);
  *c = __builtin_amdgcn_cosf(rev);
}
#else
__device__ __forceinline__ void xsincos(float x, float* s, float* c) { sincosf(x, s, c); }
#endif
__device__ __forceinline__ void xsincos(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ float xatan2(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double xatan2(double y, double x) { return atan2(y, x); }
__device__ __forceinline__ float xatan(float x) { return atanf(x); }
__device__ __forceinline__ double xatan(double x) { return atan(x); }
__device__ __forceinline__ float xsqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ double xsqrt(double x) { return sqrt(x); }
__device__ __forceinline__ float xabs(float x) { return fabsf(x); }
__device__ __forceinline__ double xabs(double x) { return fabs(x); }
__device__ __forceinline__ float xfma(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double xfma(double a, double b, double c) { return fma(a, b, c); }
template <typename T> __device__ __forceinline__ T xmin(T a, T b) { return (b < a) ? b : a; }
template <typename T> __device__ __forceinline__ T xmax(T a, T b) { return (b > a) ? b : a; }
// np.clip / PiController.sat: max(low, min(val, hi))
template <typename T> __device__ __forceinline__ T xclip(T v, T lo, T hi) { return xmax(lo, xmin(v, hi)); }

// --------------------------------------------------------------------------------------
// constants (derived on the host in double, cast once to T)
// --------------------------------------------------------------------------------------
// the float64 values of every threshold and of the gains a knife-edge re-evaluation needs
// (float32 handle: decisions whose float32 margin lies inside the float32 error band are re-taken
// in float64 from the float32 state; float64 handle: the decisions themselves).  The step kernel
// reads them from its LDS copy of the constants inside the rare branches, so they hold no
// registers across the step loop.
struct ConstsX64 {
  double los_r, windup, e_tol, arrival, rpm_max, min_dist, blackout;
  double dt, kp1, ki1, kp2, ki2, avail_prop, me_cap, hotel, load_el_gen, bias_scale, bias_max;
  double half_len, theta;
};

template <typename T>
struct Consts {
  T dt;
  // kinetics (x_g = 0 => diagonal mass matrix)
  T mass, x_du, y_dv;
  T inv_m11, inv_m22, inv_m33;
  T d_u, d_v, d_r;         // linear damping diagonal: m/T_surge, m/T_sway, I_z/T_yaw
  T ku, kv, kr;            // non-linear damping (signed, Q8)
  T vc_n, vc_e;            // current in NED
  T wind_speed, wind_sin, wind_cos;
  T wk_u, wk_v, wk_n;      // wind load factors (see ship_dynamics)
  T c_rv, c_rr, rudder_max;
  // machinery (ship_engine.py:316-395)
  T avail_prop, avail_me, avail_el, tqcap_me, tqcap_el;
  T d_me, d_hsg, r_me, r_hsg, kp_prop, jp, thrust_k;
  T me_cap, hotel, load_el_gen;
  int32_t sg_mode;
  int32_t collision_bias;
  // SimplifiedMachineryModel (ship_engine.py:398-433; SIT_MACH_SIMPLIFIED): the shaft-speed slot
  // `w` holds the thrust force, d_thrust = (p_simpl * throttle - k_thrust * thrust) / tau
  int32_t mach_simpl;
  T k_thrust, inv_tau, p_simpl;
  // controllers
  T kp1, ki1, kp2, ki2, kp_h, kd_h, ki_h;
  // LOS
  T los_r, los_r2, los_clamp, los_ki, windup;
  double ra2;
  // collision-avoidance bias (MSRL_Env.py:244-251)
  T bias_scale, bias_max, bias_rudder;
  // reward / termination (MSRL_env_ex.py)
  T e_tol, arrival_radius, rpm_max, min_dist2, theta, blackout_kw, rpm_k, half_len;
  double arrive_d2_le;   // largest double x with sqrt(x) <= arrival_radius (MSRL_env_ex.py:754, 829)
  double coll_d2;        // minimum_ship_distance ** 2 (MSRL_env_ex.py:592)
  T inv_dt, inv_e_tol, inv_maxn, inv_jp, inv_r_me, inv_r_hsg;
  T min_n, max_n, min_e, max_e;
  T pi6;
  // map index geometry (see Map)
  T gx0, gy0, ginvx, ginvy;   // grid origin and 1 / cell size
  T by0, binv;                // band origin and 1 / band height
  T hull_safe;                // half_len * sqrt(2) + 1 m: beyond it all hull corners share the centre's side
  T fx0, fy0, finvx, finvy;   // fine class grid origin and 1 / cell size
  // trajectory log only (store_simulation_data, fuel model)
  T el_cap, fuel_me_a, fuel_me_b, fuel_me_c, fuel_dg_a, fuel_dg_b, fuel_dg_c, rad2deg;
  ConstsX64 x;
};

// machinery model of a handle: a compile-time constant inside the step kernel (MACH = 0 shaft,
// 1 simplified; k_env_steps dispatches once per wave), read from the constants elsewhere (-1)
template <int MACH, typename C>
__device__ __forceinline__ bool simpl_of(const C& c) {
  if constexpr (MACH >= 0) return MACH == 1;
  else return c.mach_simpl != 0;
}

// island map (obstacle.py:92-124): edge i of the closed rings runs from (ax, ay) to (bx, by);
// coordinates are (x = east, y = north) as in obstacle.py:128.  One Edge record per edge (one
// LDS base pointer, immediate field offsets) so the predicates need no per-array registers.
//
// Spatial index (built on the host by sit_load_map, exact by construction), one u16 array:
//   idx[0 .. 4*G*G)          grid cell records, 8 bytes each: the list's first group inline
//                            (x = ids 0-3, y bits 0-7 = id 4), y bits 8-15 = number of further
//                            groups, y bits 16-31 = the first of them (in 8-byte groups from the
//                            start of idx).  The cell's first 5 candidates are then one LDS read
//                            away from the cell index, their edges two.
//   idx[kBandBase ..]        NB+1 band starts (absolute positions in idx)
//   then the band entries (edge ids), then the further grid groups (8-byte aligned).
//  * grid: G x G cells over the map extent plus a margin; cell c lists every edge that can be
//    the nearest edge of some point within 1 m of the cell (conservative prefilter, then a
//    Lipschitz-sampled refinement with a 1 m float slack; sit_load_map), so the minimum over the
//    list equals the minimum over all edges.  A list is padded to a multiple of 5 with its first
//    id and packed as 5 u8 ids per 8-byte group, so one LDS read yields 5 ids whose edge loads
//    are independent (duplicates do not change a minimum).
//  * bands: NB horizontal bands; band b lists every edge whose y-range meets the band (+-1 m).
//    GEOS's ray-crossing test only looks at edges whose y-range contains the point's y.
//  * classes (separate u32 array): kFine x kFine cells over the map extent + 100 m, 2 bits per
//    cell: 0 = no boundary within 1 m of the cell and its points are outside every polygon,
//    1 = likewise inside one, 2 = mixed.  A point outside the class grid is > 100 m off the
//    map and therefore outside every polygon.  With ~40 m cells every point farther than
//    ~31 m from the shore resolves by one lookup.
constexpr int kGrid = 32;
constexpr int kBands = 64;
constexpr int kBandBase = 4 * kGrid * kGrid;
constexpr int kIdxHead = kBandBase + kBands + 1;
constexpr int kFine = 256;
constexpr int kFineWords = kFine * kFine / 16;

template <typename T>
struct alignas(16) Edge {
  T ax, ay, bx, by;
  T il2;            // 1 / |edge|^2 (0 for a degenerate edge)
  uint32_t poly;    // polygon id
};

template <typename T>
struct Map {
  const Edge<T>* edge;      // [n_edge] (LDS copy in the step kernel)
  const uint16_t* idx;      // packed index (LDS copy in the step kernel)
  const uint32_t* fine;     // [kFineWords] 2-bit cell classes (LDS copy in the step kernel)
  int32_t n_edge;
  int32_t use_index;        // 0: full scans only
  // point-in-polygon records of the mixed class cells (LDS copy in the step kernel):
  //   frank[w]  number of mixed cells in class words [0, w)   (rank of a mixed cell)
  //   crec[r]   (x) per-polygon crossing parity that every point of the cell collects from the
  //             edges whose contribution is the same for the whole cell (checked with a 1 m
  //             margin on the host), (y) first | count << 16 of the cell's live edges in clive
  //   clive[]   edge ids (u8) whose contribution varies inside the cell
  const uint16_t* frank;
  const uint2* crec;
  const uint8_t* clive;
  int32_t use_cells;
  int32_t n_idx, n_mixed, n_live;   // entries of idx / crec / clive (bounds of the debug checks)
  // fallback scan (global memory): polygon ring offsets and bounding boxes
  const int32_t* off;       // [n_poly + 1]
  const T* bbox;            // [n_poly][4] min_x, max_x, min_y, max_y
  int32_t n_poly;
};

// --------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. SC'11)
// --------------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += W0; k1 += W1; }
    const uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
    const uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
  }
}

// 53-bit uniform in [0,1) from Philox(key=seed, ctr=(env_id, event, 0x5A4D, 0))
__device__ __forceinline__ double sampler_uniform(uint64_t seed, uint64_t env_id, uint32_t event) {
  uint32_t c[4] = {(uint32_t)env_id, event, 0x5A4Du, 0u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const double hi = (double)(c[0] >> 5), lo = (double)(c[1] >> 6);
  return (hi * 67108864.0 + lo) * (1.0 / 9007199254740992.0);
}

// standard normal from Philox(key=seed, ctr=(env_id, event, 0x504F, 0)) by Box-Muller (two
// 53-bit uniforms, u1 in (0, 1]): the policy's reparameterisation noise of a sampling event
__device__ __forceinline__ double sampler_normal(uint64_t seed, uint64_t env_id, uint32_t event) {
  uint32_t c[4] = {(uint32_t)env_id, event, 0x504Fu, 0u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const double u1 = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6) + 1.0) * (1.0 / 9007199254740992.0);
  const double u2 = ((double)(c[2] >> 5) * 67108864.0 + (double)(c[3] >> 6)) * (1.0 / 9007199254740992.0);
  return sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
}

// --------------------------------------------------------------------------------------
// route access: the body of a ship's route (waypoints 0 .. n_wpt-2) lives in a column of a
// [cap][stride] table (global or LDS); the final waypoint is held in registers because
// insertion happens at index -1 (controllers.py:298-303) and never moves it.
// --------------------------------------------------------------------------------------
//
// The active leg (waypoints k-1 and k) and the next target (k+1) are cached in registers with
// their geometry, so the waypoint switch of a step is a register select (no branch around a
// table read in the step's instruction stream); the next target is refilled by fixup() at the
// end of the step.  The table is written only by an insertion, so it stays in HBM.
// The leg's path-tangential angle and its sine and cosine (LOS_guidance.py:110-113).  float64: the
// reference's own sin(atan2(dy, dx)), cos(atan2(dy, dx)) (computed once per leg), so the
// cross-track error and the clamp decision |e_ct| >= lookahead follow the reference to the last
// bit; float32: dy / L, dx / L (the same values within float32 rounding; knife edges of the clamp
// are re-taken in float64 by los_exact).
template <typename T>
__device__ __forceinline__ void leg_geom(T pn, T pe, T cn, T ce, T& alpha, T& sa, T& ca) {
  const T dx = cn - pn, dy = ce - pe;
  alpha = xatan2(dy, dx);
  if constexpr (kIsF32<T>) {
    const T len = xsqrt(dx * dx + dy * dy);
    sa = T(0);
    ca = T(1);
    if (len > T(0)) { sa = dy / len; ca = dx / len; }
  } else {
    xsincos(alpha, &sa, &ca);
  }
}

template <typename T>
struct Route {
  T* tn;          // column base: entry i at tn[i * stride]
  T* te;
  int stride;
  int cap;        // table rows (wpt_capacity)
  T end_n, end_e;
  int nw;         // current number of waypoints
  T pn, pe;       // waypoint k-1
  T cn, ce;       // waypoint k
  // the leg's path-tangential angle and its sine/cosine (LOS_guidance.py:110-113) depend only
  // on the two waypoints: computed when the leg changes, not every step (same values)
  T alpha, sa, ca;
  T nn, ne;                 // waypoint k+1 (the target after a switch)
  T alpha_n, sa_n, ca_n;    // geometry of the leg k -> k+1
  bool fix;                 // a switch consumed the next target: refill it (fixup)
  // waypoint i: the table entry, or the final waypoint for i >= nw - 1.  The table is read
  // unconditionally at min(i, nw - 1) (inside the column: nw <= capacity), so a leg's loads issue
  // together instead of behind one branch each (one memory round trip per leg reload)
  __device__ __forceinline__ T n(int i) const {
    const T v = tn[SIT_DCLAMP(i < nw - 1 ? i : nw - 1, cap, kDbgRouteIndex) * stride];
    return (i >= nw - 1) ? end_n : v;
  }
  __device__ __forceinline__ T e(int i) const {
    const T v = te[SIT_DCLAMP(i < nw - 1 ? i : nw - 1, cap, kDbgRouteIndex) * stride];
    return (i >= nw - 1) ? end_e : v;
  }
  __device__ __forceinline__ void load_next(int k) {
    nn = n(k + 1); ne = e(k + 1);
    leg_geom(cn, ce, nn, ne, alpha_n, sa_n, ca_n);
  }
  __device__ __forceinline__ void load_leg(int k) {
    SIT_DCHECK(nw >= 2 && nw <= cap, kDbgRouteLen);
    SIT_DCHECK(k >= 1 && k < nw, kDbgWaypoint);
    pn = n(k - 1); pe = e(k - 1); cn = n(k); ce = e(k);
    leg_geom(pn, pe, cn, ce, alpha, sa, ca);
    load_next(k);
    fix = false;
  }
  // NavigationSystem.next_wpt's advance (LOS_guidance.py:88-103) as register selects
  __device__ __forceinline__ void advance(bool sw, int& k) {
    k += sw ? 1 : 0;
    pn = sw ? cn : pn; pe = sw ? ce : pe;
    cn = sw ? nn : cn; ce = sw ? ne : ce;
    alpha = sw ? alpha_n : alpha; sa = sw ? sa_n : sa; ca = sw ? ca_n : ca;
    fix = fix || sw;
  }
  // the cached leg state (k, leg, next target, geometry) of a given route length, for register
  // copies of an episode start (reset restores the construction route, Q16)
  struct Leg {
    T pn, pe, cn, ce, nn, ne, alpha, sa, ca, alpha_n, sa_n, ca_n;
  };
  __device__ __forceinline__ Leg leg() const {
    return Leg{pn, pe, cn, ce, nn, ne, alpha, sa, ca, alpha_n, sa_n, ca_n};
  }
  __device__ __forceinline__ void set_leg(const Leg& l) {
    pn = l.pn; pe = l.pe; cn = l.cn; ce = l.ce; nn = l.nn; ne = l.ne;
    alpha = l.alpha; sa = l.sa; ca = l.ca; alpha_n = l.alpha_n; sa_n = l.sa_n; ca_n = l.ca_n;
    fix = false;
  }
  __device__ __forceinline__ void fixup(int k) {
#ifdef SIT_ABL_FIXUP   // timing ablation (diagnostic builds only, results wrong): no route-table read
    if (fix) { nn = cn + T(100); ne = ce + T(100); leg_geom(cn, ce, nn, ne, alpha_n, sa_n, ca_n); fix = false; (void)k; }
#else
    if (fix) { load_next(k); fix = false; }
#endif
  }
  // update_route: insert (in_, ie) at index -1 (controllers.py:298-303); false on overflow
  __device__ __forceinline__ bool insert(T in_, T ie, int k, int cap) {
    if (nw >= cap) return false;
    const int i = nw - 1;
    tn[i * stride] = in_;
    te[i * stride] = ie;
    nw += 1;
    // the new next target is known without reading the table back: the final waypoint (k == i) or
    // the entry just written (k + 1 == i).  (load_next here put a dependent global load on the
    // obstacle's segment before guidance at most sampling events: C3 +0.3 %, C5 +0.8 % without it)
    if (k == i) {                         // the leg pointed at the final waypoint
      cn = in_; ce = ie;
      leg_geom(pn, pe, cn, ce, alpha, sa, ca);
      nn = end_n; ne = end_e;
      leg_geom(cn, ce, nn, ne, alpha_n, sa_n, ca_n);
    } else if (k + 1 == i) {              // the next target was the final waypoint
      nn = in_; ne = ie;
      leg_geom(cn, ce, nn, ne, alpha_n, sa_n, ca_n);
    }
    return true;
  }
};

// --------------------------------------------------------------------------------------
// one ship
// --------------------------------------------------------------------------------------
template <typename T>
struct Ship {
  T n, e, psi, u, v, r, w;   // pose, body velocities, shaft speed
  T i1, i2;                  // ship-speed PI and shaft-speed PI integrals
  T hi, hp;                  // heading PID integral and previous error
  T ect_int;                 // LOS cross-track integral
  T lrpm, lect, lpme;        // last stored observations (stop path)
  // float32: the low parts of the integrators (comp_add): the value is n + ln etc.  float64: unused
  T ln, le, lpsi, li1, li2, lhi, lei;
  T lu, lv, lr, lw;          // float32: the velocities' and the shaft speed's low parts (SIT_COMP_VEL / _W)
  int k;                     // next waypoint index
  int ticks;                 // simulator time in dt units
  int stop;                  // ShipAssets.stop_flag
};

// Integrators of the float32 handle as double-float values (hi + lo).  The reference integrates in
// float64; a float32 sum x += dx loses up to half an ulp of x every step, and for the integrators that
// nothing pulls back — the position along the track (ulp 4.9e-4 m at 4-8 km), the shaft-speed PI
// integral (1e5-1e6, ulp 0.008-0.06), the heading and the other PI/PID and LOS integrals, the sampling
// distance — those losses random-walk: 1e-3 - 1e-2 m of position after 2 000 steps, which moved
// waypoint switches, sampling events and terrain contacts (profiles/r04_f32_flip_attribution.json).
// comp_add carries each step's rounding error in lo and adds it back with the next increment
// (compensated summation, Fast2Sum: |hi| >= |inc| for all but zero crossings, where the terms are
// small): hi stays the float32-rounded running sum and the error no longer accumulates.  The
// decisions read hi + lo in float64 (comp_val).  float64 handles: the plain sum.
#ifndef SIT_COMP
#define SIT_COMP 1   // (0: experiment only, plain float32 sums, to price the compensation)
#endif
template <typename T>
constexpr bool kComp = kIsF32<T> && SIT_COMP != 0;

template <typename T>
__device__ __forceinline__ T comp_add(T hi, T& lo, T inc) {
  if constexpr (kComp<T>) {
#pragma clang fp reassociate(off) contract(off)
    const T y = inc + lo;
    const T t = hi + y;
    lo = y - (t - hi);
    return t;
  } else {
    (void)lo;
    return hi + inc;
  }
}
// hi + a * b as comp_add, the product fused into the low part's update: y = fma(a, b, lo), t = hi + y
// (one dependent instruction more on the integrator's chain than the plain fma; folding lo / dt into the
// factor instead kept the chain but measured C3 -2 %: more registers live across guidance)
template <typename T>
__device__ __forceinline__ T comp_fma(T hi, T& lo, T a, T b) {
  if constexpr (kComp<T>) {
#pragma clang fp reassociate(off) contract(off)
    const T y = __builtin_fmaf(a, b, lo);
    const T t = hi + y;
    lo = y - (t - hi);
    return t;
  } else {
    (void)lo;
    return hi + a * b;
  }
}
// per-integrator switches (experiments: which compensations the float32 drift needs)
#ifndef SIT_COMP_PSI
#define SIT_COMP_PSI 1   // the heading
#endif
#ifndef SIT_COMP_PI
#define SIT_COMP_PI 1    // the heading PID and the ship-speed PI integrals
#endif
#ifndef SIT_COMP_VEL
#define SIT_COMP_VEL 1   // surge, sway and yaw rate (round 6)
#endif
#ifndef SIT_COMP_W
#define SIT_COMP_W 1     // the shaft speed (the thrust force with the simplified machinery; round 6)
#endif
#ifndef SIT_PID_ERR_LO
#define SIT_PID_ERR_LO 1 // the heading PID's error from the heading's hi + lo (0: from hi alone)
#endif
template <bool ON, typename T>
__device__ __forceinline__ T comp_fma_if(T hi, T& lo, T a, T b) {
  if constexpr (ON) return comp_fma(hi, lo, a, b);
  else { (void)lo; return hi + a * b; }
}
template <typename T>
__device__ __forceinline__ double comp_val(T hi, T lo) {
  if constexpr (kComp<T>) return ieee_add((double)hi, (double)lo);
  else { (void)lo; return (double)hi; }
}
// a - b of two double-float values, rounded to T: (a_hi - b_hi) is exact for nearby float32 values
template <typename T>
__device__ __forceinline__ T comp_diff(T a, T al, T b, T bl) {
  if constexpr (kComp<T>) {
#pragma clang fp reassociate(off) contract(off)
    return (a - b) + (al - bl);
  } else {
    (void)al; (void)bl;
    return a - b;
  }
}

// rudder_angle_from_sampled_route + throttle (controllers.py:306-314, 138-143, 52-62, 81-93,
// 180-189; LOS_guidance.py:88-121).  Returns rudder, throttle and |e_ct|.
// LOS_guidance.py:110-120 in the reference's float64 arithmetic from the (float32) state: the
// cross-track error |e|, the (clamped) e / Delta and whether the integrator accepts it
// inlined: as an out-of-line call it cost 2 % of C3 (call frame and register saves around a
// branch that is almost never taken)
#ifndef SIT_LOS_EXACT_INLINE
#define SIT_LOS_EXACT_INLINE __attribute__((always_inline))
#endif
template <typename T>
__device__ SIT_LOS_EXACT_INLINE void los_exact(const ConstsX64& x, double n, double e, T pn, T pe, T cn, T ce, double ect_int,
                                                    double& ect_abs, double& q, double& sum, bool& accept) {
  // sin / cos of the leg angle as dy / L, dx / L in IEEE float64: equal to the reference's
  // math.sin / math.cos of math.atan2 (:110-113) within an ulp or two, so e_ct is within ~1e-12 m of
  // the reference's on the same float32 state (decisions closer than that to the threshold are the
  // float64 libm-ulp knife edges no other libm reproduces).  Kept free of the libm's trigonometric
  // code: this branch sits inside the step loop, whose instruction footprint is what it costs.
  const double dx = ieee_sub(cn, pn), dy = ieee_sub(ce, pe);
  const double len = ieee_sqrt(ieee_sq2(dx, dy));
  const double sa = len > 0.0 ? ieee_div(dy, len) : 0.0, ca = len > 0.0 ? ieee_div(dx, len) : 1.0;
  double ect = ieee_add(ieee_mul(-ieee_sub(n, (double)pn), sa), ieee_mul(ieee_sub(e, (double)pe), ca));
  ect_abs = fabs(ect);
  const double r2 = ieee_mul(x.los_r, x.los_r);
  if (ieee_mul(ect, ect) >= r2) ect = ieee_mul(0.99, x.los_r);
  q = ieee_div(ect, ieee_sqrt(ieee_sub(r2, ieee_mul(ect, ect))));
  sum = ieee_add(ect_int, q);
  accept = fabs(sum) <= x.windup;
}

// ect_over: |e_ct| > e_tolerance (the navigation-failure predicate, MSRL_env_ex.py:560-576) decided
// exactly (float64 inside the float32 band)
template <typename T, int MACH = -1, typename C>
__device__ __forceinline__ void guidance_control(const C& c, const ConstsX64& x, Ship<T>& s, Route<T>& rt,
                                                 T v_des, T& rudder, T& thr, T& ect_abs, T& psi_ref_out,
                                                 bool& ect_over) {
  // next_wpt: acceptance test evaluated in IEEE float64 from the stored values (the reference's
  // decision for the same state; LOS_guidance.py:96)
  // (float32: the position's double-float value; cn - n is exact in float64, then the low part)
  double acc_dn, acc_de;
  if constexpr (kComp<T>) {
    acc_dn = ieee_sub(ieee_sub(rt.cn, s.n), (double)s.ln);
    acc_de = ieee_sub(ieee_sub(rt.ce, s.e), (double)s.le);
  } else {
    acc_dn = ieee_sub(rt.cn, s.n);
    acc_de = ieee_sub(rt.ce, s.e);
  }
  rt.advance(ieee_sq2(acc_dn, acc_de) <= c.ra2 && rt.nw > s.k + 1, s.k);
  const T pn = rt.pn, pe = rt.pe;
  const T alpha = rt.alpha, sa = rt.sa, ca = rt.ca;
  T q, sum;
  T sum_lo = s.lei;
  bool accept;
  if constexpr (kIsF32<T>) {
    T ect = -(s.n - pn) * sa + (s.e - pe) * ca;
    ect_abs = xabs(ect);
    ect_over = ect_abs > c.e_tol;
    if (ect * ect >= c.los_r2) ect = c.los_clamp;         // sign lost (Q5)
    const T delta = xsqrt(c.los_r2 - ect * ect);
    q = ect / delta;
    sum = comp_add(s.ect_int, sum_lo, q);
    accept = xabs(sum) <= c.windup;
    // knife edges of the clamp (|e| = lookahead), of the navigation-failure threshold (|e| =
    // e_tolerance) and of the anti-windup limit: float32 carries ~1e-3 m of rounding in e and
    // ~3e-4 in the integral, so inside these bands the decisions are re-taken in float64
    const bool knife = kKnifeLos && (xmin(xabs(ect_abs - c.los_r), xabs(ect_abs - c.e_tol)) < T(0.05) ||
                                  xabs(xabs(sum) - c.windup) < T(0.02));
    if (knife) {
      double ex, qd, sd;
      los_exact(x, comp_val(s.n, s.ln), comp_val(s.e, s.le), pn, pe, rt.cn, rt.ce, comp_val(s.ect_int, s.lei), ex,
                qd, sd, accept);
      ect_over = ex > x.e_tol;
      ect_abs = (T)ex;
      q = (T)qd;
      sum = (T)sd;
      sum_lo = (T)ieee_sub(sd, (double)sum);
    }
  } else {
    // float64: the reference's operation order (LOS_guidance.py:112-119; no fused multiply-add,
    // sin/cos of atan2 cached with the leg), so the clamp and windup decisions are its own
    double e = ieee_add(ieee_mul(-ieee_sub(s.n, pn), sa), ieee_mul(ieee_sub(s.e, pe), ca));
    ect_abs = fabs(e);
    ect_over = ect_abs > x.e_tol;
    const double r2 = ieee_mul(x.los_r, x.los_r);
    if (ieee_mul(e, e) >= r2) e = ieee_mul(0.99, x.los_r);   // sign lost (Q5)
    q = ieee_div(e, ieee_sqrt(ieee_sub(r2, ieee_mul(e, e))));
    sum = ieee_add(s.ect_int, q);
    accept = fabs(sum) <= x.windup;
  }
  if (accept) { s.ect_int = sum; s.lei = sum_lo; }
  const T chi = xatan(-q - s.ect_int * c.los_ki);
  const T psi_ref = alpha + chi;
  psi_ref_out = psi_ref;
  // heading PID, error not wrapped (Q4).  float32: err = ((alpha - psi) - lpsi) + chi, not
  // (alpha + chi) - psi: alpha - psi is exact (Sterbenz), so neither the float32 rounding of
  // psi_ref = alpha + chi (up to 1.2e-7 rad, constant along a straight leg) nor the heading's low part
  // enters err as a bias the PID integral would accumulate.  (Measured: the heading integral's float32
  // deviation is not bounded by these biases but by the trajectory's own)
  T err;
  if constexpr (kComp<T> && SIT_PID_ERR_LO) {
#pragma clang fp reassociate(off) contract(off)
    err = ((alpha - s.psi) - s.lpsi) + chi;
  } else {
    err = psi_ref - s.psi;
  }
  const T derr = (err - s.hp) * c.inv_dt;
  s.hi = comp_fma_if<SIT_COMP_PI != 0>(s.hi, s.lhi, err, c.dt);
  s.hp = err;
  const T out = err * c.kp_h + derr * c.kd_h + s.hi * c.ki_h;
  rudder = xclip(-out, -c.rudder_max, c.rudder_max);
  // cascaded PI, shaft PI measures the ship speed (Q2), no saturation (Q3)
  const T e1 = v_des - s.u;
  s.i1 = comp_fma_if<SIT_COMP_PI != 0>(s.i1, s.li1, e1, c.dt);
  const T wdes = e1 * c.kp1 + s.i1 * c.ki1;
  if (simpl_of<MACH>(c)) {
    // ThrottleFromSpeedSetPointSimplifiedPropulsion.throttle (controllers.py:170-172): the ship-speed
    // PI alone, saturated to [0, 1.1]
    thr = xclip(wdes, T(0), T(1.1));
  } else {
    const T e2 = wdes - s.u;
    s.i2 = comp_fma(s.i2, s.li2, e2, c.dt);
    thr = e2 * c.kp2 + s.i2 * c.ki2;
  }
}

// EngineThrottleFromSpeedSetPoint.throttle (controllers.py:52-62, 138-143) in the reference's
// float64 arithmetic from the pre-step integrals i1, i2 and surge u; with the collision bias of
// MSRL_Env.py:244-251 when `bias`
template <typename T>
__device__ __forceinline__ double throttle_exact(const ConstsX64& x, T u, T v_des, double i1, double i2, bool bias,
                                                 bool simpl) {
  const double e1 = ieee_sub(v_des, u);
  const double ii1 = ieee_add(i1, ieee_mul(e1, x.dt));
  const double wdes = ieee_dot2(e1, x.kp1, ii1, x.ki1);
  double thr;
  if (simpl) {   // ThrottleFromSpeedSetPointSimplifiedPropulsion (controllers.py:170-172)
    thr = fmax(0.0, fmin(wdes, 1.1));
  } else {
    const double e2 = ieee_sub(wdes, u);
    const double ii2 = ieee_add(i2, ieee_mul(e2, x.dt));
    thr = ieee_dot2(e2, x.kp2, ii2, x.ki2);
  }
  if (bias) thr = fmax(0.0, fmin(ieee_mul(thr, x.bias_scale), x.bias_max));
  return thr;
}

// distribute_load(...).load_on_main_engine / 1000 in float64 (ship_engine.py:46-76)
__device__ __forceinline__ double power_me_kw_exact(int sg_mode, const ConstsX64& x, double thr) {
  const double total = ieee_mul(thr, x.avail_prop);
  double load_me;
  if (sg_mode == 0) load_me = fmin(total, x.me_cap);
  else if (sg_mode == 1) load_me = ieee_sub(ieee_add(total, x.hotel), x.load_el_gen);
  else load_me = total;
  return ieee_div(load_me, 1000.0);
}

// is_mechanical_failure (MSRL_env_ex.py:554-558): |shaft speed * 30 / pi| > shaft_rpm_max, with
// rpm = w * 30 / pi (ship_model.py:652) re-taken in float64 near the threshold
template <typename T, int MACH = -1>
__device__ __forceinline__ bool rpm_fails(const Consts<T>& c, const ConstsX64& x, T w, T rpm) {
  if (simpl_of<MACH>(c)) return false;   // no shaft: the observed shaft speed is 0
  if constexpr (kIsF32<T>) {
    // at or beyond the threshold's float32 band: decided in float64 (rare: a failing shaft)
    if (!kKnifeRpm) return xabs(rpm) > c.rpm_max;
    if (xabs(rpm) > c.rpm_max - T(0.01)) return fabs(ieee_div(ieee_mul(w, 30.0), M_PI)) > x.rpm_max;
    return false;
  } else {
    return fabs(ieee_div(ieee_mul(w, 30.0), M_PI)) > x.rpm_max;
  }
}

// sqrt(dn^2 + de^2) <= r (arrival, MSRL_env_ex.py:754, 829) / dn^2 + de^2 < r^2 (collision, :592)
// as the reference evaluates them in float64, decided in float32 away from the boundary
// Both evaluated in IEEE float64 every step, branch-free (a rare-path branch inside the step loop
// measured ~100 cycles per wave-step; these are ~10 VALU, and a float64 VALU instruction issues as
// fast as a float32 one at one wave per SIMD).  sqrt(d2) <= r is decided as d2 <= d2_le with d2_le
// the largest double whose correctly rounded square root is <= r (host-computed, exact).
template <typename T>
__device__ __forceinline__ bool within_radius(T n0, T e0, T n1, T e1, double d2_le) {
  if constexpr (!kKnifeRad && kIsF32<T>) {
    const T dn = n0 - n1, de = e0 - e1;
    return dn * dn + de * de <= (T)d2_le;
  }
  return ieee_sq2(ieee_sub(n0, n1), ieee_sub(e0, e1)) <= d2_le;
}
template <typename T>
__device__ __forceinline__ bool closer_than(T n0, T e0, T n1, T e1, double r2) {
  if constexpr (!kKnifeRad && kIsF32<T>) {
    const T dn = n0 - n1, de = e0 - e1;
    return dn * dn + de * de < (T)r2;
  }
  return ieee_sq2(ieee_sub(n0, n1), ieee_sub(e0, e1)) < r2;
}

// One row of ShipModelAST.store_simulation_data (ship_model.py:645-684) from the pre-integration
// state s, written to dst[key * stride] for the SIT_LOG_KEYS keys; the fuel accumulators advance
// (BaseMachineryModel.fuel_consumption, ship_engine.py:263-289; load split
// MachineryMode.distribute_load, ship_engine.py:46-76; torque :369-376; thrust :363-366).
// (An out-of-line version made the whole step kernel 2.2x slower: calls give it a stack.)
template <typename T, int MACH = -1>
__device__ __forceinline__ void store_log_row(const Consts<T>& c, T* dst, size_t stride, const Ship<T>& s, T thr,
                                              T rudder, T ect, T psi_ref, T& fuel_me, T& fuel_el, T& fuel) {
  const T total = thr * c.avail_prop;
  T load_me, load_el, lp_me, lp_el;
  if (c.sg_mode == 0) {          // MOTOR
    load_me = xmin(total, c.me_cap);
    load_el = total + c.hotel - load_me;
    lp_el = load_el / c.el_cap;
    lp_me = (c.me_cap == T(0)) ? T(0) : load_me / c.me_cap;
  } else if (c.sg_mode == 1) {   // GEN
    load_el = c.load_el_gen;
    load_me = total + c.hotel - load_el;
    lp_me = load_me / c.me_cap;
    lp_el = (c.el_cap == T(0)) ? T(0) : load_el / c.el_cap;
  } else {                       // OFF
    load_me = total;
    load_el = c.hotel;
    lp_me = load_me / c.me_cap;
    lp_el = load_el / c.el_cap;
  }
  const T rate_me = (load_me == T(0)) ? T(0)
                    : load_me * ((c.fuel_me_a * lp_me * lp_me + c.fuel_me_b * lp_me + c.fuel_me_c) / T(3.6e9));
  const T rate_el = (lp_el == T(0)) ? T(0)
                    : load_el * ((c.fuel_dg_a * lp_el * lp_el + c.fuel_dg_b * lp_el + c.fuel_dg_c) / T(3.6e9));
  fuel_me = fuel_me + rate_me * c.dt;
  fuel_el = fuel_el + rate_el * c.dt;
  fuel = fuel + (rate_me + rate_el) * c.dt;
  const T w = s.w;
  const T v[SIT_LOG_KEYS] = {
      T(s.ticks) * c.dt, s.n, s.e, s.psi * c.rad2deg, rudder * c.rad2deg, s.u, s.v, s.r * c.rad2deg,
      w * c.rpm_k, lp_me, lp_el, load_me / T(1000), c.me_cap / T(1000), load_el / T(1000),
      c.el_cap / T(1000), (load_el + load_me) / T(1000), total / T(1000), rate_me, rate_el, rate_me + rate_el,
      fuel_me, fuel_el, fuel, simpl_of<MACH>(c) ? T(0) : xmin(thr * c.avail_me / (w + T(0.1)), c.tqcap_me),
      (simpl_of<MACH>(c) ? w : c.thrust_k * w * xabs(w)) / T(1000), ect, xabs(s.psi - psi_ref)};
#pragma unroll
  for (int k = 0; k < SIT_LOG_KEYS; ++k) dst[k * stride] = v[k];
}

// distribute_load(...).load_on_main_engine / 1000 (ship_engine.py:46-76)
template <typename T>
__device__ __forceinline__ T power_me_kw(const Consts<T>& c, T thr) {
  const T total = thr * c.avail_prop;
  T load_me;
  if (c.sg_mode == 0) load_me = xmin(total, c.me_cap);                  // MOTOR
  else if (c.sg_mode == 1) load_me = total + c.hotel - c.load_el_gen;    // GEN
  else load_me = total;                                                 // OFF
  return load_me * T(0.001);
}

// update_differentials + integrate_differentials; sp, cp = sin/cos of the pre-step heading
// (computed by the caller at the start of the step, off the guidance dependency chain) (ship_model.py:624-643, ship_engine.py:355-395)
// The post-step position needs only the pre-step state (forward Euler of eta_dot = R(psi) nu):
// the step kernel computes it at the start of the step and issues the map lookups of that
// position before guidance and dynamics (their LDS latency then overlaps the step's arithmetic);
// ship_dynamics_pos stores exactly that position.
// (ln1, le1: the post-step position's low parts, comp_add)
template <typename T>
__device__ __forceinline__ void euler_position(const Consts<T>& c, const Ship<T>& s, T sp, T cp, T& n1, T& e1, T& ln1,
                                               T& le1) {
  const T d_n = cp * s.u - sp * s.v;
  const T d_e = sp * s.u + cp * s.v;
  ln1 = s.ln;
  le1 = s.le;
  n1 = comp_fma(s.n, ln1, d_n, c.dt);
  e1 = comp_fma(s.e, le1, d_e, c.dt);
}

template <typename T, int MACH = -1>
__device__ __forceinline__ void ship_dynamics_pos(const Consts<T>& c, Ship<T>& s, T thr, T rudder, T sp, T cp, T n1,
                                                  T e1, T ln1, T le1);

template <typename T, int MACH = -1>
__device__ __forceinline__ void ship_dynamics(const Consts<T>& c, Ship<T>& s, T thr, T rudder, T sp, T cp) {
  T n1, e1, ln1, le1;
  euler_position(c, s, sp, cp, n1, e1, ln1, le1);
  ship_dynamics_pos<T, MACH>(c, s, thr, rudder, sp, cp, n1, e1, ln1, le1);
}

template <typename T, int MACH>
__device__ __forceinline__ void ship_dynamics_pos(const Consts<T>& c, Ship<T>& s, T thr, T rudder, T sp, T cp, T n1,
                                                  T e1, T ln1, T le1) {
  const T u = s.u, v = s.v, r = s.r, w = s.w;
  T d_w, thrust;
  if (simpl_of<MACH>(c)) {
    // SimplifiedMachineryModel.update_thrust_force (ship_engine.py:423-428): w is the thrust force
    thrust = w;
    d_w = (thr * c.p_simpl - c.k_thrust * w) * c.inv_tau;
  } else {
    // shaft equation with pre-step omega
    const T inv_w = T(1) / (w + T(0.1));
    const T tq_me = xmin(thr * c.avail_me * inv_w, c.tqcap_me);
    const T tq_hsg = xmin(thr * c.avail_el * inv_w, c.tqcap_el);
    d_w = ((tq_me - c.d_me * w) * c.inv_r_me + (tq_hsg - c.d_hsg * w) * c.inv_r_hsg - c.kp_prop * (w * w)) * c.inv_jp;
    thrust = c.thrust_k * w * xabs(w);
  }
  // current in body frame: R(psi)^T v_c
  const T vc_u = cp * c.vc_n + sp * c.vc_e;
  const T vc_v = -sp * c.vc_n + cp * c.vc_e;
  const T ur = u - vc_u, vr = v - vc_v;
  // rudder forces (ship_model.py:608-622)
  const T f_rv = -c.c_rv * rudder * ur;
  const T f_rr = -c.c_rr * rudder * ur;
  // wind (ship_model.py:211-231): with gamma = -atan2(v_rw, u_rw), cos g = u_rw/|w|,
  // sin g = -v_rw/|w|, so tau = (-0.5 rho cx Af |w| u_rw, -0.5 rho cy Al |w| v_rw,
  // -rho cn Al L u_rw v_rw)
  const T uw = c.wind_speed * (c.wind_cos * cp + c.wind_sin * sp);   // cos(beta - psi)
  const T vw = c.wind_speed * (c.wind_sin * cp - c.wind_cos * sp);   // sin(beta - psi)
  const T urw = uw - u, vrw = vw - v;
  const T wmag = xsqrt(urw * urw + vrw * vrw);
  const T tau_u = c.wk_u * wmag * urw;
  const T tau_v = c.wk_v * wmag * vrw;
  const T tau_n = c.wk_n * urw * vrw;
  // -C_RB nu - C_A(nu_r) nu_r - (D + D_n) nu_r + tau  (ship_model.py:596-603)
  const T mv = c.mass * v, mu = c.mass * u;
  const T yv = c.y_dv * vr, xu = c.x_du * ur;
  const T f0 = mv * r - yv * r - (c.d_u + c.ku * u) * ur + tau_u + thrust;
  const T f1 = -mu * r + xu * r - (c.d_v + c.kv * v) * vr + tau_v + f_rv;
  const T f2 = -(mv * u - mu * v) - (-yv * ur + xu * vr) - (c.d_r + c.kr * r) * r + tau_n + f_rr;
  // Euler (utils.py:50-53); the position from euler_position
  s.n = n1;
  s.e = e1;
  s.ln = ln1;
  s.le = le1;
  s.psi = comp_fma_if<SIT_COMP_PSI != 0>(s.psi, s.lpsi, r, c.dt);
  s.u = comp_fma_if<SIT_COMP_VEL != 0>(u, s.lu, c.inv_m11 * f0, c.dt);
  s.v = comp_fma_if<SIT_COMP_VEL != 0>(v, s.lv, c.inv_m22 * f1, c.dt);
  s.r = comp_fma_if<SIT_COMP_VEL != 0>(r, s.lr, c.inv_m33 * f2, c.dt);
  s.w = comp_fma_if<SIT_COMP_W != 0>(w, s.lw, d_w, c.dt);
}

// ship_dynamics_pos in two parts with the same operations in the same order: DynBase holds every
// term of the pre-step state alone (ship_model.py:596-603 without the rudder forces; the shaft
// equation without the throttle; the thrust of the pre-step shaft speed), dyn_finish adds the rudder
// and throttle terms and integrates.  The step kernel computes the base before guidance, so its
// arithmetic fills the latency of guidance's serial chain.
template <typename T>
struct DynBase {
  T ur;                 // surge relative to the current (the rudder forces' speed)
  T f0, f1, f2;         // forces without the rudder terms
  T inv_w;              // 1 / (w + 0.1) (the shaft equation's torque limit)
};
template <typename T, int MACH, typename C>
__device__ __forceinline__ DynBase<T> dyn_base(const C& c, const Ship<T>& s, T sp, T cp) {
  const T u = s.u, v = s.v, r = s.r, w = s.w;
  DynBase<T> b;
  T thrust;
  if (simpl_of<MACH>(c)) {
    thrust = w;
    b.inv_w = T(0);
  } else {
    b.inv_w = T(1) / (w + T(0.1));
    thrust = c.thrust_k * w * xabs(w);
  }
  const T vc_u = cp * c.vc_n + sp * c.vc_e;
  const T vc_v = -sp * c.vc_n + cp * c.vc_e;
  const T ur = u - vc_u, vr = v - vc_v;
  b.ur = ur;
  const T uw = c.wind_speed * (c.wind_cos * cp + c.wind_sin * sp);
  const T vw = c.wind_speed * (c.wind_sin * cp - c.wind_cos * sp);
  const T urw = uw - u, vrw = vw - v;
  const T wmag = xsqrt(urw * urw + vrw * vrw);
  const T tau_u = c.wk_u * wmag * urw;
  const T tau_v = c.wk_v * wmag * vrw;
  const T tau_n = c.wk_n * urw * vrw;
  const T mv = c.mass * v, mu = c.mass * u;
  const T yv = c.y_dv * vr, xu = c.x_du * ur;
  b.f0 = mv * r - yv * r - (c.d_u + c.ku * u) * ur + tau_u + thrust;
  b.f1 = -mu * r + xu * r - (c.d_v + c.kv * v) * vr + tau_v;
  b.f2 = -(mv * u - mu * v) - (-yv * ur + xu * vr) - (c.d_r + c.kr * r) * r + tau_n;
  return b;
}
template <typename T, int MACH, typename C>
__device__ __forceinline__ void dyn_finish(const C& c, Ship<T>& s, const DynBase<T>& b, T thr, T rudder,
                                           T n1, T e1, T ln1, T le1) {
  const T u = s.u, v = s.v, r = s.r, w = s.w;
  T d_w;
  if (simpl_of<MACH>(c)) {
    d_w = (thr * c.p_simpl - c.k_thrust * w) * c.inv_tau;
  } else {
    const T tq_me = xmin(thr * c.avail_me * b.inv_w, c.tqcap_me);
    const T tq_hsg = xmin(thr * c.avail_el * b.inv_w, c.tqcap_el);
    d_w = ((tq_me - c.d_me * w) * c.inv_r_me + (tq_hsg - c.d_hsg * w) * c.inv_r_hsg - c.kp_prop * (w * w)) * c.inv_jp;
  }
  const T f_rv = -c.c_rv * rudder * b.ur;
  const T f_rr = -c.c_rr * rudder * b.ur;
  s.n = n1;
  s.e = e1;
  s.ln = ln1;
  s.le = le1;
  s.psi = comp_fma_if<SIT_COMP_PSI != 0>(s.psi, s.lpsi, r, c.dt);
  s.u = comp_fma_if<SIT_COMP_VEL != 0>(u, s.lu, c.inv_m11 * b.f0, c.dt);
  s.v = comp_fma_if<SIT_COMP_VEL != 0>(v, s.lv, c.inv_m22 * (b.f1 + f_rv), c.dt);
  s.r = comp_fma_if<SIT_COMP_VEL != 0>(r, s.lr, c.inv_m33 * (b.f2 + f_rr), c.dt);
  s.w = comp_fma_if<SIT_COMP_W != 0>(w, s.lw, d_w, c.dt);
}

// --------------------------------------------------------------------------------------
// polygon predicates (obstacle.py:126-141 -> GEOS)
// --------------------------------------------------------------------------------------
// exact sign of a*b - c*d (TwoProduct via fma, Shewchuk grow-expansion); out of line: it
// only runs when the orientation filter is uncertain
template <typename T>
__device__ __attribute__((noinline)) int exact_sign_diff(T a, T b, T c, T d) {
#pragma clang fp reassociate(off) contract(off)
  const T p1 = a * b, e1 = xfma(a, b, -p1);
  const T p2 = c * d, e2 = xfma(c, d, -p2);
  auto two_sum = [](T x, T y, T& err) { const T s = x + y; const T bb = s - x; err = (x - (s - bb)) + (y - bb); return s; };
  T h0, h1, g0, g1, g2;
  T q = two_sum(-e2, e1, h0);
  q = two_sum(q, p1, h1);
  const T h2 = q;
  T q2 = two_sum(-p2, h0, g0);
  q2 = two_sum(q2, h1, g1);
  q2 = two_sum(q2, h2, g2);
  const T comps[4] = {q2, g2, g1, g0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (comps[i] > T(0)) return 1;
    if (comps[i] < T(0)) return -1;
  }
  return 0;
}

// GEOS CGAlgorithmsDD::orientationIndex(p1, p2, q): orientationIndexFilter, exact fallback
template <typename T>
__device__ __forceinline__ int orientation(T p1x, T p1y, T p2x, T p2y, T qx, T qy) {
#pragma clang fp reassociate(off) contract(off)
  const T ax = p1x - qx, by = p2y - qy, ay = p1y - qy, bx = p2x - qx;
  const T dl = ax * by;
  const T dr = ay * bx;
  const T det = dl - dr;
  const bool same = (dl > T(0) && dr > T(0)) || (dl < T(0) && dr < T(0));
  if (!same || xabs(det) >= T(1e-15) * (xabs(dl) + xabs(dr))) return (det > T(0)) - (det < T(0));
  return exact_sign_diff(ax, by, ay, bx);
}

// GEOS RayCrossingCounter::countSegment for one segment (x = east, y = north), written with
// predication: the only branch left is the rare exact-orientation fallback.  Always evaluated in
// float64 (the reference's arithmetic): edge vertices (float32 in the float32 handle, exact for
// the reference's integer map) are promoted, and the query point is the caller's exact float64
// point (a hull corner n +- l/2 of a float32 position is exact in float64, not in float32), so the
// float32 handle decides containment exactly as the reference does for the same point.
template <typename Q>
__device__ __forceinline__ void count_segment(Q p1x, Q p1y, Q p2x, Q p2y, Q qx, Q qy, uint32_t bit, uint32_t& parity,
                                              uint32_t& onb) {
#pragma clang fp reassociate(off) contract(off)
  // GEOS order: strictly-left segments and the end vertex are resolved first, horizontal
  // segments never count, straddling segments count when the point is to their left
  if (p1x < qx && p2x < qx) return;
  const int up1 = p1y > qy, up2 = p2y > qy;          // above the ray
  const int eq1 = p1y == qy, eq2 = p2y == qy;
  const int vertex = (qx == p2x) & eq2;
  const int horiz = eq1 & eq2;
  const int on_h = horiz & (xmin(p1x, p2x) <= qx) & (qx <= xmax(p1x, p2x));
  const int straddle = (up1 & !up2) | (up2 & !up1);   // (p1y > qy && p2y <= qy) || (p2y > qy && p1y <= qy)
  int o = 0;
  if (straddle & !vertex) o = orientation(p1x, p1y, p2x, p2y, qx, qy);
  const int live = straddle & !vertex & !horiz;
  const int oo = (p2y < p1y) ? -o : o;
  onb |= (vertex | on_h | (live & (o == 0))) ? bit : 0u;
  parity ^= (live & (oo > 0)) ? bit : 0u;
}

// Polygon.contains(Point(e, n)) for any polygon by a full scan (fallback path); (qn, qe) is the
// exact float64 query point
template <typename T>
__device__ bool point_in_polys(const Map<T>& m, double qn, double qe) {
  const double qx = qe, qy = qn;
  uint32_t par = 0, onb = 0;
  for (int p = 0; p < m.n_poly; ++p) {
    const T* bb = m.bbox + 4 * p;
    if (qx < bb[0] || qx > bb[1] || qy < bb[2] || qy > bb[3]) continue;
    for (int i = m.off[p]; i < m.off[p + 1]; ++i) {
      const Edge<T> g = m.edge[i];
      count_segment<double>(g.ax, g.ay, g.bx, g.by, qx, qy, 1u << g.poly, par, onb);
    }
  }
  return (par & ~onb) != 0;
}

// squared distance from p to edge g (GEOS Distance::pointToSegment, squared form)
template <typename T>
__device__ __forceinline__ T edge_dist2(const Edge<T>& g, T px, T py) {
  const T ex = g.bx - g.ax, ey = g.by - g.ay;
  const T qx = px - g.ax, qy = py - g.ay;
  const T t = qx * ex + qy * ey;
  const T rx = px - g.bx, ry = py - g.by;
  const T cr = qy * ex - qx * ey;
  const T d_a = qx * qx + qy * qy, d_b = rx * rx + ry * ry, d_s = cr * cr * g.il2;
  // branch-free selection (all three are cheap): keeps the edge loads of a candidate group
  // independent, so they issue back to back instead of one LDS round trip per candidate
  const T d_bs = (t * g.il2 >= T(1)) ? d_b : d_s;
  return ((g.il2 == T(0)) | (t <= T(0))) ? d_a : d_bs;
}

// min over polygons of exterior.distance(Point(e, n)), full scan
template <typename T>
__device__ T distance_to_polys(const Map<T>& m, T n, T e) {
  T best = T(3.0e38);
  for (int i = 0; i < m.n_edge; ++i) best = xmin(best, edge_dist2(m.edge[i], e, n));
  return xsqrt(best);
}

// the same distance via the grid's candidate list
template <typename T>
__device__ T distance_indexed(const Consts<T>& c, const Map<T>& m, T n, T e) {
  const T fx = (e - c.gx0) * c.ginvx, fy = (n - c.gy0) * c.ginvy;
  if (!m.use_index || !(fx >= T(0) && fx < T(kGrid) && fy >= T(0) && fy < T(kGrid)))
    return distance_to_polys(m, n, e);
  const int cell = (int)fy * kGrid + (int)fx;
  // every list has >= 1 group (5 u8 ids in 8 bytes, padded by repetition); the first sits in the
  // cell record, so its edge loads depend on a single LDS read
  uint2 q = reinterpret_cast<const uint2*>(m.idx)[cell];
  const uint2* grp = reinterpret_cast<const uint2*>(m.idx) + (q.y >> 16);
  const int ng = SIT_DSPAN(4 * (int)(q.y >> 16), 4 * (int)((q.y >> 8) & 0xffu), m.n_idx, kDbgIndexEntry) / 4;
  T best = xmin(xmin(xmin(edge_dist2(m.edge[SIT_DEDGE(m, q.x & 0xffu)], e, n),
                          edge_dist2(m.edge[SIT_DEDGE(m, (q.x >> 8) & 0xffu)], e, n)),
                     xmin(edge_dist2(m.edge[SIT_DEDGE(m, (q.x >> 16) & 0xffu)], e, n),
                          edge_dist2(m.edge[SIT_DEDGE(m, q.x >> 24)], e, n))),
                edge_dist2(m.edge[SIT_DEDGE(m, q.y & 0xffu)], e, n));
#pragma unroll 1
  for (int g = 0; g < ng; ++g) {
    q = grp[g];
    const T d0 = edge_dist2(m.edge[SIT_DEDGE(m, q.x & 0xffu)], e, n);
    const T d1 = edge_dist2(m.edge[SIT_DEDGE(m, (q.x >> 8) & 0xffu)], e, n);
    const T d2 = edge_dist2(m.edge[SIT_DEDGE(m, (q.x >> 16) & 0xffu)], e, n);
    const T d3 = edge_dist2(m.edge[SIT_DEDGE(m, q.x >> 24)], e, n);
    const T d4 = edge_dist2(m.edge[SIT_DEDGE(m, q.y & 0xffu)], e, n);
    best = xmin(best, xmin(xmin(xmin(d0, d1), xmin(d2, d3)), d4));
  }
  return xsqrt(best);
}

// distance_indexed in three stages, so the step kernel can issue the LDS lookups early and use
// them late: the grid cell record and the class-grid word (pf_cell), the first candidate group's
// edge records (pf_edges), the distances (pf_finish; same candidates, same min order, same value
// as distance_indexed)
template <typename T>
__device__ __forceinline__ int fine_lookup(const Consts<T>& c, const Map<T>& m, T n, T e, int& cell, uint32_t& word);

template <typename T>
struct DistPf {
  bool ok;             // inside the grid, index present
  uint2 q;             // the cell record
  Edge<T> g[5];        // the first group's edges
  int cls, cell_f;     // class-grid lookup of the same point (fine_lookup)
  uint32_t word_f;
};
template <typename T>
__device__ __forceinline__ void pf_cell(const Consts<T>& c, const Map<T>& m, T n, T e, DistPf<T>& p) {
  const T fx = (e - c.gx0) * c.ginvx, fy = (n - c.gy0) * c.ginvy;
  p.ok = m.use_index && fx >= T(0) && fx < T(kGrid) && fy >= T(0) && fy < T(kGrid);
  const int cell = p.ok ? (int)fy * kGrid + (int)fx : 0;
  p.q = reinterpret_cast<const uint2*>(m.idx)[cell];
  p.cls = fine_lookup(c, m, n, e, p.cell_f, p.word_f);
}
template <typename T>
__device__ __forceinline__ void pf_edges(const Map<T>& m, DistPf<T>& p) {
  p.g[0] = m.edge[SIT_DEDGE(m, p.q.x & 0xffu)];
  p.g[1] = m.edge[SIT_DEDGE(m, (p.q.x >> 8) & 0xffu)];
  p.g[2] = m.edge[SIT_DEDGE(m, (p.q.x >> 16) & 0xffu)];
  p.g[3] = m.edge[SIT_DEDGE(m, p.q.x >> 24)];
  p.g[4] = m.edge[SIT_DEDGE(m, p.q.y & 0xffu)];
}
template <typename T>
__device__ __forceinline__ T pf_finish(const Map<T>& m, const DistPf<T>& p, T n, T e) {
  if (!p.ok) return distance_to_polys(m, n, e);
  const uint2* grp = reinterpret_cast<const uint2*>(m.idx) + (p.q.y >> 16);
  const int ng = SIT_DSPAN(4 * (int)(p.q.y >> 16), 4 * (int)((p.q.y >> 8) & 0xffu), m.n_idx, kDbgIndexEntry) / 4;
  T best = xmin(xmin(xmin(edge_dist2(p.g[0], e, n), edge_dist2(p.g[1], e, n)),
                     xmin(edge_dist2(p.g[2], e, n), edge_dist2(p.g[3], e, n))),
                edge_dist2(p.g[4], e, n));
#pragma unroll 1
  for (int g = 0; g < ng; ++g) {
    const uint2 q = grp[g];
    const T d0 = edge_dist2(m.edge[SIT_DEDGE(m, q.x & 0xffu)], e, n);
    const T d1 = edge_dist2(m.edge[SIT_DEDGE(m, (q.x >> 8) & 0xffu)], e, n);
    const T d2 = edge_dist2(m.edge[SIT_DEDGE(m, (q.x >> 16) & 0xffu)], e, n);
    const T d3 = edge_dist2(m.edge[SIT_DEDGE(m, q.x >> 24)], e, n);
    const T d4 = edge_dist2(m.edge[SIT_DEDGE(m, q.y & 0xffu)], e, n);
    best = xmin(best, xmin(xmin(xmin(d0, d1), xmin(d2, d3)), d4));
  }
  return xsqrt(best);
}

// Polygon.contains for two points sharing y (= n): bit 0 / bit 1 for x0 / x1 (exact float64
// query coordinates; the band index in T, its lists carry a 1 m margin)
template <typename T>
__device__ int pip_pair_indexed(const Consts<T>& c, const Map<T>& m, double n, double x0, double x1) {
  if (!m.use_index) return (int)point_in_polys(m, n, x0) | ((int)point_in_polys(m, n, x1) << 1);
  const T fb = ((T)n - c.by0) * c.binv;
  if (!(fb >= T(0) && fb < T(kBands))) return 0;   // beyond every edge's y-range
  const int b = (int)fb;
  uint32_t par0 = 0, onb0 = 0, par1 = 0, onb1 = 0;
  const int k0 = m.idx[kBandBase + b];
  const int k1 = k0 + SIT_DSPAN(k0, (int)m.idx[kBandBase + b + 1] - k0, m.n_idx, kDbgIndexEntry);
#pragma unroll 1
  for (int k = k0; k < k1; ++k) {
    const Edge<T> g = m.edge[SIT_DEDGE(m, m.idx[k])];
    const uint32_t bit = 1u << g.poly;
    count_segment<double>(g.ax, g.ay, g.bx, g.by, x0, n, bit, par0, onb0);
    count_segment<double>(g.ax, g.ay, g.bx, g.by, x1, n, bit, par1, onb1);
  }
  return ((par0 & ~onb0) != 0 ? 1 : 0) | ((par1 & ~onb1) != 0 ? 2 : 0);
}

template <typename T>
__device__ bool pip_indexed(const Consts<T>& c, const Map<T>& m, double n, double e) {
  if (!m.use_index) return point_in_polys(m, n, e);
  const T fb = ((T)n - c.by0) * c.binv;
  if (!(fb >= T(0) && fb < T(kBands))) return false;
  const int b = (int)fb;
  uint32_t par = 0, onb = 0;
  const int k0 = m.idx[kBandBase + b];
  const int k1 = k0 + SIT_DSPAN(k0, (int)m.idx[kBandBase + b + 1] - k0, m.n_idx, kDbgIndexEntry);
#pragma unroll 1
  for (int k = k0; k < k1; ++k) {
    const Edge<T> g = m.edge[SIT_DEDGE(m, m.idx[k])];
    count_segment<double>(g.ax, g.ay, g.bx, g.by, e, n, 1u << g.poly, par, onb);
  }
  return (par & ~onb) != 0;
}

// class of a point from the class grid: 0 out, 1 in, 2 mixed (built for every map); `cell`
// and `word` are what pip_cell needs for a mixed cell
template <typename T>
__device__ __forceinline__ int fine_lookup(const Consts<T>& c, const Map<T>& m, T n, T e, int& cell,
                                           uint32_t& word) {
  const T fx = (e - c.fx0) * c.finvx, fy = (n - c.fy0) * c.finvy;
  cell = 0;
  word = 0;
  if (!(fx >= T(0) && fx < T(kFine) && fy >= T(0) && fy < T(kFine))) return 0;
  cell = (int)fy * kFine + (int)fx;
  word = m.fine[SIT_DCLAMP(cell >> 4, kFineWords, kDbgClassWord)];
  return (word >> ((cell & 15) * 2)) & 3;
}

template <typename T>
__device__ __forceinline__ int fine_class(const Consts<T>& c, const Map<T>& m, T n, T e) {
  int cell;
  uint32_t word;
  return fine_lookup(c, m, n, e, cell, word);
}

// GEOS's count over a cell's live edges in float64 at the exact point (nd, ed), starting from the
// cell's constant parity.  Out of line: one copy serves every call site (it runs only where the
// float32 count is unsure, or on the float64 handle), keeping the step loop's code footprint small.
#ifndef SIT_PIP_EXACT_INLINE
#define SIT_PIP_EXACT_INLINE __attribute__((noinline))
#endif
template <typename T>
__device__ SIT_PIP_EXACT_INLINE bool pip_live_exact(const Edge<T>* edge, const uint8_t* live, int cnt,
                                                         uint32_t par, double nd, double ed, int n_edge) {
  uint32_t onb = 0;
  for (int k = 0; k < cnt; ++k) {
    const Edge<T> g = edge[SIT_DCLAMP((int)live[k], n_edge, kDbgEdgeId)];
    count_segment<double>(g.ax, g.ay, g.bx, g.by, ed, nd, 1u << g.poly, par, onb);
  }
  return (par & ~onb) != 0;
}

// float32 fast path of count_segment for a query point q known within 4e-3 m (a float32 position
// exactly, a float32-rounded hull corner within half an ulp <= 5e-4 m inside the class grid):
// the float32 decisions equal the exact ones unless a vertex coordinate lies within that
// tolerance of q's, or the orientation is inside its float32 error band; those cases set `unsure`
// and the caller re-decides the point in float64 (rare: points within millimetres of a vertex
// latitude or an edge line)
__device__ __forceinline__ void count_segment_f32(float p1x, float p1y, float p2x, float p2y, float qx, float qy,
                                                  uint32_t bit, uint32_t& parity, uint32_t& onb, bool& unsure) {
  constexpr float tol = 4e-3f;
  unsure |= xmin(xmin(xabs(p1y - qy), xabs(p2y - qy)), xmin(xabs(p1x - qx), xabs(p2x - qx))) <= tol;
  if (p1x < qx && p2x < qx) return;
  const int up1 = p1y > qy, up2 = p2y > qy;
  const int straddle = (up1 & !up2) | (up2 & !up1);
  if (straddle) {
    const float ax = p1x - qx, by = p2y - qy, ay = p1y - qy, bx = p2x - qx;
    const float dl = ax * by, dr = ay * bx, det = dl - dr;
    unsure |= xabs(det) <= 1e-5f * (xabs(dl) + xabs(dr)) + tol * (xabs(ax) + xabs(ay) + xabs(bx) + xabs(by));
    const int o = (det > 0.f) - (det < 0.f);
    parity ^= (((p2y < p1y) ? -o : o) > 0) ? bit : 0u;
  }
  (void)onb;
}

// how pip_cell may count in float32 (float32 handle; the float64 handle always counts in float64)
constexpr int kPipFar = 0;     // exact point farther than the hull diagonal + 1 m from every boundary:
                               // float32 comparisons are exact and every straddling edge's crossing is
                               // >= 57 m away, far outside the float32 orientation error
constexpr int kPipNear = 1;    // float32-rounded hull corner near the shore: float32 count with an
                               // unsure flag, float64 re-count where it is raised
constexpr int kPipExact = 2;   // no distance known (the IW point, probes): float64 count

// Polygon.contains(Point(e, n)) for a point in mixed class cell `cell` (class word `word`):
// the cell's constant crossing parity plus GEOS's count over the cell's live edges only.  (nd, ed)
// is the exact float64 point; (n, e) its value in T.
template <int MODE, typename T>
__device__ __forceinline__ bool pip_cell(const Map<T>& m, int cell, uint32_t word, T n, T e, double nd, double ed) {
  const uint32_t mixed = (word >> 1) & 0x55555555u;
  const int r = SIT_DCLAMP(m.frank[cell >> 4] + __popc(mixed & ((1u << ((cell & 15) * 2)) - 1u)), m.n_mixed,
                           kDbgCellRecord);
  const uint2 rec = m.crec[r];
  const int first = (int)(rec.y & 0xffffu);
  const int cnt = SIT_DSPAN(first, (int)(rec.y >> 16), m.n_live, kDbgCellRecord);
  if constexpr (kIsF32<T> && MODE == kPipFar) {
    uint32_t par = rec.x, onb = 0;
#pragma unroll 1
    for (int k = 0; k < cnt; ++k) {
      const Edge<T> g = m.edge[SIT_DEDGE(m, m.clive[first + k])];
      count_segment<float>(g.ax, g.ay, g.bx, g.by, e, n, 1u << g.poly, par, onb);
    }
    return (par & ~onb) != 0;
  } else {
    if constexpr (kIsF32<T> && MODE == kPipNear) {
      uint32_t par = rec.x, onb = 0;
      bool unsure = false;
#pragma unroll 1
      for (int k = 0; k < cnt; ++k) {
        const Edge<T> g = m.edge[SIT_DEDGE(m, m.clive[first + k])];
        count_segment_f32(g.ax, g.ay, g.bx, g.by, e, n, 1u << g.poly, par, onb, unsure);
      }
      if (!unsure || !kKnifePip) return par != 0;
    }
    return pip_live_exact(m.edge, m.clive + first, cnt, rec.x, nd, ed, m.n_edge);
  }
}

// Polygon.contains(Point(e, n)): fine-grid class when the cell is pure (a pure cell has no
// boundary within 1 m, far beyond float32 rounding of the cell index); the mixed cell's record
// (or, without records, a band scan) in float64 otherwise
template <typename T>
__device__ bool pip_point(const Consts<T>& c, const Map<T>& m, T n, T e) {
  int cell;
  uint32_t word;
  const int cls = fine_lookup(c, m, n, e, cell, word);
  if (cls < 2) return cls == 1;
  if (m.use_cells) return pip_cell<kPipExact>(m, cell, word, n, e, (double)n, (double)e);
  return pip_indexed(c, m, n, e);
}

// the same for a point farther than hull_safe from every boundary (float32 count is exact there)
template <typename T>
__device__ bool pip_point_far(const Consts<T>& c, const Map<T>& m, T n, T e) {
  int cell;
  uint32_t word;
  const int cls = fine_lookup(c, m, n, e, cell, word);
  if (cls < 2) return cls == 1;
  if (m.use_cells) return pip_cell<kPipFar>(m, cell, word, n, e, (double)n, (double)e);
  return pip_indexed(c, m, n, e);
}

// is_pos_inside_obstacles (MSRL_env_ex.py:490-515): any of the 4 corners (n +- h, e +- h)
// strictly inside a polygon.  When the centre is farther than h*sqrt(2) + 1 m from every
// boundary (dobst: the reward's distance), no corner-centre segment meets a boundary, so all
// corners share the centre's side and one point test decides.
template <typename T>
__device__ bool hull_corners(const Consts<T>& c, const Map<T>& m, T n, T e);


template <typename T>
__device__ bool hull_in_terrain(const Consts<T>& c, const Map<T>& m, T n, T e, T dobst) {
  if (dobst > c.hull_safe) return pip_point_far(c, m, n, e);
  return hull_corners(c, m, n, e);
}

// the same with the centre's class looked up by the caller (independent of the distance, so its
// LDS read overlaps the distance computation)
template <typename T>
__device__ __forceinline__ bool hull_in_terrain_cls(const Consts<T>& c, const Map<T>& m, T n, T e, T dobst,
                                                    int cls, int cell, uint32_t word) {
  if (dobst > c.hull_safe) {
    if (cls < 2) return cls == 1;
    if (m.use_cells) return pip_cell<kPipFar>(m, cell, word, n, e, (double)n, (double)e);
    return pip_indexed(c, m, n, e);
  }
  return hull_corners(c, m, n, e);
}

template <typename T>
__device__ bool hull_corners(const Consts<T>& c, const Map<T>& m, T n, T e) {
  const T h = c.half_len;
  // the corners as the reference forms them: n +- l/2 in float64 (exact for a float32 position);
  // their float32 roundings n -+ h pick the class cells (pure cells have a 1 m margin)
  const double hx = c.x.half_len;
  // near shore: each corner by its fine-grid class; a corner in a mixed cell by the cell's record
  // (or a band scan without records)
  if (m.use_cells) {
    int l00, l01, l10, l11;
    uint32_t w00, w01, w10, w11;
    const T nl = n - h, nh = n + h, el = e - h, eh = e + h;
    const int c00 = fine_lookup(c, m, nl, el, l00, w00), c01 = fine_lookup(c, m, nl, eh, l01, w01);
    const int c10 = fine_lookup(c, m, nh, el, l10, w10), c11 = fine_lookup(c, m, nh, eh, l11, w11);
    if (c00 == 1 || c01 == 1 || c10 == 1 || c11 == 1) return true;
    bool hit = false;
    if (c00 == 2) hit |= pip_cell<kPipNear>(m, l00, w00, nl, el, ieee_sub(n, hx), ieee_sub(e, hx));
    if (c01 == 2) hit |= pip_cell<kPipNear>(m, l01, w01, nl, eh, ieee_sub(n, hx), ieee_add(e, hx));
    if (c10 == 2) hit |= pip_cell<kPipNear>(m, l10, w10, nh, el, ieee_add(n, hx), ieee_sub(e, hx));
    if (c11 == 2) hit |= pip_cell<kPipNear>(m, l11, w11, nh, eh, ieee_add(n, hx), ieee_add(e, hx));
    return hit;
  }
  const double nlo = ieee_sub(n, hx), nhi = ieee_add(n, hx), elo = ieee_sub(e, hx), ehi = ieee_add(e, hx);
  const int c00 = fine_class(c, m, n - h, e - h), c01 = fine_class(c, m, n - h, e + h);
  const int c10 = fine_class(c, m, n + h, e - h), c11 = fine_class(c, m, n + h, e + h);
  if (c00 == 1 || c01 == 1 || c10 == 1 || c11 == 1) return true;
  bool hit = false;
  if (c00 >= 2 || c01 >= 2) hit |= pip_pair_indexed(c, m, nlo, elo, ehi) != 0;
  if (c10 >= 2 || c11 >= 2) hit |= pip_pair_indexed(c, m, nhi, elo, ehi) != 0;
  return hit;
}

}  // namespace sit
