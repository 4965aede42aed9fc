// sit_impl.h — MI355X (gfx950) kernels and host helpers of the ship-in-transit env step, shared by
// sit_kernels.hip (C ABI, float64 path, every non-step kernel) and sit_steps_f32.hip (the float32
// step kernels, compiled with device fast-math).
//
// Layout in HBM (struct of arrays, one device blob, every field 256-B aligned):
//   ship fields  [2][n_env]   index = type * n_env + env (type 0 = ship under test, 1 = obstacle)
//   env fields   [n_env]
//   route tables [2][cap][n_env]  (north and east; waypoint i of env e's ship t at
//                                  (t * cap + i) * n_env + e, so a wave reads one waypoint
//                                  index of 64 envs as one coalesced line set)
// Thread mapping of the step kernel: a 128-thread block owns 64 envs; wave 0 steps their test
// ships, wave 1 their obstacle ships (different control flow per wave, none inside a wave).
// The env-level reward needs both ships: each wave evaluates its own ship's termination
// predicates, the two waves exchange through LDS (double-buffered slots, one barrier per step)
// and the test-ship wave assembles reward/done/status in the reference's summation order.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "sit.h"
#include "sit_device.h"

using namespace sit;

// ---------------------------------------------------------------------------------------
// state blob description
// ---------------------------------------------------------------------------------------
namespace {

enum Extent { kShip = 0, kEnv = 1, kTable = 2, kObs = 3, kLogRow = 4 };
struct FieldSpec {
  const char* name;
  int dtype;
  int extent;
};

constexpr int kShipReal = 15;
constexpr int kEnvReal = 6;
const FieldSpec kFields[] = {
    {"north", SIT_DT_REAL, kShip},        {"east", SIT_DT_REAL, kShip},
    {"yaw", SIT_DT_REAL, kShip},          {"surge", SIT_DT_REAL, kShip},
    {"sway", SIT_DT_REAL, kShip},         {"yaw_rate", SIT_DT_REAL, kShip},
    {"shaft_speed", SIT_DT_REAL, kShip},  {"ship_speed_i", SIT_DT_REAL, kShip},
    {"shaft_speed_i", SIT_DT_REAL, kShip}, {"heading_i", SIT_DT_REAL, kShip},
    {"heading_prev", SIT_DT_REAL, kShip}, {"e_ct_int", SIT_DT_REAL, kShip},
    {"last_rpm", SIT_DT_REAL, kShip},     {"last_e_ct", SIT_DT_REAL, kShip},
    {"last_power_me", SIT_DT_REAL, kShip},
    {"next_wpt", SIT_DT_I32, kShip},      {"n_wpt", SIT_DT_I32, kShip},
    {"ticks", SIT_DT_I32, kShip},         {"stop", SIT_DT_I32, kShip},
    {"sampling_dist", SIT_DT_REAL, kEnv}, {"eps_dist", SIT_DT_REAL, kEnv},
    {"prev_pre_north", SIT_DT_REAL, kEnv}, {"prev_pre_east", SIT_DT_REAL, kEnv},
    {"iw_north", SIT_DT_REAL, kEnv},      {"iw_east", SIT_DT_REAL, kEnv},
    {"ep_step", SIT_DT_I32, kEnv},        {"event", SIT_DT_U32, kEnv},
    {"episodes", SIT_DT_U32, kEnv},
    {"wpt_north", SIT_DT_REAL, kTable},   {"wpt_east", SIT_DT_REAL, kTable},
    {"last_obs", SIT_DT_REAL, kObs},
    // trajectory log only: accumulated fuel per ship, the obstacle ship's last logged row
    {"fuel_me", SIT_DT_REAL, kShip},      {"fuel_el", SIT_DT_REAL, kShip},
    {"fuel", SIT_DT_REAL, kShip},         {"last_log", SIT_DT_REAL, kLogRow},
    // the IW terrain test's last result, keyed by the point it was taken at (obstacle.py's
    // Polygon.contains of a fixed map is a function of the point): single-step launches, which
    // cannot keep it in registers across steps, reuse it while the caller's IW does not change.
    // iw_key_flags bit 0 = valid, bit 1 = inside; sit_load_map clears it
    {"iw_key_north", SIT_DT_REAL, kEnv},  {"iw_key_east", SIT_DT_REAL, kEnv},
    {"iw_key_flags", SIT_DT_U32, kEnv},
    // float32 handles: the low parts of the double-float integrators (comp_add, sit_device.h): the
    // value of north is north + north_lo, and so on.  float64 handles: zero (unused)
    {"north_lo", SIT_DT_REAL, kShip},     {"east_lo", SIT_DT_REAL, kShip},
    {"yaw_lo", SIT_DT_REAL, kShip},       {"ship_speed_i_lo", SIT_DT_REAL, kShip},
    {"shaft_speed_i_lo", SIT_DT_REAL, kShip}, {"heading_i_lo", SIT_DT_REAL, kShip},
    {"e_ct_int_lo", SIT_DT_REAL, kShip},
    {"surge_lo", SIT_DT_REAL, kShip},     {"sway_lo", SIT_DT_REAL, kShip},
    {"yaw_rate_lo", SIT_DT_REAL, kShip},  {"shaft_speed_lo", SIT_DT_REAL, kShip},
    {"sampling_dist_lo", SIT_DT_REAL, kEnv},
    {"prev_pre_north_lo", SIT_DT_REAL, kEnv}, {"prev_pre_east_lo", SIT_DT_REAL, kEnv},
};
constexpr int kNumFields = (int)(sizeof(kFields) / sizeof(kFields[0]));
enum FieldId {
  F_NORTH = 0, F_LAST_PME = 14, F_K = 15, F_NW, F_TICKS, F_STOP,
  F_SAMP = 19, F_IW_E = 24, F_EP = 25, F_EVENT, F_EPISODES, F_WN, F_WE, F_LAST_OBS,
  F_FUEL_ME, F_FUEL_EL, F_FUEL, F_LAST_LOG, F_IWK_N, F_IWK_E, F_IWK_FLAGS, F_SHIP_LO, F_ENV_LO = F_SHIP_LO + 11
};
constexpr int kShipLo = 11;  // north, east, yaw, ship_speed_i, shaft_speed_i, heading_i, e_ct_int, surge, sway,
                             // yaw_rate, shaft_speed
// (the episode distance, which no decision or output reads, stays a plain float32 sum)
constexpr int kEnvLo = 3;    // sampling_dist, prev_pre_north, prev_pre_east
static_assert(F_ENV_LO + kEnvLo == kNumFields, "state field table and ids out of sync");

// per-env scenario (constant after sit_load_*), device side
template <typename T>
struct Scen {
  const T* init;          // [2][SIT_INIT_NF][n_env]
  const T* end_n;         // [2][n_env]
  const T* end_e;
  const int32_t* nw0;     // [2][n_env]
  const double* ab_len;   // [n_env]
  const double* ab_alpha; // [n_env]
  const T* initial_state; // [n_env][10]
  const T* init_lo;       // [2][SIT_INIT_NF][n_env]: float32 handles, init - (float)init (double-float starts)
};

template <typename T>
struct State {
  T* ship[kShipReal];     // [2 * n_env]
  int32_t* k;
  int32_t* nw;
  int32_t* ticks;
  int32_t* stop;
  T* env[kEnvReal];       // sampling_dist, eps_dist, prev_pre_n, prev_pre_e, iw_n, iw_e
  int32_t* ep_step;
  uint32_t* event;
  uint32_t* episodes;
  T* wn;                  // [2][cap][n_env]
  T* we;
  T* last_obs;            // [SIT_OBS_DIM][n_env]: observation before the next step
  T* fuel[3];             // [2 * n_env] each: fuel me, fuel electrical, fuel total (log only)
  T* last_log;            // [SIT_LOG_KEYS][n_env]: the obstacle's last logged row (log only)
  T* iwk[2];              // [n_env] each: the point of the cached IW test
  uint32_t* iwk_flags;    // [n_env]: kIwkValid | kIwkInside
  T* ship_lo[kShipLo];    // [2 * n_env] each: the integrators' low parts (float32 handles)
  T* env_lo[kEnvLo];      // [n_env] each
};
constexpr uint32_t kIwkValid = 1u, kIwkInside = 2u;

template <typename T>
struct StepIO {
  int32_t n_steps;
  int32_t auto_reset;
  uint64_t seed;
  int64_t env_id_offset;
  const T* action_ne;
  const uint8_t* sac_update;
  const uint8_t* init;
  T* next_state;
  T* reward;
  uint8_t* done;
  uint32_t* status;
  T* action_out;
  int32_t* done_count;
  T* transitions;
  int32_t* transition_count;
  int32_t transition_capacity;
  int32_t mask_horizon;
  // policy mode (kPolicy): per-env action slots (the request queue is built after the launch by
  // k_policy_admit, sit_actor.h, unless the step kernel serves the waiting envs itself: actor_w)
  T* policy_action;
  int32_t* policy_ready;
  int32_t* request_age;   // [n_env]: admission rounds waited (publish_ages)
  int32_t* group_counts;  // [n_env / 64][kAgeBuckets]: waiting envs per age bucket (handle scratch)
  unsigned long long* env_steps;
  const float* actor_w;   // in-kernel serving (sit_serve.h): packed actor weights, or null
  int32_t actor_det;
  unsigned long long* actor_served;
  T* log;                 // [n_steps][SIT_LOG_ROWS][n_env] or null
};

template <typename T>
struct KArgs {
  Consts<T> c;
  Map<T> map;       // global copy (base pointer = map.off, size map_bytes)
  State<T> st;
  Scen<T> sc;
  StepIO<T> io;
  int32_t n_env;
  int32_t cap;
  int32_t map_bytes;   // bytes of the map blob staged into LDS (map_stage_bytes)
  int32_t lds_bytes;   // the launch's dynamic LDS (k_env_steps_sync; checked by the serving pass in debug builds)
  int32_t fake_simds;  // test hook (SIT_TEST_FAKE_SIMDS): 0 = the waves' HW_ID SIMDs; else 0x100 | base-4 digits
};

// SIT_LDS_CELLS: the mixed-cell crossing records (frank, crec, clive: ~26 KB of the reference map's 57)
// staged into LDS with the rest (1), or read through the caches (0: they are read only for points in
// a mixed class cell, near a shore; the LDS block then holds edges, nearest-edge index and class grid)
#ifndef SIT_LDS_CELLS
#define SIT_LDS_CELLS 1
#endif

// Copy the edge records, the packed index and the class grid (and with SIT_LDS_CELLS the mixed-cell
// records: the first map_bytes of the map blob) into LDS at `dst`.
template <typename T>
__device__ __forceinline__ Map<T> stage_map(const KArgs<T>& a, unsigned char* dst) {
  const unsigned char* src = reinterpret_cast<const unsigned char*>(a.map.edge);
  const int n16 = a.map_bytes / 16;
  // LDS-DMA (global_load_lds_dwordx4): the 16-byte pieces go global -> LDS without a register
  // round trip, so all of a thread's pieces are in flight at once instead of one load latency
  // per piece.  One wave-instruction writes a wave-uniform base + lane x 16 B: the linear image.
  // The barrier after the prologue waits for them (vmcnt).
  const int lane = threadIdx.x & (kWave - 1);
  for (int i = threadIdx.x; i < n16; i += blockDim.x)
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(src) + i,
                                     (__attribute__((address_space(3))) void*)(dst + 16 * (i - lane)), 16, 0, 0);
  Map<T> m = a.map;
  m.edge = reinterpret_cast<const Edge<T>*>(dst);
  m.idx = reinterpret_cast<const uint16_t*>(dst + (reinterpret_cast<const unsigned char*>(a.map.idx) - src));
  m.fine = reinterpret_cast<const uint32_t*>(dst + (reinterpret_cast<const unsigned char*>(a.map.fine) - src));
#if SIT_LDS_CELLS
  m.frank = reinterpret_cast<const uint16_t*>(dst + (reinterpret_cast<const unsigned char*>(a.map.frank) - src));
  m.crec = reinterpret_cast<const uint2*>(dst + (reinterpret_cast<const unsigned char*>(a.map.crec) - src));
  m.clive = reinterpret_cast<const uint8_t*>(dst + (reinterpret_cast<const unsigned char*>(a.map.clive) - src));
#endif
  return m;
}

}  // namespace

namespace {   // kernels are TU-local: the float32 step kernels live in their own TU

// ---------------------------------------------------------------------------------------
// device helpers on the SoA state
// ---------------------------------------------------------------------------------------
#ifdef SIT_DEBUG
// this translation unit's failed bounds checks (sit_debug_flags), read and cleared
int debug_flags_impl(uint32_t* out) {
  unsigned int v = 0, z = 0;
  if (hipDeviceSynchronize() != hipSuccess) return SIT_E_HIP;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(sit::g_dbg_flags), sizeof(v)) != hipSuccess) return SIT_E_HIP;
  if (hipMemcpyToSymbol(HIP_SYMBOL(sit::g_dbg_flags), &z, sizeof(z)) != hipSuccess) return SIT_E_HIP;
  *out |= v;
  return SIT_OK;
}
#endif

template <typename T>
__device__ __forceinline__ void load_ship(const State<T>& st, int sid, Ship<T>& s) {
  s.n = st.ship[0][sid]; s.e = st.ship[1][sid]; s.psi = st.ship[2][sid];
  s.u = st.ship[3][sid]; s.v = st.ship[4][sid]; s.r = st.ship[5][sid]; s.w = st.ship[6][sid];
  s.i1 = st.ship[7][sid]; s.i2 = st.ship[8][sid]; s.hi = st.ship[9][sid]; s.hp = st.ship[10][sid];
  s.ect_int = st.ship[11][sid]; s.lrpm = st.ship[12][sid]; s.lect = st.ship[13][sid];
  s.lpme = st.ship[14][sid];
  s.k = st.k[sid]; s.ticks = st.ticks[sid]; s.stop = st.stop[sid];
  if constexpr (kIsF32<T>) {
    s.ln = st.ship_lo[0][sid]; s.le = st.ship_lo[1][sid]; s.lpsi = st.ship_lo[2][sid];
    s.li1 = st.ship_lo[3][sid]; s.li2 = st.ship_lo[4][sid]; s.lhi = st.ship_lo[5][sid]; s.lei = st.ship_lo[6][sid];
    s.lu = st.ship_lo[7][sid]; s.lv = st.ship_lo[8][sid]; s.lr = st.ship_lo[9][sid]; s.lw = st.ship_lo[10][sid];
  } else {
    s.ln = s.le = s.lpsi = s.li1 = s.li2 = s.lhi = s.lei = T(0);
    s.lu = s.lv = s.lr = s.lw = T(0);
  }
}

template <typename T>
__device__ __forceinline__ void store_ship(const State<T>& st, int sid, const Ship<T>& s) {
  st.ship[0][sid] = s.n; st.ship[1][sid] = s.e; st.ship[2][sid] = s.psi;
  st.ship[3][sid] = s.u; st.ship[4][sid] = s.v; st.ship[5][sid] = s.r; st.ship[6][sid] = s.w;
  st.ship[7][sid] = s.i1; st.ship[8][sid] = s.i2; st.ship[9][sid] = s.hi; st.ship[10][sid] = s.hp;
  st.ship[11][sid] = s.ect_int; st.ship[12][sid] = s.lrpm; st.ship[13][sid] = s.lect;
  st.ship[14][sid] = s.lpme;
  st.k[sid] = s.k; st.ticks[sid] = s.ticks; st.stop[sid] = s.stop;
  if constexpr (kIsF32<T>) {
    st.ship_lo[0][sid] = s.ln; st.ship_lo[1][sid] = s.le; st.ship_lo[2][sid] = s.lpsi;
    st.ship_lo[3][sid] = s.li1; st.ship_lo[4][sid] = s.li2; st.ship_lo[5][sid] = s.lhi; st.ship_lo[6][sid] = s.lei;
    st.ship_lo[7][sid] = s.lu; st.ship_lo[8][sid] = s.lv; st.ship_lo[9][sid] = s.lr; st.ship_lo[10][sid] = s.lw;
  }
}

template <typename T>
__device__ __forceinline__ T init_val(const Scen<T>& sc, int type, int f, int env, int n_env) {
  return sc.init[(type * SIT_INIT_NF + f) * n_env + env];
}
// the low part of a float32 handle's initial value (0 for float64)
template <typename T>
__device__ __forceinline__ T init_lo(const Scen<T>& sc, int type, int f, int env, int n_env) {
  if constexpr (kIsF32<T>) return sc.init_lo[(type * SIT_INIT_NF + f) * n_env + env];
  else return T(0);
}

// MultiShipRLEnv.reset for one ship (MSRL_Env.py:147-188): pose/velocities/time/route/LOS
// reset; shaft speed and every PI/PID integrator persist (Q6).
template <typename T>
__device__ __forceinline__ void reset_ship(const Scen<T>& sc, int type, int env, int n_env, Ship<T>& s,
                                           int& nw) {
  s.n = init_val(sc, type, SIT_INIT_NORTH, env, n_env);
  s.e = init_val(sc, type, SIT_INIT_EAST, env, n_env);
  s.psi = init_val(sc, type, SIT_INIT_YAW, env, n_env);
  s.u = init_val(sc, type, SIT_INIT_SURGE, env, n_env);
  s.v = init_val(sc, type, SIT_INIT_SWAY, env, n_env);
  s.r = init_val(sc, type, SIT_INIT_YAW_RATE, env, n_env);
  s.ln = init_lo(sc, type, SIT_INIT_NORTH, env, n_env);
  s.le = init_lo(sc, type, SIT_INIT_EAST, env, n_env);
  s.lpsi = init_lo(sc, type, SIT_INIT_YAW, env, n_env);
  s.lu = init_lo(sc, type, SIT_INIT_SURGE, env, n_env);
  s.lv = init_lo(sc, type, SIT_INIT_SWAY, env, n_env);
  s.lr = init_lo(sc, type, SIT_INIT_YAW_RATE, env, n_env);
  s.ect_int = T(0);
  s.lei = T(0);
  s.k = 1;
  s.ticks = 0;
  s.stop = 0;
  nw = sc.nw0[type * n_env + env];
}

// one guidance/control/update/integrate cycle without store, time or bias (MSRL_Env.py:190-217)
template <typename T>
__device__ __forceinline__ void init_step_ship(const Consts<T>& c, const ConstsX64& x, Ship<T>& s, Route<T>& rt,
                                               T v_des) {
  T rudder, thr, ect, sp, cp, psi_ref;
  bool ect_over;
  xsincos(s.psi, &sp, &cp);
  guidance_control(c, x, s, rt, v_des, rudder, thr, ect, psi_ref, ect_over);
  ship_dynamics(c, s, thr, rudder, sp, cp);
  rt.fixup(s.k);
}

// map bounds check of is_pos_outside_horizon / is_route_outside_horizon (MSRL_env_ex.py:460-542)
template <typename T>
__device__ __forceinline__ bool outside(const Consts<T>& c, T n, T e, T margin) {
  return n < c.min_n + margin || n > c.max_n - margin || e < c.min_e + margin || e > c.max_e - margin;
}

constexpr uint32_t kStopBit = 1u << 30;   // exchange-only: stop flag after this ship's checks
constexpr uint32_t kDoneBit = 1u << 29;   // exchange-only: this ship's done

template <typename T>
struct Xchg {
  T n[2][kWave];
  T e[2][kWave];
  T r_nto[kWave];
  T r_o[kWave];
  uint32_t bits[2][kWave];
  int32_t slot[kWave];    // transition record of this step (obstacle lane allocates)
};

// the action row's angle: the sampled a, or NaN when none was drawn on device.  The float32 step
// kernels are compiled with finite math, under which a NaN literal or a select against one may be
// folded away; the NaN bit pattern therefore passes an empty asm, which the optimiser cannot see
// through (tests/test_gpu_parity.py::test_f32_action_rows_nan_without_sample)
__device__ __forceinline__ float angle_or_nan(bool has, float a) {
  uint32_t nan_bits = 0x7fc00000u;
  asm volatile("" : "+v"(nan_bits));
  return __uint_as_float(has ? __float_as_uint(a) : nan_bits);
}
__device__ __forceinline__ double angle_or_nan(bool has, double a) {
  uint64_t nan_bits = 0x7ff8000000000000ull;
  asm volatile("" : "+v"(nan_bits));
  return __longlong_as_double(has ? __double_as_longlong(a) : (long long)nan_bits);
}

// ---------------------------------------------------------------------------------------
// the env step kernel: K steps of MultiShipRLEnv.step (+ optional auto-reset)
//   MODE  : kExplicit = caller's action arrays, kSynth = synthetic AST sampler on device,
//           kPolicy = actions from a policy run between launches (an env that reaches a
//           sampling event without a fresh action waits for the rest of the launch; the
//           admission kernel after the launch queues its request, and the next launch consumes
//           the action the policy wrote for it)
// ---------------------------------------------------------------------------------------
#if defined(SIT_DIAG_PATHS) || defined(SIT_DIAG_PHASES) || defined(SIT_DIAG_SYNC) || defined(SIT_DIAG_SERVE) || defined(SIT_DIAG_PLACE)
// Diagnostic builds only (tools/diag_paths.py, tools/diag_sync.py): [type][0..15] predicate path
// statistics, [type][16..23] shader-clock cycles per step phase (wave lane 0); SIT_DIAG_SYNC: cycles
// per role and segment of k_env_steps_sync (sit_sync.h).  The counters are per translation unit:
// sit_diag_read reads the float64 TU's, sit_diag_read_f32 the float32 step kernels'.
__device__ unsigned long long g_sit_diag[2][32];
int diag_read_impl(unsigned long long* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sit_diag), sizeof(g_sit_diag)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[2][32] = {};
    for (int t = 0; t < 2; ++t) z[t][28] = z[t][30] = ~0ull;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_sit_diag), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
#if defined(SIT_DIAG_PHASES) || defined(SIT_DIAG_PLACE)
// per wave of the last launch: start / end (realtime ticks), shader cycles, HW_ID | XCC_ID << 32
// (SIT_DIAG_PLACE, the two-wave kernel, tools/diag_place.py: role, block, -, HW_ID | XCC_ID << 32)
constexpr int kDiagWaves = 8192;
__device__ unsigned long long g_sit_wave[kDiagWaves][4];
int diag_read_waves_impl(unsigned long long* out, int n) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (n > kDiagWaves) n = kDiagWaves;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sit_wave), sizeof(unsigned long long) * 4 * n) != hipSuccess) return -1;
  return 0;
}
#endif
#ifdef SIT_DIAG_PHASES
// the fence makes the ship state live in registers at the timer, so arithmetic cannot be
// sunk across a phase boundary
template <typename T>
__device__ __forceinline__ void diag_fence(Ship<T>& s) {
  asm volatile("" : "+v"(s.n), "+v"(s.e), "+v"(s.psi), "+v"(s.u), "+v"(s.v), "+v"(s.r), "+v"(s.w),
                    "+v"(s.i1), "+v"(s.i2), "+v"(s.hi), "+v"(s.hp), "+v"(s.ect_int));
  asm volatile("" : "+v"(s.lrpm), "+v"(s.lect), "+v"(s.lpme), "+v"(s.k), "+v"(s.ticks), "+v"(s.stop));
}
#define SIT_PH(k) do { diag_fence(s); __builtin_amdgcn_sched_barrier(0); \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ph[k] += t_ - ph_t; ph_t = t_; \
    __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define SIT_PH(k) do { } while (0)
#endif
#ifdef SIT_DIAG_PATHS

template <typename T>
__device__ int diag_band_len(const Consts<T>& c, const Map<T>& m, T n) {
  const T fb = (n - c.by0) * c.binv;
  if (!m.use_index || !(fb >= T(0) && fb < T(kBands))) return 0;
  const int b = (int)fb;
  return m.idx[kBandBase + b + 1] - m.idx[kBandBase + b];
}

template <typename T>
__device__ void diag_lane(const Consts<T>& c, const Map<T>& m, T n, T e, T dobst, bool iw, T iwn, T iwe,
                          int* v) {
  const T fx = (e - c.gx0) * c.ginvx, fy = (n - c.gy0) * c.ginvy;
  if (m.use_index && fx >= T(0) && fx < T(kGrid) && fy >= T(0) && fy < T(kGrid)) {
    const int cell = (int)fy * kGrid + (int)fx;
    v[0] = (int)(((reinterpret_cast<const uint2*>(m.idx)[cell].y >> 8) & 0xffu) + 1u) * 5;
  }
  if (dobst <= c.hull_safe) {
    v[1] = 1;
    const T h = c.half_len;
    const int c00 = fine_class(c, m, n - h, e - h), c01 = fine_class(c, m, n - h, e + h);
    const int c10 = fine_class(c, m, n + h, e - h), c11 = fine_class(c, m, n + h, e + h);
    if (!(c00 == 1 || c01 == 1 || c10 == 1 || c11 == 1)) {
      if (c00 >= 2 || c01 >= 2) { v[2] += 1; v[3] += diag_band_len(c, m, n - h); }
      if (c10 >= 2 || c11 >= 2) { v[2] += 1; v[3] += diag_band_len(c, m, n + h); }
    }
  } else if (fine_class(c, m, n, e) >= 2) {
    v[4] = 1;
    v[3] += diag_band_len(c, m, n);
  }
  if (iw && fine_class(c, m, iwn, iwe) >= 2) { v[5] = 1; v[6] = diag_band_len(c, m, iwn); }
}

__device__ void diag_wave(int type, int lane, bool act, const int* v) {
  // lane sums and wave maxima / any-counts (the wave pays the max over its lanes)
  unsigned long long* g = g_sit_diag[type];
  int mx[7], any[7];
  for (int j = 0; j < 7; ++j) {
    int m = act ? v[j] : 0;
    for (int off = 32; off >= 1; off >>= 1) m = max(m, __shfl_xor(m, off));
    mx[j] = m;
    any[j] = __popcll(__ballot(act && v[j] != 0));
  }
  if (act) {
    for (int j = 0; j < 7; ++j) if (v[j]) atomicAdd(&g[j], (unsigned long long)v[j]);
  }
  if (lane == 0) {
    atomicAdd(&g[7], 1ull);
    atomicAdd(&g[8], (unsigned long long)mx[0]);            // max distance candidates
    atomicAdd(&g[9], (unsigned long long)(any[1] > 0));     // waves with a near-shore lane
    atomicAdd(&g[10], (unsigned long long)(any[2] > 0));    // waves with a pair scan
    atomicAdd(&g[11], (unsigned long long)mx[3]);           // max hull band trips
    atomicAdd(&g[12], (unsigned long long)(any[4] > 0));    // waves with a mixed far centre
    atomicAdd(&g[13], (unsigned long long)(any[5] > 0));    // waves with a mixed IW
    atomicAdd(&g[14], (unsigned long long)mx[6]);           // max IW band trips
  }
}
#endif

// paired output stores: a state row (SIT_OBS_DIM reals) starts 8-byte (float) / 16-byte
// (double) aligned, so pairs at even offsets go out as one 2-element store (fewer store
// instructions per wave; the scattered row stride makes store issue, not bytes, the cost)
__device__ __forceinline__ void store2(float* p, float a, float b) { *reinterpret_cast<float2*>(p) = make_float2(a, b); }
__device__ __forceinline__ void store2(double* p, double a, double b) { *reinterpret_cast<double2*>(p) = make_double2(a, b); }
// the step kernels' output rows (next_state, IW action, reward, done, status): written once and never read
// by the kernel, so the float32 kernels store them non-temporally (SIT_NT_OUT) — streaming them through the
// L2 as ordinary stores evicted what the launch reads again (the actor's W2 at the serving pass): C5 +2.2 %.
// The float64 kernels keep ordinary stores: their 16-byte row pieces, written non-temporally, reached HBM as
// partial lines (PMC traffic 1.17x the algorithmic bytes against 1.01x), for no gain (no serving pass)
#ifndef SIT_NT_OUT
#define SIT_NT_OUT 1
#endif
typedef float sit_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void out2(float* p, float a, float b) {
  if (SIT_NT_OUT) __builtin_nontemporal_store(sit_f2{a, b}, reinterpret_cast<sit_f2*>(p));
  else store2(p, a, b);
}
__device__ __forceinline__ void out2(double* p, double a, double b) { store2(p, a, b); }
template <typename T, typename V>
__device__ __forceinline__ void out1(V* p, V v) {
  if (SIT_NT_OUT && kIsF32<T>) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// four reals at a 4-real-aligned address (replay-transition records: 24 reals = six of these)
__device__ __forceinline__ void store4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void store4(double* p, double a, double b, double c, double d) {
  store2(p, a, b);
  store2(p + 2, c, d);
}

// IW = obstacle position + AB_len (cos, sin)(AB_alpha + a): float trig for the float handle
// (1e-7 relative of AB_len, inside its 1e-5 contract), double for the float64 handle
__device__ __forceinline__ void iw_point(float n, float e, double ab_len, double ab_alpha, double ang, float& iwn,
                                         float& iwe) {
  float sn, cs;
  xsincos((float)(ab_alpha + ang), &sn, &cs);
  iwn = n + (float)ab_len * cs;
  iwe = e + (float)ab_len * sn;
}
__device__ __forceinline__ void iw_point(double n, double e, double ab_len, double ab_alpha, double ang, double& iwn,
                                         double& iwe) {
  iwn = n + ab_len * cos(ab_alpha + ang);
  iwe = e + ab_len * sin(ab_alpha + ang);
}

// the same IW in two parts: the direction (cos, sin)(AB_alpha + a), which depends only on the action
// (the sync kernel draws the next event's action ahead, off its critical segment), and the point
__device__ __forceinline__ void iw_dir(double ab_alpha, double ang, float& cs, float& sn) {
  xsincos((float)(ab_alpha + ang), &sn, &cs);
}
__device__ __forceinline__ void iw_dir(double ab_alpha, double ang, double& cs, double& sn) {
  cs = cos(ab_alpha + ang);
  sn = sin(ab_alpha + ang);
}
__device__ __forceinline__ void iw_at(float n, float e, double ab_len, float cs, float sn, float& iwn, float& iwe) {
  iwn = n + (float)ab_len * cs;
  iwe = e + (float)ab_len * sn;
}
__device__ __forceinline__ void iw_at(double n, double e, double ab_len, double cs, double sn, double& iwn, double& iwe) {
  iwn = n + ab_len * cs;
  iwe = e + ab_len * sn;
}

// the sampler's seed made opaque where it is used: otherwise the compiler hoists Philox's ten-round
// key schedule (18 uniform words) out of the step loop and spills it into VGPR lanes
__device__ __forceinline__ uint64_t opaque_seed(uint64_t seed) {
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
  asm volatile("" : "+s"(lo), "+s"(hi));
  return ((uint64_t)hi << 32) | lo;
}

#ifndef SIT_PF_EDGES_EARLY
#define SIT_PF_EDGES_EARLY 0   // 1: the candidate edges loaded right after guidance (measured slower)
#endif
constexpr int kExplicit = 0, kSynth = 1, kPolicy = 2;

// Policy-mode admission (sit_actor.h): the step kernel keeps each env's request age (admission rounds
// waited) and publishes per group of kAdmitGroup consecutive envs how many of them wait with each age
// bucket (1 .. kAgeBuckets-1 exact, kAgeBuckets = that age or older)
constexpr int kAgeBuckets = 16;
constexpr int kAdmitGroup = 64;
constexpr int32_t kAgeMax = 1 << 30;
__device__ __forceinline__ int age_bucket(int32_t a) { return a < kAgeBuckets ? a : kAgeBuckets; }
// the age after this launch (age + 1 if the env ends the launch waiting, else 0) and the env group's
// bucket counts: one wave = one group of 64 envs (env = group * 64 + lane); every lane calls
__device__ __forceinline__ void publish_ages(int32_t* age, int32_t* counts, int env, bool act, bool waiting,
                                             int32_t age0) {
  const int32_t a1 = (act && waiting) ? min(age0 + 1, kAgeMax) : 0;
  if (act) age[env] = a1;
  const int lane = threadIdx.x & (kWave - 1);
  int mine = 0;
#pragma unroll
  for (int b = 1; b <= kAgeBuckets; ++b) {
    const int c = (int)__popcll(__ballot(a1 > 0 && age_bucket(a1) == b));
    if (lane == b - 1) mine = c;
  }
  if (lane < kAgeBuckets) counts[(size_t)(env / kAdmitGroup) * kAgeBuckets + lane] = mine;
}
// wave-uniform switches of the step loop (bits 0-4: the output arrays present)
constexpr uint32_t kUfTrans = 1u << 5, kUfDoneCnt = 1u << 6, kUfAutoReset = 1u << 7, kUfMaskH = 1u << 8,
                   kUfCollBias = 1u << 9, kUfBlackout = 1u << 10;
constexpr uint32_t kSampGeBit = 1u << 28;   // exchange-only: obstacle sampling distance >= AB_len

// One wave's K steps: TYPE 0 steps the ships under test, TYPE 1 the obstacle ships.  The ship type
// is a compile-time constant of each wave's loop (k_env_steps branches once, wave-uniformly, into
// one of the two instantiations), so neither loop carries the other type's registers or branches.
template <typename T, int MODE, bool LDSMAP, bool LOG, int TYPE, int MACH>
__device__ __forceinline__ void env_steps(const KArgs<T>& a, unsigned char* smem, Xchg<T>* xs, Consts<T>& cs) {
#ifdef SIT_DIAG_PHASES
  const unsigned long long w_t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long w_r0 = __builtin_amdgcn_s_memrealtime();
#endif
  // The ~70 per-step constants go kernel arguments -> LDS -> VGPRs: loaded through LDS they
  // land in vector registers (one wave per SIMD leaves ~512 per lane, AGPRs included), whereas
  // kernel-argument constants compete for the 102 SGPRs and spill to VGPR lanes (v_readlane
  // in the loop), and reading the LDS block inside the loop put ~40 dependent LDS reads on
  // each step's critical path (the register copy measured 12% faster).
  for (int i = threadIdx.x; i < (int)(sizeof(Consts<T>) / 4); i += blockDim.x)
    reinterpret_cast<uint32_t*>(&cs)[i] = reinterpret_cast<const uint32_t*>(&a.c)[i];
  __syncthreads();
  const Consts<T> c = cs;
  // LDS: the map blob (edges, index, classes).  Route tables stay in HBM (Route caches the
  // active leg); keeping the block under 64 KB of LDS matters: a larger allocation measured
  // ~1.75x slower at the same occupancy-limited grid.
  Map<T> map = LDSMAP ? stage_map(a, smem) : a.map;
  const int lane = threadIdx.x & (kWave - 1);
  constexpr int type = TYPE;
  const int n_env = a.n_env;
  const int group = kGroups > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 7) : 0;
  const int env = (blockIdx.x * kGroups + group) * kEnvsPerBlock + lane;
  xs += 2 * group;
  const bool act = lane < kEnvsPerBlock && env < n_env;
  const int sid = type * n_env + env;

  Ship<T> s{};
  Route<T> rt{};
  T v_des = T(0);
  T samp = T(0), eps = T(0), ppn = T(0), ppe = T(0), iwn = T(0), iwe = T(0);
  T samp_lo = T(0), ppn_lo = T(0), ppe_lo = T(0);   // float32: low parts (comp_add)
  // the IW's terrain test is a pure function of (iwn, iwe), which change only at sampling
  // events (or with the caller's action): cache it
  T iw_tn = T(0), iw_te = T(0);
  bool iw_valid = false, iw_in = false;
  int ep_step = 0;
  uint32_t event = 0, episodes = 0;
  double ab_len = 0.0, ab_alpha = 0.0, samp_limit = 0.0;
  T lo[6] = {};                      // this ship's part of the last observation
  const int lo_base = type == 0 ? 0 : 6, lo_n = type == 0 ? 6 : 4;
  // policy mode: both lanes of an env track whether its next step is a sampling event
  bool need = false, ready = false, stalled = false;
  T pa = T(0);
  int32_t age0 = 0;                  // policy mode: admission rounds waited (publish_ages)
  uint32_t n_stepped = 0;
  if (MODE == kPolicy && act) {
    const double samp0 = comp_val(a.st.env[0][env], kIsF32<T> ? a.st.env_lo[0][env] : T(0));
    need = a.st.ep_step[env] == 0 || (samp0 >= a.sc.ab_len[env] && a.st.stop[n_env + env] == 0);
    ready = a.io.policy_ready[env] == SIT_POLICY_READY;
    pa = a.io.policy_action[env];
    if (type == 1) age0 = a.io.request_age ? a.io.request_age[env] : 0;   // (NULL when the launch serves in-kernel)
  }
  if (act) {
    for (int j = 0; j < lo_n; ++j) lo[j] = a.st.last_obs[(size_t)(lo_base + j) * n_env + env];
    ep_step = a.st.ep_step[env];
    load_ship(a.st, sid, s);
    rt.nw = a.st.nw[sid];
    rt.end_n = a.sc.end_n[sid];
    rt.end_e = a.sc.end_e[sid];
    v_des = init_val(a.sc, type, SIT_INIT_DESIRED_SPEED, env, n_env);
    rt.tn = a.st.wn + (size_t)type * a.cap * n_env + env;
    rt.te = a.st.we + (size_t)type * a.cap * n_env + env;
    rt.stride = n_env;
    rt.cap = a.cap;
    rt.load_leg(s.k);
    if (type == 1) {
      samp = a.st.env[0][env]; eps = a.st.env[1][env];
      ppn = a.st.env[2][env]; ppe = a.st.env[3][env];
      iwn = a.st.env[4][env]; iwe = a.st.env[5][env];
      if constexpr (kIsF32<T>) {
        samp_lo = a.st.env_lo[0][env];
        ppn_lo = a.st.env_lo[1][env]; ppe_lo = a.st.env_lo[2][env];
      }
      event = a.st.event[env];
      episodes = a.st.episodes[env];
      ab_len = a.sc.ab_len[env];
      ab_alpha = a.sc.ab_alpha[env];
      samp_limit = ieee_mul(ab_len, cs.x.theta);   // is_obs_ship_navigation_failure (MSRL_env_ex.py:569)
    }
  }
  const T maxn = c.max_n;
  // episode-start values held in registers (auto-reset reloads nothing from memory): the
  // construction pose, route length, first leg with its geometry, and initial observation.  Only
  // with auto-reset: a launch without it (sit_step, explicit actions) skips these loads and the
  // first leg's geometry in its prologue
  T p0[6] = {}, p0lo[6] = {};
  T lo0[6] = {};
  int nw0 = 0;
  typename Route<T>::Leg leg0{};
  if (act && __builtin_amdgcn_readfirstlane(a.io.auto_reset)) {
    for (int j = 0; j < 6; ++j) p0[j] = init_val(a.sc, type, SIT_INIT_NORTH + j, env, n_env);
    for (int j = 0; j < 6; ++j) p0lo[j] = init_lo(a.sc, type, SIT_INIT_NORTH + j, env, n_env);
    for (int j = 0; j < lo_n; ++j) lo0[j] = a.sc.initial_state[(size_t)env * SIT_OBS_DIM + lo_base + j];
    nw0 = a.sc.nw0[sid];
    Route<T> r0 = rt;
    r0.nw = nw0;
    r0.load_leg(1);
    leg0 = r0.leg();
  }
  // per-lane output row pointers, advanced by one row block per step: the loop then needs no
  // output base pointers in SGPRs (they were re-loaded from the kernel arguments every step)
  const int outs = __builtin_amdgcn_readfirstlane((a.io.next_state ? 1 : 0) | (a.io.reward ? 2 : 0) |
                                                  (a.io.done ? 4 : 0) | (a.io.status ? 8 : 0) |
                                                  (a.io.action_out ? 16 : 0));
  // the loop's wave-uniform switches in one SGPR, made opaque at every iteration (below): the
  // compiler then tests a bit where a switch is used instead of hoisting each one out of the loop
  // as a 64-bit lane mask, which spilled ~40 SGPRs into VGPR lanes (v_readlane in the loop)
  uint32_t uf = (uint32_t)outs | (a.io.transitions ? kUfTrans : 0u) | (a.io.done_count ? kUfDoneCnt : 0u) |
                (a.io.auto_reset ? kUfAutoReset : 0u) | (a.io.mask_horizon > 0 ? kUfMaskH : 0u) |
                (c.collision_bias ? kUfCollBias : 0u) | (c.sg_mode != SIT_SG_MOTOR ? kUfBlackout : 0u);
  uf = __builtin_amdgcn_readfirstlane(uf);
  T* p_ns = (outs & 1) ? a.io.next_state + (size_t)env * SIT_OBS_DIM + (type == 0 ? 0 : 6) : nullptr;
  T* p_rw = (outs & 2) ? a.io.reward + env : nullptr;
  uint8_t* p_dn = (outs & 4) ? a.io.done + env : nullptr;
  uint32_t* p_st = (outs & 8) ? a.io.status + env : nullptr;
  T* p_ao = (outs & 16) ? a.io.action_out + (size_t)env * 4 : nullptr;
  const size_t row_step = (size_t)n_env;
  // trajectory log: this ship's column of the step's [SIT_LOG_ROWS][n_env] block
  // (LOG is a template parameter so the logging code costs the step loop nothing when off)
  T* p_lg = (LOG && a.io.log && act) ? a.io.log + (size_t)type * SIT_LOG_KEYS * n_env + env : nullptr;
  T f_me = T(0), f_el = T(0), f_tot = T(0);
  if (p_lg) { f_me = a.st.fuel[0][sid]; f_el = a.st.fuel[1][sid]; f_tot = a.st.fuel[2][sid]; }
  __syncthreads();   // map staged
#ifdef SIT_DIAG_PHASES
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long ph_t = __builtin_amdgcn_s_memtime();
#endif

  for (int step = 0; step < a.io.n_steps; ++step) {
    asm volatile("" : "+s"(uf));
    // the map's switches likewise (compared where used, not held as lane masks)
    asm volatile("" : "+s"(map.use_index), "+s"(map.use_cells), "+s"(map.n_edge), "+s"(map.n_poly));
    const size_t row = (size_t)step * n_env + env;
    Xchg<T>& x = xs[step & 1];
    // ---------------- own ship ----------------
    T o_rpm = T(0), o_ect = T(0), o_pme = T(0);
    T r_nt = T(0), r_term = T(0);
    uint32_t bits = 0;
#ifdef SIT_DIAG_PATHS
    int dv[7] = {0, 0, 0, 0, 0, 0, 0};
#endif
    bool sac = false, init_f = false;
    int tslot = -1;                    // transition record slot of this step (obstacle lane)
    double ang = 0.0;                  // the sampled angle; has_ang: drawn on device this step
    double act_n = 0.0;                // the SAC action of the event: ang / (pi / 6), in [-1, 1]
    bool has_ang = false;
    bool ect_over = false;             // |e_ct| > e_tolerance, decided exactly (guidance_control)
    bool mech = false, blk = false;    // test ship: mechanical / blackout failure (decided pre-integration)
    // sampling event without an action: the env waits for the policy for the rest of the launch
    // (both lanes decide alike); after the launch the admission kernel queues its request
    // (k_policy_admit, sit_actor.h) from the state it stops in
    if (MODE == kPolicy && act && !stalled && need && !ready) stalled = true;
    const bool live = act && !stalled;
    T sp = T(0), cp = T(1);
    if (live) xsincos(s.psi, &sp, &cp);    // heading trig of the step, off the guidance chain
    // the post-step position (a function of the pre-step state) and its map lookups, issued now:
    // their LDS latency overlaps guidance and dynamics (the predicates below use them)
    T n1 = s.n, e1 = s.e, ln1 = s.ln, le1 = s.le;
    DistPf<T> pf;
    if (live) {
      if (type == 0 || !s.stop) euler_position(c, s, sp, cp, n1, e1, ln1, le1);
      pf_cell(c, map, n1, e1, pf);
    }
    if (live) {
      ++n_stepped;
      if (type == 1) {
        // converted_action / SAC_update / init of this step
        if (MODE == kPolicy) {
          init_f = (ep_step == 0);
          sac = need;
          if (sac) {                     // the policy's squashed action scales the route angle
            act_n = (double)pa;
            ang = (double)pa * (M_PI / 6.0);
            has_ang = true;
            iw_point(s.n, s.e, ab_len, ab_alpha, ang, iwn, iwe);
            ++event;
          }
        } else if (MODE == kSynth) {
          init_f = (ep_step == 0);
          sac = init_f || (comp_val(samp, samp_lo) >= ab_len && !s.stop);
          if (sac) {                     // mode-0 action U[-1, 1] (uniform_policy.py:20-22) scaled by pi/6
            const double u01 = sampler_uniform(opaque_seed(a.io.seed), (uint64_t)(a.io.env_id_offset + env), event);
            act_n = u01 * 2.0 - 1.0;
            ang = act_n * (M_PI / 6.0);
            has_ang = true;
            iw_point(s.n, s.e, ab_len, ab_alpha, ang, iwn, iwe);
            ++event;
          }
        } else {
          init_f = a.io.init[row] != 0;
          sac = a.io.sac_update[row] != 0;
          iwn = a.io.action_ne[2 * row];
          iwe = a.io.action_ne[2 * row + 1];
        }
        // replay-transition slot of a sampling event, allocated here at the start of the step (one
        // atomic per wave, ranks by lane): its latency overlaps guidance, dynamics and predicates
        // instead of stalling the exchange before the barrier
        if (uf & kUfTrans) {
          const unsigned long long m = __ballot(sac);
          if (m) {
            const int lead = __builtin_ctzll(m);
            int base = 0;
            if (lane == lead) base = atomicAdd(a.io.transition_count, (int)__popcll(m));
            base = __shfl(base, lead);
            if (sac) tslot = base + (int)__popcll(m & ((1ull << lane) - 1ull));
          }
        }
        // obs_step (MSRL_Env.py:287-402)
        if (s.stop) {
          if (p_lg) {                    // store_last_simulation_data: last row, time updated
            p_lg[0] = T(s.ticks) * c.dt;
            for (int kk = 1; kk < SIT_LOG_KEYS; ++kk) p_lg[kk * row_step] = a.st.last_log[kk * row_step + env];
          }
          s.ticks += 2;                  // stop path: next_time() twice, no integration (Q10)
          o_rpm = s.lrpm; o_ect = s.lect; o_pme = s.lpme;
          ect_over = (double)o_ect > cs.x.e_tol;
          if (SIT_PF_EDGES_EARLY) pf_edges(map, pf);
        } else {
          if (sac) {                     // update_route: insert at index -1 (Q16)
            if (!rt.insert(iwn, iwe, s.k, a.cap)) bits |= SIT_ST_ROUTE_OVERFLOW;
            samp = T(0);
            samp_lo = T(0);
          }
          const T pre_n = s.n, pre_e = s.e, pre_ln = s.ln, pre_le = s.le;
          T rudder, thr, psi_ref;
          guidance_control<T, MACH>(c, cs.x, s, rt, v_des, rudder, thr, o_ect, psi_ref, ect_over);
          if (SIT_PF_EDGES_EARLY) pf_edges(map, pf);
          o_rpm = s.w * c.rpm_k;
          o_pme = power_me_kw(c, thr);
          s.lrpm = o_rpm; s.lect = o_ect; s.lpme = o_pme;
          if (p_lg) {
            store_log_row<T, MACH>(c, p_lg, row_step, s, thr, rudder, o_ect, psi_ref, f_me, f_el, f_tot);
            for (int kk = 0; kk < SIT_LOG_KEYS; ++kk) a.st.last_log[kk * row_step + env] = p_lg[kk * row_step];
          }
          ship_dynamics_pos<T, MACH>(c, s, thr, rudder, sp, cp, n1, e1, ln1, le1);
          if (!init_f) {                 // distance between the last two stored positions
            const T dn = comp_diff(pre_n, pre_ln, ppn, ppn_lo), de = comp_diff(pre_e, pre_le, ppe, ppe_lo);
            const T d = xsqrt(dn * dn + de * de);
            eps = eps + d;
            samp = comp_add(samp, samp_lo, d);
          }
          ppn = pre_n; ppe = pre_e; ppn_lo = pre_ln; ppe_lo = pre_le;
          s.ticks += 1;
        }
      } else {
        // test_step (MSRL_Env.py:219-285)
        T rudder, thr, psi_ref;
        const double i1_0 = comp_val(s.i1, s.li1), i2_0 = comp_val(s.i2, s.li2);   // pre-step integrals (blackout knife edge)
        guidance_control<T, MACH>(c, cs.x, s, rt, v_des, rudder, thr, o_ect, psi_ref, ect_over);
        if (SIT_PF_EDGES_EARLY) pf_edges(map, pf);
        if (uf & kUfCollBias) {          // is_collision_imminent() on all-zero states (Q1)
          thr = xclip(thr * c.bias_scale, T(0), c.bias_max);
          rudder = xclip(rudder + c.bias_rudder, -c.rudder_max, c.rudder_max);
        }
        o_rpm = s.w * c.rpm_k;
        o_pme = power_me_kw(c, thr);
        // failure predicates on pre-integration values (MSRL_env_ex.py:554-558, 578-582), exact:
        // float64 where the float32 margin is inside the float32 band (always for the float64 handle)
        mech = rpm_fails<T, MACH>(c, cs.x, s.w, o_rpm);
        // MOTOR (PTI): load_me = min(total, ME capacity) <= ME capacity, so no blackout ever (Q7)
        if (uf & kUfBlackout) {
          blk = o_pme > c.blackout_kw;
          if (!kIsF32<T> || xabs(o_pme - c.blackout_kw) <= T(1e-4) * (xabs(o_pme) + T(1)))
            blk = power_me_kw_exact(c.sg_mode, cs.x, throttle_exact(cs.x, s.u, v_des, i1_0, i2_0,
                                                                    c.collision_bias != 0, MACH == 1))
                  > cs.x.blackout;
        }
        s.lrpm = o_rpm; s.lect = o_ect; s.lpme = o_pme;
        if (p_lg) store_log_row<T, MACH>(c, p_lg, row_step, s, thr, rudder, o_ect, psi_ref, f_me, f_el, f_tot);
        ship_dynamics_pos<T, MACH>(c, s, thr, rudder, sp, cp, n1, e1, ln1, le1);
        s.ticks += 1;
      }

      // ---------------- own termination predicates (MSRL_env_ex.py:628-881) ----------------
#if defined(SIT_ABLATE_PREDICATES)   // diagnostic builds only (tools/ablate.sh): polygon work removed
      const T dobst = T(1000);
      const bool terrain = false;
#elif defined(SIT_ABLATE_HULL)        // diagnostic: distance kept, hull test removed
      const T dobst = distance_indexed(c, map, s.n, s.e);
      const bool terrain = false;
#elif defined(SIT_ABLATE_DIST)        // diagnostic: distance removed, hull test by its four corners
      const T dobst = T(1000);
      const bool terrain = hull_corners(c, map, s.n, s.e);
#else
      SIT_PH(0);
      if (!SIT_PF_EDGES_EARLY) pf_edges(map, pf);
      const T dobst = pf_finish(map, pf, s.n, s.e);
      SIT_PH(1);
      const bool terrain = hull_in_terrain_cls(c, map, s.n, s.e, dobst, pf.cls, pf.cell_f, pf.word_f);
      SIT_PH(2);
#endif
#ifdef SIT_DIAG_PATHS
      diag_lane(c, map, s.n, s.e, dobst, type == 1, iwn, iwe, dv);
#endif
      const bool arrive = within_radius(s.n, s.e, rt.end_n, rt.end_e, c.arrive_d2_le);
      const bool horizon = outside(c, s.n, s.e, c.half_len);
      int stop = s.stop;
      bool done = false;
      if (type == 0) {
        r_nt = xabs(o_ect) * c.inv_e_tol + (T(1) - dobst * c.inv_maxn) * T(0.01);
        if (p_lg) {                      // reward_results terms of the ship under test (:640-643)
          T* t = p_lg + (size_t)(2 * SIT_LOG_KEYS) * row_step;                 // rows 54-56
          t[0] = xabs(o_ect) / c.e_tol;
          t[row_step] = (T(1) - dobst / c.max_n) / T(100);
          t[2 * row_step] = r_nt;
        }
        const bool pred[6] = {arrive, horizon, terrain, mech, ect_over, blk};
        const T rew[6] = {T(0), T(0), T(1000), T(1000), T(1000), T(1000)};
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          if (pred[i]) {
            if (!stop) r_term = r_term + rew[i];
            stop = 1;
            done = true;
            bits |= 1u << i;
          }
        }
        if (done) bits |= SIT_ST_TEST_DONE;
      } else {
        if (!stop)
          r_nt = T(0.1) - xabs(o_ect) * c.inv_e_tol * T(0.01) - (T(1) - dobst * c.inv_maxn) * T(0.01);
        if (p_lg) {                      // reward_results terms of the obstacle ship (:656-669)
          T* t = p_lg + (size_t)(SIT_LOG_KEYS + 3) * row_step;   // rows 57-60
          t[0] = stop ? T(0) : T(0.1);
          t[row_step] = stop ? T(0) : -(xabs(o_ect) / c.e_tol) / T(100);
          t[2 * row_step] = stop ? T(0) : -(T(1) - dobst / c.max_n) / T(100);
          t[3 * row_step] = r_nt;
        }
        if (arrive) { stop = 1; bits |= SIT_ST_OBS_ENDPOINT; }
        if (horizon) { stop = 1; done = true; bits |= SIT_ST_OBS_HORIZON; }
        if (terrain) {                   // done without stop flag (Q12)
          if (!stop) r_term = r_term - T(1000);
          done = true;
          bits |= SIT_ST_OBS_TERRAIN;
        }
#if defined(SIT_ABLATE_PREDICATES) || defined(SIT_ABLATE_HULL)
        if (outside(c, iwn, iwe, T(0))) {
#else
        if (!iw_valid || iwn != iw_tn || iwe != iw_te) {
          iw_in = pip_point(c, map, iwn, iwe);
          iw_tn = iwn; iw_te = iwe; iw_valid = true;
        }
        if (outside(c, iwn, iwe, T(0)) || iw_in) {   // Q11
#endif
          if (!stop) r_term = r_term - T(1000);
          stop = 1; done = true;
          bits |= SIT_ST_OBS_IW_TERMINAL;
        }
        if (ect_over || comp_val(samp, samp_lo) > samp_limit) {
          if (!stop) r_term = r_term - T(1000);
          stop = 1; done = true;
          bits |= SIT_ST_OBS_NAVIGATION;
        }
        if (done) bits |= SIT_ST_OBS_DONE;
      }
      s.stop = stop;
      if (type == 1) x.slot[lane] = tslot;
      x.n[type][lane] = s.n;
      x.e[type][lane] = s.e;
      x.bits[type][lane] = bits | (stop ? kStopBit : 0u) | (done ? kDoneBit : 0u) |
                           ((MODE == kPolicy && type == 1 && comp_val(samp, samp_lo) >= ab_len) ? kSampGeBit : 0u);
      if (type == 1) { x.r_nto[lane] = r_nt; x.r_o[lane] = r_term; }
    }
    SIT_PH(3);
    __syncthreads();
    SIT_PH(4);
#ifdef SIT_DIAG_PATHS
    diag_wave(type, lane, act, dv);
#endif
    // ---------------- env level: shared reward, outputs ----------------
    bool env_done = false;
    if (MODE == kPolicy && act && !live && type == 0) {   // no step taken this row
      if (uf & 8) *p_st = SIT_ST_NO_STEP;
      if (uf & 4) *p_dn = 0;
    }
    if (live) {
      const T dn = x.n[0][lane] - x.n[1][lane], de = x.e[0][lane] - x.e[1][lane];
      const bool coll = closer_than(x.n[0][lane], x.e[0][lane], x.n[1][lane], x.e[1][lane], c.coll_d2);
      const uint32_t bt = x.bits[0][lane], bo = x.bits[1][lane];
      env_done = ((bt | bo) & kDoneBit) || coll;
      if (coll) s.stop = 1;
      if (type == 0) {
        const T r_snt = (bo & kStopBit) ? T(0) : (T(1) - xsqrt(dn * dn + de * de) * c.inv_maxn) * T(0.001);
        if (p_lg) p_lg[(size_t)(2 * SIT_LOG_KEYS + 7) * row_step] = r_snt;   // shared term (:714-731)
        const T rs = coll ? T(2000) : T(0);
        const T reward = r_nt + r_term + x.r_nto[lane] + x.r_o[lane] + r_snt + rs;
        const uint32_t status = ((bt | bo) & ~(kStopBit | kDoneBit | kSampGeBit)) | (coll ? SIT_ST_COLLISION : 0u);
#ifndef SIT_ABLATE_STORES
        if (uf & 2) *p_rw = reward;
        if (uf & 4) *p_dn = env_done ? 1 : 0;
#endif
        const int slot = x.slot[lane];
        if (slot >= 0 && slot < a.io.transition_capacity) {
          T* rec = a.io.transitions + (size_t)slot * SIT_TRANSITION_DIM;
          for (int j = 0; j < 6; ++j) rec[j] = lo[j];
          rec[11] = reward;
          rec[12] = s.n; rec[13] = s.e; rec[14] = s.psi; rec[15] = o_rpm; rec[16] = o_ect; rec[17] = o_pme;
          const bool horizon_hit = (uf & kUfMaskH) && ep_step + 2 == a.io.mask_horizon;
          rec[22] = (horizon_hit || !env_done) ? T(1) : T(0);
        }
#ifndef SIT_ABLATE_STORES
        if (uf & 8) *p_st = status;
#endif
#ifndef SIT_ABLATE_STORES
        if (uf & 1) { store2(p_ns, s.n, s.e); store2(p_ns + 2, s.psi, o_rpm); store2(p_ns + 4, o_ect, o_pme); }
#endif
      } else {
#ifndef SIT_ABLATE_STORES
        if (uf & 1) { store2(p_ns, s.n, s.e); store2(p_ns + 2, s.psi, o_ect); }
#endif
#ifndef SIT_ABLATE_STORES
        if (uf & 16) { store2(p_ao, iwn, iwe); store2(p_ao + 2, angle_or_nan(has_ang, (T)ang), sac ? T(1) : T(0)); }
#endif
        const int slot = x.slot[lane];
        if (slot >= 0 && slot < a.io.transition_capacity) {
          T* rec = a.io.transitions + (size_t)slot * SIT_TRANSITION_DIM;
          for (int j = 0; j < 4; ++j) rec[6 + j] = lo[j];
          // the SAC action of the event in [-1, 1] (memory.push(state, action, ...), main_ast.py:395):
          // the sampler's U[-1, 1] draw or the policy's squashed action; NaN without a device draw
          rec[10] = angle_or_nan(has_ang, (T)act_n);
          rec[18] = s.n; rec[19] = s.e; rec[20] = s.psi; rec[21] = o_ect;
          rec[23] = (T)(a.io.env_id_offset + env);
        }
      }
      // the observation becomes the next step's state
      if (type == 0) { lo[0] = s.n; lo[1] = s.e; lo[2] = s.psi; lo[3] = o_rpm; lo[4] = o_ect; lo[5] = o_pme; }
      else { lo[0] = s.n; lo[1] = s.e; lo[2] = s.psi; lo[3] = o_ect; }
      if (MODE == kPolicy) {
        if (need) ready = false;       // this step's sampling event consumed the action (both lanes)
        // the next step is a sampling event at an episode start or once the sampling distance
        // reaches AB_len while the obstacle ship runs (the obstacle lane's own test, exchanged)
        const bool obs_stop = (bo & kStopBit) || coll;
        need = ((bo & kSampGeBit) && !obs_stop) || ((uf & kUfAutoReset) && env_done);
      }
    }
    // episode-done count: one ballot + popcount per wave, one atomic per wave
    if (type == 0 && (uf & kUfDoneCnt)) {
      const unsigned long long m = __ballot(env_done);
      if (lane == 0 && m) atomicAdd(a.io.done_count + step, (int)__popcll(m));
    }
    SIT_PH(5);
    // ---------------- auto reset: reset() + init_step() (test_beds/main_ast.py:314-329) ----------------
    if (live) {
      rt.fixup(s.k);
      ep_step += 1;
#ifdef SIT_ABLATE_RESET
      if (false) {
#else
      if ((uf & kUfAutoReset) && env_done) {
#endif
        // reset() (MSRL_Env.py:147-188) from the register copies
        s.n = p0[0]; s.e = p0[1]; s.psi = p0[2]; s.u = p0[3]; s.v = p0[4]; s.r = p0[5];
        s.ln = p0lo[0]; s.le = p0lo[1]; s.lpsi = p0lo[2]; s.lu = p0lo[3]; s.lv = p0lo[4]; s.lr = p0lo[5];
        s.ect_int = T(0); s.lei = T(0); s.k = 1; s.ticks = 0; s.stop = 0;
        rt.nw = nw0;
        rt.set_leg(leg0);
        ep_step = 0;
        if (type == 1) { samp = T(0); eps = T(0); samp_lo = T(0); ++episodes; }
        for (int j = 0; j < 6; ++j) lo[j] = lo0[j];
        init_step_ship(c, cs.x, s, rt, v_des);
      }
    }
    SIT_PH(6);
    p_ns += row_step * SIT_OBS_DIM;
    p_rw += row_step;
    p_dn += row_step;
    p_st += row_step;
    p_ao += row_step * 4;
    if (p_lg) p_lg += row_step * SIT_LOG_ROWS;
  }
#ifdef SIT_DIAG_PHASES
  if (lane == 0)
    for (int k = 0; k < 7; ++k) atomicAdd(&g_sit_diag[type][16 + k], ph[k]);
  const unsigned long long w_loop = ph_t;
#endif

  // ---------------- write back ----------------
  if (LOG && a.io.log && act) { a.st.fuel[0][sid] = f_me; a.st.fuel[1][sid] = f_el; a.st.fuel[2][sid] = f_tot; }
  if (MODE == kPolicy) {
    if (act && type == 1) a.io.policy_ready[env] = ready ? SIT_POLICY_READY : (stalled ? SIT_POLICY_WAITING : 0);
    static_assert(kEnvsPerBlock == kAdmitGroup || MODE != kPolicy, "one wave = one admission group");
    if (type == 1) publish_ages(a.io.request_age, a.io.group_counts, env, act, stalled, age0);
    if (a.io.env_steps && type == 0) {   // env-steps executed: one atomic per wave
      unsigned long long v = act ? n_stepped : 0;
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0 && v) atomicAdd(a.io.env_steps, v);
    }
  }
  if (act) {
    store_ship(a.st, sid, s);
    a.st.nw[sid] = rt.nw;
    for (int j = 0; j < lo_n; ++j) a.st.last_obs[(size_t)(lo_base + j) * n_env + env] = lo[j];
    if (type == 1) {
      a.st.env[0][env] = samp; a.st.env[1][env] = eps;
      a.st.env[2][env] = ppn; a.st.env[3][env] = ppe;
      a.st.env[4][env] = iwn; a.st.env[5][env] = iwe;
      if constexpr (kIsF32<T>) {
        a.st.env_lo[0][env] = samp_lo;
        a.st.env_lo[1][env] = ppn_lo; a.st.env_lo[2][env] = ppe_lo;
      }
      a.st.ep_step[env] = ep_step;
      a.st.event[env] = event;
      a.st.episodes[env] = episodes;
    }
  }
#ifdef SIT_DIAG_PHASES
  // whole-wave timing: [24] sum of wave cycles, [25] max wave cycles, [26] sum of prologue
  // cycles, [27] sum of epilogue cycles, [28]/[29] min/max start (realtime), [30]/[31] min/max end
  if (lane == 0) {
    const unsigned long long w_t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long w_r1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* g = g_sit_diag[type];
    atomicAdd(&g[24], w_t1 - w_t0);
    atomicMax(&g[25], w_t1 - w_t0);
    atomicAdd(&g[26], w_loop - w_t0 - (ph[0] + ph[1] + ph[2] + ph[3] + ph[4] + ph[5] + ph[6]));
    atomicAdd(&g[27], w_t1 - w_loop);
    atomicMin(&g[28], w_r0);
    atomicMax(&g[29], w_r0);
    atomicMin(&g[30], w_r1);
    atomicMax(&g[31], w_r1);
    const int wid = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (wid < kDiagWaves) {
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);     // HW_REG_HW_ID
      const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);   // HW_REG_XCC_ID
      g_sit_wave[wid][0] = w_r0; g_sit_wave[wid][1] = w_r1; g_sit_wave[wid][2] = w_t1 - w_t0;
      g_sit_wave[wid][3] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    }
  }
#endif
}

// MACH: the handle's machinery model as a kernel template argument (a runtime branch on it inside
// the step loop measured ~4% slower: it splits the scheduling regions of guidance and dynamics)
template <typename T, int MODE, bool LDSMAP, bool LOG, int MACH>
__global__ __launch_bounds__(128 * kGroups, SIT_MIN_WAVES) void k_env_steps(const KArgs<T> a) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ Xchg<T> xs[2 * kGroups];
  __shared__ Consts<T> cs;
  if ((__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 1) == 0) env_steps<T, MODE, LDSMAP, LOG, 0, MACH>(a, smem, xs, cs);
  else env_steps<T, MODE, LDSMAP, LOG, 1, MACH>(a, smem, xs, cs);
}

#include "sit_sync.h"

// this translation unit's count of k_env_steps_sync blocks whose waves shared a SIMD (sit_role_fallbacks)
int role_fallbacks_impl(unsigned long long* out, int reset) {
#if SIT_SIMD_ROLES
  unsigned long long v = 0, z = 0;
  if (hipDeviceSynchronize() != hipSuccess) return SIT_E_HIP;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_role_fallback), sizeof(v)) != hipSuccess) return SIT_E_HIP;
  if (reset && hipMemcpyToSymbol(HIP_SYMBOL(g_role_fallback), &z, sizeof(z)) != hipSuccess) return SIT_E_HIP;
  *out += v;
#else
  (void)out; (void)reset;
#endif
  return SIT_OK;
}

// MultiShipRLEnv.init_step for masked envs (one thread per ship)
template <typename T>
__global__ __launch_bounds__(256) void k_init_step(const KArgs<T> a, const uint8_t* mask) {
  const int sid = blockIdx.x * blockDim.x + threadIdx.x;
  const int n_env = a.n_env;
  if (sid >= 2 * n_env) return;
  const int type = sid / n_env, env = sid - type * n_env;
  if (mask && !mask[env]) return;
  Ship<T> s;
  load_ship(a.st, sid, s);
  Route<T> rt;
  rt.nw = a.st.nw[sid];
  rt.end_n = a.sc.end_n[sid];
  rt.end_e = a.sc.end_e[sid];
  rt.tn = a.st.wn + (size_t)type * a.cap * n_env + env;
  rt.te = a.st.we + (size_t)type * a.cap * n_env + env;
  rt.stride = n_env;
  rt.cap = a.cap;
  rt.load_leg(s.k);
  init_step_ship(a.c, a.c.x, s, rt, init_val(a.sc, type, SIT_INIT_DESIRED_SPEED, env, n_env));
  store_ship(a.st, sid, s);
}

// MultiShipRLEnv.reset for masked envs (one thread per env)
template <typename T>
__global__ __launch_bounds__(256) void k_reset(const KArgs<T> a, const uint8_t* mask, T* initial_state) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  const int n_env = a.n_env;
  if (env >= n_env) return;
  if (!mask || mask[env]) {
    for (int type = 0; type < 2; ++type) {
      const int sid = type * n_env + env;
      Ship<T> s;
      load_ship(a.st, sid, s);
      int nw;
      reset_ship(a.sc, type, env, n_env, s, nw);
      store_ship(a.st, sid, s);
      a.st.nw[sid] = nw;
    }
    a.st.env[0][env] = T(0);
    a.st.env[1][env] = T(0);
    a.st.env_lo[0][env] = T(0);
    a.st.ep_step[env] = 0;
    for (int j = 0; j < SIT_OBS_DIM; ++j)
      a.st.last_obs[(size_t)j * n_env + env] = a.sc.initial_state[(size_t)env * SIT_OBS_DIM + j];
  }
  // the construction-time observation (constant per env) is returned for every env
  if (initial_state)
    for (int j = 0; j < SIT_OBS_DIM; ++j)
      initial_state[(size_t)env * SIT_OBS_DIM + j] = a.sc.initial_state[(size_t)env * SIT_OBS_DIM + j];
}

// map predicates of arbitrary points (test/diagnostic entry sit_probe_map, one thread per
// point): boundary distance, Polygon.contains of the point, is_pos_inside_obstacles hull test
template <typename T>
__global__ __launch_bounds__(256) void k_probe_map(const KArgs<T> a, int n, const T* pts, T* dist,
                                                   uint8_t* inside, uint8_t* hull) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const T pn = pts[2 * i], pe = pts[2 * i + 1];
  const T d = distance_indexed(a.c, a.map, pn, pe);
  if (dist) dist[i] = d;
  if (inside) inside[i] = pip_point(a.c, a.map, pn, pe) ? 1 : 0;
  if (hull) hull[i] = hull_in_terrain(a.c, a.map, pn, pe, d) ? 1 : 0;
}

// the IEEE float64 helpers of the knife-edge decisions (sit_selftest_f64, one thread per input):
// compiled into both translation units, so the fast-math one is checked bitwise against numpy
__global__ __launch_bounds__(256) void k_selftest_f64(int op, int n, const double* a, const double* b, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = a[i], y = b[i];
  double r;
  switch (op) {
    case 0: r = ieee_div(x, y); break;
    case 1: r = ieee_sqrt(x); break;
    case 2: r = ieee_sq2(x, y); break;
    case 3: r = ieee_sub(ieee_add(x, y), x); break;
    case 4: r = ieee_dot2(x, y, y, x); break;
    case 5: r = sin(x); break;            // the transcendental functions the float64 path and the
    case 6: r = cos(x); break;            // knife-edge re-evaluations call (ocml): compared with
    case 7: r = atan2(x, y); break;       // the reference's libm in tests/test_gpu_parity.py
    // the float32 functions of the float32 step (this TU's build flags): the heading / IW-direction
    // sine and cosine (xsincos: v_sin / v_cos under SIT_FAST_TRIG), the LOS course (atan) and the leg
    // angle (atan2) of float32 arguments, returned as float64 (test_f32_fast_trig_accuracy)
    case 9: case 10: {
      float sf, cf;
      xsincos((float)x, &sf, &cf);
      r = op == 9 ? (double)sf : (double)cf;
      break;
    }
    case 11: r = (double)xatan((float)x); break;
    case 12: r = (double)xatan2((float)x, (float)y); break;
    default: {                            // 8: k_env_steps_sync's roles for the SIMD assignment x
      // (base 4: SIMD of wave v = digit v) and CU ticket y: role of wave v in base-4 digit v
      const int s = (int)x, tk = (int)y;
      int packed = 0;
      for (int v = 0; v < 4; ++v)
        packed |= sync_role_of(s & 3, (s >> 2) & 3, (s >> 4) & 3, (s >> 6) & 3, v, tk, SIT_SIMD_MIRROR) << (2 * v);
      r = (double)packed;
    }
  }
  out[i] = r;
}

// policy head + scatter (sit_policy_apply, one thread per request row): the squashed Gaussian
// action tanh(mu + exp(clip(log_sigma, -20, 2)) * noise) (normal.py:88-101, gaussian_policy.py:
// 71-72) of each queued env, written into its action slot and marked ready
template <typename T>
__global__ __launch_bounds__(256) void k_policy_apply(int cap, const T* head, int head_stride, const T* noise,
                                                      const int32_t* req_env, const int32_t* req_count,
                                                      int deterministic, T* policy_action, int32_t* policy_ready,
                                                      unsigned long long* served, int n_env) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int cnt = *req_count;
  if (i == 0 && served) atomicAdd(served, (unsigned long long)(cnt < cap ? cnt : cap));
  if (i >= cap || i >= cnt) return;
  const int e = req_env[i];
  if (e < 0 || e >= n_env) return;
  const T mu = head[(size_t)i * head_stride];
  const T ls = xclip(head[(size_t)i * head_stride + 1], T(-20), T(2));
  const T x = deterministic ? mu : mu + exp(ls) * noise[i];
  policy_action[e] = tanh(x);
  policy_ready[e] = 1;
}

// construction-time state (one thread per env)
template <typename T>
__global__ __launch_bounds__(256) void k_restart(const KArgs<T> a) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  const int n_env = a.n_env;
  if (env >= n_env) return;
  for (int type = 0; type < 2; ++type) {
    const int sid = type * n_env + env;
    Ship<T> s{};
    int nw;
    reset_ship(a.sc, type, env, n_env, s, nw);
    s.w = init_val(a.sc, type, SIT_INIT_SHAFT_SPEED, env, n_env);
    s.lw = init_lo(a.sc, type, SIT_INIT_SHAFT_SPEED, env, n_env);
    s.i1 = init_val(a.sc, type, SIT_INIT_SHIP_SPEED_I, env, n_env);
    s.i2 = init_val(a.sc, type, SIT_INIT_SHAFT_SPEED_I, env, n_env);
    s.li1 = init_lo(a.sc, type, SIT_INIT_SHIP_SPEED_I, env, n_env);
    s.li2 = init_lo(a.sc, type, SIT_INIT_SHAFT_SPEED_I, env, n_env);
    s.hi = T(0); s.hp = T(0); s.lrpm = T(0); s.lect = T(0); s.lpme = T(0); s.lhi = T(0);
    store_ship(a.st, sid, s);
    a.st.nw[sid] = nw;
  }
  for (int j = 0; j < kEnvReal; ++j) a.st.env[j][env] = T(0);
  for (int j = 0; j < kEnvLo; ++j) a.st.env_lo[j][env] = T(0);
  a.st.ep_step[env] = 0;
  a.st.event[env] = 0;
  a.st.episodes[env] = 0;
  for (int j = 0; j < SIT_OBS_DIM; ++j)
    a.st.last_obs[(size_t)j * n_env + env] = a.sc.initial_state[(size_t)env * SIT_OBS_DIM + j];
}

}  // namespace

// =======================================================================================
// host side
// =======================================================================================
struct sit_handle {
  int precision = SIT_F32;
  int n_env = 0;
  int cap = 0;
  int device = 0;
  sit_params p{};
  std::string err;
  // state blob
  unsigned char* blob = nullptr;
  size_t blob_bytes = 0;
  size_t off[kNumFields] = {};
  int64_t count[kNumFields] = {};
  // scenario
  unsigned char* scen = nullptr;
  size_t scen_init = 0, scen_init_lo = 0, scen_end_n = 0, scen_end_e = 0, scen_nw0 = 0, scen_ab_len = 0,
         scen_ab_alpha = 0, scen_initial = 0, scen_admit = 0, scen_serve = 0, scen_bytes = 0;
  // map
  unsigned char* map = nullptr;
  int n_poly = 0, n_vert = 0;
  size_t map_idx = 0, map_fine = 0, map_off = 0, map_bbox = 0, map_frank = 0, map_crec = 0, map_clive = 0;
  int use_cells = 0;
  int64_t n_mixed = 0, n_live = 0, n_idx = 0;
  int lds_attr[24] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                      -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};   // dynamic-LDS size per step-kernel variant
  size_t map_bytes = 0;      // bytes staged into LDS: Edge[n_edge] + packed index
  int lds_attr_sync[12] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};   // k_env_steps_sync [mode][mach][lds]
  // step-kernel selection, read once at sit_create (diagnostics / A-B runs only):
  //   SIT_STEP_KERNEL=classic  k_env_steps for every mode (default: k_env_steps_sync where it applies)
  //   SIT_LDS_MAP=0|1          map read through the caches / staged in LDS for every launch
  //                            (default: staged when the launch has >= kLdsMinSteps steps)
  int kernel_classic = 0;
  int lds_map_sel = -1;
  int fake_simds = 0;                // SIT_TEST_FAKE_SIMDS (test hook): 0x100 | base-4 SIMD assignment
  char last_kernel[96] = {};         // the step kernel of the last sit_step / sit_rollout launch
  int use_index = 0;
  double gx0 = 0, gy0 = 0, ginvx = 0, ginvy = 0, by0 = 0, binv = 0;
  double fx0 = 0, fy0 = 0, finvx = 0, finvy = 0;
  double min_n = 0, max_n = 0, min_e = 0, max_e = 0;
  bool have_map = false, have_routes = false, have_init = false;
  unsigned char* stage = nullptr;       // sit_step_host: pinned coherent host staging
  unsigned char* stage_dev = nullptr;   // its device address
};

namespace {

thread_local std::string g_create_err;

int fail(sit_handle* h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (h) h->err = buf; else g_create_err = buf;
  return code;
}

#define HIP_TRY(h, call)                                                                    \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess) return fail((h), SIT_E_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

// Device memory of the setup calls (sit_create / sit_load_* / sit_destroy).  Sanitizer builds
// (-DSIT_HOST_MEMORY_TEST, tools/sanitize.sh: host ASan/UBSan) back it with host memory, so that
// the host logic -- argument checks, blob layout, the map index, route and scenario staging --
// runs and is checked on a machine without a GPU; kernels are not launched in that build.
#ifdef SIT_HOST_MEMORY_TEST
hipError_t setup_device(int* d) { *d = 0; return hipSuccess; }
hipError_t setup_alloc(unsigned char** p, size_t n) {
  *p = static_cast<unsigned char*>(std::malloc(n ? n : 1));
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t setup_free(void* p) { std::free(p); return hipSuccess; }
hipError_t setup_zero(void* p, size_t n) { std::memset(p, 0, n); return hipSuccess; }
hipError_t setup_upload(void* dst, const void* src, size_t n) { std::memcpy(dst, src, n); return hipSuccess; }
#else
hipError_t setup_device(int* d) { return hipGetDevice(d); }
hipError_t setup_alloc(unsigned char** p, size_t n) { return hipMalloc(p, n); }
hipError_t setup_free(void* p) { return hipFree(p); }
hipError_t setup_zero(void* p, size_t n) { return hipMemset(p, 0, n); }
hipError_t setup_upload(void* dst, const void* src, size_t n) { return hipMemcpy(dst, src, n, hipMemcpyHostToDevice); }
#endif

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }
size_t real_size(const sit_handle* h) { return h->precision == SIT_F64 ? 8 : 4; }

// Derived constants, computed like the reference constructors (ship_model.py:71-130,
// ship_engine.py:32-44, 316-325; controllers; MSRL_env_ex.py).
template <typename T>
Consts<T> make_consts(const sit_handle* h) {
  const sit_params& p = h->p;
  Consts<T> c{};
  const double dwt = p.dead_weight_tonnage;
  const double payload = 0.9 * (dwt - p.bunkers);
  const double lsw = dwt / p.coefficient_of_deadweight_to_displacement - dwt;
  const double mass = lsw + payload + p.bunkers + p.ballast;
  const double l = p.length_of_ship, w = p.width_of_ship;
  const double i_z = mass * (l * l + w * w) / 12;
  const double x_du = mass * p.added_mass_coefficient_in_surge;
  const double y_dv = mass * p.added_mass_coefficient_in_sway;
  const double n_dr = i_z * p.added_mass_coefficient_in_yaw;
  const double area_f = w * p.front_height, area_l = l * p.side_height;
  c.dt = (T)p.integration_step;
  c.mass = (T)mass; c.x_du = (T)x_du; c.y_dv = (T)y_dv;
  c.inv_m11 = (T)(1.0 / (mass + x_du));
  c.inv_m22 = (T)(1.0 / (mass + y_dv));
  c.inv_m33 = (T)(1.0 / (i_z + n_dr));
  c.d_u = (T)(mass / p.mass_over_linear_friction_coefficient_in_surge);
  c.d_v = (T)(mass / p.mass_over_linear_friction_coefficient_in_sway);
  c.d_r = (T)(i_z / p.mass_over_linear_friction_coefficient_in_yaw);
  c.ku = (T)p.nonlinear_friction_coefficient_in_surge;
  c.kv = (T)p.nonlinear_friction_coefficient_in_sway;
  c.kr = (T)p.nonlinear_friction_coefficient_in_yaw;
  c.vc_n = (T)p.current_velocity_component_from_north;
  c.vc_e = (T)p.current_velocity_component_from_east;
  c.wind_speed = (T)p.wind_speed;
  c.wind_sin = (T)std::sin(p.wind_direction);
  c.wind_cos = (T)std::cos(p.wind_direction);
  c.wk_u = (T)(-0.5 * p.rho_air * p.cx * area_f);
  c.wk_v = (T)(-0.5 * p.rho_air * p.cy * area_l);
  c.wk_n = (T)(-p.rho_air * p.cn * area_l * l);
  c.c_rv = (T)p.rudder_angle_to_sway_force_coefficient;
  c.c_rr = (T)p.rudder_angle_to_yaw_force_coefficient;
  c.rudder_max = (T)(p.max_rudder_angle_degrees * M_PI / 180);
  const double me = p.main_engine_capacity, el = p.electrical_capacity, hotel = p.hotel_load;
  double avail = 0, avail_me = 0, avail_el = 0;
  if (hotel != 0.0) {   // BaseMachineryModel only sets the powers for a truthy hotel load
    if (p.shaft_generator_state == SIT_SG_MOTOR) { avail = me + el - hotel; avail_me = me; avail_el = el - hotel; }
    else if (p.shaft_generator_state == SIT_SG_GEN) { avail = me - hotel; avail_me = me - hotel; avail_el = 0; }
    else { avail = me; avail_me = me; avail_el = 0; }
  }
  c.avail_prop = (T)avail; c.avail_me = (T)avail_me; c.avail_el = (T)avail_el;
  c.tqcap_me = (T)(avail_me / 5 * M_PI / 30);
  c.tqcap_el = (T)(avail_el / 5 * M_PI / 30);
  c.d_me = (T)p.linear_friction_main_engine;
  c.d_hsg = (T)p.linear_friction_hybrid_shaft_generator;
  c.r_me = (T)p.gear_ratio_between_main_engine_and_propeller;
  c.r_hsg = (T)p.gear_ratio_between_hybrid_shaft_generator_and_propeller;
  c.kp_prop = (T)p.propeller_speed_to_torque_coefficient;
  c.jp = (T)p.propeller_inertia;
  c.thrust_k = (T)(std::pow(p.propeller_diameter, 4.0) * p.propeller_speed_to_thrust_force_coefficient);
  c.me_cap = (T)me; c.hotel = (T)hotel; c.load_el_gen = (T)std::min(hotel, el);
  c.sg_mode = p.shaft_generator_state;
  c.mach_simpl = p.machinery_model == SIT_MACH_SIMPLIFIED;
  // SimplifiedMachineryModel (ship_engine.py:420-428): power = load_perc * (available propulsion
  // power of the main engine + of the electrical side), k_thrust = 2160 / 790
  c.k_thrust = (T)(2160.0 / 790.0);
  c.inv_tau = (T)(1.0 / p.thrust_force_dynamic_time_constant);
  c.p_simpl = (T)(avail_me + avail_el);
  c.collision_bias = p.collision_bias;
  c.kp1 = (T)p.kp_ship_speed; c.ki1 = (T)p.ki_ship_speed;
  c.kp2 = (T)p.kp_shaft_speed; c.ki2 = (T)p.ki_shaft_speed;
  c.kp_h = (T)p.heading_kp; c.kd_h = (T)p.heading_kd; c.ki_h = (T)p.heading_ki;
  c.los_r = (T)p.lookahead_distance;
  c.los_r2 = (T)(p.lookahead_distance * p.lookahead_distance);
  c.los_clamp = (T)(0.99 * p.lookahead_distance);
  c.los_ki = (T)p.los_integral_gain;
  c.windup = (T)p.integrator_windup_limit;
  c.ra2 = p.radius_of_acceptance * p.radius_of_acceptance;
  c.bias_scale = (T)p.bias_throttle_scale;
  c.bias_max = (T)p.bias_throttle_max;
  c.bias_rudder = (T)(p.bias_rudder_degrees * (M_PI / 180.0));
  c.e_tol = (T)p.e_tolerance;
  c.arrival_radius = (T)p.arrival_radius;
  c.rpm_max = (T)p.shaft_rpm_max;
  c.min_dist2 = (T)(p.minimum_ship_distance * p.minimum_ship_distance);
  c.coll_d2 = p.minimum_ship_distance * p.minimum_ship_distance;
  {  // sqrt(x) <= r  <=>  x <= d2_le (IEEE sqrt is correctly rounded and monotone)
    const double r = p.arrival_radius;
    double v = r * r;
    // (towards +-DBL_MAX, not infinity: the float32 TU's device pass parses this with finite math)
    while (std::sqrt(std::nextafter(v, DBL_MAX)) <= r) v = std::nextafter(v, DBL_MAX);
    while (v > 0 && std::sqrt(v) > r) v = std::nextafter(v, -DBL_MAX);
    c.arrive_d2_le = v;
  }
  c.theta = (T)p.theta;
  c.blackout_kw = (T)(me / 1000);
  c.rpm_k = c.mach_simpl ? T(0) : (T)(30.0 / M_PI);   // SimplifiedMachineryModel: no shaft
  c.inv_dt = (T)(1.0 / p.integration_step);
  c.inv_e_tol = (T)(1.0 / p.e_tolerance);
  c.inv_maxn = (T)(1.0 / h->max_n);
  c.inv_jp = (T)(1.0 / p.propeller_inertia);
  c.inv_r_me = (T)(1.0 / p.gear_ratio_between_main_engine_and_propeller);
  c.inv_r_hsg = (T)(1.0 / p.gear_ratio_between_hybrid_shaft_generator_and_propeller);
  c.half_len = (T)(l / 2);
  c.min_n = (T)h->min_n; c.max_n = (T)h->max_n; c.min_e = (T)h->min_e; c.max_e = (T)h->max_e;
  c.pi6 = (T)(M_PI / 6.0);
  c.gx0 = (T)h->gx0; c.gy0 = (T)h->gy0; c.ginvx = (T)h->ginvx; c.ginvy = (T)h->ginvy;
  c.by0 = (T)h->by0; c.binv = (T)h->binv;
  c.hull_safe = (T)(l / 2 * std::sqrt(2.0) + 1.0);
  c.fx0 = (T)h->fx0; c.fy0 = (T)h->fy0; c.finvx = (T)h->finvx; c.finvy = (T)h->finvy;
  c.el_cap = (T)el;
  c.fuel_me_a = (T)p.fuel_me_a; c.fuel_me_b = (T)p.fuel_me_b; c.fuel_me_c = (T)p.fuel_me_c;
  c.fuel_dg_a = (T)p.fuel_dg_a; c.fuel_dg_b = (T)p.fuel_dg_b; c.fuel_dg_c = (T)p.fuel_dg_c;
  c.rad2deg = (T)(180.0 / M_PI);
  // float64 thresholds and gains (knife-edge decisions; MSRL_env_ex.py:119, 554-603, 754, 829)
  c.x.los_r = p.lookahead_distance;
  c.x.windup = p.integrator_windup_limit;
  c.x.e_tol = p.e_tolerance;
  c.x.arrival = p.arrival_radius;
  c.x.rpm_max = p.shaft_rpm_max;
  c.x.min_dist = p.minimum_ship_distance;
  c.x.blackout = me / 1000;
  c.x.dt = p.integration_step;
  c.x.kp1 = p.kp_ship_speed; c.x.ki1 = p.ki_ship_speed;
  c.x.kp2 = p.kp_shaft_speed; c.x.ki2 = p.ki_shaft_speed;
  c.x.avail_prop = avail; c.x.me_cap = me; c.x.hotel = hotel; c.x.load_el_gen = std::min(hotel, el);
  c.x.bias_scale = p.bias_throttle_scale; c.x.bias_max = p.bias_throttle_max;
  c.x.half_len = l / 2;
  c.x.theta = p.theta;
  return c;
}

// bytes of the map blob the fused step kernels stage into LDS (SIT_LDS_CELLS)
size_t map_stage_bytes(const sit_handle* h) { return SIT_LDS_CELLS ? h->map_bytes : h->map_frank; }

template <typename T>
KArgs<T> make_args(const sit_handle* h) {
  KArgs<T> a{};
  a.c = make_consts<T>(h);
  a.n_env = h->n_env;
  a.cap = h->cap;
  auto fp = [&](int f) { return reinterpret_cast<T*>(h->blob + h->off[f]); };
  auto ip = [&](int f) { return reinterpret_cast<int32_t*>(h->blob + h->off[f]); };
  for (int i = 0; i < kShipReal; ++i) a.st.ship[i] = fp(F_NORTH + i);
  a.st.k = ip(F_K); a.st.nw = ip(F_NW); a.st.ticks = ip(F_TICKS); a.st.stop = ip(F_STOP);
  for (int i = 0; i < kEnvReal; ++i) a.st.env[i] = fp(F_SAMP + i);
  a.st.ep_step = ip(F_EP);
  a.st.event = reinterpret_cast<uint32_t*>(h->blob + h->off[F_EVENT]);
  a.st.episodes = reinterpret_cast<uint32_t*>(h->blob + h->off[F_EPISODES]);
  a.st.wn = fp(F_WN); a.st.we = fp(F_WE);
  a.st.last_obs = fp(F_LAST_OBS);
  for (int i = 0; i < 3; ++i) a.st.fuel[i] = fp(F_FUEL_ME + i);
  a.st.last_log = fp(F_LAST_LOG);
  a.st.iwk[0] = fp(F_IWK_N); a.st.iwk[1] = fp(F_IWK_E);
  a.st.iwk_flags = reinterpret_cast<uint32_t*>(h->blob + h->off[F_IWK_FLAGS]);
  for (int i = 0; i < kShipLo; ++i) a.st.ship_lo[i] = fp(F_SHIP_LO + i);
  for (int i = 0; i < kEnvLo; ++i) a.st.env_lo[i] = fp(F_ENV_LO + i);
  a.sc.init = reinterpret_cast<const T*>(h->scen + h->scen_init);
  a.sc.end_n = reinterpret_cast<const T*>(h->scen + h->scen_end_n);
  a.sc.end_e = reinterpret_cast<const T*>(h->scen + h->scen_end_e);
  a.sc.nw0 = reinterpret_cast<const int32_t*>(h->scen + h->scen_nw0);
  a.sc.ab_len = reinterpret_cast<const double*>(h->scen + h->scen_ab_len);
  a.sc.ab_alpha = reinterpret_cast<const double*>(h->scen + h->scen_ab_alpha);
  a.sc.initial_state = reinterpret_cast<const T*>(h->scen + h->scen_initial);
  a.sc.init_lo = reinterpret_cast<const T*>(h->scen + h->scen_init_lo);
  a.map.n_poly = h->n_poly;
  a.map.n_edge = h->n_vert;
  a.map.use_index = h->use_index;
  a.map.edge = reinterpret_cast<const Edge<T>*>(h->map);
  a.map.idx = reinterpret_cast<const uint16_t*>(h->map + h->map_idx);
  a.map.fine = reinterpret_cast<const uint32_t*>(h->map + h->map_fine);
  a.map.frank = reinterpret_cast<const uint16_t*>(h->map + h->map_frank);
  a.map.crec = reinterpret_cast<const uint2*>(h->map + h->map_crec);
  a.map.clive = reinterpret_cast<const uint8_t*>(h->map + h->map_clive);
  a.map.use_cells = h->use_cells;
  a.map.n_idx = (int32_t)h->n_idx;
  a.map.n_mixed = (int32_t)h->n_mixed;
  a.map.n_live = (int32_t)h->n_live;
  a.map.off = reinterpret_cast<const int32_t*>(h->map + h->map_off);
  a.map.bbox = reinterpret_cast<const T*>(h->map + h->map_bbox);
  a.map_bytes = (int32_t)map_stage_bytes(h);
  return a;
}

// policy-mode admission scratch: [n_groups][kAgeBuckets] counts, [n_groups][2] plan, header
int32_t* admit_counts(const sit_handle* h) { return reinterpret_cast<int32_t*>(h->scen + h->scen_admit); }
// in-kernel serving's fallback queue (logged launches run the one-wave kernel): capacity n_env
struct ServeQueue {
  int32_t* env;
  int32_t* age;
  int32_t* count;
  void* obs;
  void* noise;
};
ServeQueue serve_queue(const sit_handle* h) {
  unsigned char* b = h->scen + h->scen_serve;
  const size_t n = (size_t)h->n_env, rs = h->precision == SIT_F64 ? 8 : 4;
  ServeQueue q;
  q.env = reinterpret_cast<int32_t*>(b);
  q.age = q.env + n;
  q.count = q.age + n;
  q.obs = b + ((3 * n * 4 + 255) & ~size_t(255));
  q.noise = static_cast<unsigned char*>(q.obs) + n * SIT_OBS_DIM * rs;
  return q;
}

int ready(sit_handle* h) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (!h->have_map) return fail(h, SIT_E_STATE, "sit_load_map has not been called");
  if (!h->have_routes) return fail(h, SIT_E_STATE, "sit_load_routes has not been called");
  if (!h->have_init) return fail(h, SIT_E_STATE, "sit_load_initial has not been called");
  return SIT_OK;
}

// LDS budget of one step-kernel block: two blocks (4 waves, one per SIMD) must fit the CU's
// 160 KB; above 80 KB only one block fits and the grid runs in two rounds (~1.75x slower)
constexpr size_t kLdsBudget = 80 * 1024;
constexpr size_t kLdsCu = 160 * 1024;       // the CU's LDS (k_env_steps_sync: two 256-thread blocks per CU)
// launches of fewer steps read the map through the caches instead of staging it into LDS: staging
// 57 KB per block is a prologue that a single step (sit_step, the scalar drop-in) cannot amortise
#ifndef SIT_LDS_MIN_STEPS
#define SIT_LDS_MIN_STEPS 8
#endif
constexpr int kLdsMinSteps = SIT_LDS_MIN_STEPS;
size_t map_lds_bytes(const sit_handle* h) { return (map_stage_bytes(h) + 255) & ~size_t(255); }

// the step kernel of a launch as a readable instantiation name (sit_step_kernel)
template <typename T>
void set_kernel_name(sit_handle* h, bool sync, int mode, bool lds, bool log, int mach) {
  static const char* const modes[3] = {"kExplicit", "kSynth", "kPolicy"};
  const char* t = kIsF32<T> ? "float" : "double";
  if (sync) snprintf(h->last_kernel, sizeof(h->last_kernel), "k_env_steps_sync<%s,%s,%s,MACH=%d>", t, modes[mode],
                     lds ? "map=LDS" : "map=global", mach);
  else snprintf(h->last_kernel, sizeof(h->last_kernel), "k_env_steps<%s,%s,%s,%s,MACH=%d>", t, modes[mode],
                lds ? "map=LDS" : "map=global", log ? "log" : "nolog", mach);
}

// the launch's k_env_steps_sync map placement and dynamic LDS (0: the launch takes k_env_steps);
// *attr: the kernel's dynamic-LDS attribute (policy mode: the in-kernel serving size, whether or not
// the launch serves, so one attribute covers both)
template <typename T>
size_t sync_launch_lds(const sit_handle* h, const StepIO<T>& io, bool* lds_map, size_t* attr) {
  const bool sync_lds = h->lds_map_sel == 1 || (h->lds_map_sel < 0 && io.n_steps >= kLdsMinSteps);
  const size_t map = sync_lds ? map_stage_bytes(h) : 0;
  const bool policy = io.policy_action && !io.action_ne;
  const size_t lds = io.actor_w ? serve_lds_bytes<T>(map)
                     : policy   ? sync_lds_bytes<T, kPolicy>(map)
                     : io.action_ne ? sync_lds_bytes<T, kExplicit>(map) : sync_lds_bytes<T, kSynth>(map);
  const size_t at_serve = (policy ? serve_lds_bytes<T>(map) : lds) + SIT_DYN_OFF;
  const size_t at = at_serve + sizeof(Consts<T>) + 256 <= kLdsCu ? at_serve : lds + SIT_DYN_OFF;
  if (lds_map) *lds_map = sync_lds;
  if (attr) *attr = at;
  // (the fit check on the LDS the launch uses: a queue-path policy launch is not refused for serving LDS)
  if (h->kernel_classic || io.log || !h->use_index || lds + SIT_DYN_OFF + sizeof(Consts<T>) + 256 > kLdsCu) return 0;
  return lds + SIT_DYN_OFF;
}

template <typename T>
int launch_steps(sit_handle* h, const StepIO<T>& io, hipStream_t stream) {
  KArgs<T> a = make_args<T>(h);
  a.io = io;
  const int mode = io.action_ne ? kExplicit : (io.policy_action ? kPolicy : kSynth);
  const int mach = a.c.mach_simpl ? 1 : 0;
  if (io.actor_w && mode != kPolicy) return fail(h, SIT_E_INVALID, "in-kernel serving needs policy mode");
  // k_env_steps_sync (sit_sync.h), two waves per ship with the map predicates on their own wave, for
  // every launch without the trajectory log: synthetic sampler (C3/C4), policy (C5) and explicit
  // actions (sit_step, the drop-in MultiShipRLEnv.step).  k_env_steps (one wave per ship) runs the
  // logged launches, and every launch under SIT_STEP_KERNEL=classic.  The sync kernel stages the map
  // into LDS for fused launches; single-step launches read it through the caches.
  bool sync_lds = false;
  size_t lds_attr = 0;
  const size_t lds_sync = sync_launch_lds<T>(h, io, &sync_lds, &lds_attr);
  if (lds_sync > 0) {
    const void* kern = nullptr;
    auto pick = [&](auto mode_tag, auto mach_tag, auto lds_tag) {
      constexpr int M = decltype(mode_tag)::value, K = decltype(mach_tag)::value;
      constexpr bool L = decltype(lds_tag)::value;
      kern = reinterpret_cast<const void*>(&k_env_steps_sync<T, M, K, L>);
    };
    auto pick_lds = [&](auto mode_tag, auto mach_tag) {
      if (sync_lds) pick(mode_tag, mach_tag, std::true_type{});
      else pick(mode_tag, mach_tag, std::false_type{});
    };
    auto pick_mach = [&](auto mode_tag) {
      if (mach) pick_lds(mode_tag, std::integral_constant<int, 1>{});
      else pick_lds(mode_tag, std::integral_constant<int, 0>{});
    };
    if (mode == kPolicy) pick_mach(std::integral_constant<int, kPolicy>{});
    else if (mode == kSynth) pick_mach(std::integral_constant<int, kSynth>{});
    else pick_mach(std::integral_constant<int, kExplicit>{});
    const int slot = ((mode * 2 + mach) * 2) + (sync_lds ? 1 : 0);
    if (h->lds_attr_sync[slot] != (int)lds_attr) {
      HIP_TRY(h, hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_attr));
      h->lds_attr_sync[slot] = (int)lds_attr;
    }
    const int blocks = (h->n_env + kSyncLanes - 1) / kSyncLanes;
    a.lds_bytes = (int32_t)(lds_sync - SIT_DYN_OFF);
    a.fake_simds = h->fake_simds;
    void* args[] = {&a};
    HIP_TRY(h, hipLaunchKernel(kern, dim3(blocks), dim3(256), args, lds_sync, stream));
    set_kernel_name<T>(h, true, mode, sync_lds, false, mach);
    return SIT_OK;
  }
  if (io.actor_w) return fail(h, SIT_E_INVALID, "in-kernel serving runs on k_env_steps_sync only");
  const int blocks = (h->n_env + kEnvsPerBlock * kGroups - 1) / (kEnvsPerBlock * kGroups);
  // the map (edges, index, classes) is staged in LDS when it fits the budget next to the static
  // exchange buffers and the launch has enough steps to amortise the staging; otherwise the
  // predicates read it through the caches
  const size_t stat = sizeof(Xchg<T>) * 2 * kGroups + sizeof(Consts<T>) + 256;
  const bool fits = map_lds_bytes(h) + stat <= kLdsBudget;
  const bool lds_map = fits && (h->lds_map_sel == 1 || (h->lds_map_sel < 0 && io.n_steps >= kLdsMinSteps));
  const size_t lds = lds_map ? map_lds_bytes(h) : 0;
  auto go = [&](auto kern) -> int {
    // the dynamic-LDS attribute is set once per kernel and size (not per launch: launches may be
    // captured into HIP graphs)
    const int slot = ((mode * 2 + (lds_map ? 1 : 0)) * 2 + (io.log ? 1 : 0)) * 2 + mach;
    if (lds_map && h->lds_attr[slot] != (int)lds) {
      HIP_TRY(h, hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      h->lds_attr[slot] = (int)lds;
    }
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(128 * kGroups), lds, stream, a);
    return SIT_OK;
  };
  auto pick_mach = [&](auto mode_tag, auto mach_tag) -> int {
    constexpr int M = decltype(mode_tag)::value, K = decltype(mach_tag)::value;
    if (io.log) return lds_map ? go(k_env_steps<T, M, true, true, K>) : go(k_env_steps<T, M, false, true, K>);
    return lds_map ? go(k_env_steps<T, M, true, false, K>) : go(k_env_steps<T, M, false, false, K>);
  };
  auto pick = [&](auto mode_tag) -> int {
    if (mach) return pick_mach(mode_tag, std::integral_constant<int, 1>{});
    return pick_mach(mode_tag, std::integral_constant<int, 0>{});
  };
  int rc;
  if (mode == kSynth) rc = pick(std::integral_constant<int, kSynth>{});
  else if (mode == kPolicy) rc = pick(std::integral_constant<int, kPolicy>{});
  else rc = pick(std::integral_constant<int, kExplicit>{});
  if (rc) return rc;
  HIP_TRY(h, hipGetLastError());
  set_kernel_name<T>(h, false, mode, lds_map, io.log != nullptr, mach);
  return SIT_OK;
}

template <typename T>
int launch_probe(sit_handle* h, int n, const void* pts_ne, void* dist, uint8_t* inside, uint8_t* hull,
                 hipStream_t stream) {
  const KArgs<T> a = make_args<T>(h);
  const int blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_probe_map<T>, dim3(blocks), dim3(256), 0, stream, a, n, (const T*)pts_ne, (T*)dist,
                     inside, hull);
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

int launch_selftest(int op, int n, const double* a, const double* b, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(k_selftest_f64, dim3((n + 255) / 256), dim3(256), 0, stream, op, n, a, b, out);
  return hipGetLastError() == hipSuccess ? SIT_OK : SIT_E_HIP;
}

}  // namespace

