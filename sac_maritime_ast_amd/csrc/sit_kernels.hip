// sit_kernels.hip — MI355X (gfx950) kernels and C ABI of the ship-in-transit env step.
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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
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
};
constexpr int kNumFields = (int)(sizeof(kFields) / sizeof(kFields[0]));
enum FieldId {
  F_NORTH = 0, F_LAST_PME = 14, F_K = 15, F_NW, F_TICKS, F_STOP,
  F_SAMP = 19, F_IW_E = 24, F_EP = 25, F_EVENT, F_EPISODES, F_WN, F_WE, F_LAST_OBS,
  F_FUEL_ME, F_FUEL_EL, F_FUEL, F_LAST_LOG
};

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
};

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
  // policy mode (kPolicy): per-env action slots and the request queue of waiting envs
  const T* policy_action;
  int32_t* policy_ready;
  int32_t* request_env;
  T* request_noise;
  T* request_obs;
  int32_t* request_count;
  int32_t request_capacity;
  unsigned long long* env_steps;
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
  int32_t map_bytes;
};

// Copy the edge records, the packed index and the class grid (the first map_bytes of the map
// blob) into LDS at `dst`.
template <typename T>
__device__ __forceinline__ Map<T> stage_map(const KArgs<T>& a, unsigned char* dst) {
  const unsigned char* src = reinterpret_cast<const unsigned char*>(a.map.edge);
  const int n16 = a.map_bytes / 16;
  for (int i = threadIdx.x; i < n16; i += blockDim.x)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  Map<T> m = a.map;
  m.edge = reinterpret_cast<const Edge<T>*>(dst);
  m.idx = reinterpret_cast<const uint16_t*>(dst + (reinterpret_cast<const unsigned char*>(a.map.idx) - src));
  m.fine = reinterpret_cast<const uint32_t*>(dst + (reinterpret_cast<const unsigned char*>(a.map.fine) - src));
  m.frank = reinterpret_cast<const uint16_t*>(dst + (reinterpret_cast<const unsigned char*>(a.map.frank) - src));
  m.crec = reinterpret_cast<const uint2*>(dst + (reinterpret_cast<const unsigned char*>(a.map.crec) - src));
  m.clive = reinterpret_cast<const uint8_t*>(dst + (reinterpret_cast<const unsigned char*>(a.map.clive) - src));
  return m;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// device helpers on the SoA state
// ---------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void load_ship(const State<T>& st, int sid, Ship<T>& s) {
  s.n = st.ship[0][sid]; s.e = st.ship[1][sid]; s.psi = st.ship[2][sid];
  s.u = st.ship[3][sid]; s.v = st.ship[4][sid]; s.r = st.ship[5][sid]; s.w = st.ship[6][sid];
  s.i1 = st.ship[7][sid]; s.i2 = st.ship[8][sid]; s.hi = st.ship[9][sid]; s.hp = st.ship[10][sid];
  s.ect_int = st.ship[11][sid]; s.lrpm = st.ship[12][sid]; s.lect = st.ship[13][sid];
  s.lpme = st.ship[14][sid];
  s.k = st.k[sid]; s.ticks = st.ticks[sid]; s.stop = st.stop[sid];
}

template <typename T>
__device__ __forceinline__ void store_ship(const State<T>& st, int sid, const Ship<T>& s) {
  st.ship[0][sid] = s.n; st.ship[1][sid] = s.e; st.ship[2][sid] = s.psi;
  st.ship[3][sid] = s.u; st.ship[4][sid] = s.v; st.ship[5][sid] = s.r; st.ship[6][sid] = s.w;
  st.ship[7][sid] = s.i1; st.ship[8][sid] = s.i2; st.ship[9][sid] = s.hi; st.ship[10][sid] = s.hp;
  st.ship[11][sid] = s.ect_int; st.ship[12][sid] = s.lrpm; st.ship[13][sid] = s.lect;
  st.ship[14][sid] = s.lpme;
  st.k[sid] = s.k; st.ticks[sid] = s.ticks; st.stop[sid] = s.stop;
}

template <typename T>
__device__ __forceinline__ T init_val(const Scen<T>& sc, int type, int f, int env, int n_env) {
  return sc.init[(type * SIT_INIT_NF + f) * n_env + env];
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
  s.ect_int = T(0);
  s.k = 1;
  s.ticks = 0;
  s.stop = 0;
  nw = sc.nw0[type * n_env + env];
}

// one guidance/control/update/integrate cycle without store, time or bias (MSRL_Env.py:190-217)
template <typename T>
__device__ __forceinline__ void init_step_ship(const Consts<T>& c, Ship<T>& s, Route<T>& rt, T v_des) {
  T rudder, thr, ect, sp, cp, psi_ref;
  xsincos(s.psi, &sp, &cp);
  guidance_control(c, s, rt, v_des, rudder, thr, ect, psi_ref);
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

// ---------------------------------------------------------------------------------------
// the env step kernel: K steps of MultiShipRLEnv.step (+ optional auto-reset)
//   MODE  : kExplicit = caller's action arrays, kSynth = synthetic AST sampler on device,
//           kPolicy = actions from a policy run between launches (an env that reaches a
//           sampling event without a fresh action waits for the rest of the launch and queues
//           a request; the next launch consumes the action the policy wrote for it)
// ---------------------------------------------------------------------------------------
#if defined(SIT_DIAG_PATHS) || defined(SIT_DIAG_PHASES)
// Diagnostic builds only (tools/diag_paths.py): [type][0..15] predicate path statistics,
// [type][16..23] shader-clock cycles per step phase (wave lane 0).
__device__ unsigned long long g_sit_diag[2][32];
#endif
#ifdef SIT_DIAG_PHASES
// per wave of the last launch: start / end (realtime ticks), shader cycles, HW_ID | XCC_ID << 32
constexpr int kDiagWaves = 8192;
__device__ unsigned long long g_sit_wave[kDiagWaves][4];
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
    v[0] = (int)(reinterpret_cast<const uint32_t*>(m.idx)[cell] >> 16) * 5;
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

// IW = obstacle position + AB_len (cos, sin)(AB_alpha + a): float trig for the float handle
// (1e-7 relative of AB_len, inside its 1e-5 contract), double for the float64 handle
__device__ __forceinline__ void iw_point(float n, float e, double ab_len, double ab_alpha, double ang, float& iwn,
                                         float& iwe) {
  float sn, cs;
  sincosf((float)(ab_alpha + ang), &sn, &cs);
  iwn = n + (float)ab_len * cs;
  iwe = e + (float)ab_len * sn;
}
__device__ __forceinline__ void iw_point(double n, double e, double ab_len, double ab_alpha, double ang, double& iwn,
                                         double& iwe) {
  iwn = n + ab_len * cos(ab_alpha + ang);
  iwe = e + ab_len * sin(ab_alpha + ang);
}

constexpr int kExplicit = 0, kSynth = 1, kPolicy = 2;
constexpr uint32_t kSampGeBit = 1u << 28;   // exchange-only: obstacle sampling distance >= AB_len

template <typename T, int MODE, bool LDSMAP, bool LOG>
__global__ __launch_bounds__(128) void k_env_steps(const KArgs<T> a) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ Xchg<T> xs[2];
#ifdef SIT_DIAG_PHASES
  const unsigned long long w_t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long w_r0 = __builtin_amdgcn_s_memrealtime();
#endif
  // The ~70 per-step constants go kernel arguments -> LDS -> VGPRs: loaded through LDS they
  // land in vector registers (one wave per SIMD leaves ~512 per lane, AGPRs included), whereas
  // kernel-argument constants compete for the 102 SGPRs and spill to VGPR lanes (v_readlane
  // in the loop), and reading the LDS block inside the loop put ~40 dependent LDS reads on
  // each step's critical path (the register copy measured 12% faster).
  __shared__ Consts<T> cs;
  for (int i = threadIdx.x; i < (int)(sizeof(Consts<T>) / 4); i += blockDim.x)
    reinterpret_cast<uint32_t*>(&cs)[i] = reinterpret_cast<const uint32_t*>(&a.c)[i];
  __syncthreads();
  const Consts<T> c = cs;
  // LDS: the map blob (edges, index, classes).  Route tables stay in HBM (Route caches the
  // active leg); keeping the block under 64 KB of LDS matters: a larger allocation measured
  // ~1.75x slower at the same occupancy-limited grid.
  const Map<T> map = LDSMAP ? stage_map(a, smem) : a.map;
  const int lane = threadIdx.x & (kWave - 1);
  const int type = threadIdx.x >> 6;             // wave-uniform
  const int n_env = a.n_env;
  const int env = blockIdx.x * kEnvsPerBlock + lane;
  const bool act = lane < kEnvsPerBlock && env < n_env;
  const int sid = type * n_env + env;

  Ship<T> s{};
  Route<T> rt{};
  T v_des = T(0);
  T samp = T(0), eps = T(0), ppn = T(0), ppe = T(0), iwn = T(0), iwe = T(0);
  // the IW's terrain test is a pure function of (iwn, iwe), which change only at sampling
  // events (or with the caller's action): cache it
  T iw_tn = T(0), iw_te = T(0);
  bool iw_valid = false, iw_in = false;
  int ep_step = 0;
  uint32_t event = 0, episodes = 0;
  double ab_len = 0.0, ab_alpha = 0.0;
  T lo[6] = {};                      // this ship's part of the last observation
  const int lo_base = type == 0 ? 0 : 6, lo_n = type == 0 ? 6 : 4;
  // policy mode: both lanes of an env track whether its next step is a sampling event
  bool need = false, ready = false, stalled = false;
  T pa = T(0);
  uint32_t n_stepped = 0;
  if (MODE == kPolicy && act) {
    const double samp0 = (double)a.st.env[0][env];
    need = a.st.ep_step[env] == 0 || (samp0 >= a.sc.ab_len[env] && a.st.stop[n_env + env] == 0);
    ready = a.io.policy_ready[env] != 0;
    pa = a.io.policy_action[env];
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
    rt.load_leg(s.k);
    if (type == 1) {
      samp = a.st.env[0][env]; eps = a.st.env[1][env];
      ppn = a.st.env[2][env]; ppe = a.st.env[3][env];
      iwn = a.st.env[4][env]; iwe = a.st.env[5][env];
      event = a.st.event[env];
      episodes = a.st.episodes[env];
      ab_len = a.sc.ab_len[env];
      ab_alpha = a.sc.ab_alpha[env];
    }
  }
  const T maxn = c.max_n;
  // episode-start values held in registers (auto-reset reloads nothing from memory): the
  // construction pose, route length, first leg with its geometry, and initial observation
  T p0[6] = {};
  T lo0[6] = {};
  int nw0 = 0;
  typename Route<T>::Leg leg0{};
  if (act) {
    for (int j = 0; j < 6; ++j) p0[j] = init_val(a.sc, type, SIT_INIT_NORTH + j, env, n_env);
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
    double ang = NAN;
    bool stall_now = false;
    if (MODE == kPolicy && act && !stalled && need && !ready) {
      // sampling event without an action: wait for the policy; the obstacle lane queues the
      // request with this event's standard-normal draw (reparameterised sample, normal.py:96-101)
      // and its half of the observation; the test lane adds its half after the exchange
      stalled = stall_now = true;
      if (type == 1) {
        const int q = atomicAdd(a.io.request_count, 1);
        x.slot[lane] = q;
        if (q < a.io.request_capacity) {
          a.io.request_env[q] = env;
          a.io.request_noise[q] = (T)sampler_normal(a.io.seed, (uint64_t)(a.io.env_id_offset + env), event);
          for (int j = 0; j < 4; ++j) a.io.request_obs[(size_t)q * SIT_OBS_DIM + 6 + j] = lo[j];
        }
      }
    }
    const bool live = act && !stalled;
    T sp = T(0), cp = T(1);
    if (live) xsincos(s.psi, &sp, &cp);    // heading trig of the step, off the guidance chain
    if (live) {
      ++n_stepped;
      if (type == 1) {
        // converted_action / SAC_update / init of this step
        if (MODE == kPolicy) {
          init_f = (ep_step == 0);
          sac = need;
          if (sac) {                     // the policy's squashed action scales the route angle
            ang = (double)pa * (M_PI / 6.0);
            iw_point(s.n, s.e, ab_len, ab_alpha, ang, iwn, iwe);
            ++event;
          }
        } else if (MODE == kSynth) {
          init_f = (ep_step == 0);
          sac = init_f || ((double)samp >= ab_len && !s.stop);
          if (sac) {
            const double u01 = sampler_uniform(a.io.seed, (uint64_t)(a.io.env_id_offset + env), event);
            ang = (u01 * 2.0 - 1.0) * (M_PI / 6.0);
            iw_point(s.n, s.e, ab_len, ab_alpha, ang, iwn, iwe);
            ++event;
          }
        } else {
          init_f = a.io.init[row] != 0;
          sac = a.io.sac_update[row] != 0;
          iwn = a.io.action_ne[2 * row];
          iwe = a.io.action_ne[2 * row + 1];
        }
        // obs_step (MSRL_Env.py:287-402)
        if (s.stop) {
          if (p_lg) {                    // store_last_simulation_data: last row, time updated
            p_lg[0] = T(s.ticks) * c.dt;
            for (int kk = 1; kk < SIT_LOG_KEYS; ++kk) p_lg[kk * row_step] = a.st.last_log[kk * row_step + env];
          }
          s.ticks += 2;                  // stop path: next_time() twice, no integration (Q10)
          o_rpm = s.lrpm; o_ect = s.lect; o_pme = s.lpme;
        } else {
          if (sac) {                     // update_route: insert at index -1 (Q16)
            if (!rt.insert(iwn, iwe, s.k, a.cap)) bits |= SIT_ST_ROUTE_OVERFLOW;
            samp = T(0);
          }
          const T pre_n = s.n, pre_e = s.e;
          T rudder, thr, psi_ref;
          guidance_control(c, s, rt, v_des, rudder, thr, o_ect, psi_ref);
          o_rpm = s.w * c.rpm_k;
          o_pme = power_me_kw(c, thr);
          s.lrpm = o_rpm; s.lect = o_ect; s.lpme = o_pme;
          if (p_lg) {
            store_log_row(c, p_lg, row_step, s, thr, rudder, o_ect, psi_ref, f_me, f_el, f_tot);
            for (int kk = 0; kk < SIT_LOG_KEYS; ++kk) a.st.last_log[kk * row_step + env] = p_lg[kk * row_step];
          }
          ship_dynamics(c, s, thr, rudder, sp, cp);
          if (!init_f) {                 // distance between the last two stored positions
            const T dn = pre_n - ppn, de = pre_e - ppe;
            const T d = xsqrt(dn * dn + de * de);
            eps = eps + d;
            samp = samp + d;
          }
          ppn = pre_n; ppe = pre_e;
          s.ticks += 1;
        }
      } else {
        // test_step (MSRL_Env.py:219-285)
        T rudder, thr, psi_ref;
        guidance_control(c, s, rt, v_des, rudder, thr, o_ect, psi_ref);
        if (c.collision_bias) {          // is_collision_imminent() on all-zero states (Q1)
          thr = xclip(thr * c.bias_scale, T(0), c.bias_max);
          rudder = xclip(rudder + c.bias_rudder, -c.rudder_max, c.rudder_max);
        }
        o_rpm = s.w * c.rpm_k;
        o_pme = power_me_kw(c, thr);
        s.lrpm = o_rpm; s.lect = o_ect; s.lpme = o_pme;
        if (p_lg) store_log_row(c, p_lg, row_step, s, thr, rudder, o_ect, psi_ref, f_me, f_el, f_tot);
        ship_dynamics(c, s, thr, rudder, sp, cp);
        s.ticks += 1;
      }

      // ---------------- own termination predicates (MSRL_env_ex.py:628-881) ----------------
#if defined(SIT_ABLATE_PREDICATES)   // diagnostic builds only (tools/ablate.sh): polygon work removed
      const T dobst = T(1000);
      const bool terrain = false;
#elif defined(SIT_ABLATE_HULL)        // diagnostic: distance kept, hull test removed
      const T dobst = distance_indexed(c, map, s.n, s.e);
      const bool terrain = false;
#else
      SIT_PH(0);
      int cell_c;
      uint32_t word_c;
      const int cls_c = fine_lookup(c, map, s.n, s.e, cell_c, word_c);
      const T dobst = distance_indexed(c, map, s.n, s.e);
      SIT_PH(1);
      const bool terrain = hull_in_terrain_cls(c, map, s.n, s.e, dobst, cls_c, cell_c, word_c);
      SIT_PH(2);
#endif
#ifdef SIT_DIAG_PATHS
      diag_lane(c, map, s.n, s.e, dobst, type == 1, iwn, iwe, dv);
#endif
      const T dn_end = s.n - rt.end_n, de_end = s.e - rt.end_e;
      const bool arrive = xsqrt(dn_end * dn_end + de_end * de_end) <= c.arrival_radius;
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
        const bool pred[6] = {arrive, horizon, terrain, xabs(o_rpm) > c.rpm_max, xabs(o_ect) > c.e_tol,
                              o_pme > c.blackout_kw};
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
        if (xabs(o_ect) > c.e_tol || (double)samp > ab_len * (double)c.theta) {
          if (!stop) r_term = r_term - T(1000);
          stop = 1; done = true;
          bits |= SIT_ST_OBS_NAVIGATION;
        }
        if (done) bits |= SIT_ST_OBS_DONE;
      }
      s.stop = stop;
      if (type == 1) {
        int slot = -1;
        if (a.io.transitions && sac) slot = atomicAdd(a.io.transition_count, 1);
        x.slot[lane] = slot;
      }
      x.n[type][lane] = s.n;
      x.e[type][lane] = s.e;
      x.bits[type][lane] = bits | (stop ? kStopBit : 0u) | (done ? kDoneBit : 0u) |
                           ((MODE == kPolicy && type == 1 && (double)samp >= ab_len) ? kSampGeBit : 0u);
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
      if (outs & 8) *p_st = SIT_ST_NO_STEP;
      if (outs & 4) *p_dn = 0;
      if (stall_now) {
        const int q = x.slot[lane];
        if (q < a.io.request_capacity)
          for (int j = 0; j < 6; ++j) a.io.request_obs[(size_t)q * SIT_OBS_DIM + j] = lo[j];
      }
    }
    if (live) {
      const T dn = x.n[0][lane] - x.n[1][lane], de = x.e[0][lane] - x.e[1][lane];
      const bool coll = dn * dn + de * de < c.min_dist2;
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
        if (outs & 2) *p_rw = reward;
        if (outs & 4) *p_dn = env_done ? 1 : 0;
#endif
        const int slot = x.slot[lane];
        if (slot >= 0 && slot < a.io.transition_capacity) {
          T* rec = a.io.transitions + (size_t)slot * SIT_TRANSITION_DIM;
          for (int j = 0; j < 6; ++j) rec[j] = lo[j];
          rec[11] = reward;
          rec[12] = s.n; rec[13] = s.e; rec[14] = s.psi; rec[15] = o_rpm; rec[16] = o_ect; rec[17] = o_pme;
          const bool horizon_hit = a.io.mask_horizon > 0 && ep_step + 2 == a.io.mask_horizon;
          rec[22] = (horizon_hit || !env_done) ? T(1) : T(0);
        }
#ifndef SIT_ABLATE_STORES
        if (outs & 8) *p_st = status;
#endif
#ifndef SIT_ABLATE_STORES
        if (outs & 1) { store2(p_ns, s.n, s.e); store2(p_ns + 2, s.psi, o_rpm); store2(p_ns + 4, o_ect, o_pme); }
#endif
      } else {
#ifndef SIT_ABLATE_STORES
        if (outs & 1) { store2(p_ns, s.n, s.e); store2(p_ns + 2, s.psi, o_ect); }
#endif
#ifndef SIT_ABLATE_STORES
        if (outs & 16) { store2(p_ao, iwn, iwe); store2(p_ao + 2, (T)ang, sac ? T(1) : T(0)); }
#endif
        const int slot = x.slot[lane];
        if (slot >= 0 && slot < a.io.transition_capacity) {
          T* rec = a.io.transitions + (size_t)slot * SIT_TRANSITION_DIM;
          for (int j = 0; j < 4; ++j) rec[6 + j] = lo[j];
          rec[10] = (T)ang;
          rec[18] = s.n; rec[19] = s.e; rec[20] = s.psi; rec[21] = o_ect;
          if (MODE == kPolicy) rec[10] = pa;   // the policy's action (memory.push, main_ast.py:395)
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
        need = ((bo & kSampGeBit) && !obs_stop) || (a.io.auto_reset && env_done);
      }
    }
    // episode-done count: one ballot + popcount per wave, one atomic per wave
    if (type == 0 && a.io.done_count) {
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
      if (a.io.auto_reset && env_done) {
#endif
        // reset() (MSRL_Env.py:147-188) from the register copies
        s.n = p0[0]; s.e = p0[1]; s.psi = p0[2]; s.u = p0[3]; s.v = p0[4]; s.r = p0[5];
        s.ect_int = T(0); s.k = 1; s.ticks = 0; s.stop = 0;
        rt.nw = nw0;
        rt.set_leg(leg0);
        ep_step = 0;
        if (type == 1) { samp = T(0); eps = T(0); ++episodes; }
        for (int j = 0; j < 6; ++j) lo[j] = lo0[j];
        init_step_ship(c, s, rt, v_des);
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
    if (act && type == 1) a.io.policy_ready[env] = ready ? 1 : 0;
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
  rt.load_leg(s.k);
  init_step_ship(a.c, s, rt, init_val(a.sc, type, SIT_INIT_DESIRED_SPEED, env, n_env));
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

// policy head + scatter (sit_policy_apply, one thread per request row): the squashed Gaussian
// action tanh(mu + exp(clip(log_sigma, -20, 2)) * noise) (normal.py:88-101, gaussian_policy.py:
// 71-72) of each queued env, written into its action slot and marked ready
template <typename T>
__global__ __launch_bounds__(256) void k_policy_apply(int cap, const T* head, int head_stride, const T* noise,
                                                      const int32_t* req_env, const int32_t* req_count,
                                                      int deterministic, T* policy_action, int32_t* policy_ready,
                                                      int n_env) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap || i >= *req_count) return;
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
    s.i1 = init_val(a.sc, type, SIT_INIT_SHIP_SPEED_I, env, n_env);
    s.i2 = init_val(a.sc, type, SIT_INIT_SHAFT_SPEED_I, env, n_env);
    s.hi = T(0); s.hp = T(0); s.lrpm = T(0); s.lect = T(0); s.lpme = T(0);
    store_ship(a.st, sid, s);
    a.st.nw[sid] = nw;
  }
  for (int j = 0; j < kEnvReal; ++j) a.st.env[j][env] = T(0);
  a.st.ep_step[env] = 0;
  a.st.event[env] = 0;
  a.st.episodes[env] = 0;
  for (int j = 0; j < SIT_OBS_DIM; ++j)
    a.st.last_obs[(size_t)j * n_env + env] = a.sc.initial_state[(size_t)env * SIT_OBS_DIM + j];
}

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
  size_t scen_init = 0, scen_end_n = 0, scen_end_e = 0, scen_nw0 = 0, scen_ab_len = 0,
         scen_ab_alpha = 0, scen_initial = 0, scen_bytes = 0;
  // map
  unsigned char* map = nullptr;
  int n_poly = 0, n_vert = 0;
  size_t map_idx = 0, map_fine = 0, map_off = 0, map_bbox = 0, map_frank = 0, map_crec = 0, map_clive = 0;
  int use_cells = 0;
  int64_t n_mixed = 0, n_live = 0;
  int lds_attr[12] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};   // dynamic-LDS size per step-kernel variant
  size_t map_bytes = 0;      // bytes staged into LDS: Edge[n_edge] + packed index
  int use_index = 0;
  double gx0 = 0, gy0 = 0, ginvx = 0, ginvy = 0, by0 = 0, binv = 0;
  double fx0 = 0, fy0 = 0, finvx = 0, finvy = 0;
  double min_n = 0, max_n = 0, min_e = 0, max_e = 0;
  bool have_map = false, have_routes = false, have_init = false;
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
  c.theta = (T)p.theta;
  c.blackout_kw = (T)(me / 1000);
  c.rpm_k = (T)(30.0 / M_PI);
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
  return c;
}

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
  a.sc.init = reinterpret_cast<const T*>(h->scen + h->scen_init);
  a.sc.end_n = reinterpret_cast<const T*>(h->scen + h->scen_end_n);
  a.sc.end_e = reinterpret_cast<const T*>(h->scen + h->scen_end_e);
  a.sc.nw0 = reinterpret_cast<const int32_t*>(h->scen + h->scen_nw0);
  a.sc.ab_len = reinterpret_cast<const double*>(h->scen + h->scen_ab_len);
  a.sc.ab_alpha = reinterpret_cast<const double*>(h->scen + h->scen_ab_alpha);
  a.sc.initial_state = reinterpret_cast<const T*>(h->scen + h->scen_initial);
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
  a.map.off = reinterpret_cast<const int32_t*>(h->map + h->map_off);
  a.map.bbox = reinterpret_cast<const T*>(h->map + h->map_bbox);
  a.map_bytes = (int32_t)h->map_bytes;
  return a;
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
size_t map_lds_bytes(const sit_handle* h) { return (h->map_bytes + 255) & ~size_t(255); }

template <typename T>
int launch_steps(sit_handle* h, const StepIO<T>& io, hipStream_t stream) {
  KArgs<T> a = make_args<T>(h);
  a.io = io;
  const int blocks = (h->n_env + kEnvsPerBlock - 1) / kEnvsPerBlock;
  const int mode = io.action_ne ? kExplicit : (io.policy_action ? kPolicy : kSynth);
  // the map (edges, index, classes) is staged in LDS when it fits the budget next to the
  // static exchange buffers; otherwise the predicates read it through the caches
  const size_t stat = sizeof(Xchg<T>) * 2 + sizeof(Consts<T>) + 256;
  const bool lds_map = map_lds_bytes(h) + stat <= kLdsBudget;
  const size_t lds = lds_map ? map_lds_bytes(h) : 0;
  auto go = [&](auto kern) -> int {
    // the dynamic-LDS attribute is set once per kernel and size (not per launch: launches may be
    // captured into HIP graphs)
    const int slot = (mode * 2 + (lds_map ? 1 : 0)) * 2 + (io.log ? 1 : 0);
    if (lds_map && h->lds_attr[slot] != (int)lds) {
      HIP_TRY(h, hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      h->lds_attr[slot] = (int)lds;
    }
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(128), lds, stream, a);
    return SIT_OK;
  };
  auto pick = [&](auto mode_tag) -> int {
    constexpr int M = decltype(mode_tag)::value;
    if (io.log) return lds_map ? go(k_env_steps<T, M, true, true>) : go(k_env_steps<T, M, false, true>);
    return lds_map ? go(k_env_steps<T, M, true, false>) : go(k_env_steps<T, M, false, false>);
  };
  int rc;
  if (mode == kSynth) rc = pick(std::integral_constant<int, kSynth>{});
  else if (mode == kPolicy) rc = pick(std::integral_constant<int, kPolicy>{});
  else rc = pick(std::integral_constant<int, kExplicit>{});
  if (rc) return rc;
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

}  // namespace

// =======================================================================================
// C ABI
// =======================================================================================
extern "C" {

#if defined(SIT_DIAG_PATHS) || defined(SIT_DIAG_PHASES)
#ifdef SIT_DIAG_PHASES
int sit_diag_read_waves(unsigned long long* out, int n) {   // [n][4], diagnostic builds only
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (n > kDiagWaves) n = kDiagWaves;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sit_wave), sizeof(unsigned long long) * 4 * n) != hipSuccess) return -1;
  return 0;
}
#endif
int sit_diag_read(unsigned long long* out, int reset) {   // diagnostic builds only
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

int sit_probe_map(sit_handle* h, int32_t n, const void* pts_ne, void* dist, uint8_t* inside, uint8_t* hull,
                  void* stream) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (!h->have_map) return fail(h, SIT_E_STATE, "sit_load_map has not been called");
  if (n < 0 || (n > 0 && !pts_ne)) return fail(h, SIT_E_INVALID, "need n >= 0 points");
  if (n == 0) return SIT_OK;
  const int blocks = (n + 255) / 256;
  if (h->precision == SIT_F64) {
    const KArgs<double> a = make_args<double>(h);
    hipLaunchKernelGGL(k_probe_map<double>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a, n,
                       (const double*)pts_ne, (double*)dist, inside, hull);
  } else {
    const KArgs<float> a = make_args<float>(h);
    hipLaunchKernelGGL(k_probe_map<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a, n,
                       (const float*)pts_ne, (float*)dist, inside, hull);
  }
  HIP_TRY(h, hipGetLastError());
  return SIT_OK;
}

int sit_policy_apply(sit_handle* h, int32_t capacity, const void* head, int32_t head_stride, const void* noise,
                     const int32_t* request_env, const int32_t* request_count, int32_t deterministic,
                     void* policy_action, int32_t* policy_ready, void* stream) {
  if (!h) return fail(nullptr, SIT_E_INVALID, "null handle");
  if (capacity <= 0 || !head || head_stride < 2 || !request_env || !request_count || !policy_action ||
      !policy_ready || (!deterministic && !noise))
    return fail(h, SIT_E_INVALID, "policy_apply: bad arguments");
  const int blocks = (capacity + 255) / 256;
  if (h->precision == SIT_F64)
    hipLaunchKernelGGL(k_policy_apply<double>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, capacity,
                       (const double*)head, head_stride, (const double*)noise, request_env, request_count,
                       deterministic, (double*)policy_action, policy_ready, h->n_env);
  else
    hipLaunchKernelGGL(k_policy_apply<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, capacity,
                       (const float*)head, head_stride, (const float*)noise, request_env, request_count,
                       deterministic, (float*)policy_action, policy_ready, h->n_env);
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
}

const char* sit_last_error(const sit_handle* h) { return h ? h->err.c_str() : g_create_err.c_str(); }
int32_t sit_precision(const sit_handle* h) { return h ? h->precision : 0; }
int32_t sit_n_env(const sit_handle* h) { return h ? h->n_env : 0; }
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
  sit_handle* h = new sit_handle();
  h->precision = precision;
  h->n_env = n_env;
  h->cap = wpt_capacity;
  h->p = *p;
  hipError_t e = hipGetDevice(&h->device);
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
  h->scen_end_n = so; so = align256(so + (size_t)2 * n_env * rs);
  h->scen_end_e = so; so = align256(so + (size_t)2 * n_env * rs);
  h->scen_nw0 = so; so = align256(so + (size_t)2 * n_env * 4);
  h->scen_ab_len = so; so = align256(so + (size_t)n_env * 8);
  h->scen_ab_alpha = so; so = align256(so + (size_t)n_env * 8);
  h->scen_initial = so; so = align256(so + (size_t)n_env * SIT_OBS_DIM * rs);
  h->scen_bytes = so;
  if (hipMalloc(&h->blob, h->blob_bytes) != hipSuccess || hipMalloc(&h->scen, h->scen_bytes) != hipSuccess) {
    fail(nullptr, SIT_E_NOMEM, "hipMalloc of %zu + %zu bytes failed", h->blob_bytes, h->scen_bytes);
    sit_destroy(h);
    return SIT_E_NOMEM;
  }
  if (hipMemset(h->blob, 0, h->blob_bytes) != hipSuccess || hipMemset(h->scen, 0, h->scen_bytes) != hipSuccess) {
    fail(nullptr, SIT_E_HIP, "hipMemset failed");
    sit_destroy(h);
    return SIT_E_HIP;
  }
  *out = h;
  return SIT_OK;
}

void sit_destroy(sit_handle* h) {
  if (!h) return;
  if (h->blob) (void)hipFree(h->blob);
  if (h->scen) (void)hipFree(h->scen);
  if (h->map) (void)hipFree(h->map);
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
  const size_t head = (size_t)kIdxHead;
  const size_t gbase = (head + bentries.size() + 3) & ~size_t(3);   // 8-byte aligned groups
  const size_t n_idx = gbase + gentries.size();
  h->use_index = (n_idx < 65535 && n_idx * 2 <= 48 * 1024) ? 1 : 0;
  h->gx0 = gx0; h->gy0 = gy0; h->ginvx = 1.0 / sx; h->ginvy = 1.0 / sy;
  h->by0 = by0; h->binv = 1.0 / bh;
  std::vector<uint16_t> idx(h->use_index ? n_idx : 2, 0);
  if (h->use_index) {
    for (int c = 0; c < kGrid * kGrid; ++c) {
      idx[2 * c] = (uint16_t)((gbase + gstart[c]) / 4);             // first group
      idx[2 * c + 1] = (uint16_t)((gstart[c + 1] - gstart[c]) / 4); // group count
    }
    for (int b = 0; b <= kBands; ++b) idx[kBandBase + b] = (uint16_t)(head + bstart[b]);
    std::copy(bentries.begin(), bentries.end(), idx.begin() + head);
    std::copy(gentries.begin(), gentries.end(), idx.begin() + gbase);
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
  if (h->map) { (void)hipFree(h->map); h->map = nullptr; }
  HIP_TRY(h, hipMalloc(&h->map, o));
  HIP_TRY(h, hipMemcpy(h->map, host.data(), o, hipMemcpyHostToDevice));
  h->n_poly = n_poly;
  h->n_vert = nv;
  h->have_map = true;
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
  HIP_TRY(h, hipMemcpy(h->blob + h->off[F_WN], tn.data(), tn.size(), hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->blob + h->off[F_WE], te.data(), te.size(), hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->scen + h->scen_end_n, en.data(), en.size(), hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->scen + h->scen_end_e, ee.data(), ee.size(), hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->scen + h->scen_nw0, nw0.data(), nw0.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->scen + h->scen_ab_len, ab_len.data(), (size_t)n * 8, hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->scen + h->scen_ab_alpha, ab_alpha.data(), (size_t)n * 8, hipMemcpyHostToDevice));
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
  HIP_TRY(h, hipMemcpy(h->scen + h->scen_init, a.data(), a.size(), hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->scen + h->scen_initial, b.data(), b.size(), hipMemcpyHostToDevice));
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
  return launch_steps<float>(h, io, (hipStream_t)stream);
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
  if (ra->policy_action && ra->action_ne)
    return fail(h, SIT_E_INVALID, "policy mode and explicit actions are exclusive");
  if (ra->policy_action && (!ra->policy_ready || !ra->request_env || !ra->request_noise || !ra->request_obs ||
                            !ra->request_count || ra->request_capacity <= 0))
    return fail(h, SIT_E_INVALID, "policy mode needs policy_ready, request_env, request_noise, "
                                  "request_obs, request_count and a positive request_capacity");
  auto fill = [&](auto* io, auto* tag) {
    using R = std::remove_pointer_t<decltype(tag)>;
    io->n_steps = ra->n_steps; io->auto_reset = ra->auto_reset; io->seed = ra->seed;
    io->env_id_offset = ra->env_id_offset;
    io->action_ne = (const R*)ra->action_ne; io->sac_update = ra->sac_update; io->init = ra->init;
    io->next_state = (R*)ra->next_state; io->reward = (R*)ra->reward; io->done = ra->done;
    io->status = ra->status; io->action_out = (R*)ra->action_out; io->done_count = ra->done_count;
    io->transitions = (R*)ra->transitions; io->transition_count = ra->transition_count;
    io->transition_capacity = ra->transition_capacity; io->mask_horizon = ra->mask_horizon;
    io->policy_action = (const R*)ra->policy_action; io->policy_ready = ra->policy_ready;
    io->request_env = ra->request_env; io->request_noise = (R*)ra->request_noise;
    io->request_obs = (R*)ra->request_obs;
    io->request_count = ra->request_count; io->request_capacity = ra->request_capacity;
    io->env_steps = reinterpret_cast<unsigned long long*>(ra->env_steps);
    io->log = (R*)ra->log;
  };
  if (h->precision == SIT_F64) {
    StepIO<double> io{};
    fill(&io, (double*)nullptr);
    return launch_steps<double>(h, io, (hipStream_t)stream);
  }
  StepIO<float> io{};
  fill(&io, (float*)nullptr);
  return launch_steps<float>(h, io, (hipStream_t)stream);
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
  return SIT_OK;
}

}  // extern "C"
