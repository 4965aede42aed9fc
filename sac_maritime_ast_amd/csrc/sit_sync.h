// sit_sync.h — the step kernel with each ship's map predicates on a wave of their own, in the
// same step (no speculation): rollouts with auto-reset whose actions come from the synthetic AST
// sampler (configs C3/C4) or from the SAC policy between launches (config C5).
//
// Included from sit_impl.h (inside its anonymous namespace, after k_env_steps).
//
// Forward Euler moves a ship with its pre-step velocities and heading (ship_model.py:632-643), so
// the post-step position is known at the start of the step.  The D wave of each ship publishes it
// (and the obstacle's IW of the step) before barrier A, then runs guidance, control, machinery and
// kinetics; meanwhile the ship's P wave evaluates the map predicates of that position (boundary
// distance, hull in terrain, the IW test; MSRL_env_ex.py:490-542, 628-881) and every other predicate
// of a position alone (arrival, map horizon, and P0 the ship-ship collision).  Barrier B joins them:
// D decides the episode's end and runs the auto reset; P turns its predicates into the reward terms
// and writes its ship's next_state columns (P1 also the IW action row); P0, one step behind, writes
// reward / done / status and the replay transition.  The D waves carry the step's serial chain
// (guidance, control, machinery, kinetics), so everything that needs only a position runs on P.
//
// Roles: a 256-thread block is one env group of kSyncLanes envs x {D0, D1, P0, P1}; odd blocks take
// the roles in mirrored order (P0 P1 D0 D1), which aims each SIMD at one D and one P wave.
//
// Policy mode (MODE == kPolicy, the sampler of samplers.PolicySampler): at a sampling event D1
// consumes the env's action slot if the policy has filled it; otherwise the env takes no further
// step in this launch (all four waves skip it: D1 publishes the decision before barrier A), P0 writes
// the ST_NO_STEP rows, and D1 marks the env SIT_POLICY_WAITING at the end of the launch.  The request
// queue is built after the launch, deterministically (k_policy_admit, sit_actor.h), from the state
// the env stopped in — or, with sit_rollout_args.actor_weights, by the block itself: after barrier C
// the waiting envs are published to LDS and all four waves evaluate the actor for them
// (sit_serve.h), so the next launch finds every waiting env's action ready.
#pragma once

#ifndef SIT_SYNC_LANES
#define SIT_SYNC_LANES 64   // envs per group (active lanes of each of the group's four waves)
#endif
#ifndef SIT_SYNC_CREF
#define SIT_SYNC_CREF 1     // D waves read the constants from their LDS copy (no VGPR spills; +2.5 %)
#endif
constexpr int kSyncLanes = SIT_SYNC_LANES;

// Issue priority per role (s_setprio 0-3).  The two blocks on a CU put their waves on the SIMDs in
// D/P pairs of different env groups — (D0, P0) and (D1, P1) — and the two waves of a SIMD compete for
// its issue slots where both are ready.  Round 4, with P0 the longest chain: P0 > P1 > D1 > D0
// measured C3 +3.3 % and C5 +4.8 % (same-box A/B, two rounds; favouring the D waves instead cost
// 1 - 2 %).  Round 5: the double-float integrators made D1 the critical role, and D1 above
// its partner P1 — P0 > D1 > P1 > D0 — measured C5 +0.7 %, C3 +0.1 % (three rounds, gpurun_out/r05s)
#ifndef SIT_PRIO_P0
#define SIT_PRIO_P0 3
#endif
#ifndef SIT_PRIO_P1
#define SIT_PRIO_P1 1
#endif
#ifndef SIT_PRIO_D1
#define SIT_PRIO_D1 2
#endif
#ifndef SIT_PRIO_D0
#define SIT_PRIO_D0 0
#endif


// SIT_DIAG_SYNC (diagnostic builds only, tools/diag_sync.py): shader cycles per role and loop segment,
// lane 0 of each wave, summed into g_sit_diag[role >> 1][(role & 1) * 16 + segment]: 0 work before
// barrier A, 1 wait at A, 2 work A -> B, 3 wait at B, 4 work after B, 5 wave-steps; 6 and 7 P0's
// outputs of the previous step up to the row stores / the rest (part of 2); 8-11 sub-segments; D1 also
// 6 / 7 / 14 (tools/diag_sync.py names them per role)
#ifdef SIT_DIAG_SYNC
#define SY_INIT() unsigned long long sy_t = __builtin_amdgcn_s_memtime(), sy_acc[16] = {}
#define SY_MARK(k) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    sy_acc[k] += t_ - sy_t; sy_t = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#define SY_STEP() (sy_acc[5] += 1)
#define SY_FLUSH(role) do { if ((threadIdx.x & 63) == 0) for (int q_ = 0; q_ < 16; ++q_) \
    atomicAdd(&g_sit_diag[(role) >> 1][((role) & 1) * 16 + q_], sy_acc[q_]); } while (0)
#else
#define SY_INIT() do { } while (0)
#define SY_MARK(k) do { } while (0)
#define SY_STEP() do { } while (0)
#define SY_FLUSH(role) do { } while (0)
#endif
static_assert(kSyncLanes >= 1 && kSyncLanes <= kWave, "SIT_SYNC_LANES must be in [1, 64]");

// D-wave flags of a step (kSf*), per ship: the predicates of the ship's own step
constexpr uint32_t kSfNav = 1u << 2, kSfMech = 1u << 3, kSfEct = 1u << 4, kSfBlk = 1u << 5, kSfStopPre = 1u << 8,
                   kSfSac = 1u << 10, kSfOverflow = 1u << 11;
constexpr uint32_t kSfDone = kSfNav | kSfMech | kSfEct | kSfBlk;   // end the episode
// P-wave bits of a step (kPb*), per ship: the predicates of the post-step position
constexpr uint32_t kPbTerrain = 1u << 0, kPbIw = 1u << 1, kPbArrive = 1u << 2, kPbHorizon = 1u << 3,
                   kPbColl = 1u << 4;   // kPbColl: the ship-ship collision, in the test ship's word (P0)
// the episode ends: test ship arrival / horizon / terrain; obstacle horizon / terrain / IW; collision
constexpr uint32_t kPbDoneTest = kPbArrive | kPbHorizon | kPbTerrain | kPbColl, kPbDoneObs = kPbHorizon | kPbTerrain | kPbIw;
// the step's policy-mode decision (SyncSlot::q): the env steps / it waits for its action
constexpr int32_t kQLive = -1, kQStalled = -2;

template <typename T>
struct SyncSlot {             // one step of the envs of a group (ring of 2)
  T pn[2][kWave], pe[2][kWave];   // post-step position per ship (D, before A)
  T iwn[kWave], iwe[kWave];       // the obstacle's IW of the step (D1, before A)
  T ang[kWave];                   // the route angle of the step's sampling event (D1, before A)
  int32_t q[kWave];               // policy mode: kQLive / kQStalled / request slot (D1, before A)
  T t[6][kWave];              // test ship: n, e, psi, rpm, |e_ct|, P_me (D0, before B)
  T o[5][kWave];              // obstacle: n, e, psi, |e_ct|, SAC action (D1, before B)
  uint32_t f[2][kWave];       // kSf* flags per ship (D, before B)
  int32_t ep[kWave];          // episode step before the step (D1)
  uint32_t pb[2][kWave];      // kPb* bits per ship (P, before B)
  T r_nto[kWave], r_o[kWave]; // P1 after B: the obstacle's reward terms
  uint32_t bo[kWave];         // P1 after B: the obstacle's status bits | stop | done
};
template <typename T>
struct SyncShared {
  SyncSlot<T> d[2];
};

// P0's replay-transition ring (records of sampling events, SIT_TRANSITION_DIM reals each): buffered
// in LDS and appended to the caller's buffer by one atomic per flush.  (One atomic per step with
// events made P0 wait for the slot on its critical segment — and, gfx9 counting stores in vmcnt,
// for the reward / done / status stores issued just before it: C3 paid 4.8 % for the stream; the ring
// measured C3 +2.3 %.)  Synthetic-sampler launches only: policy launches are 64 steps long, and the
// ring's last flush put an atomic round trip before their serving barrier (C5 -2.7 %); they append
// per step (kTrRing 0).
template <int MODE>
constexpr int kTrRing = MODE == kSynth ? 64 : 0;
template <typename T, int MODE>
__host__ __device__ constexpr size_t sync_ring_bytes() {
  return ((size_t)kTrRing<MODE> * SIT_TRANSITION_DIM * sizeof(T) + 255) & ~size_t(255);
}
// the sync kernel's dynamic LDS: [staged map | exchange slots | transition ring]
template <typename T, int MODE>
__host__ __device__ constexpr size_t sync_lds_bytes(size_t map_bytes) {
  return ((map_bytes + 255) & ~size_t(255)) + ((sizeof(SyncShared<T>) + 255) & ~size_t(255)) + sync_ring_bytes<T, MODE>();
}

#include "sit_serve.h"   // in-kernel serving (its LDS layout follows the exchange slots')

// ------------------------------------------------------------------------------------------
// D waves
// ------------------------------------------------------------------------------------------
template <typename T, int MODE, int TYPE, int MACH>
__device__ __forceinline__ void sync_d(const KArgs<T>& a, const Consts<T>& cs, SyncShared<T>& X, ServePub* pub, int env,
                                      bool act) {
#if SIT_SYNC_CREF
  const Consts<T>& c = cs;
#else
  const Consts<T> c = cs;
#endif
  // (a register copy of the guidance / control / dynamics constants measured 1.8 % slower at C3: 221
  // instead of 174 VGPRs, more SGPR spills; the LDS reads are off the critical chain)
  const Consts<T>& hc = cs;
  const int lane = threadIdx.x & (kWave - 1);
  const int n_env = a.n_env;
  const int sid = TYPE * n_env + env;
  const int n = a.io.n_steps;
  SY_INIT();

  Ship<T> s{};
  Route<T> rt{};
  T v_des = T(0);
  T samp = T(0), eps = T(0), ppn = T(0), ppe = T(0), iwn = T(0), iwe = T(0);
  T samp_lo = T(0), ppn_lo = T(0), ppe_lo = T(0);   // float32: low parts (comp_add)
  int ep_step = 0;
  uint32_t event = 0, episodes = 0;
  double ab_len = 0.0, ab_alpha = 0.0, samp_limit = 0.0;
  // policy mode: the env's action slot (D1), and whether the env stopped for the policy
  bool ready = false, stalled = false;
  T pa = T(0);
  int32_t age0 = 0;              // policy mode (D1): admission rounds waited (publish_ages)
  // D1: the next sampling event's action and IW direction, drawn ahead (after the dynamics of the
  // step that consumed the previous one, or in the prologue) so that the event itself, on the
  // critical segment before barrier A, costs two multiply-adds
  double nx_act = 0.0;
  T nx_cs = T(0), nx_sn = T(0);
  // explicit mode (D1): the caller's inputs of the next step, loaded one step ahead (the first step's
  // with the prologue's loads), so no global load sits on the segment before barrier A
  bool x_sac = false, x_init = false;
  T x_an = T(0), x_ae = T(0);
  auto load_inputs = [&](int step) {
    const size_t row = (size_t)step * n_env + env;
    x_sac = a.io.sac_update[row] != 0;
    x_init = a.io.init[row] != 0;
    x_an = a.io.action_ne[2 * row];
    x_ae = a.io.action_ne[2 * row + 1];
  };
  if (act) {
    ep_step = a.st.ep_step[env];
    load_ship(a.st, sid, s);
    rt.nw = a.st.nw[sid];
    rt.end_n = a.sc.end_n[sid];
    rt.end_e = a.sc.end_e[sid];
    v_des = init_val(a.sc, TYPE, SIT_INIT_DESIRED_SPEED, env, n_env);
    rt.tn = a.st.wn + (size_t)TYPE * a.cap * n_env + env;
    rt.te = a.st.we + (size_t)TYPE * a.cap * n_env + env;
    rt.stride = n_env;
    rt.cap = a.cap;
    rt.load_leg(s.k);
    if (TYPE == 1) {
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
      samp_limit = ieee_mul(ab_len, cs.x.theta);   // MSRL_env_ex.py:569
      if (MODE == kPolicy) {
        ready = a.io.policy_ready[env] == SIT_POLICY_READY;
        pa = a.io.policy_action[env];
        age0 = a.io.request_age ? a.io.request_age[env] : 0;   // (NULL when the launch serves in-kernel)
      }
    }
  }
  // the next event's draw: mode-0 action U[-1, 1] (uniform_policy.py:20-22) from the sampler, or the
  // policy's squashed action in [-1, 1]; the route angle is the action scaled by pi / 6
  auto draw_next = [&]() {
#if defined(SIT_ABL_CHEAPDRAW)   // timing ablation (results wrong): a hash draw instead of Philox
    const uint32_t hh = (uint32_t)(env * 2654435761u) ^ (event * 0x9E3779B9u);
    nx_act = MODE == kPolicy ? (double)pa : (double)(hh >> 8) * (2.0 / 16777216.0) - 1.0;
#else
    nx_act = MODE == kPolicy ? (double)pa
                             : sampler_uniform(opaque_seed(a.io.seed), (uint64_t)(a.io.env_id_offset + env), event) * 2.0 - 1.0;
#endif
#if defined(SIT_ABL_NOTRIG)      // timing ablation (results wrong): no sincos of the IW direction
    nx_cs = (T)(0.5 + 0.1 * nx_act); nx_sn = (T)(0.5 - 0.1 * nx_act);
#else
    iw_dir(ab_alpha, nx_act * (M_PI / 6.0), nx_cs, nx_sn);
#endif
  };
  if (TYPE == 1 && act && (MODE == kSynth || (MODE == kPolicy && ready))) draw_next();
  if (MODE == kExplicit && TYPE == 1 && act && n > 0) load_inputs(0);
  T p0[6] = {}, p0lo[6] = {};
  int nw0 = 0;
  typename Route<T>::Leg leg0{};
  const bool auto_reset = __builtin_amdgcn_readfirstlane(a.io.auto_reset) != 0;
  if (act && auto_reset) {   // the episode start the auto reset restores (not loaded without it)
    for (int j = 0; j < 6; ++j) p0[j] = init_val(a.sc, TYPE, SIT_INIT_NORTH + j, env, n_env);
    for (int j = 0; j < 6; ++j) p0lo[j] = init_lo(a.sc, TYPE, SIT_INIT_NORTH + j, env, n_env);
    nw0 = a.sc.nw0[sid];
    Route<T> r0 = rt;
    r0.nw = nw0;
    r0.load_leg(1);
    leg0 = r0.leg();
  }
  uint32_t uf = __builtin_amdgcn_readfirstlane((c.collision_bias ? kUfCollBias : 0u) |
                                               (c.sg_mode != SIT_SG_MOTOR ? kUfBlackout : 0u) |
                                               (auto_reset ? kUfAutoReset : 0u));
  // sine and cosine of the heading the next step starts from, taken where the heading is set (after
  // the dynamics, which end before barrier B, where the D wave usually waits for the P wave; after an
  // auto reset): the segment from B to A, on the step's critical path, then needs only the Euler
  // position (its four multiply-adds) before publishing it
  T sp_n = T(0), cp_n = T(1);
  if (act) xsincos(s.psi, &sp_n, &cp_n);

  SY_MARK(12);   // prologue
  for (int it = 0; it < n; ++it) {
    asm volatile("" : "+s"(uf));
    SyncSlot<T>& xd = X.d[it & 1];
    const T sp = sp_n, cp = cp_n;
    T n1 = s.n, e1 = s.e, ln1 = s.ln, le1 = s.le;
    bool sac = false, init_x = false;
    double ang = 0.0, act_n = 0.0;
    if (act && !stalled) {
      if (TYPE == 0 || !s.stop) euler_position(c, s, sp, cp, n1, e1, ln1, le1);
      SY_MARK(10);
      if (TYPE == 1 && MODE == kExplicit) {
        // the caller's converted_action, SAC_update and init of this step (MultiShipRLEnv.step)
        sac = x_sac;
        init_x = x_init;
        iwn = x_an;
        iwe = x_ae;
        if (it + 1 < n) load_inputs(it + 1);
        xd.iwn[lane] = iwn; xd.iwe[lane] = iwe;
        xd.ang[lane] = angle_or_nan(false, T(0));   // no device draw
      } else if (TYPE == 1) {
        // a sampling event: the episode's first step, or the sampling distance reaching AB_len while
        // the obstacle ship runs (test_beds/main_ast.py:337-349 with the SURVEY 8(d) converter)
        sac = ep_step == 0 || (comp_val(samp, samp_lo) >= ab_len && !s.stop);
        int32_t q = kQLive;
        if (MODE == kPolicy && sac && !ready) {
          // no action yet: the env waits for the policy for the rest of the launch (the admission
          // kernel after the launch queues its request, k_policy_admit)
          stalled = true;
          sac = false;
          q = kQStalled;
        } else if (sac) {                 // the action drawn ahead (draw_next)
          act_n = nx_act;
          if (MODE == kPolicy) ready = false;
          ang = act_n * (M_PI / 6.0);
          iw_at(s.n, s.e, ab_len, nx_cs, nx_sn, iwn, iwe);
          ++event;
        }
        if (MODE == kPolicy) xd.q[lane] = q;
        xd.iwn[lane] = iwn; xd.iwe[lane] = iwe;
        xd.ang[lane] = angle_or_nan(sac, (T)ang);
      }
      xd.pn[TYPE][lane] = n1; xd.pe[TYPE][lane] = e1;
    } else if (MODE == kPolicy && TYPE == 1 && act) {
      xd.q[lane] = kQStalled;
    }
    SY_MARK(0);
#ifndef SIT_ABL_NO_A   // timing ablation (diagnostic builds only, results wrong): no barrier A
    __syncthreads();   // A: positions (and the IW, and in policy mode the step's decision) published
#endif
    SY_MARK(1);
    if (MODE == kPolicy && TYPE == 0 && act && !stalled) stalled = xd.q[lane] != kQLive;
    if (act && !stalled) {
      T o_rpm, o_ect, o_pme = T(0);
      bool ect_over = false;
      uint32_t fl = s.stop ? kSfStopPre : 0u;
      if (TYPE == 1) {
        const bool init_f = MODE == kExplicit ? init_x : ep_step == 0;
        if (sac) fl |= kSfSac;
        if (s.stop) {                    // obs_step (MSRL_Env.py:287-402): stop path (Q10)
          s.ticks += 2;
          o_rpm = s.lrpm; o_ect = s.lect; o_pme = s.lpme;
          ect_over = (double)o_ect > cs.x.e_tol;
        } else {
          if (sac) {                     // update_route: insert at index -1 (Q16)
            if (!rt.insert(iwn, iwe, s.k, a.cap)) fl |= kSfOverflow;
            samp = T(0);
            samp_lo = T(0);
          }
          const T pre_n = s.n, pre_e = s.e, pre_ln = s.ln, pre_le = s.le;
          const DynBase<T> db = dyn_base<T, MACH>(hc, s, sp, cp);   // independent of guidance: fills its latency
          T rudder, thr, psi_ref;
#ifdef SIT_ABL_DG   // timing ablation (diagnostic builds only): no guidance / control
          rudder = T(0); thr = T(0.5); o_ect = T(0); psi_ref = T(0);
#else
          guidance_control<T, MACH>(hc, cs.x, s, rt, v_des, rudder, thr, o_ect, psi_ref, ect_over);
#endif
          SY_MARK(8);
          o_rpm = s.w * c.rpm_k;
          o_pme = power_me_kw(c, thr);
          s.lrpm = o_rpm; s.lect = o_ect; s.lpme = o_pme;
#ifdef SIT_ABL_DK   // timing ablation: no machinery / kinetics (the position still moves)
          s.n = n1; s.e = e1; s.psi = s.psi + T(1e-3) * rudder;
#else
          dyn_finish<T, MACH>(hc, s, db, thr, rudder, n1, e1, ln1, le1);
#endif
          xsincos(s.psi, &sp_n, &cp_n);
          SY_MARK(9);
          if (!init_f) {
            const T dn = comp_diff(pre_n, pre_ln, ppn, ppn_lo), de = comp_diff(pre_e, pre_le, ppe, ppe_lo);
            const T d = xsqrt(dn * dn + de * de);
            eps = eps + d;
            samp = comp_add(samp, samp_lo, d);
          }
          ppn = pre_n; ppe = pre_e; ppn_lo = pre_ln; ppe_lo = pre_le;
          s.ticks += 1;
        }
        SY_MARK(6);
        // is_obs_ship_navigation_failure (MSRL_env_ex.py:566-576); arrival and the map horizon are
        // the P wave's (a function of the position)
        const bool nav = ect_over || comp_val(samp, samp_lo) > samp_limit;
        fl |= nav ? kSfNav : 0u;
        xd.o[0][lane] = s.n; xd.o[1][lane] = s.e; xd.o[2][lane] = s.psi; xd.o[3][lane] = o_ect;
        xd.o[4][lane] = MODE == kExplicit ? angle_or_nan(false, T(0)) : (T)act_n;
        xd.f[1][lane] = fl;
        xd.ep[lane] = ep_step;
        SY_MARK(7);
        if (MODE == kSynth && sac) draw_next();   // the next event's action (its counter is event)
        SY_MARK(14);
      } else {
        // test_step (MSRL_Env.py:219-285)
        T rudder, thr, psi_ref;
        const T i1_0 = s.i1, i2_0 = s.i2, li1_0 = s.li1, li2_0 = s.li2;
        const DynBase<T> db = dyn_base<T, MACH>(hc, s, sp, cp);
#ifdef SIT_ABL_DG
        rudder = T(0); thr = T(0.5); o_ect = T(0); psi_ref = T(0);
#else
        guidance_control<T, MACH>(hc, cs.x, s, rt, v_des, rudder, thr, o_ect, psi_ref, ect_over);
#endif
        SY_MARK(8);
        if (uf & kUfCollBias) {          // is_collision_imminent() on all-zero states (Q1)
          thr = xclip(thr * c.bias_scale, T(0), c.bias_max);
          rudder = xclip(rudder + c.bias_rudder, -c.rudder_max, c.rudder_max);
        }
        o_rpm = s.w * c.rpm_k;
        o_pme = power_me_kw(c, thr);
        const bool mech = rpm_fails<T, MACH>(c, cs.x, s.w, o_rpm);
        bool blk = false;
        if (uf & kUfBlackout) {
          blk = o_pme > c.blackout_kw;
          if (!kIsF32<T> || xabs(o_pme - c.blackout_kw) <= T(1e-4) * (xabs(o_pme) + T(1)))
            blk = power_me_kw_exact(c.sg_mode, cs.x, throttle_exact(cs.x, s.u, v_des, comp_val(i1_0, li1_0),
                                                                    comp_val(i2_0, li2_0), c.collision_bias != 0,
                                                                    MACH == 1))
                  > cs.x.blackout;
        }
        s.lrpm = o_rpm; s.lect = o_ect; s.lpme = o_pme;
#ifdef SIT_ABL_DK
        s.n = n1; s.e = e1; s.psi = s.psi + T(1e-3) * rudder;
#else
        dyn_finish<T, MACH>(hc, s, db, thr, rudder, n1, e1, ln1, le1);
#endif
        xsincos(s.psi, &sp_n, &cp_n);
        SY_MARK(9);
        s.ticks += 1;
        fl |= (mech ? kSfMech : 0u) | (ect_over ? kSfEct : 0u) | (blk ? kSfBlk : 0u);
        xd.t[0][lane] = s.n; xd.t[1][lane] = s.e; xd.t[2][lane] = s.psi;
        xd.t[3][lane] = o_rpm; xd.t[4][lane] = o_ect; xd.t[5][lane] = o_pme;
        xd.f[0][lane] = fl;
      }
    }
    SY_MARK(2);
    __syncthreads();   // B: both ships' step and their map predicates
    SY_MARK(3);
#ifdef SIT_PRIO_D1_B   // (experiment) D1's priority from barrier B to barrier A
    if (TYPE == 1) __builtin_amdgcn_s_setprio(SIT_PRIO_D1_B);
#endif
    // the episode's end (every predicate, the collision) and the auto reset (main_ast.py:314-333)
    if (act && !stalled) {
      const uint32_t pb0 = xd.pb[0][lane], pb1 = xd.pb[1][lane];
      const bool env_done = ((xd.f[0][lane] | xd.f[1][lane]) & kSfDone) || (pb0 & kPbDoneTest) || (pb1 & kPbDoneObs);
      // the stop flags (MSRL_env_ex.py:742-899): the test ship stops with any of its predicates, the
      // obstacle at arrival, the map horizon, an IW terminal (Q11) and navigation failure, not at the
      // terrain (Q12); both at a collision.  (A test-ship predicate ends the episode: reset below.)
      if (TYPE == 0) { if ((xd.f[0][lane] & kSfDone) || (pb0 & kPbDoneTest)) s.stop = 1; }
      else if ((xd.f[1][lane] & kSfNav) || (pb1 & (kPbArrive | kPbHorizon | kPbIw)) || (pb0 & kPbColl)) s.stop = 1;
      rt.fixup(s.k);
      ep_step += 1;
      SY_MARK(11);
      if ((uf & kUfAutoReset) && env_done) {
        // reset() (MSRL_Env.py:147-188; shaft speed and every PI/PID integrator persist, Q6) + init_step()
        s.n = p0[0]; s.e = p0[1]; s.psi = p0[2]; s.u = p0[3]; s.v = p0[4]; s.r = p0[5];
        s.ln = p0lo[0]; s.le = p0lo[1]; s.lpsi = p0lo[2]; s.lu = p0lo[3]; s.lv = p0lo[4]; s.lr = p0lo[5];
        s.ect_int = T(0); s.lei = T(0); s.k = 1; s.ticks = 0; s.stop = 0;
        rt.nw = nw0;
        rt.set_leg(leg0);
        ep_step = 0;
        if (TYPE == 1) { samp = T(0); eps = T(0); samp_lo = T(0); ++episodes; }
        init_step_ship(c, cs.x, s, rt, v_des);
        xsincos(s.psi, &sp_n, &cp_n);
      }
    }
    SY_MARK(4);
    SY_STEP();
#ifdef SIT_PRIO_D1_B
    if (TYPE == 1) __builtin_amdgcn_s_setprio(SIT_PRIO_D1);
#endif
  }
  __syncthreads();   // C: P1's reward terms of the last step (P0 writes that step's outputs)
  if (act) {
    store_ship(a.st, sid, s);
    a.st.nw[sid] = rt.nw;
    if (TYPE == 1) {
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
      // (served in this launch's epilogue: the waiting env's action is ready for the next launch)
      if (MODE == kPolicy)
        a.io.policy_ready[env] = (ready || (stalled && pub)) ? SIT_POLICY_READY : (stalled ? SIT_POLICY_WAITING : 0);
    }
  }
  static_assert(kSyncLanes == kAdmitGroup || MODE != kPolicy, "one wave = one admission group");
  if (MODE == kPolicy && TYPE == 1) {
    if (pub) {   // in-kernel serving: the waiting envs' ids and their events' normal draws, in lane order
      const bool w = act && stalled;
      const unsigned long long m = __ballot(w);
      if (w) {
        const int r = (int)__popcll(m & ((1ull << lane) - 1ull));
        pub->env[r] = env;
        pub->noise[r] = (float)(T)sampler_normal(a.io.seed, (uint64_t)(a.io.env_id_offset + env), event);
      }
      if (lane == 0) pub->count = (int32_t)__popcll(m);
    } else {
      publish_ages(a.io.request_age, a.io.group_counts, env, act, stalled, age0);
    }
  }
  SY_MARK(13);   // epilogue (the wait at barrier C, the state write-back)
  SY_FLUSH(TYPE);
}

// ------------------------------------------------------------------------------------------
// P waves
// ------------------------------------------------------------------------------------------
template <typename T, int MODE, int TYPE, bool LDSMAP>
__device__ __forceinline__ void sync_p(const KArgs<T>& a, const Consts<T>& cs, const Map<T>& map_in,
                                      SyncShared<T>& X, ServePub* pub, T* ring, int env, bool act) {
  const Consts<T> c = cs;   // a register copy (reading the LDS copy where used measured 11 % slower)
  Map<T> map = map_in;
  const int lane = threadIdx.x & (kWave - 1);
  const int n_env = a.n_env;
  const int n = a.io.n_steps;
  SY_INIT();
  // P1: the IW test's cache (the IW changes at sampling events).  Single-step launches (the map read
  // through the caches, LDSMAP false) carry it across launches in the state (iw_key_*): there the
  // test's chain of dependent map reads is the step's longest path, and the drop-in's caller passes
  // the same IW until its next sampling event.  (Fused launches keep it in registers only: carrying
  // it cost C3 1.4 %, a load, a store and three more SGPR spills.)
  T iw_tn = T(0), iw_te = T(0);
  bool iw_valid = false, iw_in = false;
  if (!LDSMAP && TYPE == 1 && act) {
    const uint32_t f = a.st.iwk_flags[env];
    iw_tn = a.st.iwk[0][env]; iw_te = a.st.iwk[1][env];
    iw_valid = (f & kIwkValid) != 0;
    iw_in = (f & kIwkInside) != 0;
  }
  T lo[SIT_OBS_DIM] = {};           // P0: the observation before the step (replay transition)
  // P0: the episode's initial observation, held in registers: a load of it inside the loop left a
  // global load pending on lo's registers, and the next step's LDS reads into them waited for every
  // outstanding memory operation (s_waitcnt vmcnt(0)), the step's output stores included (~1 000 cycles)
  T li[SIT_OBS_DIM] = {};
  const bool auto_reset = __builtin_amdgcn_readfirstlane(a.io.auto_reset) != 0;
  if (TYPE == 0 && act)
    for (int j = 0; j < SIT_OBS_DIM; ++j) {
      lo[j] = a.st.last_obs[(size_t)j * n_env + env];
      if (auto_reset) li[j] = a.sc.initial_state[(size_t)env * SIT_OBS_DIM + j];
    }
  // (drained here, so that no load is pending on li's registers when the loop first reads them)
  __builtin_amdgcn_s_waitcnt(0);
  T r_nt_t = T(0), r_term_t = T(0); // P0: the test ship's reward terms and bits of the last step
  uint32_t bits_t = 0;
  bool coll_t = false;              // P0: the last step's ship-ship collision
  T dobst = T(0);
  uint32_t pbits = 0;               // this step's kPb* predicates of the ship's post-step position
  bool stalled = false;             // policy mode: the env stopped for the policy in this launch
  uint32_t n_stepped = 0;           // policy mode (P0): env-steps executed
  // the ship's final waypoint (the arrival predicate, MSRL_env_ex.py:750-754, 825-829)
  const T end_n = act ? a.sc.end_n[TYPE * n_env + env] : T(0), end_e = act ? a.sc.end_e[TYPE * n_env + env] : T(0);
  uint32_t uf = __builtin_amdgcn_readfirstlane((a.io.next_state ? 1u : 0u) | (a.io.reward ? 2u : 0u) |
                                               (a.io.done ? 4u : 0u) | (a.io.status ? 8u : 0u) |
                                               (a.io.action_out ? 16u : 0u) | (a.io.transitions ? kUfTrans : 0u) |
                                               (a.io.done_count ? kUfDoneCnt : 0u) |
                                               (a.io.mask_horizon > 0 ? kUfMaskH : 0u) |
                                               (auto_reset ? kUfAutoReset : 0u));
  // this ship's next_state columns (P0: 0-5, P1: 6-9) and, P1, the IW action row, one row block per step
  T* p_ns = (uf & 1) ? a.io.next_state + (size_t)env * SIT_OBS_DIM + (TYPE == 0 ? 0 : 6) : nullptr;
  T* p_ao = (TYPE == 1 && (uf & 16)) ? a.io.action_out + (size_t)env * 4 : nullptr;
  const size_t row_step = (size_t)n_env;

  // P0's output rows, one row per step: per-lane pointers advanced by n_env (kernel-argument pointers
  // reloaded inside the loop cost a scalar load and its wait per store)
  T* p_rw = (TYPE == 0 && (uf & 2)) ? a.io.reward + env : nullptr;
  uint8_t* p_dn = (TYPE == 0 && (uf & 4)) ? a.io.done + env : nullptr;
  uint32_t* p_st = (TYPE == 0 && (uf & 8)) ? a.io.status + env : nullptr;
  int* p_dc = (TYPE == 0 && (uf & kUfDoneCnt)) ? a.io.done_count : nullptr;

  SY_MARK(12);   // prologue
  // P0: the transition ring's records appended to the caller's buffer (one atomic for all of them;
  // records past transition_capacity are counted, not written)
  constexpr int kRing = kTrRing<MODE>;
  int ring_n = 0;                   // records in the ring (wave-uniform)
  auto flush = [&]() {
    if (ring_n == 0) return;
    int base = 0;
    if (lane == 0) base = atomicAdd(a.io.transition_count, ring_n);
    base = __shfl(base, 0);
    const int tcap = a.io.transition_capacity;
    for (int i = lane; i < ring_n * (SIT_TRANSITION_DIM / 4); i += kWave) {
      const int r = i / (SIT_TRANSITION_DIM / 4), q = i - r * (SIT_TRANSITION_DIM / 4);
      const T* src = ring + (size_t)r * SIT_TRANSITION_DIM + 4 * q;
      if (base + r < tcap) store4(a.io.transitions + (size_t)(base + r) * SIT_TRANSITION_DIM + 4 * q, src[0], src[1], src[2], src[3]);
    }
    ring_n = 0;
  };
  // P0: reward, done, status, replay transition and done count of step j (MSRL_env_ex.py:906-980);
  // called once per step, in order
  auto outputs = [&](int j) {
    const SyncSlot<T>& xd = X.d[j & 1];
    bool env_done = false;
    bool live = act;
    if (MODE == kPolicy && act) {
      const int32_t q = xd.q[lane];
      live = q == kQLive;
      if (!live) {                     // no step in this row: the env waits for its action
        if (uf & 8) out1<T>(p_st, (uint32_t)SIT_ST_NO_STEP);
        if (uf & 4) out1<T>(p_dn, (uint8_t)0);
      } else {
        ++n_stepped;
      }
    }
    // (outside the live branch: the transition ring is driven with every lane active — its flush
    // copies by all 64 lanes and lane 0 takes the slots)
    T nt[6], no[4];
    T reward = T(0);
    bool sac = false;
    if (live) {
      // every LDS value of the step read up front (one wait; the empty asm keeps the reads out of
      // the branches below)
      for (int q = 0; q < 6; ++q) nt[q] = xd.t[q][lane];
      for (int q = 0; q < 4; ++q) no[q] = xd.o[q][lane];
      const uint32_t bo = xd.bo[lane], f1 = xd.f[1][lane];
      const T r_nto = xd.r_nto[lane], r_o = xd.r_o[lane];
      asm volatile("" :: "v"(nt[0]), "v"(nt[1]), "v"(no[0]), "v"(no[1]), "v"(bo), "v"(f1), "v"(r_nto), "v"(r_o));
      const bool coll = coll_t;
      env_done = (bits_t & SIT_ST_TEST_DONE) || (bo & kDoneBit) || coll;
      const T dn = nt[0] - no[0], de = nt[1] - no[1];
      const T snt = (T(1) - xsqrt(dn * dn + de * de) * c.inv_maxn) * T(0.001);
      const T r_snt = (bo & kStopBit) ? T(0) : snt;
      const T rs = coll ? T(2000) : T(0);
      reward = r_nt_t + r_term_t + r_nto + r_o + r_snt + rs;
      const uint32_t status = ((bits_t | bo) & ~(kStopBit | kDoneBit)) | (coll ? SIT_ST_COLLISION : 0u);
      if (uf & 2) out1<T>(p_rw, reward);
      if (uf & 4) out1<T>(p_dn, (uint8_t)(env_done ? 1 : 0));
      if (uf & 8) out1<T>(p_st, status);
      sac = (f1 & kSfSac) != 0;
    }
    SY_MARK(6);
    if (uf & kUfTrans) {               // replay transition of a sampling event (main_ast.py:385-396)
      const unsigned long long m = __ballot(sac);
      if (m) {
        const int nn = (int)__popcll(m), rank = (int)__popcll(m & ((1ull << lane) - 1ull));
        if (kRing > 0 && ring_n + nn > kRing) flush();
        T* rec = nullptr;
        if (kRing > 0 && nn <= kRing) {  // into the ring
          if (sac) rec = ring + (size_t)(ring_n + rank) * SIT_TRANSITION_DIM;
          ring_n += nn;
        } else {                         // a burst larger than the ring: appended directly
          int base = 0;
          if (lane == 0) base = atomicAdd(a.io.transition_count, nn);
          base = __shfl(base, 0);
          if (sac && base + rank < a.io.transition_capacity)
            rec = a.io.transitions + (size_t)(base + rank) * SIT_TRANSITION_DIM;
        }
        if (rec) {
          // the 24-real record (include/sit.h) as six 4-real stores (a record starts 4-real aligned)
          const bool horizon_hit = (uf & kUfMaskH) && xd.ep[lane] + 2 == a.io.mask_horizon;
          const T mask = (horizon_hit || !env_done) ? T(1) : T(0);
          store4(rec, lo[0], lo[1], lo[2], lo[3]);
          store4(rec + 4, lo[4], lo[5], lo[6], lo[7]);
          store4(rec + 8, lo[8], lo[9], xd.o[4][lane], reward);
          store4(rec + 12, nt[0], nt[1], nt[2], nt[3]);
          store4(rec + 16, nt[4], nt[5], no[0], no[1]);
          store4(rec + 20, no[2], no[3], mask, (T)(a.io.env_id_offset + env));
        }
      }
    }
    // (the observation before the next step: every step when transitions or policy requests read
    // it, else only at the last step, for last_obs)
    if (live && (MODE == kPolicy || (uf & kUfTrans) || j == n - 1)) {
      const bool restart = (uf & kUfAutoReset) && env_done;   // the auto reset's initial observation
      for (int q = 0; q < 6; ++q) lo[q] = restart ? li[q] : nt[q];
      for (int q = 0; q < 4; ++q) lo[6 + q] = restart ? li[6 + q] : no[q];
    }
    if (uf & kUfDoneCnt) {
      const unsigned long long m = __ballot(env_done);
      if (lane == 0 && m) atomicAdd(p_dc, (int)__popcll(m));
    }
    p_rw += row_step; p_dn += row_step; p_st += row_step; ++p_dc;
  };

  for (int it = 0; it < n; ++it) {
    asm volatile("" : "+s"(uf));
    asm volatile("" : "+s"(map.use_index), "+s"(map.use_cells), "+s"(map.n_edge), "+s"(map.n_poly));
    SyncSlot<T>& xd = X.d[it & 1];
    SY_MARK(0);
#ifndef SIT_ABL_NO_A
    __syncthreads();   // A: this step's positions
#endif
    SY_MARK(1);
#ifndef SIT_ABL_PO   // timing ablation: P0 writes no outputs
    if (TYPE == 0 && it >= 1) outputs(it - 1);
#endif
    SY_MARK(7);
    if (MODE == kPolicy && act && !stalled) stalled = xd.q[lane] != kQLive;
    // the predicates of the post-step position (MSRL_env_ex.py:460-603, 628-881): the map's (boundary
    // distance, hull in terrain, the IW test), arrival within 200 m of the final waypoint, the map
    // horizon, and (P0) the ship-ship collision.  (Reading the cell record and first edges before
    // P0's outputs, to overlap their latency, measured 3 % slower.)
#ifdef SIT_ABL_PP   // timing ablation: no position predicates
    if (act && !stalled) xd.pb[TYPE][lane] = 0u;
    if (false) {
#else
    if (act && !stalled) {
#endif
      const T sn = xd.pn[TYPE][lane], se = xd.pe[TYPE][lane];
      DistPf<T> pf;
      pf_cell(c, map, sn, se, pf);
      pf_edges(map, pf);
      SY_MARK(8);
      dobst = pf_finish(map, pf, sn, se);
      SY_MARK(9);
      const bool terrain = hull_in_terrain_cls(c, map, sn, se, dobst, pf.cls, pf.cell_f, pf.word_f);
      SY_MARK(10);
      pbits = (terrain ? kPbTerrain : 0u) | (within_radius(sn, se, end_n, end_e, c.arrive_d2_le) ? kPbArrive : 0u) |
              (outside(c, sn, se, c.half_len) ? kPbHorizon : 0u);
      if (TYPE == 1) {
        const T wn = xd.iwn[lane], we = xd.iwe[lane];
        if (!iw_valid || wn != iw_tn || we != iw_te) {
          iw_in = pip_point(c, map, wn, we);
          iw_tn = wn; iw_te = we; iw_valid = true;
        }
        if (outside(c, wn, we, T(0)) || iw_in) pbits |= kPbIw;   // Q11
        SY_MARK(11);
      } else {
        coll_t = closer_than(sn, se, xd.pn[1][lane], xd.pe[1][lane], c.coll_d2);   // MSRL_env_ex.py:584-603
        if (coll_t) pbits |= kPbColl;
      }
      xd.pb[TYPE][lane] = pbits;
    }
    SY_MARK(2);
    __syncthreads();   // B: the D waves' step results
    SY_MARK(3);
#ifdef SIT_PRIO_P1_B   // (experiment) P1's priority from barrier B to barrier A
    if (TYPE == 1) __builtin_amdgcn_s_setprio(SIT_PRIO_P1_B);
#endif
    if (act && !stalled) {
      const uint32_t fl = xd.f[TYPE][lane];
      int stop = (fl & kSfStopPre) ? 1 : 0;
      bool done = false;
      T r_nt = T(0), r_term = T(0);
      uint32_t bits = 0;
      const bool terrain = (pbits & kPbTerrain) != 0;
      if (TYPE == 0) {
        const T t4 = xd.t[4][lane];
        if (uf & 1) {                    // next_state columns 0-5 (MSRL_Env.py:426-437)
          out2(p_ns, xd.t[0][lane], xd.t[1][lane]); out2(p_ns + 2, xd.t[2][lane], xd.t[3][lane]);
          out2(p_ns + 4, t4, xd.t[5][lane]);
        }
        r_nt = xabs(t4) * c.inv_e_tol + (T(1) - dobst * c.inv_maxn) * T(0.01);
        const bool pred[6] = {(pbits & kPbArrive) != 0, (pbits & kPbHorizon) != 0, terrain, (fl & kSfMech) != 0,
                              (fl & kSfEct) != 0, (fl & kSfBlk) != 0};
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
        r_nt_t = r_nt; r_term_t = r_term; bits_t = bits;
      } else {
        const T o3 = xd.o[3][lane];
        if (uf & 1) { out2(p_ns, xd.o[0][lane], xd.o[1][lane]); out2(p_ns + 2, xd.o[2][lane], o3); }
        if (uf & 16) {                   // the IW action row: north, east, route angle, SAC_update
          const bool sac = (fl & kSfSac) != 0;
          out2(p_ao, xd.iwn[lane], xd.iwe[lane]); out2(p_ao + 2, xd.ang[lane], sac ? T(1) : T(0));
        }
        if (!stop)
          r_nt = T(0.1) - xabs(o3) * c.inv_e_tol * T(0.01) - (T(1) - dobst * c.inv_maxn) * T(0.01);
        bits = (fl & kSfOverflow) ? SIT_ST_ROUTE_OVERFLOW : 0u;
        if (pbits & kPbArrive) { stop = 1; bits |= SIT_ST_OBS_ENDPOINT; }
        if (pbits & kPbHorizon) { stop = 1; done = true; bits |= SIT_ST_OBS_HORIZON; }
        if (terrain) {                   // done without stop flag (Q12)
          if (!stop) r_term = r_term - T(1000);
          done = true;
          bits |= SIT_ST_OBS_TERRAIN;
        }
        if (pbits & kPbIw) {
          if (!stop) r_term = r_term - T(1000);
          stop = 1; done = true;
          bits |= SIT_ST_OBS_IW_TERMINAL;
        }
        if (fl & kSfNav) {
          if (!stop) r_term = r_term - T(1000);
          stop = 1; done = true;
          bits |= SIT_ST_OBS_NAVIGATION;
        }
        if (done) bits |= SIT_ST_OBS_DONE;
        xd.r_nto[lane] = r_nt;
        xd.r_o[lane] = r_term;
        xd.bo[lane] = bits | (stop ? kStopBit : 0u) | (done ? kDoneBit : 0u);
      }
    }
    p_ns += row_step * SIT_OBS_DIM;
    p_ao += row_step * 4;
#ifdef SIT_PRIO_P1_B
    if (TYPE == 1) __builtin_amdgcn_s_setprio(SIT_PRIO_P1);
#endif
    SY_MARK(4);
    SY_STEP();
  }
  __syncthreads();   // C
  if (TYPE == 0) {
    if (n >= 1) outputs(n - 1);
    if (kRing > 0 && (uf & kUfTrans)) flush();
    if (act)
      for (int j = 0; j < SIT_OBS_DIM; ++j) a.st.last_obs[(size_t)j * n_env + env] = lo[j];
    if (MODE == kPolicy && pub) {   // in-kernel serving: the observations the waiting envs wait at
      const bool w = act && stalled;
      const unsigned long long m = __ballot(w);
      if (w) {
        const int r = (int)__popcll(m & ((1ull << lane) - 1ull));
        for (int j = 0; j < SIT_OBS_DIM; ++j) pub->obs[r][j] = (float)lo[j];
      }
    }
    if (MODE == kPolicy && a.io.env_steps) {   // env-steps executed: one atomic per wave
      unsigned long long v = act ? n_stepped : 0;
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0 && v) atomicAdd(a.io.env_steps, v);
    }
  }
  if (!LDSMAP && TYPE == 1 && act) {
    a.st.iwk[0][env] = iw_tn; a.st.iwk[1][env] = iw_te;
    a.st.iwk_flags[env] = iw_valid ? (kIwkValid | (iw_in ? kIwkInside : 0u)) : 0u;
  }
  SY_MARK(13);   // epilogue (the wait at barrier C, P0's last outputs and last_obs)
  SY_FLUSH(2 + TYPE);
}

// LDSMAP: the island map staged into LDS per block (fused launches) or read through the caches
// (single-step launches, whose prologue cannot amortise staging 57 KB per block)
// SIT_SYNC_WAVES_PER_EU: the occupancy the kernel's registers are allocated for (waves per SIMD; 0 = the
// compiler's choice).  Three blocks per CU need <= 168 VGPRs and <= 53 KB of LDS per block
#ifndef SIT_SYNC_WAVES_PER_EU
#define SIT_SYNC_WAVES_PER_EU 0
#endif
// SIT_F64_WAVES_PER_EU: the same for the float64 instantiations alone (they live in the strict TU,
// sit_kernels.hip, built with SIT_F32_TU defined; the float32 ones in sit_steps_f32.hip)
#ifndef SIT_F64_WAVES_PER_EU
#define SIT_F64_WAVES_PER_EU 0
#endif
#if SIT_SYNC_WAVES_PER_EU > 0
#define SIT_SYNC_OCC __attribute__((amdgpu_waves_per_eu(SIT_SYNC_WAVES_PER_EU, SIT_SYNC_WAVES_PER_EU)))
#elif SIT_F64_WAVES_PER_EU > 0 && defined(SIT_F32_TU)
#define SIT_SYNC_OCC __attribute__((amdgpu_waves_per_eu(SIT_F64_WAVES_PER_EU, SIT_F64_WAVES_PER_EU)))
#else
#define SIT_SYNC_OCC
#endif
// Roles by SIMD (fused launches): round 3 observed a block's four waves on four different SIMDs and a
// CU holding two blocks (i and i + 256), so fixed roles by wave index left a quarter of the SIMDs with
// two D waves and a quarter with two P waves.  Each wave takes its role from the SIMD it runs on
// (HW_ID), mirrored for the second block of its CU (a per-CU ticket, one atomic per block while the
// map stages), so every SIMD holds one D and one P wave — which the issue priorities above then order.
// Measured C3 +3.3 % with the priorities (without them, round 3: -0.3 %), C5 unchanged.  Single-step
// launches (map through the caches, nothing staged to hide the ticket's round trip behind) keep the
// fixed order.
// Placement independence: the hardware does not guarantee that placement (another kernel on the CU,
// RCCL beside the step at N > 1, a second stream group can change it).  So the role is not the SIMD
// itself but the rank of the wave's (SIMD, wave index) among the block's four (sync_role_of,
// sit_device.h): always a permutation of D0, D1, P0, P1 — every role runs exactly once per block,
// whatever the placement — and equal to the SIMD when the four differ.  Blocks whose waves share a
// SIMD are counted (g_role_fallback, sit_role_fallbacks): results are unaffected, only the priorities'
// pairing.  (The per-CU ticket is shared by concurrent launches; that, too, only affects speed.)
#ifndef SIT_DYN_OFF
#define SIT_DYN_OFF 0
#endif
#if SIT_SIMD_ROLES
__device__ int g_cu_ticket[2048];
__device__ unsigned long long g_role_fallback;   // blocks whose four waves did not sit on four SIMDs
#endif
template <typename T, int MODE, int MACH, bool LDSMAP>
__global__ __launch_bounds__(256) SIT_SYNC_OCC void k_env_steps_sync(const KArgs<T> a) {
  extern __shared__ __align__(16) unsigned char smem_dyn[];
  unsigned char* const smem = smem_dyn + SIT_DYN_OFF;   // (SIT_DYN_OFF: experiment, the LDS layout's offset)
  __shared__ Consts<T> cs;
#ifdef SIT_DIAG_SYNC
  const unsigned long long sy_k0 = __builtin_amdgcn_s_memtime();
#endif
  for (int i = threadIdx.x; i < (int)(sizeof(Consts<T>) / 4); i += blockDim.x)
    reinterpret_cast<uint32_t*>(&cs)[i] = reinterpret_cast<const uint32_t*>(&a.c)[i];
  const Map<T> map = LDSMAP ? stage_map(a, smem) : a.map;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if SIT_SIMD_ROLES
  __shared__ int s_tk;
  __shared__ int s_simd[4];   // the SIMD of each wave of the block (HW_ID[5:4])
  if (LDSMAP) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);     // HW_REG_HW_ID
    const int fk = __builtin_amdgcn_readfirstlane(a.fake_simds);
    if ((threadIdx.x & (kWave - 1)) == 0)
      s_simd[w] = fk ? (((fk >> (2 * w)) ^ (int)blockIdx.x) & 3) : (int)((hw >> 4) & 3);
    if (threadIdx.x == 0) {
      const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);   // HW_REG_XCC_ID
      const unsigned key = ((((xcc & 7) * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15)) & 2047;
      s_tk = atomicAdd(&g_cu_ticket[key], 1) & 1;
    }
  }
#endif
  const int lane = threadIdx.x & (kWave - 1);
  const int env = blockIdx.x * kSyncLanes + lane;
  const bool act = lane < kSyncLanes && env < a.n_env;
  SyncShared<T>& X = *reinterpret_cast<SyncShared<T>*>(smem + (LDSMAP ? (((size_t)a.map_bytes + 255) & ~size_t(255)) : 0));
  __syncthreads();   // constants copied, map staged, SIMDs published
#if SIT_SIMD_ROLES
  int role;
  if (LDSMAP) {
    const int s0 = __builtin_amdgcn_readfirstlane(s_simd[0]), s1 = __builtin_amdgcn_readfirstlane(s_simd[1]);
    const int s2 = __builtin_amdgcn_readfirstlane(s_simd[2]), s3 = __builtin_amdgcn_readfirstlane(s_simd[3]);
    role = __builtin_amdgcn_readfirstlane(
        sync_role_of(s0, s1, s2, s3, w, __builtin_amdgcn_readfirstlane(s_tk), SIT_SIMD_MIRROR));
    if (threadIdx.x == 0 && !sync_simds_distinct(s0, s1, s2, s3)) atomicAdd(&g_role_fallback, 1ull);
  } else {
    role = (blockIdx.x & 1) == 0 ? w : (w ^ 2);
  }
#else
  const int role = (blockIdx.x & 1) == 0 ? w : (w ^ 2);
#endif
#ifdef SIT_DIAG_SYNC   // slot 15: kernel start to the staged map (per launch)
  if (lane == 0) atomicAdd(&g_sit_diag[role >> 1][(role & 1) * 16 + 15], __builtin_amdgcn_s_memtime() - sy_k0);
#endif
#ifdef SIT_DIAG_PLACE
  if (lane == 0 && blockIdx.x * 4 + w < kDiagWaves) {   // which SIMD each role's wave sits on
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);     // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);   // HW_REG_XCC_ID
    unsigned long long* g = g_sit_wave[blockIdx.x * 4 + w];
    g[0] = role; g[1] = blockIdx.x; g[2] = 0; g[3] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
  }
#endif
  // policy mode with in-kernel serving: the published requests after the map and exchange slots
  // (serve_lds_bytes; the host sized the launch's LDS for it)
  ServePub* pub = (MODE == kPolicy && a.io.actor_w)
                      ? reinterpret_cast<ServePub*>(smem + serve_pub_offset<T>(LDSMAP ? (size_t)a.map_bytes : 0))
                      : nullptr;
  // P0's transition ring after the exchange slots
  T* ring = reinterpret_cast<T*>(reinterpret_cast<unsigned char*>(&X) + ((sizeof(SyncShared<T>) + 255) & ~size_t(255)));
  {  // the role's issue priority (s_setprio, SIT_PRIO_*)
    constexpr int prio[4] = {SIT_PRIO_D0, SIT_PRIO_D1, SIT_PRIO_P0, SIT_PRIO_P1};
    if (prio[role] == 1) __builtin_amdgcn_s_setprio(1);
    else if (prio[role] == 2) __builtin_amdgcn_s_setprio(2);
    else if (prio[role] == 3) __builtin_amdgcn_s_setprio(3);
  }
#ifdef SIT_ONLY_ROLE   // diagnostic builds only (register report per role; results wrong): one role's code
  if (SIT_ONLY_ROLE == 0) sync_d<T, MODE, 0, MACH>(a, cs, X, pub, env, act);
  else if (SIT_ONLY_ROLE == 1) sync_d<T, MODE, 1, MACH>(a, cs, X, pub, env, act);
  else if (SIT_ONLY_ROLE == 2) sync_p<T, MODE, 0, LDSMAP>(a, cs, map, X, pub, ring, env, act);
  else sync_p<T, MODE, 1, LDSMAP>(a, cs, map, X, pub, ring, env, act);
  (void)role;
#else
  if (role == 0) sync_d<T, MODE, 0, MACH>(a, cs, X, pub, env, act);
  else if (role == 1) sync_d<T, MODE, 1, MACH>(a, cs, X, pub, env, act);
  else if (role == 2) sync_p<T, MODE, 0, LDSMAP>(a, cs, map, X, pub, ring, env, act);
  else sync_p<T, MODE, 1, LDSMAP>(a, cs, map, X, pub, ring, env, act);
#endif
  if (MODE == kPolicy && pub) {
#ifdef SIT_DIAG_SYNC
    const unsigned long long sy_s0 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();   // D: the block's waiting envs published; the map and exchange slots are dead
#ifdef SIT_DEBUG   // the serving LDS (ServeWork at 0, ServePub after it) inside the launch's dynamic LDS
    if (serve_lds_bytes<T>(LDSMAP ? (size_t)a.map_bytes : 0) > (size_t)a.lds_bytes) {
      if (threadIdx.x == 0) SIT_DCHECK(false, kDbgServeCount);
      return;
    }
#endif
    serve_block<T>(a.io.actor_w, a.io.actor_det != 0, smem, *pub, a.io.policy_action, a.io.actor_served, a.n_env);
#ifdef SIT_ABL_SERVE_REPEAT   // timing ablation (served counts wrong): the serving pass run again, to price one
    for (int rep = 1; rep < SIT_ABL_SERVE_REPEAT; ++rep) {   // more serving round per launch
      __syncthreads();
      serve_block<T>(a.io.actor_w, a.io.actor_det != 0, smem, *pub, a.io.policy_action, nullptr, a.n_env);
    }
#endif
#ifdef SIT_DIAG_SYNC   // slot 14: the wait at barrier D and the serving (per launch)
    if (lane == 0) atomicAdd(&g_sit_diag[role >> 1][(role & 1) * 16 + 14], __builtin_amdgcn_s_memtime() - sy_s0);
#endif
  }
}
