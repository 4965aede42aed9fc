// sit_split.h — the pipelined step kernel of the synthetic-sampler rollout (configs C3/C4): each
// ship's step split over two waves, so C3's 65 536 ships run as 2 048 waves (two per SIMD).
//
// Included from sit_impl.h (inside its anonymous namespace, after k_env_steps).
//
// Why: at C3 the one-wave-per-ship kernel (k_env_steps) holds one wave per SIMD, and a wave alone
// issues a VALU instruction at most every 4 cycles and hides none of its own LDS / memory latency:
// it ran at ~0.18 of the chip's VALU issue rate.  Two waves per SIMD measured 1.42x the per-SIMD
// throughput (tools/occ.sh, n_env = 65 536), and the polygon predicates (boundary distance, hull
// test, IW test) are 47 % of the one-wave step (ablation).  They are functions of a position only.
//
// Roles (one 512-thread block = 2 env groups x 4 waves; group 0 waves 0-3 are D0 D1 P0 P1 and
// group 1's are P0 P1 D0 D1, so each SIMD holds one D and one P wave):
//   D0 / D1  step the ship under test / the obstacle ship (sampler, guidance, control, machinery,
//            kinetics, Euler) and decide every predicate that needs no map: arrival, horizon,
//            mechanical, navigation and blackout failures, ship-ship collision, and run the auto
//            reset (MSRL_Env.py:147-442; MSRL_env_ex.py:554-592, 628-881; main_ast.py:314-333).
//   P0 / P1  one step behind: the map predicates of their ship's position (obstacles_distance,
//            is_pos_inside_obstacles, the obstacle's IW test, MSRL_env_ex.py:490-542, 628-881) and
//            the rewards that depend on them; P0, two steps behind, assembles the env's reward,
//            done and status in the reference's order and writes them with the replay transition.
// Speculation: D computes step j before P has decided step j-1's terrain / IW predicates.  Those
// predicates only ever end the episode (done -> auto reset), so D assumes "no" and, when P says
// "yes" for an env not already reset, restores the state the reset keeps (shaft speed, PI/PID
// integrals, sampler counter), applies reset() + init_step() and recomputes step j (rare: a
// terrain or IW termination).  The results equal the sequential kernel's step for step.
//
// Per iteration two barriers: A (P's predicates of step j-1 are visible to D's redo check) and B
// (D's step j, redone if needed, is visible to D's collision test and to P).  Exchange slots are a
// ring of 4 steps in LDS.  Selected by SIT_STEP_KERNEL=pipelined for the synthetic sampler with
// auto-reset and the LDS map, without the trajectory log.
//
// Measured (C3, MI355X): 1.47e10 env-steps/s against k_env_steps' 1.62e10.  The split adds 21 %
// VALU and 60 % SALU per ship-step (exchange, duplicated collision test, redo checks), redoes 5 %
// of wave-steps, and its waves spend 57 % of their cycles at the two barriers / waitcnt: the
// obstacle D wave stays the critical chain and sharing its SIMD with a P wave stretches it
// (priorities measured no different).  Kept as a tested alternative; k_env_steps is the default.
#pragma once

#ifndef SIT_SPLIT_CREF
#define SIT_SPLIT_CREF 1   // D waves read the constants from LDS (no VGPR spills; +2.5 %)
#endif
constexpr int kSplitRing = 4;
// D-wave flags of a step (kSf*), per ship
constexpr uint32_t kSfArrive = 1u << 0, kSfHorizon = 1u << 1, kSfNav = 1u << 2, kSfMech = 1u << 3,
                   kSfEct = 1u << 4, kSfBlk = 1u << 5, kSfStopPre = 1u << 8, kSfDoneNt = 1u << 9,
                   kSfSac = 1u << 10, kSfOverflow = 1u << 11;
constexpr uint32_t kPbReset = 1u << 28;   // P: terrain / IW terminal ended the episode at this step

template <typename T>
struct SplitDSlot {           // one step's D-wave results for the 64 envs of a group
  T t[6][kWave];              // ship under test: n, e, psi, rpm, |e_ct|, P_me (next_state 0-5)
  T o[7][kWave];              // obstacle: n, e, psi, |e_ct| (next_state 6-9), IW n, IW e, SAC action
  uint32_t f[2][kWave];       // kSf* flags of each ship
  int32_t ep[kWave];          // episode step before this step
};
template <typename T>
struct SplitPSlot {           // one step's P-wave results
  uint32_t b[2][kWave];       // [0] test: kPbReset; [1] obstacle: status bits | stop | done | kPbReset
  T r_nto[kWave], r_o[kWave]; // the obstacle's non-terminal and terminal reward
};
template <typename T>
struct SplitShared {
  SplitDSlot<T> d[kSplitRing];
  SplitPSlot<T> p[kSplitRing];
};

#ifdef SIT_DIAG_SPLIT
// diagnostic builds only (tools/diag_split.py): shader cycles per role and phase, lane 0 of each
// wave, summed into g_sit_diag[role >> 1][(role & 1) * 8 + phase]
#define SPL_T0() unsigned long long spl_t = __builtin_amdgcn_s_memtime(); unsigned long long spl_acc[8] = {}
#define SPL_MARK(ph) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); spl_acc[ph] += t_ - spl_t; spl_t = t_; } while (0)
#define SPL_FLUSH(role) do { if ((threadIdx.x & 63) == 0) for (int q_ = 0; q_ < 8; ++q_) \
    atomicAdd(&g_sit_diag[(role) >> 1][((role) & 1) * 8 + q_], spl_acc[q_]); } while (0)
#else
#define SPL_T0() do {} while (0)
#define SPL_MARK(ph) do {} while (0)
#define SPL_FLUSH(role) do {} while (0)
#endif

template <typename T>
__host__ __device__ constexpr size_t split_lds_bytes(size_t map_bytes) {
  return ((map_bytes + 255) & ~size_t(255)) + 2 * ((sizeof(SplitShared<T>) + 255) & ~size_t(255));
}

// ------------------------------------------------------------------------------------------
// D waves
// ------------------------------------------------------------------------------------------
template <typename T, int TYPE, int MACH>
__device__ __forceinline__ void split_d(const KArgs<T>& a, const Consts<T>& cs, SplitShared<T>& X, int env,
                                       bool act) {
#if SIT_SPLIT_CREF
  const Consts<T>& c = cs;     // constants read from LDS where used (registers for the state)
#else
  const Consts<T> c = cs;
#endif
  const int lane = threadIdx.x & (kWave - 1);
  const int n_env = a.n_env;
  const int sid = TYPE * n_env + env;
  const int n = a.io.n_steps;

  Ship<T> s{};
  Route<T> rt{};
  T v_des = T(0);
  T samp = T(0), eps = T(0), ppn = T(0), ppe = T(0), iwn = T(0), iwe = T(0);
  int ep_step = 0;
  uint32_t event = 0, episodes = 0;
  double ab_len = 0.0, ab_alpha = 0.0, samp_limit = 0.0;
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
    rt.load_leg(s.k);
    if (TYPE == 1) {
      samp = a.st.env[0][env]; eps = a.st.env[1][env];
      ppn = a.st.env[2][env]; ppe = a.st.env[3][env];
      iwn = a.st.env[4][env]; iwe = a.st.env[5][env];
      event = a.st.event[env];
      episodes = a.st.episodes[env];
      ab_len = a.sc.ab_len[env];
      ab_alpha = a.sc.ab_alpha[env];
      samp_limit = ieee_mul(ab_len, cs.x.theta);   // MSRL_env_ex.py:569
    }
  }
  // episode-start values (reset() reloads nothing from memory)
  T p0[6] = {};
  int nw0 = 0;
  typename Route<T>::Leg leg0{};
  if (act) {
    for (int j = 0; j < 6; ++j) p0[j] = init_val(a.sc, TYPE, SIT_INIT_NORTH + j, env, n_env);
    nw0 = a.sc.nw0[sid];
    Route<T> r0 = rt;
    r0.nw = nw0;
    r0.load_leg(1);
    leg0 = r0.leg();
  }
  uint32_t uf = __builtin_amdgcn_readfirstlane((a.io.next_state ? 1u : 0u) | (a.io.action_out ? 16u : 0u) |
                                               (c.collision_bias ? kUfCollBias : 0u) |
                                               (c.sg_mode != SIT_SG_MOTOR ? kUfBlackout : 0u));
  T* p_ns = (uf & 1) ? a.io.next_state + (size_t)env * SIT_OBS_DIM + (TYPE == 0 ? 0 : 6) : nullptr;
  T* p_ao = (uf & 16) ? a.io.action_out + (size_t)env * 4 : nullptr;
  const size_t row_step = (size_t)n_env;

  // reset() (MSRL_Env.py:147-188; shaft speed and every PI/PID integrator persist, Q6) + init_step()
  auto reset_env = [&]() {
    s.n = p0[0]; s.e = p0[1]; s.psi = p0[2]; s.u = p0[3]; s.v = p0[4]; s.r = p0[5];
    s.ect_int = T(0); s.k = 1; s.ticks = 0; s.stop = 0;
    rt.nw = nw0;
    rt.set_leg(leg0);
    ep_step = 0;
    if (TYPE == 1) { samp = T(0); eps = T(0); ++episodes; }
    init_step_ship(c, cs.x, s, rt, v_des);
  };

  bool done_prev = false;   // env_done of the previous step without the map predicates (already reset)
  SPL_T0();
  for (int it = 0; it < n + 2; ++it) {
    asm volatile("" : "+s"(uf));
    const bool stepping = it < n;
    SplitDSlot<T>& xd = X.d[it & (kSplitRing - 1)];
    // the state reset() keeps, as it was before this step (restored if the step is redone)
    const T sw = s.w, si1 = s.i1, si2 = s.i2, shi = s.hi, shp = s.hp;
    const uint32_t sev = event;
    bool pend = act && stepping;
    for (int pass = 0; pass < 2; ++pass) {
      if (pass == 1) {
        SPL_MARK(0);
        __syncthreads();   // A: P's map predicates of step it - 1
        SPL_MARK(1);
        bool redo = false;
        if (act && it >= 1 && it - 1 < n && !done_prev) {
          const SplitPSlot<T>& xp = X.p[(it - 1) & (kSplitRing - 1)];
          redo = ((xp.b[0][lane] | xp.b[1][lane]) & kPbReset) != 0;
        }
        if (!__ballot(redo)) break;
#ifdef SIT_DIAG_SPLIT
        spl_acc[5] += 1;
#endif
        // the episode ended at step it - 1 (terrain or IW terminal): the auto reset of that step,
        // then this step again
        pend = redo && stepping;
        if (redo) {
          s.w = sw; s.i1 = si1; s.i2 = si2; s.hi = shi; s.hp = shp;
          event = sev;
          reset_env();
        }
      }
      if (!pend) continue;
      T sp, cp;
      xsincos(s.psi, &sp, &cp);
      T o_rpm, o_ect, o_pme = T(0);
      bool ect_over = false;
      uint32_t fl = s.stop ? kSfStopPre : 0u;
      if (TYPE == 1) {
        // synthetic AST sampler (uniform_policy.py:20-22 scaled by pi/6)
        const bool init_f = ep_step == 0;
        const bool sac = init_f || ((double)samp >= ab_len && !s.stop);
        double ang = 0.0, act_n = 0.0;
        if (sac) {
          const double u01 = sampler_uniform(opaque_seed(a.io.seed), (uint64_t)(a.io.env_id_offset + env), event);
          act_n = u01 * 2.0 - 1.0;
          ang = act_n * (M_PI / 6.0);
          iw_point(s.n, s.e, ab_len, ab_alpha, ang, iwn, iwe);
          ++event;
          fl |= kSfSac;
        }
        // obs_step (MSRL_Env.py:287-402)
        if (s.stop) {
          s.ticks += 2;                  // stop path: next_time() twice, no integration (Q10)
          o_rpm = s.lrpm; o_ect = s.lect; o_pme = s.lpme;
          ect_over = (double)o_ect > cs.x.e_tol;
        } else {
          if (sac) {                     // update_route: insert at index -1 (Q16)
            if (!rt.insert(iwn, iwe, s.k, a.cap)) fl |= kSfOverflow;
            samp = T(0);
          }
          const T pre_n = s.n, pre_e = s.e;
          T rudder, thr, psi_ref;
          guidance_control<T, MACH>(c, cs.x, s, rt, v_des, rudder, thr, o_ect, psi_ref, ect_over);
          o_rpm = s.w * c.rpm_k;
          o_pme = power_me_kw(c, thr);
          s.lrpm = o_rpm; s.lect = o_ect; s.lpme = o_pme;
          ship_dynamics<T, MACH>(c, s, thr, rudder, sp, cp);
          if (!init_f) {                 // distance between the last two stored positions
            const T dn = pre_n - ppn, de = pre_e - ppe;
            const T d = xsqrt(dn * dn + de * de);
            eps = eps + d;
            samp = samp + d;
          }
          ppn = pre_n; ppe = pre_e;
          s.ticks += 1;
        }
        const bool arrive = within_radius(s.n, s.e, rt.end_n, rt.end_e, c.arrive_d2_le);
        const bool horizon = outside(c, s.n, s.e, c.half_len);
        const bool nav = ect_over || (double)samp > samp_limit;
        fl |= (arrive ? kSfArrive : 0u) | (horizon ? kSfHorizon : 0u) | (nav ? kSfNav : 0u) |
              ((horizon || nav) ? kSfDoneNt : 0u);
        if (arrive || horizon || nav) s.stop = 1;   // (the IW terminal stops it too: P, then reset)
        xd.o[0][lane] = s.n; xd.o[1][lane] = s.e; xd.o[2][lane] = s.psi; xd.o[3][lane] = o_ect;
        xd.o[4][lane] = iwn; xd.o[5][lane] = iwe; xd.o[6][lane] = (T)act_n;
        xd.f[1][lane] = fl;
        xd.ep[lane] = ep_step;
        if (uf & 1) { store2(p_ns, s.n, s.e); store2(p_ns + 2, s.psi, o_ect); }
        if (uf & 16) { store2(p_ao, iwn, iwe); store2(p_ao + 2, angle_or_nan(sac, (T)ang), sac ? T(1) : T(0)); }
      } else {
        // test_step (MSRL_Env.py:219-285)
        T rudder, thr, psi_ref;
        const T i1_0 = s.i1, i2_0 = s.i2;
        guidance_control<T, MACH>(c, cs.x, s, rt, v_des, rudder, thr, o_ect, psi_ref, ect_over);
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
            blk = power_me_kw_exact(c.sg_mode, cs.x, throttle_exact(cs.x, s.u, v_des, i1_0, i2_0,
                                                                    c.collision_bias != 0, MACH == 1))
                  > cs.x.blackout;
        }
        s.lrpm = o_rpm; s.lect = o_ect; s.lpme = o_pme;
        ship_dynamics<T, MACH>(c, s, thr, rudder, sp, cp);
        s.ticks += 1;
        const bool arrive = within_radius(s.n, s.e, rt.end_n, rt.end_e, c.arrive_d2_le);
        const bool horizon = outside(c, s.n, s.e, c.half_len);
        const bool any = arrive || horizon || mech || ect_over || blk;
        fl |= (arrive ? kSfArrive : 0u) | (horizon ? kSfHorizon : 0u) | (mech ? kSfMech : 0u) |
              (ect_over ? kSfEct : 0u) | (blk ? kSfBlk : 0u) | (any ? kSfDoneNt : 0u);
        if (any) s.stop = 1;
        xd.t[0][lane] = s.n; xd.t[1][lane] = s.e; xd.t[2][lane] = s.psi;
        xd.t[3][lane] = o_rpm; xd.t[4][lane] = o_ect; xd.t[5][lane] = o_pme;
        xd.f[0][lane] = fl;
        if (uf & 1) { store2(p_ns, s.n, s.e); store2(p_ns + 2, s.psi, o_rpm); store2(p_ns + 4, o_ect, o_pme); }
      }
    }
    SPL_MARK(2);
    __syncthreads();   // B: both ships' step it (redone if needed)
    SPL_MARK(3);
    // env level without the map predicates: collision, the episode's end, the auto reset
    if (act && stepping) {
      const T tn = xd.t[0][lane], te = xd.t[1][lane], on = xd.o[0][lane], oe = xd.o[1][lane];
      const bool coll = closer_than(tn, te, on, oe, c.coll_d2);
      done_prev = ((xd.f[0][lane] | xd.f[1][lane]) & kSfDoneNt) || coll;
      if (coll) s.stop = 1;
      rt.fixup(s.k);
      ep_step += 1;
      if (done_prev) reset_env();
    } else {
      done_prev = false;
    }
    if (stepping) {
      p_ns += row_step * SIT_OBS_DIM;
      p_ao += row_step * 4;
    }
    SPL_MARK(4);
  }
  SPL_FLUSH(TYPE);
  if (act) {
    store_ship(a.st, sid, s);
    a.st.nw[sid] = rt.nw;
    if (TYPE == 1) {
      a.st.env[0][env] = samp; a.st.env[1][env] = eps;
      a.st.env[2][env] = ppn; a.st.env[3][env] = ppe;
      a.st.env[4][env] = iwn; a.st.env[5][env] = iwe;
      a.st.ep_step[env] = ep_step;
      a.st.event[env] = event;
      a.st.episodes[env] = episodes;
    }
  }
}

// ------------------------------------------------------------------------------------------
// P waves
// ------------------------------------------------------------------------------------------
template <typename T, int TYPE>
__device__ __forceinline__ void split_p(const KArgs<T>& a, const Consts<T>& cs, const Map<T>& map_in,
                                       SplitShared<T>& X, int env, bool act) {
  const Consts<T> c = cs;
  Map<T> map = map_in;
  const int lane = threadIdx.x & (kWave - 1);
  const int n_env = a.n_env;
  const int n = a.io.n_steps;
  // P1: the IW terrain test is a function of (iwn, iwe), which change only at sampling events
  T iw_tn = T(0), iw_te = T(0);
  bool iw_valid = false, iw_in = false;
  // P0: the observation before the step (the replay transition's state) and the test ship's
  // reward terms and status bits of the previous step
  T lo[SIT_OBS_DIM] = {};
  if (TYPE == 0 && act)
    for (int j = 0; j < SIT_OBS_DIM; ++j) lo[j] = a.st.last_obs[(size_t)j * n_env + env];
  T r_nt_t = T(0), r_term_t = T(0);
  uint32_t bits_t = 0;
  uint32_t uf = __builtin_amdgcn_readfirstlane((a.io.reward ? 2u : 0u) | (a.io.done ? 4u : 0u) |
                                               (a.io.status ? 8u : 0u) | (a.io.transitions ? kUfTrans : 0u) |
                                               (a.io.done_count ? kUfDoneCnt : 0u) |
                                               (a.io.mask_horizon > 0 ? kUfMaskH : 0u));

  SPL_T0();
  for (int it = 0; it < n + 2; ++it) {
    asm volatile("" : "+s"(uf));
    asm volatile("" : "+s"(map.use_index), "+s"(map.use_cells), "+s"(map.n_edge), "+s"(map.n_poly));
    // ---- P0: the env's outputs of step it - 2 ----
    if (TYPE == 0 && it >= 2 && it - 2 < n) {
      const int j2 = it - 2;
      const SplitDSlot<T>& xd = X.d[j2 & (kSplitRing - 1)];
      const SplitPSlot<T>& xp = X.p[j2 & (kSplitRing - 1)];
      bool env_done = false;
      if (act) {
        const T tn = xd.t[0][lane], te = xd.t[1][lane], on = xd.o[0][lane], oe = xd.o[1][lane];
        const bool coll = closer_than(tn, te, on, oe, c.coll_d2);
        const uint32_t bo = xp.b[1][lane];
        env_done = (bits_t & SIT_ST_TEST_DONE) || (bo & kDoneBit) || coll;
        const T dn = tn - on, de = te - oe;
        const T r_snt = (bo & kStopBit) ? T(0) : (T(1) - xsqrt(dn * dn + de * de) * c.inv_maxn) * T(0.001);
        const T rs = coll ? T(2000) : T(0);
        const T reward = r_nt_t + r_term_t + xp.r_nto[lane] + xp.r_o[lane] + r_snt + rs;
        const uint32_t status = ((bits_t | bo) & ~(kStopBit | kDoneBit | kPbReset)) | (coll ? SIT_ST_COLLISION : 0u);
        const size_t row = (size_t)j2 * n_env + env;
        if (uf & 2) a.io.reward[row] = reward;
        if (uf & 4) a.io.done[row] = env_done ? 1 : 0;
        if (uf & 8) a.io.status[row] = status;
        const bool sac = (xd.f[1][lane] & kSfSac) != 0;
        if (uf & kUfTrans) {           // replay transition of a sampling event (main_ast.py:385-396)
          const unsigned long long m = __ballot(sac);
          if (m) {
            const int lead = __builtin_ctzll(m);
            int base = 0;
            if (lane == lead) base = atomicAdd(a.io.transition_count, (int)__popcll(m));
            base = __shfl(base, lead);
            const int slot = base + (int)__popcll(m & ((1ull << lane) - 1ull));
            if (sac && slot < a.io.transition_capacity) {
              T* rec = a.io.transitions + (size_t)slot * SIT_TRANSITION_DIM;
              for (int j = 0; j < SIT_OBS_DIM; ++j) rec[j] = lo[j];
              rec[10] = xd.o[6][lane];
              rec[11] = reward;
              for (int j = 0; j < 6; ++j) rec[12 + j] = xd.t[j][lane];
              for (int j = 0; j < 4; ++j) rec[18 + j] = xd.o[j][lane];
              const bool horizon_hit = (uf & kUfMaskH) && xd.ep[lane] + 2 == a.io.mask_horizon;
              rec[22] = (horizon_hit || !env_done) ? T(1) : T(0);
              rec[23] = (T)(a.io.env_id_offset + env);
            }
          }
        }
        // the observation becomes the next step's state; the auto reset's initial observation
        if (env_done) {
          for (int j = 0; j < SIT_OBS_DIM; ++j) lo[j] = a.sc.initial_state[(size_t)env * SIT_OBS_DIM + j];
        } else {
          for (int j = 0; j < 6; ++j) lo[j] = xd.t[j][lane];
          for (int j = 0; j < 4; ++j) lo[6 + j] = xd.o[j][lane];
        }
      }
      if (uf & kUfDoneCnt) {           // episode-done count: one ballot + one atomic per wave
        const unsigned long long m = __ballot(env_done);
        if (lane == 0 && m) atomicAdd(a.io.done_count + j2, (int)__popcll(m));
      }
    }
    SPL_MARK(0);
    // ---- the map predicates of step it - 1 (MSRL_env_ex.py:490-542, 628-881) ----
    if (it >= 1 && it - 1 < n) {
      const int j = it - 1;
      const SplitDSlot<T>& xd = X.d[j & (kSplitRing - 1)];
      SplitPSlot<T>& xp = X.p[j & (kSplitRing - 1)];
      if (act) {
        const T sn = TYPE == 0 ? xd.t[0][lane] : xd.o[0][lane];
        const T se = TYPE == 0 ? xd.t[1][lane] : xd.o[1][lane];
        const T o_ect = TYPE == 0 ? xd.t[4][lane] : xd.o[3][lane];
        const uint32_t fl = xd.f[TYPE][lane];
        int cell_c;
        uint32_t word_c;
        const int cls_c = fine_lookup(c, map, sn, se, cell_c, word_c);
        const T dobst = distance_indexed(c, map, sn, se);
        const bool terrain = hull_in_terrain_cls(c, map, sn, se, dobst, cls_c, cell_c, word_c);
        int stop = (fl & kSfStopPre) ? 1 : 0;
        bool done = false;
        T r_nt = T(0), r_term = T(0);
        uint32_t bits = 0;
        if (TYPE == 0) {
          r_nt = xabs(o_ect) * c.inv_e_tol + (T(1) - dobst * c.inv_maxn) * T(0.01);
          const bool pred[6] = {(fl & kSfArrive) != 0, (fl & kSfHorizon) != 0, terrain, (fl & kSfMech) != 0,
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
          xp.b[0][lane] = terrain ? kPbReset : 0u;
        } else {
          const T iwn = xd.o[4][lane], iwe = xd.o[5][lane];
          if (!iw_valid || iwn != iw_tn || iwe != iw_te) {
            iw_in = pip_point(c, map, iwn, iwe);
            iw_tn = iwn; iw_te = iwe; iw_valid = true;
          }
          const bool iw_term = outside(c, iwn, iwe, T(0)) || iw_in;   // Q11
          if (!stop)
            r_nt = T(0.1) - xabs(o_ect) * c.inv_e_tol * T(0.01) - (T(1) - dobst * c.inv_maxn) * T(0.01);
          bits = (fl & kSfOverflow) ? SIT_ST_ROUTE_OVERFLOW : 0u;
          if (fl & kSfArrive) { stop = 1; bits |= SIT_ST_OBS_ENDPOINT; }
          if (fl & kSfHorizon) { stop = 1; done = true; bits |= SIT_ST_OBS_HORIZON; }
          if (terrain) {                 // done without stop flag (Q12)
            if (!stop) r_term = r_term - T(1000);
            done = true;
            bits |= SIT_ST_OBS_TERRAIN;
          }
          if (iw_term) {
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
          xp.b[1][lane] = bits | (stop ? kStopBit : 0u) | (done ? kDoneBit : 0u) |
                          ((terrain || iw_term) ? kPbReset : 0u);
          xp.r_nto[lane] = r_nt;
          xp.r_o[lane] = r_term;
        }
      }
    }
    SPL_MARK(1);
    __syncthreads();   // A
    SPL_MARK(2);
    __syncthreads();   // B
    SPL_MARK(3);
  }
  SPL_FLUSH(2 + TYPE);
  if (TYPE == 0 && act)
    for (int j = 0; j < SIT_OBS_DIM; ++j) a.st.last_obs[(size_t)j * n_env + env] = lo[j];
}

// 512 threads = 2 env groups of 64 envs x {D0, D1, P0, P1}; one map copy per block
template <typename T, int MACH>
__global__ __launch_bounds__(512) void k_env_steps_split(const KArgs<T> a) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ Consts<T> cs;
  for (int i = threadIdx.x; i < (int)(sizeof(Consts<T>) / 4); i += blockDim.x)
    reinterpret_cast<uint32_t*>(&cs)[i] = reinterpret_cast<const uint32_t*>(&a.c)[i];
  const Map<T> map = stage_map(a, smem);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int group = w >> 2;
  const int role = group == 0 ? (w & 3) : ((w & 3) ^ 2);
  const int lane = threadIdx.x & (kWave - 1);
  const int env = (blockIdx.x * 2 + group) * kWave + lane;
  const bool act = env < a.n_env;
  SplitShared<T>* xsh =
      reinterpret_cast<SplitShared<T>*>(smem + (((size_t)a.map_bytes + 255) & ~size_t(255)));
  SplitShared<T>& X = *reinterpret_cast<SplitShared<T>*>(reinterpret_cast<unsigned char*>(xsh) +
                                                         (size_t)group * ((sizeof(SplitShared<T>) + 255) & ~size_t(255)));
#ifdef SIT_DIAG_SPLIT
  __shared__ int spl_simd[8];
  if (lane == 0) spl_simd[w] = (int)((__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) >> 4) & 3);
#endif
  __syncthreads();   // constants copied, map staged
#ifdef SIT_DIAG_SPLIT
  if (threadIdx.x == 0) {   // blocks whose SIMDs each hold one D and one P wave
    int dcount[4] = {0, 0, 0, 0};
    for (int q = 0; q < 8; ++q) {
      const int rq = (q >> 2) == 0 ? (q & 3) : ((q & 3) ^ 2);
      if (rq < 2) dcount[spl_simd[q]] += 1;
    }
    const bool bal = dcount[0] == 1 && dcount[1] == 1 && dcount[2] == 1 && dcount[3] == 1;
    atomicAdd(&g_sit_diag[1][16], bal ? 1ull : 0ull);
    atomicAdd(&g_sit_diag[1][17], 1ull);
    for (int q = 0; q < 8; ++q) atomicAdd(&g_sit_diag[1][18 + q], (unsigned long long)spl_simd[q]);
  }
#endif
#ifndef SIT_SPLIT_PRIO
#define SIT_SPLIT_PRIO 0   // 1, 2: measured no different from 0
#endif
  // issue priority per SIMD pair: D1 + P1 and D0 + P0 share a SIMD; the longer chain of each pair
  // (the obstacle's step, the test-ship predicates with the env's outputs) issues first
  if (SIT_SPLIT_PRIO == 1) {
    if (role == 1 || role == 2) __builtin_amdgcn_s_setprio(1);
  } else if (SIT_SPLIT_PRIO == 2) {
    if (role < 2) __builtin_amdgcn_s_setprio(1);
  }
  if (role == 0) split_d<T, 0, MACH>(a, cs, X, env, act);
  else if (role == 1) split_d<T, 1, MACH>(a, cs, X, env, act);
  else if (role == 2) split_p<T, 0>(a, cs, map, X, env, act);
  else split_p<T, 1>(a, cs, map, X, env, act);
}
