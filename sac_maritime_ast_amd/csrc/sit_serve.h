// sit_serve.h — the SAC-AST actor evaluated by the policy-mode step kernel itself, at the end of
// its launch, for the envs of the block that wait for an action (sit_rollout_args.actor_weights).
//
// Included from sit_sync.h (inside sit_impl.h's anonymous namespace).  The network and head are
// sit_policy_actor's (sit_actor.h, include/sit.h): ast_core/nn_models/mlp.py:95-148 (ReLU MLP, obs
// 10 -> 256 -> 256 -> (mu, log_sigma)), the squashed Gaussian head of ast_core/distributions/
// normal.py:88-101 and ast_core/policies/gaussian_policy.py:71-72, in float32.  Both kernels share
// the per-row arithmetic below (the same products in the same order, the head's exp / tanh written
// out in explicit instructions), so an env served here gets the same action bits as through the
// request queue and sit_policy_actor — in the strict translation unit and in the float32 step TU,
// which is compiled with device fast-math.
//
// Why in the step kernel: a 256-thread step block is one group of 64 envs, the actor's block shape;
// at C5 about 10 of its envs end a 64-step launch waiting.  Serving them in the block's epilogue
// replaces the admission and actor launches (~23 us of dependent latency per launch) by a few us at
// the end of a kernel whose blocks finish at different times, and needs no queue capacity: every
// waiting env is served every launch.
#pragma once

constexpr int kActorObs = SIT_OBS_DIM;
constexpr int kActorHidden = SIT_ACTOR_HIDDEN;
// packed weights (float32): W1 [H][obs] (torch Linear layout), b1 [H], W2^T [H in][H out],
// b2 [H], W3 [2][H], b3 [2]
constexpr int kActorW1 = 0;
constexpr int kActorB1 = kActorW1 + kActorHidden * kActorObs;
constexpr int kActorW2T = kActorB1 + kActorHidden;
constexpr int kActorB2 = kActorW2T + kActorHidden * kActorHidden;
constexpr int kActorW3 = kActorB2 + kActorHidden;
constexpr int kActorB3 = kActorW3 + 2 * kActorHidden;
static_assert(kActorB3 + 2 == SIT_ACTOR_WEIGHTS, "packed actor layout");
static_assert(kActorHidden == 256, "one thread per hidden unit, 256 threads per block");

typedef float f32x2 __attribute__((ext_vector_type(2)));

// exp(x) for the clipped log sigma (x in [-20, 2]): Cody-Waite reduction by ln 2 and a degree-7
// Taylor polynomial on |r| <= ln(2)/2 (truncation < 2e-9 relative), ldexp back.  Explicit fma /
// multiply / rint / ldexp only, so no translation unit's fast-math flags change a bit of it.
__device__ __forceinline__ float actor_exp(float x) {
#pragma clang fp reassociate(off) contract(off)
  const float n = __builtin_rintf(x * 1.44269504f);
  float r = __builtin_fmaf(-n, 0.693145752f, x);      // ln 2, high part (exact product for |n| < 2^12)
  r = __builtin_fmaf(-n, 1.42860677e-6f, r);           // ln 2, low part
  float p = 1.98412698e-4f;                             // 1/7!
  p = __builtin_fmaf(p, r, 1.38888889e-3f);
  p = __builtin_fmaf(p, r, 8.33333333e-3f);
  p = __builtin_fmaf(p, r, 4.16666667e-2f);
  p = __builtin_fmaf(p, r, 1.66666667e-1f);
  p = __builtin_fmaf(p, r, 0.5f);
  p = __builtin_fmaf(p, r, 1.0f);
  p = __builtin_fmaf(p, r, 1.0f);
  return __builtin_ldexpf(p, (int)n);
}

// tanh(x) = sign(x) e / (e + 2), e = expm1(2|x|): expm1 by its Taylor series below 0.35 (no
// cancellation near 0), exp - 1 above; the quotient by the hardware reciprocal (1 ulp) and a
// multiply, |x| >= 9 gives +-1 (tanh(9) rounds to 1 - 6e-8).  Relative error a few float32 ulp
// (tests/test_gpu_policy.py checks the actor against float64 PyTorch at 1e-5).
__device__ __forceinline__ float actor_tanh(float x) {
#pragma clang fp reassociate(off) contract(off)
  const float ax = __builtin_fminf(__builtin_fabsf(x), 9.0f);
  const float t = ax + ax;
  float em;
  if (t < 0.35f) {
    float p = 2.48015873e-5f;                           // 1/8!
    p = __builtin_fmaf(p, t, 1.98412698e-4f);
    p = __builtin_fmaf(p, t, 1.38888889e-3f);
    p = __builtin_fmaf(p, t, 8.33333333e-3f);
    p = __builtin_fmaf(p, t, 4.16666667e-2f);
    p = __builtin_fmaf(p, t, 1.66666667e-1f);
    p = __builtin_fmaf(p, t, 0.5f);
    p = __builtin_fmaf(p, t, 1.0f);
    em = p * t;
  } else {
    em = actor_exp(t) - 1.0f;
  }
  const float y = em * __builtin_amdgcn_rcpf(em + 2.0f);
  return __builtin_copysignf(ax >= 9.0f ? 1.0f : y, x);
}

// the squashed Gaussian head of one row: x = mu + exp(clip(log_sigma, -20, 2)) * noise (x = mu when
// deterministic), action = tanh(x)
__device__ __forceinline__ float actor_head(float mu, float ls_raw, float noise, bool deterministic) {
#pragma clang fp reassociate(off) contract(off)
  const float ls = __builtin_fminf(__builtin_fmaxf(ls_raw, -20.0f), 2.0f);
  const float x = deterministic ? mu : __builtin_fmaf(actor_exp(ls), noise, mu);
  return actor_tanh(x);
}

// ------------------------------------------------------------------------------------------
// In-kernel serving
// ------------------------------------------------------------------------------------------
constexpr int kServeRows = 16;   // request rows per pass of the block's actor
constexpr int kServeKB = 8;      // W2^T float4 rows per prefetch batch and lane (two batches in flight)

// the block's waiting envs, written after barrier C: env id and the event's normal draw by the
// obstacle's D wave, the observation the env waits at by P0; rows in lane order
struct ServePub {
  float obs[kWave][kActorObs];
  float noise[kWave];
  int32_t env[kWave];
  int32_t count;
};
// the actor's working set, at LDS offset 0 over the staged map and the exchange slots (dead after
// barrier D)
struct ServeWork {
  f32x2 h1[kServeRows / 2][kActorHidden];       // layer-1 activations, row pairs interleaved (16 KB)
  float part[2][kServeRows][kActorHidden];      // layer-2 half sums (32 KB)
  float head[2 * kServeRows];                   // (mu, log_sigma) per row
};
static_assert(sizeof(f32x2) * (kServeRows / 2) * kActorHidden == sizeof(float) * kServeRows * kActorHidden,
              "layer-2 activations alias h1");

__host__ __device__ constexpr size_t serve_align(size_t b) { return (b + 255) & ~size_t(255); }
// the dynamic LDS of a serving launch: [map | exchange slots | transition ring] (or the actor's
// working set, whichever is larger), then the published requests
template <typename T>
__host__ __device__ constexpr size_t serve_pub_offset(size_t map_bytes) {
  return sync_lds_bytes<T, kPolicy>(map_bytes) > serve_align(sizeof(ServeWork)) ? sync_lds_bytes<T, kPolicy>(map_bytes)
                                                                                : serve_align(sizeof(ServeWork));
}
template <typename T>
__host__ __device__ constexpr size_t serve_lds_bytes(size_t map_bytes) {
  return serve_pub_offset<T>(map_bytes) + serve_align(sizeof(ServePub));
}

// One pass of the actor over published rows [row0, row0 + kServeRows) by the block's 256 threads:
// layer 1 (thread j = hidden unit j), layer 2 split over K (wave q sums inputs [64 q, 64 q + 64) for
// all 256 units, lane l owning units 4l..4l+3: one coalesced float4 of W2^T per k, the activations
// wave-uniform LDS broadcasts feeding packed FMAs), the two half sums combined in sit_policy_actor's
// order ((q0 + q1) + (q2 + q3)) + b2, layer 3 by 16 lanes per (row, output).  Rows past `count` are
// computed on whatever the published rows hold and never written.  Leaves (mu, log_sigma) in W.head.
__device__ __forceinline__ void serve_pass(const float* __restrict__ w, const ServePub& P, ServeWork& W, int row0,
                                           const float (&wr)[kActorObs], float b1, float b2) {
#pragma clang fp reassociate(off) contract(off)
  constexpr int H = kActorHidden, R = kServeRows, KB = kServeKB;
  const int j = threadIdx.x, q = j >> 6, l = j & 63;
  // layer 1: h1 = relu(W1 obs + b1), one row pair at a time (unrolled over all rows, the compiler
  // held every row's observation in registers at once)
#pragma unroll 1
  for (int p = 0; p < R / 2; ++p) {
    float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
    for (int i = 0; i < kActorObs; ++i) {
      a0 = __builtin_fmaf(wr[i], P.obs[row0 + 2 * p][i], a0);
      a1 = __builtin_fmaf(wr[i], P.obs[row0 + 2 * p + 1][i], a1);
    }
    W.h1[p][j] = f32x2{__builtin_fmaxf(a0 + b1, 0.0f), __builtin_fmaxf(a1 + b1, 0.0f)};
  }
  __syncthreads();
  // layer 2
  const int kq = q * 64;
  // each batch's rows from a base the compiler cannot see through: with plain indexing it hoisted all
  // 64 row addresses (128 registers) out of the pass loop and spilled
  auto batch = [&](int k0, float4 (&dst)[KB]) {
    const float4* b = reinterpret_cast<const float4*>(w + kActorW2T) + (size_t)k0 * (H / 4) + l;
    asm volatile("" : "+v"(b));
#pragma unroll
    for (int i = 0; i < KB; ++i) dst[i] = b[i * (H / 4)];
  };
  float4 wa[KB], wb[KB];
  batch(kq, wa);
  f32x2 acc[4][R / 2];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int p = 0; p < R / 2; ++p) acc[n][p] = f32x2{0.0f, 0.0f};
#pragma unroll
  for (int c = 0; c < 64 / KB; ++c) {
    if (c + 1 < 64 / KB) batch(kq + (c + 1) * KB, wb);
#pragma unroll
    for (int g = 0; g < KB / 2; ++g) {
      const int k = kq + c * KB + g * 2;
      // (h[2p][k], h[2p+1][k], h[2p][k+1], h[2p+1][k+1]): one b128 broadcast read per row pair
      f32x2 hp[R / 2][2];
#pragma unroll
      for (int p = 0; p < R / 2; ++p) {
        const float4 v = *reinterpret_cast<const float4*>(&W.h1[p][k]);
        hp[p][0] = f32x2{v.x, v.y};
        hp[p][1] = f32x2{v.z, v.w};
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float4 wk = wa[g * 2 + i];
        const float wn[4] = {wk.x, wk.y, wk.z, wk.w};
#pragma unroll
        for (int p = 0; p < R / 2; ++p)
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[n][p] = __builtin_elementwise_fma(hp[p][i], f32x2{wn[n], wn[n]}, acc[n][p]);
      }
    }
#pragma unroll
    for (int i = 0; i < KB; ++i) wa[i] = wb[i];
  }
  // the K quarters: q1 and q3 store, q0 and q2 add theirs, then (q0 + q1) + (q2 + q3)
  if (q == 1 || q == 3) {
    float(*dst)[H] = W.part[q >> 1];
#pragma unroll
    for (int p = 0; p < R / 2; ++p) {
      *reinterpret_cast<float4*>(&dst[2 * p][4 * l]) = float4{acc[0][p].x, acc[1][p].x, acc[2][p].x, acc[3][p].x};
      *reinterpret_cast<float4*>(&dst[2 * p + 1][4 * l]) = float4{acc[0][p].y, acc[1][p].y, acc[2][p].y, acc[3][p].y};
    }
  }
  __syncthreads();
  if (q == 0 || q == 2) {
    float(*dst)[H] = W.part[q >> 1];
#pragma unroll
    for (int p = 0; p < R / 2; ++p) {
      float4 a0 = *reinterpret_cast<const float4*>(&dst[2 * p][4 * l]);
      float4 a1 = *reinterpret_cast<const float4*>(&dst[2 * p + 1][4 * l]);
      a0 = float4{acc[0][p].x + a0.x, acc[1][p].x + a0.y, acc[2][p].x + a0.z, acc[3][p].x + a0.w};
      a1 = float4{acc[0][p].y + a1.x, acc[1][p].y + a1.y, acc[2][p].y + a1.z, acc[3][p].y + a1.w};
      *reinterpret_cast<float4*>(&dst[2 * p][4 * l]) = a0;
      *reinterpret_cast<float4*>(&dst[2 * p + 1][4 * l]) = a1;
    }
  }
  __syncthreads();
  float(*h2)[H] = reinterpret_cast<float(*)[H]>(&W.h1[0][0]);
#pragma unroll
  for (int r = 0; r < R; ++r) h2[r][j] = __builtin_fmaxf((W.part[0][r][j] + W.part[1][r][j]) + b2, 0.0f);
  __syncthreads();
  // layer 3: (row, output) pairs x 16 lanes, each lane 16 units, then a 16-lane reduction
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int pr = (j >> 4) + 16 * half, c = j & 15;
    const int r = pr >> 1, o = pr & 1;
    const float* v = w + kActorW3 + o * H + c * 16;
    float sum = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) sum = __builtin_fmaf(h2[r][c * 16 + i], v[i], sum);
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 16);
    if (c == 0) W.head[pr] = sum + w[kActorB3 + o];
  }
  __syncthreads();
}

// The block's waiting envs served: every pass of kServeRows rows, then each row's head and the
// action slot of its env.  Called by all 256 threads after barrier D (block-uniform count).
// Debug builds check the published count against the 64 rows ServePub holds and every served env id
// against n_env (kDbgServeCount, kDbgServeEnv: clamped, so no access leaves its table).
template <typename T>
__device__ __forceinline__ void serve_block(const float* __restrict__ w, bool deterministic, unsigned char* smem,
                                            const ServePub& P, T* policy_action, unsigned long long* served,
                                            int n_env) {
  int count = __builtin_amdgcn_readfirstlane(P.count);
#ifdef SIT_DEBUG
  if (count < 0 || count > kWave) {
    SIT_DCHECK(false, kDbgServeCount);
    count = count < 0 ? 0 : kWave;
  }
#endif
  if (count <= 0) return;
  ServeWork& W = *reinterpret_cast<ServeWork*>(smem);
  const int j = threadIdx.x;
  if (served && j == 0) atomicAdd(served, (unsigned long long)count);
  float wr[kActorObs];
#pragma unroll
  for (int i = 0; i < kActorObs; ++i) wr[i] = w[kActorW1 + j * kActorObs + i];
  const float b1 = w[kActorB1 + j], b2 = w[kActorB2 + j];
  for (int row0 = 0; row0 < count; row0 += kServeRows) {
    serve_pass(w, P, W, row0, wr, b1, b2);
    if (j < kServeRows && row0 + j < count) {
      const int e = SIT_DCLAMP(P.env[row0 + j], n_env, kDbgServeEnv);
      policy_action[e] = (T)actor_head(W.head[2 * j], W.head[2 * j + 1], P.noise[row0 + j], deterministic);
    }
    __syncthreads();   // W reused by the next pass
  }
}

// ------------------------------------------------------------------------------------------
// Concurrent serving (sit_rollout_args.actor_concurrent)
// ------------------------------------------------------------------------------------------
// A small persistent kernel, k_actor_server, runs beside the policy-mode step kernel (a second
// stream, launched right after it) and serves the waiting envs while the launch goes on: an env that
// stops at a sampling event steps again a few steps later instead of at the next launch.  The two
// kernels share only tagged 8-byte granules {tag, 32-bit value} (MI355X_MICROARCH.md § visibility,
// R2), written and read with agent-scope relaxed atomics (global sc1 stores / loads), plus one mask
// word per step block and a count of finished step blocks (agent-scope atomics):
//   request  req[i][e] = {tag, obs_i bits}, i < SIT_OBS_DIM, and req[SIT_OBS_DIM][e] = {tag, the event's
//            normal draw}: the obstacle's predicate wave P1 of env e's block stores them at the step the
//            env stops (D1 publishes the stop before barrier A), then, one step later and after its own
//            vmcnt(0) wait, sets bit e of mask[block]; tag = event + 1 (bit 31 in granule 0: the
//            episode's initial observation, which the server reads from initial_state itself).  P1
//            has slack at that point of the step; D1 only polls.
//   action   slot[e] = {event + 1, action bits}: the server's answer; D1 polls it (one sc1 load per
//            step for each waiting lane) and steps again when the tag matches its event
// Tags grow with the env's event counter, so a stale granule never matches, and a request whose tag
// is not above its slot's was served already.  The step kernel never waits for the server (it only
// polls), so a server that is not resident delays actions, never the launch; the server leaves when
// every step block has finished and it holds no request, or after a bounded time (stats[0]).
// Arithmetic: the rows of serve_pass (the same products in the same order: layer 1 as there; layer 2
// per unit as four K-quarter sums combined ((q0 + q1) + (q2 + q3)) + b2; layer 3 by 16-lane groups and
// the same butterfly), so a row served here equals the in-kernel and queue paths bit for bit.
typedef __attribute__((address_space(1))) unsigned long long srv_gu64;
typedef __attribute__((address_space(1))) unsigned int srv_gu32;
__device__ __forceinline__ unsigned long long srv_ld(const unsigned long long* p) {
  return __hip_atomic_load((const srv_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void srv_st(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((srv_gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned srv_ld32(const unsigned* p) {
  return __hip_atomic_load((const srv_gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr uint32_t kSrvInit = 0x80000000u;   // request tag bit: the episode's initial observation
constexpr size_t kSrvLds = sizeof(float) * kActorHidden * 8 * 3;   // k_actor_server's dynamic LDS (kSrvRows 8)
constexpr int kSrvRows = 8;                  // request rows per pass of a server block
constexpr int kSrvAssign = 64;               // step blocks per server block, at most (one per lane of wave 0)
#ifndef SIT_SRV_BLOCKS
#define SIT_SRV_BLOCKS 64                    // server blocks (at least ceil(step blocks / kSrvAssign))
#endif
#ifndef SIT_SRV_SLEEP
#define SIT_SRV_SLEEP 8                      // s_sleep units (64 clocks each) between idle polls
#endif

template <typename T>
struct SrvArgs {
  const float* w;                  // packed actor weights (sit_policy_actor's layout)
  const T* initial_state;          // [n_env][SIT_OBS_DIM]: the observation at an episode start
  unsigned long long* slot;        // [n_env] action granules
  const unsigned long long* req;   // [SIT_OBS_DIM + 1][n_env] request granules (the last: the normal draw)
  unsigned long long* mask;        // [n_blocks]
  const unsigned* done;            // finished step blocks
  unsigned long long* stats;       // [4]: timeouts, passes, rows, polls (kept across launches)
  unsigned long long* served;      // actor_served or null
  uint64_t seed;
  int64_t env_id_offset;
  uint64_t timeout;                // s_memrealtime ticks (100 MHz)
  int32_t n_env, n_blocks, n_srv, det;
};

// <= 64 VGPRs (8 waves per SIMD, the most gfx950 runs): one server wave fits beside the two step waves
// (<= 224 VGPRs each, policy mode) of a SIMD; with 24 KB of LDS beside their 2 x 67 KB
#ifndef SIT_SRV_WPE
#define SIT_SRV_WPE 8
#endif
#if SIT_SRV_WPE > 0
#define SIT_SRV_OCC __attribute__((amdgpu_waves_per_eu(SIT_SRV_WPE, SIT_SRV_WPE)))
#else
#define SIT_SRV_OCC
#endif
template <typename T>
__global__ __launch_bounds__(256) SIT_SRV_OCC
void k_actor_server(const SrvArgs<T> s) {
#pragma clang fp reassociate(off) contract(off)
  constexpr int H = kActorHidden, R = kSrvRows;
  static_assert(sizeof(float) * H * R * 3 == kSrvLds, "server LDS");
  // dynamic LDS (a static size would let the compiler plan for the occupancy that size allows and
  // spend registers accordingly): hb, layer 1 [unit][row]; part, layer 2 per unit in the unit's thread
  // only (LDS instead of registers): [0] q0 + q1, [1] q2, then the activation [row][unit]
  extern __shared__ __align__(16) unsigned char srv_dyn[];
  float* const hb = reinterpret_cast<float*>(srv_dyn);
  float (*const part)[R][H] = reinterpret_cast<float (*)[R][H]>(srv_dyn + sizeof(float) * H * R);
  __shared__ float obs[R][kActorObs];
  __shared__ float nz[R];
  __shared__ int32_t renv[R];
  __shared__ uint32_t rkey[R];
  __shared__ float head[2 * R];
  __shared__ int32_t ctl[2];
  __builtin_amdgcn_s_setprio(0);
  const int j = threadIdx.x, lane = j & 63, wv = j >> 6;
  const int n_as = (s.n_blocks - (int)blockIdx.x + s.n_srv - 1) / s.n_srv;   // assigned step blocks (<= 64)
  unsigned long long pend = 0;     // wave 0, lane i: the waiting envs of assigned block i not served yet
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (wv == 0) {
      // the finished count before the masks: a block counted finished has set all its bits
      const unsigned d = __builtin_amdgcn_readfirstlane(lane == 0 ? srv_ld32(s.done) : 0u);
      const int b = (int)blockIdx.x + lane * s.n_srv;
      if (lane < n_as && srv_ld(&s.mask[b]) != 0ull)
        pend |= __hip_atomic_exchange((srv_gu64*)&s.mask[b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // rows of this pass: the pending envs of the assigned blocks in order, up to R of them
      int rows = 0;
      unsigned long long busy = __ballot(pend != 0ull);
      while (busy && rows < R) {
        const int i = __builtin_ctzll(busy);
        busy &= busy - 1;
        const unsigned long long m = __shfl(pend, i);            // block i's pending envs
        const int e = ((int)blockIdx.x + i * s.n_srv) * 64 + lane;
        bool valid = false, drop = false, init = false;
        uint32_t tag = 0;
        if ((m >> lane) & 1ull) {
          const unsigned long long g0 = srv_ld(&s.req[e]);
          const uint32_t st = (uint32_t)(srv_ld(&s.slot[e]) >> 32);
          tag = (uint32_t)(g0 >> 32) & ~kSrvInit;
          init = ((uint32_t)(g0 >> 32) & kSrvInit) != 0;
          if (tag <= st) {
            drop = true;                                          // served already
          } else {
            valid = (uint32_t)(srv_ld(&s.req[(size_t)kActorObs * s.n_env + e]) >> 32) == tag;   // the draw
            if (!init)
#pragma unroll 1
              for (int q = 1; q < kActorObs; ++q)
                valid = valid && (uint32_t)(srv_ld(&s.req[(size_t)q * s.n_env + e]) >> 32) == tag;
          }
        }
        const unsigned long long vm = __ballot(valid), dm = __ballot(drop);
        const int take = min(R - rows, (int)__popcll(vm));
        // the lowest `take` valid lanes
        const bool mine = valid && (int)__popcll(vm & ((1ull << lane) - 1ull)) < take;
        if (mine) {
          const int r = rows + (int)__popcll(vm & ((1ull << lane) - 1ull));
          // (the granules of a waiting env do not change until it is answered: read again)
#pragma unroll 1
          for (int q = 0; q < kActorObs; ++q)
            obs[r][q] = init ? (float)s.initial_state[(size_t)e * kActorObs + q]
                             : __uint_as_float((uint32_t)srv_ld(&s.req[(size_t)q * s.n_env + e]));
          renv[r] = e;
          rkey[r] = tag;
          nz[r] = __uint_as_float((uint32_t)srv_ld(&s.req[(size_t)kActorObs * s.n_env + e]));
        }
        const unsigned long long gone = __ballot(mine) | dm;
        if (lane == i) pend &= ~gone;
        rows += take;
      }
      const bool idle = __ballot(pend != 0ull) == 0ull;
      const bool timeout = __builtin_amdgcn_s_memrealtime() - t0 > s.timeout;
      if (lane == 0) {
        ctl[0] = rows;
        ctl[1] = ((d >= (unsigned)s.n_blocks && idle && rows == 0) || timeout) ? 1 + (timeout ? 1 : 0) : 0;
        if (timeout) atomicAdd(&s.stats[0], 1ull);
        atomicAdd(&s.stats[3], 1ull);
      }
    }
    __syncthreads();
    const int rows = ctl[0], quit = ctl[1];
    if (quit) break;
    if (rows == 0) {
      if (wv == 0) __builtin_amdgcn_s_sleep(SIT_SRV_SLEEP);
      __syncthreads();   // (ctl is rewritten by the next poll)
      continue;
    }
    // layer 1: unit j of every row
    {
      const float* w1 = s.w + kActorW1 + j * kActorObs;
      const float b1 = s.w[kActorB1 + j];
#pragma clang loop vectorize(disable) unroll(disable)
      for (int r = 0; r < R; ++r) {
        float a = 0.0f;
#pragma unroll
        for (int i = 0; i < kActorObs; ++i) a = __builtin_fmaf(w1[i], obs[r][i], a);
        hb[j * R + r] = __builtin_fmaxf(a + b1, 0.0f);
      }
    }
    __syncthreads();
    // layer 2: unit j, the four K-quarter sums in order, then ((q0 + q1) + (q2 + q3)) + b2.  W2^T is
    // streamed from L2 in batches of kPf rows, the next batch in flight while one is consumed (the pass
    // is bound by the bytes it keeps in flight: 2 x kPf loads of 256 B per wave)
    {
      constexpr int kPf = 16;   // W2^T rows per batch: four batches per K-quarter, two in flight
      const float b2 = s.w[kActorB2 + j];
      // W2^T through a buffer descriptor: the row offset k * H in the instruction's scalar operand, the
      // unit's in one VGPR (64-bit addresses per row were hoisted out of the loop and spilled)
      const __amdgpu_buffer_rsrc_t w2 =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(s.w + kActorW2T), 0, H * H * (int)sizeof(float), 0x00020000);
      const int vo = j * (int)sizeof(float);
      auto load = [&](float (&dst)[kPf], int c) {
#pragma unroll
        for (int i = 0; i < kPf; ++i)
          dst[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(w2, vo, (c * kPf + i) * H * (int)sizeof(float), 0));
      };
      float acc[R];
      auto consume = [&](const float (&src)[kPf], int c) {
#pragma unroll
        for (int i = 0; i < kPf; ++i) {
          const int k = c * kPf + i;
          const float wk = src[i];
          const float4 h0 = *reinterpret_cast<const float4*>(&hb[k * R]);
          const float4 h1 = *reinterpret_cast<const float4*>(&hb[k * R + 4]);
          const float hv[R] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r] = __builtin_fmaf(hv[r], wk, acc[r]);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      float wa[kPf], wb[kPf];
      load(wa, 0);
#pragma unroll 1
      for (int q = 0; q < 4; ++q) {   // K-quarter q: batches c0 .. c0 + 3, wa holding c0
        const int c0 = 4 * q;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = 0.0f;
        load(wb, c0 + 1);
        consume(wa, c0);
        load(wa, c0 + 2);
        consume(wb, c0 + 1);
        load(wb, c0 + 3);
        consume(wa, c0 + 2);
        if (q < 3) load(wa, c0 + 4);
        consume(wb, c0 + 3);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float x = acc[r];
            if (q == 0) part[0][r][j] = x;
            else if (q == 1) part[0][r][j] = part[0][r][j] + x;
            else if (q == 2) part[1][r][j] = x;
            else part[1][r][j] = __builtin_fmaxf((part[0][r][j] + (part[1][r][j] + x)) + b2, 0.0f);
          }
      }
    }
    __syncthreads();
    // layer 3: (row, output) pairs x 16 lanes, each lane 16 units, then a 16-lane butterfly
    {
      const int pr = j >> 4, c = j & 15;
      const int r = pr >> 1, o = pr & 1;
      const float* v = s.w + kActorW3 + o * H + c * 16;
      float sum = 0.0f;
#pragma unroll 4
      for (int i = 0; i < 16; ++i) sum = __builtin_fmaf(part[1][r][c * 16 + i], v[i], sum);
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 16);
      if (c == 0) head[pr] = sum + s.w[kActorB3 + o];
    }
    __syncthreads();
    if (j < rows) {
      const float act = actor_head(head[2 * j], head[2 * j + 1], nz[j], s.det != 0);
      // (T)act as the in-kernel and queue paths store it; a float carries it exactly
      srv_st(&s.slot[renv[j]], ((unsigned long long)rkey[j] << 32) | (unsigned long long)__float_as_uint(act));
    }
    if (j == 0) {
      atomicAdd(&s.stats[1], 1ull);
      atomicAdd(&s.stats[2], (unsigned long long)rows);
      if (s.served) atomicAdd(s.served, (unsigned long long)rows);
    }
    __syncthreads();   // LDS reused by the next pass
  }
}
