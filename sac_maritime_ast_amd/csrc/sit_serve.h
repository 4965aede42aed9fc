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
#ifndef SIT_SERVE_ROWS
#define SIT_SERVE_ROWS 16
#endif
constexpr int kServeRows = SIT_SERVE_ROWS;   // request rows per pass of the block's actor (even)
#ifndef SIT_SERVE_VAR
#define SIT_SERVE_VAR 1   // passes of 4 / 8 / 12 / kServeRows rows by the rows left (0: always kServeRows)
#endif
#ifndef SIT_SERVE_KB
#define SIT_SERVE_KB 8
#endif
constexpr int kServeKB = SIT_SERVE_KB;   // W2^T float4 rows per prefetch batch and lane (two batches in flight)

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
  f32x2 h1[kServeRows / 2][kActorHidden];       // layer-1 activations, row pairs interleaved (1 KB per row)
  float part[2][kServeRows][kActorHidden];      // layer-2 half sums (2 KB per row)
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

// SIT_DIAG_SERVE (diagnostic builds only, tools/diag_serve.py; not with SIT_DIAG_SYNC): per pass, lane 0 of
// wave 0 counts the pass in g_sit_diag[1][R / 4] and sums its duration in s_memtime / s_memrealtime (100 MHz)
// ticks into g_sit_diag[1][8] / [1][9].  (Stamps between the pass's phases were tried: their waits serialize
// the W2^T stream and tripled the pass, so only the whole pass is timed.)

// One pass of the actor over published rows [row0, row0 + kServeRows) by the block's 256 threads:
// layer 1 (thread j = hidden unit j), layer 2 split over K (wave q sums inputs [64 q, 64 q + 64) for
// all 256 units, lane l owning units 4l..4l+3: one coalesced float4 of W2^T per k, the activations
// wave-uniform LDS broadcasts feeding packed FMAs), the two half sums combined in sit_policy_actor's
// order ((q0 + q1) + (q2 + q3)) + b2, layer 3 by 16 lanes per (row, output).  Rows past `count` are
// computed on whatever the published rows hold and never written.  Leaves (mu, log_sigma) in W.head.
// R (even, <= kServeRows): the rows of this pass; each row's arithmetic is the same for every R.
template <int R>
__device__ __forceinline__ void serve_pass(const float* __restrict__ w, const ServePub& P, ServeWork& W, int row0,
                                           const float (&wr)[kActorObs], float b1, float b2) {
#pragma clang fp reassociate(off) contract(off)
  static_assert(R % 2 == 0 && R <= kServeRows, "pass rows");
  constexpr int H = kActorHidden, KB = kServeKB;
  const int j = threadIdx.x, q = j >> 6, l = j & 63;
#ifdef SIT_DIAG_SERVE
  const unsigned long long sv_m0 = __builtin_amdgcn_s_memtime(), sv_r0 = __builtin_amdgcn_s_memrealtime();
#endif
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
  for (int half = 0; half < (2 * R + 15) / 16; ++half) {
    const int pr = (j >> 4) + 16 * half, c = j & 15;
    if (2 * R % 16 != 0 && pr >= 2 * R) break;   // (uniform per 16-lane group)
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
#ifdef SIT_DIAG_SERVE
  if (j == 0) {
    atomicAdd(&g_sit_diag[1][R / 4], 1ull);
    atomicAdd(&g_sit_diag[1][8], __builtin_amdgcn_s_memtime() - sv_m0);
    atomicAdd(&g_sit_diag[1][9], __builtin_amdgcn_s_memrealtime() - sv_r0);
  }
#endif
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
    // the pass sized to the rows left, rounded up to 4 (a block serves ~10 rows per 64-step launch at C5:
    // a fixed 16-row pass computed ~35 % padding rows, and the pass is FLOP-bound)
    const int rem = count - row0;
#if SIT_SERVE_VAR
    if (rem <= 4) serve_pass<4>(w, P, W, row0, wr, b1, b2);
    else if (rem <= 8) serve_pass<8>(w, P, W, row0, wr, b1, b2);
    else if (rem <= 12) serve_pass<12>(w, P, W, row0, wr, b1, b2);
    else serve_pass<kServeRows>(w, P, W, row0, wr, b1, b2);
#else
    (void)rem;
    serve_pass<kServeRows>(w, P, W, row0, wr, b1, b2);
#endif
    if (j < kServeRows && row0 + j < count) {
      const int e = SIT_DCLAMP(P.env[row0 + j], n_env, kDbgServeEnv);
      policy_action[e] = (T)actor_head(W.head[2 * j], W.head[2 * j + 1], P.noise[row0 + j], deterministic);
    }
    __syncthreads();   // W reused by the next pass
  }
}
