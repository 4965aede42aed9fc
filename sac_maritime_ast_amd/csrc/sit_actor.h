// sit_actor.h — the SAC-AST actor fused into one kernel (sit_policy_actor, include/sit.h).
//
// Policy mode (config C5) evaluates the Gaussian policy on the envs that queued a request during
// the last fused env launch: ast_core/nn_models/mlp.py:95-148 (ReLU MLP, obs 10 -> 256 -> 256 ->
// 2 = (mu, log_sigma)), the squashed Gaussian head of ast_core/distributions/normal.py:88-101 and
// ast_core/policies/gaussian_policy.py:71-72, then the scatter into the env action slots.  As
// separate library GEMMs plus elementwise kernels that was ~8 launches per act, ~40 % of C5's GPU
// time; here it is one launch whose blocks past the device-side request count exit at once.
//
// Layout: one block of 256 threads (4 waves) per kActorRows request rows.  Layer 1: thread j = hidden
// unit j.  Layer 2 (99 % of the flops) is split over K: wave q takes inputs [64 q, 64 q + 64) for
// all 256 units, lane l units 4l..4l+3, so each k is one coalesced 1 KiB float4 read of W2^T
// (L2-resident across blocks, 16 rows in flight per lane) and one wave-uniform LDS broadcast of
// the rows' activations feeds 16 packed FMAs; the four quarter sums meet in LDS in a fixed order.
// Layer 3: 16 lanes per (row, output), then a 16-lane shuffle reduction.  FP32 throughout (the
// reference actor's dtype); deterministic; summation order differs from a GEMM library's, well
// within 1e-5.
#pragma once

#include "sit_device.h"

namespace {

// (the packed weight layout, f32x2 and the head are sit_serve.h's, shared with the step kernel's
// in-kernel serving)
constexpr int kActorRows = 8;
#ifndef SIT_ACTOR_KB
#define SIT_ACTOR_KB 8    // W2^T float4 rows per prefetch batch and lane (2 batches in flight): 8 = 144 VGPRs, three
                          // blocks per CU (C5 +2.6 % over 32: 188 VGPRs, two; 16: 168 VGPRs, +1.8 %)
#endif
static_assert(64 % SIT_ACTOR_KB == 0 && SIT_ACTOR_KB % 4 == 0, "actor prefetch batch");

template <typename T>
__global__ __launch_bounds__(256) void k_policy_actor(int cap, const float* __restrict__ w, const T* __restrict__ obs,
                                                      const T* __restrict__ noise, const int32_t* __restrict__ req_env,
                                                      const int32_t* __restrict__ req_count, int deterministic,
                                                      T* policy_action, int32_t* policy_ready, int n_env,
                                                      unsigned long long* served, int32_t* clear_count) {
  constexpr int H = kActorHidden, R = kActorRows;
  __shared__ float s_obs[R][kActorObs];
  __shared__ __align__(16) f32x2 s_h1[R / 2][H];     // layer-1 activations, row pairs interleaved
  __shared__ __align__(16) float s_h[R][H];          // layer-2 activations
  __shared__ __align__(16) float s_part[4][R][H];    // layer-2 partial sums of the 4 K quarters
  const int j = threadIdx.x;
  const int row0 = blockIdx.x * R;
  if (row0 >= cap) return;
  // every independent global read is issued up front (one memory round trip instead of a chain):
  // the request count, this block's observation rows (read whether or not they are valid), the
  // layer-1 weights and the first W2^T batch
  const int raw_count = *req_count;
  const int orow = j / kActorObs, oi = j % kActorObs;
  const bool oload = j < R * kActorObs && row0 + orow < cap;
  const float ov = oload ? (float)obs[(size_t)(row0 + orow) * kActorObs + oi] : 0.0f;
  float wr[kActorObs];
#pragma unroll
  for (int i = 0; i < kActorObs; ++i) wr[i] = w[kActorW1 + j * kActorObs + i];
  const float b1 = w[kActorB1 + j];
  const int q = j >> 6, l = j & 63;
  const float4* w2 = reinterpret_cast<const float4*>(w + kActorW2T) + l;
  const int kq = q * 64;
  constexpr int KB = SIT_ACTOR_KB;       // W2^T rows in flight per lane (two batches)
  float4 wa[KB], wb[KB];
#pragma unroll
  for (int i = 0; i < KB; ++i) wa[i] = w2[(kq + i) * (H / 4)];
  const int count = min(raw_count, cap);
  if (blockIdx.x == 0 && j == 0) {
    if (served) atomicAdd(served, (unsigned long long)max(count, 0));
    // the other slot of the two-slot request counter: consumed by the previous actor launch,
    // appended to by the next env launch (no block of this launch reads it)
    if (clear_count) *clear_count = 0;
  }
  if (row0 < count) {
    const int nrow = min(R, count - row0);
    if (j < R * kActorObs) s_obs[orow][oi] = orow < nrow ? ov : 0.0f;
    __syncthreads();
    // layer 1 (thread j = hidden unit j): h1 = relu(W1 obs + b1)
    {
      const float b = b1;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < kActorObs; ++i) acc = fmaf(wr[i], s_obs[r][i], acc);
        s_h1[r >> 1][j][r & 1] = fmaxf(acc + b, 0.0f);
      }
    }
    __syncthreads();
    // layer 2, split-K: wave q sums inputs k in [64 q, 64 q + 64) for all 256 units, lane l owning
    // units 4l..4l+3 (one coalesced float4 of W2^T per k); the layer-1 activations are wave-uniform
    // LDS broadcast reads, each feeding 16 packed FMAs (row pairs)
    {
      f32x2 acc[4][R / 2];
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int p = 0; p < R / 2; ++p) acc[n][p] = f32x2{0.0f, 0.0f};
#pragma unroll
      for (int c = 0; c < 64 / KB; ++c) {
        if (c + 1 < 64 / KB) {
#pragma unroll
          for (int i = 0; i < KB; ++i) wb[i] = w2[(kq + (c + 1) * KB + i) * (H / 4)];
        }
#pragma unroll
        for (int g = 0; g < KB / 4; ++g) {
          const int k = kq + c * KB + g * 4;
          // (h[2p][k], h[2p+1][k]) pairs for k..k+3: two b128 broadcast reads per row pair
          f32x2 hp[R / 2][4];
#pragma unroll
          for (int p = 0; p < R / 2; ++p) {
            const float4 lo = *reinterpret_cast<const float4*>(&s_h1[p][k]);
            const float4 hi = *reinterpret_cast<const float4*>(&s_h1[p][k + 2]);
            hp[p][0] = f32x2{lo.x, lo.y}; hp[p][1] = f32x2{lo.z, lo.w};
            hp[p][2] = f32x2{hi.x, hi.y}; hp[p][3] = f32x2{hi.z, hi.w};
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float4 wk = wa[g * 4 + i];
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
#pragma unroll
      for (int p = 0; p < R / 2; ++p) {
        *reinterpret_cast<float4*>(&s_part[q][2 * p][4 * l]) = float4{acc[0][p].x, acc[1][p].x, acc[2][p].x, acc[3][p].x};
        *reinterpret_cast<float4*>(&s_part[q][2 * p + 1][4 * l]) = float4{acc[0][p].y, acc[1][p].y, acc[2][p].y, acc[3][p].y};
      }
    }
    __syncthreads();
    {
      const float b2 = w[kActorB2 + j];
#pragma unroll
      for (int r = 0; r < R; ++r)
        s_h[r][j] = fmaxf(((s_part[0][r][j] + s_part[1][r][j]) + (s_part[2][r][j] + s_part[3][r][j])) + b2, 0.0f);
    }
    __syncthreads();
    // layer 3: 16 (row, output) pairs x 16 lanes, each lane 16 units, then a 16-lane reduction
    {
      const int pr = j >> 4, c = j & 15;
      const int r = pr >> 1, o = pr & 1;
      const float* v = w + kActorW3 + o * H + c * 16;
      float sum = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; ++i) sum = fmaf(s_h[r][c * 16 + i], v[i], sum);
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 16);
      if (c == 0) s_part[0][0][pr] = sum + w[kActorB3 + o];
    }
    __syncthreads();
    if (j < nrow) {
      // normal.py:88-101 (log_sigma clipped to [-20, 2], reparameterised sample), tanh squash
      const int qrow = row0 + j;
      const float a = actor_head(s_part[0][0][2 * j], s_part[0][0][2 * j + 1],
                                 deterministic ? 0.0f : (float)noise[qrow], deterministic != 0);
      const int e = req_env[qrow];
      if (e >= 0 && e < n_env) {
        policy_action[e] = (T)a;
        policy_ready[e] = 1;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Admission: the request queue of a policy-mode launch, built after the step kernel.
//
// The reference's loop never lets an env wait: every step gets an action (test_beds/main_ast.py:
// 335-348, 378).  Here an env stopped at a sampling event waits until the actor has served it, and
// the actor serves at most `cap` envs per launch; which ones is decided deterministically: oldest
// request first (age = admission rounds waited, request_age[e]), ties by env id.  An env that starts
// waiting in launch L is then admitted by round L + ceil(n / cap) - 1 (every round admits cap envs
// that were ahead of it, and later requests never are), so per-env progress is a function of the
// data and the capacity, not of wave scheduling (an atomic append decided it before round 4).
//
// The step kernel keeps the ages (age + 1 for an env that ends the launch waiting, else 0) and
// publishes, per 64-env group, the waiting envs per age bucket (kAgeBuckets wave ballots,
// publish_ages in sit_impl.h).  k_policy_admit then needs no global synchronisation: every block
// reads the whole count table (32 KB at 32 768 envs, L2-resident), sums the buckets, finds the cutoff
// bucket from the oldest down, and scans the groups in order for the first queue row of its own
// groups and how many of their cutoff-bucket envs get in; each of its waves then ranks its group's
// lanes with two ballots and writes their queue rows in env order with the observation each env
// waits at (last_obs) and its event's normal draw, and clears the admitted envs' ages.  (A separate
// one-block plan kernel measured 8.6 us per launch, latency-bound; redundant plans cost ~32 KB of L2
// reads per block.)  Ages 1..kAgeBuckets-1 are ordered exactly; older ones share the last bucket
// (env-id order there), which the FIFO bound keeps unreachable while ceil(n / cap) < kAgeBuckets.
// ------------------------------------------------------------------------------------------
constexpr int kAdmitThreads = 256;                             // 4 waves = 4 env groups per block
constexpr int kAdmitGroups = kAdmitThreads / kAdmitGroup;
constexpr int kAdmitPerThread = 2;                             // groups per thread and pass of the plan
constexpr int kAdmitPass = kAdmitThreads * kAdmitPerThread;    // 512 groups = 32 768 envs per pass

// exclusive prefix over the block (kAdmitThreads threads, thread order); *total = block sum.  s[8].
__device__ __forceinline__ int admit_scan(int v, int* s, int* total) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
  constexpr int kW = kAdmitThreads / kWave;
  int x = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) s[w] = x;
  __syncthreads();
  int before = x - v, tot = 0;
#pragma unroll
  for (int i = 0; i < kW; ++i) {
    before += i < w ? s[i] : 0;
    tot += s[i];
  }
  *total = tot;
  __syncthreads();   // s reusable
  return before;
}

// the age-bucket counts of group g (zeros past the last group)
__device__ __forceinline__ void admit_row(const int32_t* __restrict__ counts, int g, int n_groups, int* row) {
  if (g < n_groups) {
    const int4* p = reinterpret_cast<const int4*>(counts + (size_t)g * kAgeBuckets);
#pragma unroll
    for (int i = 0; i < kAgeBuckets / 4; ++i) {
      const int4 x = p[i];
      row[4 * i] = x.x; row[4 * i + 1] = x.y; row[4 * i + 2] = x.z; row[4 * i + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int b = 0; b < kAgeBuckets; ++b) row[b] = 0;
  }
}

template <typename T>
__global__ __launch_bounds__(kAdmitThreads) void k_policy_admit(const KArgs<T> a, int cap,
                                                                const int32_t* __restrict__ counts,
                                                                int32_t* __restrict__ age, int32_t* __restrict__ req_env,
                                                                int32_t* __restrict__ req_count, T* __restrict__ obs,
                                                                T* __restrict__ noise) {
  static_assert(kAgeBuckets % 4 == 0 && kAgeBuckets <= kWave, "bucket layout");
  __shared__ int s[8];
  __shared__ int tot[kAgeBuckets];
  __shared__ int cut[2];
  __shared__ int my_plan[kAdmitGroups][2];   // this block's groups: first queue row, admitted cutoff envs
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t >> 6;
  const int n_env = a.n_env;
  const int n_groups = (n_env + kAdmitGroup - 1) / kAdmitGroup;
  // this wave's env (issued first: its load overlaps the plan)
  const int g_me = blockIdx.x * kAdmitGroups + w;
  const int e = g_me * kAdmitGroup + lane;
  const bool in = e < n_env;
  const int32_t a1 = in ? age[e] : 0;
  if (t < kAgeBuckets) tot[t] = 0;
  // bucket totals over every group
  int rows[kAdmitPerThread][kAgeBuckets];
#pragma unroll
  for (int j = 0; j < kAdmitPerThread; ++j) admit_row(counts, t * kAdmitPerThread + j, n_groups, rows[j]);
  int acc[kAgeBuckets];
#pragma unroll
  for (int b = 0; b < kAgeBuckets; ++b) acc[b] = rows[0][b] + rows[1][b];
  for (int p0 = kAdmitPass; p0 < n_groups; p0 += kAdmitPass) {
#pragma unroll
    for (int j = 0; j < kAdmitPerThread; ++j) {
      int r[kAgeBuckets];
      admit_row(counts, p0 + t * kAdmitPerThread + j, n_groups, r);
#pragma unroll
      for (int b = 0; b < kAgeBuckets; ++b) acc[b] += r[b];
    }
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < kAgeBuckets; ++b) {
    int x = acc[b];
#pragma unroll
    for (int off = kWave / 2; off >= 1; off >>= 1) x += __shfl_xor(x, off);
    if (lane == 0 && x) atomicAdd(&tot[b], x);
  }
  __syncthreads();
  if (t == 0) {   // the cutoff, oldest bucket first
    int total = 0;
    for (int b = 0; b < kAgeBuckets; ++b) total += tot[b];
    int bcut = 1, rem = 0x7fffffff;   // default: every waiting env is admitted
    if (total > cap) {
      int cum = 0;
      for (int b = kAgeBuckets; b >= 1; --b) {
        if (cum + tot[b - 1] >= cap) { bcut = b; rem = cap - cum; break; }
        cum += tot[b - 1];
      }
    }
    cut[0] = bcut; cut[1] = rem;
    if (blockIdx.x == 0) *req_count = min(total, cap);
  }
  __syncthreads();
  const int bcut = cut[0], rem = cut[1];
  // every group in order: the cutoff-bucket envs before it and the queue rows before it
  int pre_base = 0, row_base = 0;
  for (int p0 = 0; p0 < n_groups; p0 += kAdmitPass) {
    int cc[kAdmitPerThread], above[kAdmitPerThread];
#pragma unroll
    for (int j = 0; j < kAdmitPerThread; ++j) {
      int r[kAgeBuckets];
      if (p0 == 0) {
#pragma unroll
        for (int b = 0; b < kAgeBuckets; ++b) r[b] = rows[j][b];
      } else {
        admit_row(counts, p0 + t * kAdmitPerThread + j, n_groups, r);
      }
      cc[j] = 0; above[j] = 0;
#pragma unroll
      for (int b = 1; b <= kAgeBuckets; ++b) {
        cc[j] += b == bcut ? r[b - 1] : 0;
        above[j] += b > bcut ? r[b - 1] : 0;
      }
    }
    int tc, ta;
    int pre = pre_base + admit_scan(cc[0] + cc[1], s, &tc);
    int cq[kAdmitPerThread], adm[kAdmitPerThread];
#pragma unroll
    for (int j = 0; j < kAdmitPerThread; ++j) {
      cq[j] = max(0, min(cc[j], rem - pre));
      adm[j] = above[j] + cq[j];
      pre += cc[j];
    }
    int base = row_base + admit_scan(adm[0] + adm[1], s, &ta);
#pragma unroll
    for (int j = 0; j < kAdmitPerThread; ++j) {
      const int g = p0 + t * kAdmitPerThread + j;
      const int k = g - blockIdx.x * kAdmitGroups;
      if (k >= 0 && k < kAdmitGroups) { my_plan[k][0] = base; my_plan[k][1] = cq[j]; }
      base += adm[j];
    }
    pre_base += tc;
    row_base += ta;
  }
  __syncthreads();
  if (g_me >= n_groups) return;
  // this wave's group: ranks by ballot, rows in env order
  const int gbase = my_plan[w][0], gcq = my_plan[w][1];
  const bool waiting = a1 > 0;
  const int b = age_bucket(a1);
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int rank = (int)__popcll(__ballot(waiting && b == bcut) & lt);
  const bool admit = waiting && (b > bcut || (b == bcut && rank < gcq));
  const int row = gbase + (int)__popcll(__ballot(admit) & lt);
  if (!admit) return;
  // (loading every lane's observation before the plan, to overlap its latency, measured no faster)
  T v[SIT_OBS_DIM];
#pragma unroll
  for (int k = 0; k < SIT_OBS_DIM; ++k) v[k] = a.st.last_obs[(size_t)k * n_env + e];
  const uint32_t ev = a.st.event[e];
  req_env[row] = e;
  age[e] = 0;
#pragma unroll
  for (int k = 0; k < SIT_OBS_DIM; ++k) obs[(size_t)row * SIT_OBS_DIM + k] = v[k];
  noise[row] = (T)sampler_normal(a.io.seed, (uint64_t)(a.io.env_id_offset + e), ev);
}

template <typename T>
int launch_policy_admit(sit_handle* h, const sit_rollout_args* ra, hipStream_t stream) {
  static_assert(kAdmitPerThread == 2, "admit_scan sums two groups per thread");
  const int n_groups = (h->n_env + kAdmitGroup - 1) / kAdmitGroup;
  KArgs<T> a = make_args<T>(h);
  a.io.seed = ra->seed;
  a.io.env_id_offset = ra->env_id_offset;
  const int blocks = (n_groups + kAdmitGroups - 1) / kAdmitGroups;
  hipLaunchKernelGGL(k_policy_admit<T>, dim3(blocks), dim3(kAdmitThreads), 0, stream, a, ra->request_capacity,
                     admit_counts(h), ra->request_age, ra->request_env, ra->request_count, (T*)ra->request_obs,
                     (T*)ra->request_noise);
  return SIT_OK;
}

template <typename T>
int launch_policy_actor(sit_handle* h, int cap, const float* w, const void* obs, const void* noise,
                        const int32_t* req_env, const int32_t* req_count, int det, void* act, int32_t* ready,
                        int64_t* served, int32_t* clear_count, hipStream_t stream) {
  const int blocks = (cap + kActorRows - 1) / kActorRows;
  hipLaunchKernelGGL(k_policy_actor<T>, dim3(blocks), dim3(kActorHidden), 0, stream, cap, w, (const T*)obs,
                     (const T*)noise, req_env, req_count, det, (T*)act, ready, h->n_env,
                     reinterpret_cast<unsigned long long*>(served), clear_count);
  return SIT_OK;
}

}  // namespace
