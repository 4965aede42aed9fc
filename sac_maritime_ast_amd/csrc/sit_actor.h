// sit_actor.h — the SAC-AST actor fused into one kernel (sit_policy_actor, include/sit.h).
//
// Policy mode (config C5) evaluates the Gaussian policy on the envs that queued a request during
// the last fused env launch: ast_core/nn_models/mlp.py:95-148 (ReLU MLP, obs 10 -> 256 -> 256 ->
// 2 = (mu, log_sigma)), the squashed Gaussian head of ast_core/distributions/normal.py:88-101 and
// ast_core/policies/gaussian_policy.py:71-72, then the scatter into the env action slots.  As
// separate library GEMMs plus elementwise kernels that was ~8 launches per act, ~40 % of C5's GPU
// time; here it is one launch whose blocks past the device-side request count exit at once.
//
// Layout: one block of 256 threads (4 waves) per kActorRows request rows; thread j owns hidden
// unit j of both layers.  Layer 1 reads the rows' observations from LDS; layer 2 streams W2^T
// (row k = the 256 weights of input k, so one k is one coalesced 1 KiB read, L2-resident across
// blocks) against the rows' layer-1 activations (LDS broadcast reads), two rows per packed FMA;
// layer 3 is a block reduction (lane shuffles, then LDS across the waves).  FP32 throughout (the
// reference actor's dtype); summation order differs from a GEMM library's, within 1e-5.
#pragma once

#include "sit_device.h"

namespace {

constexpr int kActorObs = SIT_OBS_DIM;
constexpr int kActorHidden = SIT_ACTOR_HIDDEN;
constexpr int kActorRows = 8;
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

template <typename T>
__global__ __launch_bounds__(256) void k_policy_actor(int cap, const float* __restrict__ w, const T* __restrict__ obs,
                                                      const T* __restrict__ noise, const int32_t* __restrict__ req_env,
                                                      int32_t* req_count, int deterministic, T* policy_action,
                                                      int32_t* policy_ready, int n_env, unsigned long long* served,
                                                      int32_t* blocks_done) {
  __shared__ float s_obs[kActorRows][kActorObs];
  __shared__ __align__(16) float s_h1[kActorRows][kActorHidden];
  __shared__ float s_red[4][2 * kActorRows];
  const int j = threadIdx.x;
  const int count = min(*req_count, cap);
  const int row0 = blockIdx.x * kActorRows;
  if (blockIdx.x == 0 && j == 0 && served) atomicAdd(served, (unsigned long long)max(count, 0));
  if (row0 < count) {
    const int nrow = min(kActorRows, count - row0);
    if (j < kActorRows * kActorObs) {
      const int r = j / kActorObs, i = j % kActorObs;
      s_obs[r][i] = r < nrow ? (float)obs[(size_t)(row0 + r) * kActorObs + i] : 0.0f;
    }
    __syncthreads();
    // layer 1: h1 = relu(W1 obs + b1)
    {
      float wr[kActorObs];
#pragma unroll
      for (int i = 0; i < kActorObs; ++i) wr[i] = w[kActorW1 + j * kActorObs + i];
      const float b = w[kActorB1 + j];
#pragma unroll
      for (int r = 0; r < kActorRows; ++r) {
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < kActorObs; ++i) acc = fmaf(wr[i], s_obs[r][i], acc);
        s_h1[r][j] = fmaxf(acc + b, 0.0f);
      }
    }
    __syncthreads();
    // layer 2: h2 = relu(W2 h1 + b2), rows in pairs (packed FMA)
    f32x2 acc[kActorRows / 2];
#pragma unroll
    for (int p = 0; p < kActorRows / 2; ++p) acc[p] = f32x2{0.0f, 0.0f};
    const float* w2t = w + kActorW2T + j;
#pragma unroll 2
    for (int k = 0; k < kActorHidden; k += 4) {
      const float w0 = w2t[(k + 0) * kActorHidden], w1 = w2t[(k + 1) * kActorHidden];
      const float w2 = w2t[(k + 2) * kActorHidden], w3 = w2t[(k + 3) * kActorHidden];
#pragma unroll
      for (int p = 0; p < kActorRows / 2; ++p) {
        const float4 ha = *reinterpret_cast<const float4*>(&s_h1[2 * p][k]);
        const float4 hb = *reinterpret_cast<const float4*>(&s_h1[2 * p + 1][k]);
        acc[p] = __builtin_elementwise_fma(f32x2{ha.x, hb.x}, f32x2{w0, w0}, acc[p]);
        acc[p] = __builtin_elementwise_fma(f32x2{ha.y, hb.y}, f32x2{w1, w1}, acc[p]);
        acc[p] = __builtin_elementwise_fma(f32x2{ha.z, hb.z}, f32x2{w2, w2}, acc[p]);
        acc[p] = __builtin_elementwise_fma(f32x2{ha.w, hb.w}, f32x2{w3, w3}, acc[p]);
      }
    }
    const float b2 = w[kActorB2 + j];
    const float v0 = w[kActorW3 + j], v1 = w[kActorW3 + kActorHidden + j];
    // layer 3 partials: out[r][o] = b3[o] + sum_j W3[o][j] h2[r][j]
    float part[2 * kActorRows];
#pragma unroll
    for (int p = 0; p < kActorRows / 2; ++p) {
      const float h0 = fmaxf(acc[p].x + b2, 0.0f), h1 = fmaxf(acc[p].y + b2, 0.0f);
      part[4 * p + 0] = h0 * v0;
      part[4 * p + 1] = h0 * v1;
      part[4 * p + 2] = h1 * v0;
      part[4 * p + 3] = h1 * v1;
    }
#pragma unroll
    for (int q = 0; q < 2 * kActorRows; ++q) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) part[q] += __shfl_xor(part[q], off, 64);
    }
    if ((j & 63) == 0) {
#pragma unroll
      for (int q = 0; q < 2 * kActorRows; ++q) s_red[j >> 6][q] = part[q];
    }
    __syncthreads();
    if (j < nrow) {
      const int r = j;
      const float mu = w[kActorB3 + 0] + ((s_red[0][2 * r] + s_red[1][2 * r]) + (s_red[2][2 * r] + s_red[3][2 * r]));
      const float ls_raw = w[kActorB3 + 1] + ((s_red[0][2 * r + 1] + s_red[1][2 * r + 1]) +
                                              (s_red[2][2 * r + 1] + s_red[3][2 * r + 1]));
      // normal.py:88-101 (log_sigma clipped to [-20, 2], reparameterised sample), tanh squash
      const float ls = fminf(fmaxf(ls_raw, -20.0f), 2.0f);
      const int q = row0 + r;
      const float x = deterministic ? mu : fmaf(expf(ls), (float)noise[q], mu);
      const int e = req_env[q];
      if (e >= 0 && e < n_env) {
        policy_action[e] = (T)tanhf(x);
        policy_ready[e] = 1;
      }
    }
  }
  // the last block to finish clears the request count for the next env launch
  if (blocks_done) {
    __syncthreads();
    if (j == 0) {
      __threadfence();
      if (atomicAdd(blocks_done, 1) == (int)gridDim.x - 1) {
        atomicExch(req_count, 0);
        atomicExch(blocks_done, 0);
      }
    }
  }
}

template <typename T>
int launch_policy_actor(sit_handle* h, int cap, const float* w, const void* obs, const void* noise,
                        const int32_t* req_env, int32_t* req_count, int det, void* act, int32_t* ready,
                        int64_t* served, int32_t* blocks_done, hipStream_t stream) {
  const int blocks = (cap + kActorRows - 1) / kActorRows;
  hipLaunchKernelGGL(k_policy_actor<T>, dim3(blocks), dim3(kActorHidden), 0, stream, cap, w, (const T*)obs,
                     (const T*)noise, req_env, req_count, det, (T*)act, ready, h->n_env,
                     reinterpret_cast<unsigned long long*>(served), blocks_done);
  return SIT_OK;
}

}  // namespace
