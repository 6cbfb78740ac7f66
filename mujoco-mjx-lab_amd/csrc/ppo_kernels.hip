// PPO host-loop kernels (reference train_ppo.py), same translation unit as capi.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace mjl {

// GAE reverse scan (train_ppo.py:171-202 compute_gae), one lane per env. Inputs [T, B] row-major
// (values [T+1, B]); each time step's loads are independent of the carry, so the unrolled loop
// issues them ahead of the serial recurrence. Contraction is off so every op rounds as the
// reference's elementwise jnp expression does: bit-identical to the torch restatement. gl is
// gamma * lam formed in double on the host, as the Python expression `gamma * lam * (...)` does.
#pragma clang fp contract(off)
__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                  const float* __restrict__ term, const float* __restrict__ trunc,
                                                  int T, int B, float gamma, float gl, float* __restrict__ adv,
                                                  float* __restrict__ ret) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float carry = 0.f;
  float vnext = val[(size_t)T * B + b];
  int t = T - 1;
  constexpr int U = 8;
  for (; t >= U - 1; t -= U) {
    float r[U], v[U], te[U], tr[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t o = (size_t)(t - u) * B + b;
      r[u] = rew[o]; v[u] = val[o]; te[u] = term[o]; tr[u] = trunc[o];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t o = (size_t)(t - u) * B + b;
      const float delta = r[u] + gamma * vnext * (1.f - te[u]) - v[u];
      carry = delta + gl * (1.f - fmaxf(te[u], tr[u])) * carry;
      adv[o] = carry;
      ret[o] = carry + v[u];
      vnext = v[u];
    }
  }
  for (; t >= 0; t--) {
    const size_t o = (size_t)t * B + b;
    const float v = val[o], te = term[o];
    const float delta = rew[o] + gamma * vnext * (1.f - te) - v;
    carry = delta + gl * (1.f - fmaxf(te, trunc[o])) * carry;
    adv[o] = carry;
    ret[o] = carry + v;
    vnext = v;
  }
}
#pragma clang fp contract(on)

// Rollout-step elementwise work of train_ppo.py:128-169 in two launches instead of ~20 torch ops.
// normalize_obs + clip (training_utils.py:52-56, train_ppo.py:134-135): y = clip((x - mean) /
// sqrt(var + 1e-8), -clip, clip).
#pragma clang fp contract(off)
__global__ __launch_bounds__(256) void obs_normalize_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                                            const float* __restrict__ var, int n, int dim, float clip,
                                                            float* __restrict__ y) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * dim) return;
  const int j = t % dim;
  const float v = __fdiv_rn(x[t] - mean[j], __fsqrt_rn(var[j] + 1e-8f));
  y[t] = fminf(fmaxf(v, -clip), clip);
}

// Gaussian policy head (networks.py:82-112 GaussianPolicy, train_ppo.py:121-126,136-139), one lane
// per env: mean = tanh(z), s = clip(log_std, -20, 2), act = mean + exp(s) eps,
// logp = -0.5 sum_j ((act - mean)^2 / exp(2 s) + 2 s + log 2 pi).
__global__ __launch_bounds__(256) void policy_head_kernel(const float* __restrict__ z, const float* __restrict__ log_std,
                                                          const float* __restrict__ eps, int B, int A,
                                                          float* __restrict__ act, float* __restrict__ logp) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float log2pi = 1.8378770664093453f;
  float acc = 0.f;
  for (int j = 0; j < A; j++) {
    const size_t o = (size_t)b * A + j;
    const float s = fminf(fmaxf(log_std[j], -20.f), 2.f);
    const float mu = tanhf(z[o]);
    const float a = mu + expf(s) * eps[o];
    act[o] = a;
    const float d = a - mu;
    acc += __fdiv_rn(d * d, expf(2.f * s)) + 2.f * s + log2pi;
  }
  logp[b] = -0.5f * acc;
}
#pragma clang fp contract(on)

// Column sums of a row-major [n, d] matrix (the PPO update's bias gradients dY.sum(0) over a
// 65,536-row minibatch, and the split-K weight-gradient sum over its splits), in a fixed order.
// A 256-thread block covers a tile of dc = min(d, tile) columns with G = 256 / dc row groups;
// blockIdx.y takes rows [y * chunk, (y + 1) * chunk), row group g the rows g, g + G, ... of it,
// eight independent partial sums per thread so the loads of a trip issue together. The G group
// sums combine through LDS in group order; the block writes out[y][col] (one row per chunk: the
// caller reduces those rows again when there is more than one). torch's sum(0) takes 33 us for
// [65536, 256] and 169 us for [65536, 21] on MI355X (tools/colsum_probe.py).
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ x, int n, int d, int dc, int chunk,
                                                     float* __restrict__ out) {
  __shared__ float red[256];
  const int G = 256 / dc, t = threadIdx.x, g = t / dc, c = t - g * dc;
  const int col = blockIdx.x * dc + c;
  const int r0 = blockIdx.y * chunk, r1 = min(n, r0 + chunk);
  float s = 0.f;
  if (g < G && col < d) {
    constexpr int U = 8;
    float p[U];
#pragma unroll
    for (int u = 0; u < U; u++) p[u] = 0.f;
    int r = r0 + g;
    for (; r + (U - 1) * G < r1; r += U * G) {
#pragma unroll
      for (int u = 0; u < U; u++) p[u] += x[(size_t)(r + u * G) * d + col];
    }
    for (; r < r1; r += G) p[0] += x[(size_t)r * d + col];
    s = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
  }
  red[t] = s;
  __syncthreads();
  if (t < dc && col < d) {
    float acc = red[t];
    for (int q = 1; q < G; q++) acc += red[q * dc + t];
    out[(size_t)blockIdx.y * d + col] = acc;
  }
}

// launch geometry shared by mjl_colsum and mjl_colsum_scratch: stage 1 over the rows in chunks of
// 128 (one chunk when n <= 256), stage 2 (when there is more than one chunk) over the chunk rows
// with 16-column tiles, i.e. 16 row groups per column
struct ColsumPlan {
  int dc1, chunk, R, dc2;
  ColsumPlan(int n, int d) {
    dc1 = d < 256 ? d : 256;
    chunk = n <= 256 ? (n > 0 ? n : 1) : 128;
    R = (n + chunk - 1) / chunk;
    dc2 = d < 16 ? d : 16;
  }
};

}  // namespace mjl
