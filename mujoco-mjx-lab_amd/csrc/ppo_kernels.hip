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

}  // namespace mjl
