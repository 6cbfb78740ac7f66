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

}  // namespace mjl
