// APG rollout bookkeeping (mjx_amd/apg.py's native path; reference train_apg.py:161-209): the
// observation + normalisation, the post-step guard / discount / return update, and the
// observation's backward, each one elementwise launch per rollout step instead of ~10-30 torch ops.
#pragma once
#include <hip/hip_runtime.h>

#include "model_dev.h"

namespace mjl {

// IEEE-rounded sqrt and division for the normalisation, as the torch restatement computes them (this
// translation unit is built with -fapprox-func, which lets the compiler emit the 1-ulp
// v_sqrt_f32 / v_rcp_f32 alone; a truncated-solver rollout amplifies one ulp): the hardware
// estimate, then the neighbour / residual correction by fma (finite, normal-range operands)
__device__ __forceinline__ float sqrt_rn(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  if (!(x > 0.f) || !isfinite(x)) return s;
  const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
  if (fmaf(-sd, s, x) <= 0.f) s = sd;
  if (fmaf(-su, s, x) > 0.f) s = su;
  return s;
}
__device__ __forceinline__ float div_rn(float a, float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  const float q0 = a * r;
  const float q1 = fmaf(fmaf(-b, q0, a), r, q0);
  return fmaf(fmaf(-b, q1, a), r, q1);
}

// x clipped to [-c, c] with NaN kept (torch.clamp semantics)
__device__ __forceinline__ float clamp_keep_nan(float x, float c) { return x < -c ? -c : (x > c ? c : x); }

// o = [qpos | qvel] of env e; on = the policy input: x = alive ? o : 0, normalised as
// clip((x - mean) / (sqrt(var) + 1e-8), -10, 10) if use_norm (train_apg.py:171-176); alive_snap
// keeps this step's alive flags for the backward
__global__ void apg_obs_kernel(StateBuf S, int B, int nq, int nv, const uint8_t* __restrict__ alive,
                               const float* __restrict__ mean, const float* __restrict__ var, int use_norm,
                               float* __restrict__ o, float* __restrict__ on, uint8_t* __restrict__ alive_snap) {
  const int w = nq + nv;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * w) return;
  const int e = (int)(i / w), j = (int)(i % w);
  const float v = j < nq ? S.qpos[(size_t)e * nq + j] : S.qvel[(size_t)e * nv + (j - nq)];
  const bool al = alive[e] != 0;
  o[i] = v;
  const float x = al ? v : 0.f;
  on[i] = use_norm ? clamp_keep_nan(div_rn(x - mean[j], sqrt_rn(var[j]) + 1e-8f), 10.f) : x;
  if (j == 0) alive_snap[e] = al;
}

// after env e's step: the non-finite / divergence guard, the discount and the return
// (apg.py _loss_and_grad, in the same order of float operations)
__global__ void apg_post_kernel(StateBuf S, int B, int nq, int nv, const float* __restrict__ rew,
                                const float* __restrict__ term, const float* __restrict__ trunc, float gamma,
                                float diverge_qvel, uint8_t* __restrict__ alive, float* __restrict__ disc,
                                float* __restrict__ ret, float* __restrict__ dropped, float* __restrict__ grew,
                                float* __restrict__ rfin) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B) return;
  const float r = rew[e];
  bool ok = isfinite(r);
  for (int j = 0; j < nq; j++) ok = ok && isfinite(S.qpos[(size_t)e * nq + j]);
  float vmax = 0.f;
  for (int j = 0; j < nv; j++) {
    const float v = S.qvel[(size_t)e * nv + j];
    ok = ok && isfinite(v);
    vmax = fmaxf(vmax, fabsf(v));
  }
  if (diverge_qvel > 0.f) ok = ok && vmax <= diverge_qvel;
  bool al = alive[e] != 0;
  const bool bad = al && !ok;
  if (bad) dropped[e] += 1.f;
  al = al && !bad;
  const float d = al ? disc[e] : 0.f;
  grew[e] = div_rn(-d, (float)B);
  ret[e] = ret[e] + (al ? d * r : 0.f);
  rfin[e] = isfinite(r) ? r : 0.f;
  const float nd = d * gamma * (1.f - fmaxf(term[e], trunc[e]));
  disc[e] = nd;
  alive[e] = al && nd != 0.f;
}

// backward of apg_obs_kernel's on w.r.t. o, accumulated: g_qpos / g_qvel += d on / d o * go
// (where: zero for envs not alive; clamp: zero outside [-10, 10]; the division: go / (sqrt(var) + 1e-8))
__global__ void apg_obs_vjp_kernel(int B, int nq, int nv, const float* __restrict__ o,
                                   const uint8_t* __restrict__ alive_snap, const float* __restrict__ mean,
                                   const float* __restrict__ var, int use_norm, const float* __restrict__ go,
                                   float* __restrict__ g_qpos, float* __restrict__ g_qvel) {
  const int w = nq + nv;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * w) return;
  const int e = (int)(i / w), j = (int)(i % w);
  float g = 0.f;
  if (alive_snap[e]) {
    g = go[i];
    if (use_norm) {
      const float den = sqrt_rn(var[j]) + 1e-8f;
      const float y = div_rn(o[i] - mean[j], den);
      g = (y >= -10.f && y <= 10.f) ? div_rn(g, den) : 0.f;
    }
  }
  if (j < nq) g_qpos[(size_t)e * nq + j] = g_qpos[(size_t)e * nq + j] + g;
  else g_qvel[(size_t)e * nv + (j - nq)] = g_qvel[(size_t)e * nv + (j - nq)] + g;
}

}  // namespace mjl
