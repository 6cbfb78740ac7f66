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
// (apg.py _loss_and_grad, in the same order of float operations), from env e's wave: fin = this lane's
// qpos / qvel entries are finite, vmax = their max |qvel|; the finite test by ballot, max |qvel| by a
// wave max (fmaxf is order-free: the serial loop's value); lane 0 updates the env's scalars (r, te,
// tr: its reward, terminated and truncated flags). Shared by apg_post_kernel and the APG record kernel
// (adjoint.hip vjp_record_kernel, which runs it on the state it just wrote back).
struct ApgPostArgs {
  float gamma, diverge_qvel;
  uint8_t* alive;  // null: no post-step update
  float *disc, *ret, *dropped, *grew, *rfin;
  int B;
};
// env e's scalars before the update (loaded where the caller can hide their latency)
struct ApgPostEnv {
  bool alive;
  float disc, ret, dropped;
};
__device__ __forceinline__ ApgPostEnv apg_post_load(const ApgPostArgs& a, int e) {
  return ApgPostEnv{a.alive[e] != 0, a.disc[e], a.ret[e], a.dropped[e]};
}
// (returns the env's new alive flag in lane 0)
__device__ __forceinline__ bool apg_post_wave(const ApgPostArgs& a, int e, int lane, bool fin, float vmax, float r,
                                              float te, float tr, const ApgPostEnv& pe) {
  const bool allfin = __ballot(!fin) == 0ull;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
  if (lane != 0) return false;
  bool ok = isfinite(r) && allfin;
  if (a.diverge_qvel > 0.f) ok = ok && vmax <= a.diverge_qvel;
  bool al = pe.alive;
  const bool bad = al && !ok;
  if (bad) a.dropped[e] = pe.dropped + 1.f;
  al = al && !bad;
  const float d = al ? pe.disc : 0.f;
  a.grew[e] = div_rn(-d, (float)a.B);
  a.ret[e] = pe.ret + (al ? d * r : 0.f);
  a.rfin[e] = isfinite(r) ? r : 0.f;
  const float nd = d * a.gamma * (1.f - fmaxf(te, tr));
  a.disc[e] = nd;
  a.alive[e] = al && nd != 0.f;
  return al && nd != 0.f;
}

// One wave per env: lane j loads qpos[j] / qvel[j] (coalesced). (A thread per env looped over the env's
// nq + nv words: 55 strided loads per lane, 9.4 us per 2048-env launch on 8 workgroups.)
constexpr int kPostEnvs = 4;  // envs (waves) per block
__global__ __launch_bounds__(64 * kPostEnvs) void apg_post_kernel(StateBuf S, int nq, int nv, const float* __restrict__ rew,
                                                                  const float* __restrict__ term,
                                                                  const float* __restrict__ trunc, ApgPostArgs a) {
  const int lane = threadIdx.x & 63, e = blockIdx.x * kPostEnvs + (threadIdx.x >> 6);
  if (e >= a.B) return;  // wave-uniform
  bool fin = true;
  float vmax = 0.f;
  for (int j = lane; j < nq; j += 64) fin &= isfinite(S.qpos[(size_t)e * nq + j]);
  for (int j = lane; j < nv; j += 64) {
    const float v = S.qvel[(size_t)e * nv + j];
    fin &= isfinite(v);
    vmax = fmaxf(vmax, fabsf(v));
  }
  apg_post_wave(a, e, lane, fin, vmax, rew[e], term[e], trunc[e], apg_post_load(a, e));
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

// The APG policy's per-step passes (networks.py:63-80: a tanh MLP with a tanh-squashed output;
// mjx_amd APGPolicy) as one launch each, where torch ran three GEMMs and three tanh launches forward
// and three GEMMs and three tanh-backward launches for the observation cotangent (~4.5 us each at
// 2048 rows: 12 launches per rollout step). A block takes kSmlThreads / U rows, thread (row, unit
// < U) one output unit; each layer's weights are staged through LDS (transposed for the forward so
// the units read consecutive words), activations through LDS, sums in k order from the bias.
// (Measured slower and not kept: every layer's weights, biases and stored activations loaded at the
// kernel's start, 10.0 -> 11.0 us forward and 8.1 -> 8.9 us backward (fused forms); each layer's
// weights loaded into registers with all loads issued together and the next layer's loaded during
// this one, 8.2 -> 11.4 us forward and 7.2 -> 8.9 us backward (plain forms, tools/prof_target.py apgmlp).)
constexpr int kSmlMaxW = 64, kSmlMaxL = 4, kSmlThreads = 256;
struct SmallMlp {
  int nl, k0, u;            // layers, input width, units per row slot (32 or 64: >= every width)
  int n[kSmlMaxL];          // layer widths; layer l reads k = l ? n[l - 1] : k0
  const float* w[kSmlMaxL];  // [n_l, k_l] row-major (torch Linear.weight)
  const float* b[kSmlMaxL];
  float* y[kSmlMaxL];       // [B, n_l] tanh outputs: written by the forward, read by the backward
};

// the APG observation feeding the policy forward (mjl_apg_obs_policy_fwd): apg_obs_kernel's o / on /
// alive_snap for the block's rows, written as there, with on staged as the first layer's input
struct ObsIn {
  const float *qpos, *qvel;
  int nq, nv, use_norm;
  const uint8_t* alive;
  const float *mean, *var;
  float *o, *on;
  uint8_t* snap;
};
// the next rollout step's observation and policy forward, fused into the APG record after its post-step
// update (mjl_env_step_record_apg_next): mjl_apg_obs_policy_fwd's o / on / alive_snap and layer outputs
// for this env, the same float operations; P.w[l] hold the layers' weights TRANSPOSED ([k_l, n_l], so
// the wave's lanes read a k row coalesced); o null: none
struct ApgNextArgs {
  int use_norm;
  const float *mean, *var;
  float *o, *on;
  uint8_t* snap;
  SmallMlp P;
};
// the policy's input backward + the observation's backward (mjl_apg_policy_bwd_obs_vjp's arithmetic) fused
// into the APG replay's tail (mjl_env_step_vjp_replay_apg): P.w row-major as the torch weights, P.y the
// step's layer outputs; o / alive_snap the step's observation and flags; P.nl 0: none
struct ApgPolicyBwd {
  int use_norm;
  const float *o, *mean, *var;
  const uint8_t* snap;
  SmallMlp P;
};
// the observation's backward fused into the policy's input backward (mjl_apg_policy_bwd_obs_vjp):
// apg_obs_vjp_kernel on the input cotangent where small_mlp_bwd_input_kernel wrote g_x
struct ObsVjp {
  int nq, nv, use_norm;
  const float* o;
  const uint8_t* snap;
  const float *mean, *var;
  float *g_qpos, *g_qvel;
};

template <bool OBS>
__global__ __launch_bounds__(kSmlThreads) void small_mlp_fwd_kernel(const float* __restrict__ x, int B, SmallMlp P,
                                                                    ObsIn O) {
  __shared__ float wt[kSmlMaxW * kSmlMaxW];
  __shared__ float h[2][kSmlThreads / 32][kSmlMaxW];
  const int U = P.u, R = kSmlThreads / U, t = threadIdx.x, r = t / U, j = t - r * U;
  const int row0 = blockIdx.x * R, row = row0 + r;
  for (int e = t; e < R * P.k0; e += kSmlThreads) {
    const int rr = e / P.k0, k = e - rr * P.k0, rw = row0 + rr;
    if constexpr (OBS) {  // apg_obs_kernel's element (rw, k), the same float operations
      float in = 0.f;
      if (rw < B) {
        const size_t i = (size_t)rw * P.k0 + k;
        const float v = k < O.nq ? O.qpos[(size_t)rw * O.nq + k] : O.qvel[(size_t)rw * O.nv + (k - O.nq)];
        const bool al = O.alive[rw] != 0;
        O.o[i] = v;
        const float xv = al ? v : 0.f;
        in = O.use_norm ? clamp_keep_nan(div_rn(xv - O.mean[k], sqrt_rn(O.var[k]) + 1e-8f), 10.f) : xv;
        O.on[i] = in;
        if (k == 0) O.snap[rw] = al;
      }
      h[0][rr][k] = in;
    } else {
      h[0][rr][k] = rw < B ? x[(size_t)rw * P.k0 + k] : 0.f;
    }
  }
  int K = P.k0, cur = 0;
  for (int l = 0; l < P.nl; l++) {
    const int N = P.n[l];
    const float* __restrict__ W = P.w[l];
    __syncthreads();  // the previous layer's activations written, its weights no longer read
    for (int e = t; e < N * K; e += kSmlThreads) {
      const int jj = e / K, k = e - jj * K;
      wt[k * N + jj] = W[e];
    }
    __syncthreads();
    if (j < N) {
      float s = P.b[l][j];
      for (int k = 0; k < K; k++) s = fmaf(wt[k * N + j], h[cur][r][k], s);
      const float y = tanhf(s);
      h[cur ^ 1][r][j] = y;
      if (row < B) P.y[l][(size_t)row * N + j] = y;
    }
    cur ^= 1;
    K = N;
  }
}

// d loss / d x from d loss / d y_L (ga): g = ga (1 - y_L^2), then per layer from the top
// g_in = W_l^T g, times (1 - y_{l-1}^2) below the first layer; gx = W_0^T g
template <bool OBS>
__global__ __launch_bounds__(kSmlThreads) void small_mlp_bwd_input_kernel(const float* __restrict__ ga, int B,
                                                                          SmallMlp P, float* __restrict__ gx,
                                                                          ObsVjp O) {
  __shared__ float wl[kSmlMaxW * kSmlMaxW];
  __shared__ float g[2][kSmlThreads / 32][kSmlMaxW];
  const int U = P.u, R = kSmlThreads / U, t = threadIdx.x, r = t / U, u = t - r * U;
  const int row = blockIdx.x * R + r;
  const int L = P.nl, NL = P.n[L - 1];
  if (u < NL) {
    const float y = row < B ? P.y[L - 1][(size_t)row * NL + u] : 0.f;
    g[0][r][u] = row < B ? ga[(size_t)row * NL + u] * (1.f - y * y) : 0.f;
  }
  int cur = 0;
  for (int l = L - 1; l >= 0; l--) {
    const int N = P.n[l], K = l ? P.n[l - 1] : P.k0;
    const float* __restrict__ W = P.w[l];
    __syncthreads();
    for (int e = t; e < N * K; e += kSmlThreads) wl[e] = W[e];
    __syncthreads();
    if (u < K) {
      float s = 0.f;
      for (int jj = 0; jj < N; jj++) s = fmaf(wl[jj * K + u], g[cur][r][jj], s);
      if (l) {
        const float y = row < B ? P.y[l - 1][(size_t)row * K + u] : 0.f;
        g[cur ^ 1][r][u] = s * (1.f - y * y);
      } else if (row < B) {
        if constexpr (OBS) {  // apg_obs_vjp_kernel's element (row, u) with go = s
          float gg = 0.f;
          if (O.snap[row]) {
            gg = s;
            if (O.use_norm) {
              const float den = sqrt_rn(O.var[u]) + 1e-8f;
              const float y = div_rn(O.o[(size_t)row * K + u] - O.mean[u], den);
              gg = (y >= -10.f && y <= 10.f) ? div_rn(gg, den) : 0.f;
            }
          }
          if (u < O.nq) O.g_qpos[(size_t)row * O.nq + u] = O.g_qpos[(size_t)row * O.nq + u] + gg;
          else O.g_qvel[(size_t)row * O.nv + (u - O.nq)] = O.g_qvel[(size_t)row * O.nv + (u - O.nq)] + gg;
        } else {
          gx[(size_t)row * K + u] = s;
        }
      }
    }
    cur ^= 1;
  }
}

}  // namespace mjl
