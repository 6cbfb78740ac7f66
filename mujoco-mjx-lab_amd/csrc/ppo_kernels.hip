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

// The rollout step's whole policy forward (train_ppo.py:134-139: normalize_obs + clip, the
// GaussianPolicy MLP of src/networks.py:22-61,82-112, the tanh head, sampling and gaussian_logprob)
// as one launch on the matrix cores, instead of the normalisation launch, four library GEMMs,
// three tanh launches and the head launch (~45 us per step at 2048 envs).
// One workgroup of kPolWaves waves per 16 envs. Layer l: Y = act(X W_l^T + b_l), X [16, K] in
// LDS, each wave taking every kPolWaves-th 16-column block of Y as v_mfma_f32_16x16x4_f32 over K in
// chunks of 16: lane group g = lane >> 4 supplies k = 16 c + 4 g + t to MFMA t of chunk c, so the
// lane's A values (X row lane & 15) and B values are 16-B contiguous: the weights come packed as
// WP[k / 4][n][k % 4] (zero-padded to K, N multiples of 16: mjl_policy_pack's layout), b after
// each layer's WP. Output C[4 g + r][n] of a block sits in lane (g, n) register r.
// (A vector-ALU variant, 8 envs per 256-thread workgroup and thread n owning column n, packed weights
// read as b128 per 4 k: twice the workgroups, measured 33.2 against 20.5 us at 1024 envs and 34.1-35.0
// against 21.2 us at 2048; not kept. Split-K of the 21-wide output layer over the 14 waves its two
// column blocks leave idle — each wave 2 of the 16 K chunks, the partials summed through LDS in part
// order — measured 21.2 against 20.3 us at 1024 envs (round 6): the output layer's
// 64-MFMA chain was not on the critical path once the other waves' barriers are counted; not kept.
// Four envs per workgroup on v_mfma_f32_4x4x1_16b_f32, so that 1024 envs fill all 256 CUs, bit-identical
// to this kernel: 18.3-19.0 against 20.3 us at 1024 envs, 22.1-22.4 against 20.3 at 2048 -- the 4x4x1
// form issues at ~40 cycles for a quarter of 16x16x4's MACs, so the CUs gained are spent on issue
// (tools/pol4_kernel.inc, tools/pol_micro.hip, profiles/r6/pol_micro.txt); not kept.)
constexpr int kPolMaxLayers = 6;
constexpr int kPolLdx = 260;  // LDS row stride (floats): rows 4 banks apart, conflict-free b128
#ifndef MJL_POL_WAVES
#define MJL_POL_WAVES 16
#endif
constexpr int kPolWaves = MJL_POL_WAVES;        // waves per 16-env workgroup
constexpr int kPolBpw = 16 / kPolWaves;         // 16-column blocks per wave per pass (256 columns)
#ifndef MJL_POL_PD
#define MJL_POL_PD 4
#endif
constexpr int kPolPD = MJL_POL_PD;  // K chunks (16 k each) of weights and activations in flight per wave
struct PolicyDims {
  int nlayer, obs_dim, act_dim;
  int K[kPolMaxLayers], N[kPolMaxLayers];  // padded (multiples of 16), K[0] >= obs_dim
  long long off[kPolMaxLayers];             // float offset of layer l's WP in the parameter buffer
};
#pragma clang fp contract(off)
__global__ __launch_bounds__(64 * MJL_POL_WAVES) void policy_rollout_kernel(const float* __restrict__ obs, const float* __restrict__ mean,
                                                             const float* __restrict__ var, float clip,
                                                             const float* __restrict__ params, PolicyDims pd,
                                                             const float* __restrict__ log_std,
                                                             const float* __restrict__ eps, int B,
                                                             float* __restrict__ act, float* __restrict__ logp) {
  __shared__ __attribute__((aligned(16))) float X[2][16 * kPolLdx];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * 16;
  {  // normalised, clipped observations (obs_normalize_kernel's arithmetic), zero-padded to K[0]
    const int K0 = pd.K[0], D = pd.obs_dim;
    for (int e = tid; e < 16 * K0; e += 64 * kPolWaves) {
      const int r = e / K0, j = e - r * K0, b = row0 + r;
      float v = 0.f;
      if (j < D && b < B) {
        v = __fdiv_rn(obs[(size_t)b * D + j] - mean[j], __fsqrt_rn(var[j] + 1e-8f));
        v = fminf(fmaxf(v, -clip), clip);
      }
      X[0][r * kPolLdx + j] = v;
    }
  }
  __syncthreads();
  const int g = lane >> 4, c16 = lane & 15;
  int cur = 0;
  typedef float f4 __attribute__((ext_vector_type(4)));
  for (int l = 0; l < pd.nlayer; l++) {
    const int K = pd.K[l], N = pd.N[l];
    const float* WP = params + pd.off[l];
    const float* bias = WP + (size_t)K * N;
    const bool last = l == pd.nlayer - 1;
    const int nblk = N >> 4;
    for (int nb0 = wave; nb0 < nblk; nb0 += kPolWaves * kPolBpw) {  // kPolBpw blocks per wave per pass
      f4 acc[kPolBpw];
      int nbs[kPolBpw];
#pragma unroll
      for (int q = 0; q < kPolBpw; q++) {
        nbs[q] = nb0 + kPolWaves * q;
        acc[q] = (f4){0.f, 0.f, 0.f, 0.f};
      }
      // one chunk (16 k) of A from LDS and B from the packed weights; the next chunk's loads issue
      // before this chunk's MFMAs (two register sets, alternating)
      auto load = [&](int c, f4& a, f4 (&b)[kPolBpw]) {
        a = *(const f4*)&X[cur][c16 * kPolLdx + c + 4 * g];
#pragma unroll
        for (int q = 0; q < kPolBpw; q++) {
          const int nb = nbs[q] < nblk ? nbs[q] : 0;
          b[q] = *(const f4*)&WP[((size_t)((c >> 2) + g) * N + nb * 16 + c16) * 4];
        }
      };
      auto mac = [&](const f4& a, const f4 (&b)[kPolBpw]) {  // the blocks' accumulators alternate
#pragma unroll
        for (int t = 0; t < 4; t++) {
#pragma unroll
          for (int q = 0; q < kPolBpw; q++)
            if (nbs[q] < nblk) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[q][t], acc[q], 0, 0, 0);
        }
      };
      // a ring of kPolPD chunks in flight: chunk c + kPolPD - 1's loads issue before chunk c's MFMAs
      // (one chunk ahead: 21.6 us per 1024-env launch, 22.0 at 2048; three ahead 20.7 / 21.2; five the
      // same as three: tools/r5/gpu_polpd.sh). The MFMA sequence, and so every bit, is unchanged.
      f4 ra[kPolPD], rb[kPolPD][kPolBpw];
      const int nc = K >> 4;
#pragma unroll
      for (int p = 0; p < kPolPD - 1; p++)
        if (p < nc) load(16 * p, ra[p], rb[p]);
      for (int c0 = 0; c0 < nc; c0 += kPolPD) {
#pragma unroll
        for (int p = 0; p < kPolPD; p++) {
          const int c = c0 + p;
          if (c < nc) {
            const int pn = (p + kPolPD - 1) % kPolPD;
            if (c + kPolPD - 1 < nc) load(16 * (c + kPolPD - 1), ra[pn], rb[pn]);
            mac(ra[p], rb[p]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < kPolBpw; q++) {
        if (nbs[q] >= nblk) continue;
        const int n = nbs[q] * 16 + c16;
        const float bn = bias[n];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const float y = acc[q][r] + bn;
          X[cur ^ 1][(4 * g + r) * kPolLdx + n] = last ? y : tanhf(y);
        }
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  // head (policy_head_kernel's arithmetic): one thread per (env, action) for the action and its
  // log-density term, then one thread per env sums its terms in action order
  {
    const int A = pd.act_dim;
    const float log2pi = 1.8378770664093453f;
    float* term = &X[cur ^ 1][0];  // the other activation buffer is free now
    for (int e = tid; e < 16 * A; e += 64 * kPolWaves) {
      const int r = e / A, j = e - r * A, b = row0 + r;
      if (b < B) {
        const size_t o = (size_t)b * A + j;
        const float s = fminf(fmaxf(log_std[j], -20.f), 2.f);
        const float mu = tanhf(X[cur][r * kPolLdx + j]);
        const float a = mu + expf(s) * eps[o];
        act[o] = a;
        const float d = a - mu;
        term[r * kPolLdx + j] = __fdiv_rn(d * d, expf(2.f * s)) + 2.f * s + log2pi;
      }
    }
    __syncthreads();
    if (tid < 16 && row0 + tid < B) {
      float accl = 0.f;
      for (int j = 0; j < A; j++) accl += term[tid * kPolLdx + j];
      logp[row0 + tid] = -0.5f * accl;
    }
  }
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
// with 4-column tiles, i.e. 64 row groups per column (at 65,536 rows: 512 chunk rows, one trip of 8
// loads per thread; 16-column tiles took 4 dependent trips, 12 us)
struct ColsumPlan {
  int dc1, chunk, R, dc2;
  ColsumPlan(int n, int d) {
    dc1 = d < 256 ? d : 256;
    chunk = n <= 256 ? (n > 0 ? n : 1) : 128;
    R = (n + chunk - 1) / chunk;
    dc2 = d < 4 ? d : 4;
  }
};

// The backward of y = tanh(z) fused with the bias gradient's first column-sum stage (the PPO
// update's hidden layers: [65,536, 256] per minibatch): dz = g (1 - y^2) row-major [n, d], and per
// chunk of `chunk` rows the column sums of dz into out[chunk index][d] (ColsumPlan's stage-1 layout;
// colsum_kernel reduces those rows). Where torch ran tanh_backward (28 us) and then re-read dz for the
// column sum (15-17 us). d % 4 == 0: thread t takes column quad t % dq of a dq-quad tile and rows
// t / dq, + G, ... of the chunk, U rows in flight per trip; the G row-group sums combine through LDS
// in group order (fixed order: deterministic).
__global__ __launch_bounds__(256) void tanh_bwd_colsum_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                              int n, int d, int dq, int chunk, float* __restrict__ dz,
                                                              float* __restrict__ out) {
  __shared__ float4 red[256];
  const int G = 256 / dq, t = threadIdx.x, grp = t / dq, q = t - grp * dq;
  const int col = (blockIdx.x * dq + q) * 4;
  const int r0 = blockIdx.y * chunk, r1 = min(n, r0 + chunk);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (grp < G && col < d) {
    constexpr int U = 4;
    int r = r0 + grp;
    auto one = [&](int row) {
      const size_t o = (size_t)row * d + col;
      const float4 gv = *reinterpret_cast<const float4*>(g + o), yv = *reinterpret_cast<const float4*>(y + o);
      float4 z;
      z.x = gv.x * (1.f - yv.x * yv.x);
      z.y = gv.y * (1.f - yv.y * yv.y);
      z.z = gv.z * (1.f - yv.z * yv.z);
      z.w = gv.w * (1.f - yv.w * yv.w);
      *reinterpret_cast<float4*>(dz + o) = z;
      return z;
    };
    for (; r + (U - 1) * G < r1; r += U * G) {
      float4 z[U];
#pragma unroll
      for (int u = 0; u < U; u++) z[u] = one(r + u * G);
#pragma unroll
      for (int u = 0; u < U; u++) { s.x += z[u].x; s.y += z[u].y; s.z += z[u].z; s.w += z[u].w; }
    }
    for (; r < r1; r += G) {
      const float4 z = one(r);
      s.x += z.x; s.y += z.y; s.z += z.z; s.w += z.w;
    }
  }
  red[t] = s;
  __syncthreads();
  if (t < dq && col < d) {
    float4 acc = red[t];
    for (int k = 1; k < G; k++) {
      const float4 v = red[k * dq + t];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *reinterpret_cast<float4*>(out + (size_t)blockIdx.y * d + col) = acc;
  }
}

}  // namespace mjl
