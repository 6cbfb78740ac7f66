// The twin PPO update's two thin ends as single launches (mjx_amd/twin.py; reference run_ppo_updates,
// train_ppo.py:233-252, over the src/networks.py:82-131 MLPs). At C5's 8,192-row per-rank minibatch
// each library GEMM on a thin shape is a launch of its own on a ~5 us floor; here:
//
//  * twin_gather_in_kernel: the minibatch gather (the observations written twice, one copy per net,
//    the actions / old log-probs / returns / advantages once) fused with BOTH nets' input layer,
//    H1 = tanh(obs W0^T + b0) — replaces the gather launch, the batched [2, M, K0] x [2, K0, N] GEMM
//    and the bias + tanh pass;
//  * twin_head_bwd_kernel: the output layers' backward fused with the last hidden layer's tanh
//    backward — dZ = (dz W_out) (1 - H^2), its column-sum partials (the hidden bias gradient's first
//    stage) and the output weight gradient's per-chunk partials dz^T H — replaces the split-K output
//    weight-gradient GEMM, the dH GEMM and the tanh-backward pass.
//
// Both are f32 FMA chains in a fixed order (deterministic: graph replays equal eager runs bit for
// bit); the second stages of the partials are summed with every other slice in mjl_slice_sum_multi.
#pragma once
#include <hip/hip_runtime.h>

namespace mjl {

typedef float tw_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ tw_f2 tw_fma(tw_f2 a, float b, tw_f2 c) {
  return __builtin_elementwise_fma(a, tw_f2{b, b}, c);
}

// ------------------------------------------------------------------ gather + input layer
constexpr int kTinRows = 32;  // minibatch rows per block
constexpr int kTinK0 = 54;    // instantiated input width (the humanoid observation)
constexpr int kTinN = 256;    // instantiated hidden width (src/config.json)

struct TwinInArgs {
  const long long* idx;  // [n] row indices, or an [n_minibatches, n] table read at row *idx_row
  const int* idx_row;
  int n, A;
  long long nsrc;
  const float *obs, *act, *logp, *ret, *adv;  // the rollout arrays [nsrc, K0] / [nsrc, A] / [nsrc]
  float *o2, *a, *ol, *r, *ad;                // gathered: o2 [2, n, K0] (twice), a [n, A], [n] x 3
  const float* W;                              // input layer weights [2, N, K0], biases [2, N]
  const float* b;
  float* h;                                    // out: [2, n, N] = tanh(o W^T + b) per net
};

// block: kTinRows rows, N threads = N / 64 waves. Wave w takes rows 8w .. 8w + 7 (their observations
// are wave-uniform: 16-byte LDS broadcasts), lane l the 8 columns l + 64 c of the two nets' 2N outputs
// (c < N / 64: the policy's, the rest the value's), so a k step reads 8 conflict-free words of the
// transposed weights and 2 broadcasts, for 32 packed FMAs — LDS and VALU time balanced (one lane per
// column pair and 32 rows was LDS-bound). Every global load of the gather and of the weight staging
// is issued before the first wait (one wave per SIMD: nothing else hides their latency).
template <int K0, int N>
__global__ __launch_bounds__(N) void twin_gather_in_kernel(TwinInArgs p) {
  constexpr int XS = kTinRows + 4;  // xs row stride (16-byte aligned: 144 B)
  constexpr int WS = 2 * N + 1;     // ws row stride (odd: the transposing writes spread over banks)
  constexpr int NC = 2 * N / 64;    // columns per lane
  constexpr int RPW = 8;            // rows per wave
  static_assert(K0 % 2 == 0 && N % 64 == 0 && (N / 64) * RPW == kTinRows, "tile shape");
  constexpr int WF2 = K0;           // float2 of the [2N, K0] weights per thread: 2N K0 / 2 / N
  constexpr int OBS_IT = (kTinRows * K0 + N - 1) / N;
  constexpr int ACT_IT = (kTinRows * 32 + N - 1) / N;  // A <= 32
  __shared__ float ws[K0 * WS];
  __shared__ __attribute__((aligned(16))) float xs[K0 * XS];
  __shared__ long long sidx[kTinRows];
  const int t = threadIdx.x, n = p.n, r0 = blockIdx.x * kTinRows, A = p.A;
  const int rows = min(kTinRows, n - r0);
  const long long* idx = p.idx + (p.idx_row ? (size_t)*p.idx_row * n : 0);
  long long my_idx = -1;
  if (t < rows) my_idx = idx[r0 + t];
  float2 wv[WF2];  // the weights, coalesced: float2 f = t + i N of W viewed as [2N, K0]
  const float2* W2 = reinterpret_cast<const float2*>(p.W);
#pragma unroll
  for (int i = 0; i < WF2; i++) wv[i] = W2[t + i * N];
  if (t < kTinRows) sidx[t] = my_idx;
  __syncthreads();
  const long long nsrc = p.nsrc;
  const float nan = __builtin_nanf("");
  float ov[OBS_IT], av[ACT_IT];
#pragma unroll
  for (int i = 0; i < OBS_IT; i++) {
    const int e = t + i * N, r = e / K0, k = e - r * K0;
    const long long s = e < kTinRows * K0 ? sidx[r] : -1;
    ov[i] = (s >= 0 && s < nsrc) ? p.obs[(size_t)s * K0 + k] : nan;
  }
#pragma unroll
  for (int i = 0; i < ACT_IT; i++) {
    const int e = t + i * N, r = e / A, k = e - r * A;
    const long long s = e < rows * A ? sidx[r] : -1;
    av[i] = (s >= 0 && s < nsrc) ? p.act[(size_t)s * A + k] : nan;
  }
  float olv = nan, rv = nan, adv = nan;
  const bool own = t < rows && my_idx >= 0 && my_idx < nsrc;
  if (own) {
    olv = p.logp[my_idx];
    rv = p.ret[my_idx];
    adv = p.adv[my_idx];
  }
#pragma unroll
  for (int i = 0; i < WF2; i++) {
    const int f = t + i * N, row = f / (K0 / 2), k = 2 * (f - row * (K0 / 2));
    ws[k * WS + row] = wv[i].x;
    ws[(k + 1) * WS + row] = wv[i].y;
  }
#pragma unroll
  for (int i = 0; i < OBS_IT; i++) {
    const int e = t + i * N, r = e / K0, k = e - r * K0;
    if (e < kTinRows * K0) {
      xs[k * XS + r] = ov[i];
      if (r < rows) {
        p.o2[(size_t)(r0 + r) * K0 + k] = ov[i];
        p.o2[((size_t)n + r0 + r) * K0 + k] = ov[i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < ACT_IT; i++) {
    const int e = t + i * N;
    if (e < rows * A) p.a[(size_t)r0 * A + e] = av[i];
  }
  if (t < rows) {
    p.ol[r0 + t] = olv;
    p.r[r0 + t] = rv;
    p.ad[r0 + t] = adv;
  }
  __syncthreads();
  const int lane = t & 63, rg = t >> 6;
  tw_f2 acc[NC][RPW / 2];
#pragma unroll
  for (int c = 0; c < NC; c++)
#pragma unroll
    for (int i = 0; i < RPW / 2; i++) acc[c][i] = tw_f2{0.f, 0.f};
#pragma unroll 2
  for (int k = 0; k < K0; k++) {
    const float4 x0 = *reinterpret_cast<const float4*>(&xs[k * XS + RPW * rg]);
    const float4 x1 = *reinterpret_cast<const float4*>(&xs[k * XS + RPW * rg + 4]);
    const tw_f2 xp[4] = {{x0.x, x0.y}, {x0.z, x0.w}, {x1.x, x1.y}, {x1.z, x1.w}};
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const float w = ws[k * WS + lane + 64 * c];
#pragma unroll
      for (int i = 0; i < RPW / 2; i++) acc[c][i] = tw_fma(xp[i], w, acc[c][i]);
    }
  }
#pragma unroll
  for (int c = 0; c < NC; c++) {
    const int col = lane + 64 * c, net = col / N, cn = col - net * N;
    const float b = p.b[col];
    float* hr = p.h + ((size_t)net * n + r0 + RPW * rg) * N + cn;
#pragma unroll
    for (int i = 0; i < RPW / 2; i++) {
      if (RPW * rg + 2 * i < rows) hr[(size_t)(2 * i) * N] = tanhf(acc[c][i].x + b);
      if (RPW * rg + 2 * i + 1 < rows) hr[(size_t)(2 * i + 1) * N] = tanhf(acc[c][i].y + b);
    }
  }
}

// ------------------------------------------------------------------ output layers' backward
constexpr int kHbRows = 128;     // rows per block (= the weight-gradient / column-sum partial chunk)
constexpr int kHbCols = 64;      // columns per block: 16 quads
constexpr int kHbGroups = 16;    // row groups: thread t = quad t % 16, group t / 16 (8 rows each)
constexpr int kHbA = 21;         // instantiated output width (the humanoid's 21 actions)
constexpr int kHbDzStride = 24;  // LDS row stride of the staged dz rows (16-byte aligned)
constexpr int kHbPass = 7;       // output rows of the weight-gradient reduction per LDS pass

struct TwinHeadBwdArgs {
  const float* dz;  // [2, n, A]: the output layers' dZ (mjl_twin_loss_head)
  const float* W;   // [2, A, N]: the output layers' weights
  const float* y;   // [2, n, N]: the last hidden layer's outputs tanh(.)
  float* dzh;       // out [2, n, N]: that layer's dZ = (dz W) (1 - y^2)
  float* cs;        // out [2, n / kHbRows, N]: its column sums per row chunk
  float* gw;        // out [2, n / kHbRows, A, N]: the output weight gradient dz^T y per row chunk
  int n, N;
};

// block: 128 rows x 64 columns of one net, 256 threads (quad q = 4 columns, 8 rows of group g);
// every y row the thread reads is issued before the first FMA (two blocks per CU: 16 quad-rows in
// flight per lane pair); the group partials reduce through LDS in a fixed order, the weight gradient's
// in passes of kHbPass output rows.
template <int A>
__global__ __launch_bounds__(256, 2) void twin_head_bwd_kernel(TwinHeadBwdArgs p) {
  constexpr int RPT = kHbRows / kHbGroups;  // rows per thread
  static_assert(A % kHbPass == 0, "reduction passes");
  __shared__ __attribute__((aligned(16))) float sdz[kHbRows * kHbDzStride];
  __shared__ float4 red[kHbGroups * kHbPass * 16];
  const int t = threadIdx.x, q = t & 15, g = t >> 4;
  const int chunk = blockIdx.x, net = blockIdx.z, n = p.n, N = p.N;
  const int col = blockIdx.y * kHbCols + 4 * q;
  const int r0 = chunk * kHbRows;
  const float* yb = p.y + ((size_t)net * n + r0) * N + col;
  float4 yv[RPT];
#pragma unroll
  for (int u = 0; u < RPT; u++) yv[u] = *reinterpret_cast<const float4*>(yb + (size_t)(g + u * kHbGroups) * N);
  tw_f2 wl[A], wh[A];  // this thread's 4 columns of W_out
#pragma unroll
  for (int a = 0; a < A; a++) {
    const float4 w = *reinterpret_cast<const float4*>(p.W + ((size_t)net * A + a) * N + col);
    wl[a] = tw_f2{w.x, w.y};
    wh[a] = tw_f2{w.z, w.w};
  }
  const float* dzb = p.dz + ((size_t)net * n + r0) * A;
  for (int e = t; e < kHbRows * A; e += 256) {
    const int r = e / A, a = e - r * A;
    sdz[r * kHbDzStride + a] = dzb[e];
  }
  __syncthreads();
  tw_f2 gl[A], gh[A];
#pragma unroll
  for (int a = 0; a < A; a++) gl[a] = gh[a] = tw_f2{0.f, 0.f};
  tw_f2 csl{0.f, 0.f}, csh{0.f, 0.f};
  float* zb = p.dzh + ((size_t)net * n + r0) * N + col;
#pragma unroll
  for (int u = 0; u < RPT; u++) {
    const int r = g + u * kHbGroups;
    const float* d = &sdz[r * kHbDzStride];
    const tw_f2 yl{yv[u].x, yv[u].y}, yh{yv[u].z, yv[u].w};
    tw_f2 hl{0.f, 0.f}, hh{0.f, 0.f};
#pragma unroll
    for (int a = 0; a < A; a++) {
      const float da = d[a];
      hl = tw_fma(wl[a], da, hl);
      hh = tw_fma(wh[a], da, hh);
      gl[a] = tw_fma(yl, da, gl[a]);
      gh[a] = tw_fma(yh, da, gh[a]);
    }
    const tw_f2 zl = hl * (tw_f2{1.f, 1.f} - yl * yl), zh = hh * (tw_f2{1.f, 1.f} - yh * yh);
    *reinterpret_cast<float4*>(zb + (size_t)r * N) = make_float4(zl.x, zl.y, zh.x, zh.y);
    csl += zl;
    csh += zh;
  }
  // the 16 row groups' partials, summed in group order (fixed: deterministic)
  red[g * 16 + q] = make_float4(csl.x, csl.y, csh.x, csh.y);
  __syncthreads();
  if (t < 16) {
    float4 s = red[t];
    for (int k = 1; k < kHbGroups; k++) {
      const float4 v = red[k * 16 + t];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const int R = n / kHbRows;
    *reinterpret_cast<float4*>(p.cs + ((size_t)net * R + chunk) * N + blockIdx.y * kHbCols + 4 * t) = s;
  }
  const int S = n / kHbRows;
#pragma unroll
  for (int a0 = 0; a0 < A; a0 += kHbPass) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kHbPass; j++)
      red[(g * kHbPass + j) * 16 + q] = make_float4(gl[a0 + j].x, gl[a0 + j].y, gh[a0 + j].x, gh[a0 + j].y);
    __syncthreads();
    if (t < kHbPass * 16) {
      const int j = t >> 4, qq = t & 15;
      float4 s = red[j * 16 + qq];
      for (int k = 1; k < kHbGroups; k++) {
        const float4 v = red[(k * kHbPass + j) * 16 + qq];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      *reinterpret_cast<float4*>(p.gw + (((size_t)net * S + chunk) * A + a0 + j) * N + blockIdx.y * kHbCols + 4 * qq) = s;
    }
  }
}

}  // namespace mjl
