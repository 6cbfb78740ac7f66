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

// block: kTinRows rows; thread t: net t / (N/2), output columns 2 (t mod N/2) and +1 of that net.
// Both nets' weights staged transposed in LDS (ws[k][net N + c]: a thread's two columns are one 8-byte
// read per k), the gathered observations transposed too (xs[k][row]: 4 rows per 16-byte broadcast
// read); two rows per packed FMA, 32 rows x 2 columns of accumulators per thread. (Weights held in
// registers instead spilled: the unrolled k loop's hoisted LDS reads took every VGPR.)
template <int K0, int N>
__global__ __launch_bounds__(N) void twin_gather_in_kernel(TwinInArgs p) {
  constexpr int XS = kTinRows + 4;  // padded row stride (16-byte aligned: 144 B)
  constexpr int TH = N / 2;
  static_assert(K0 % 2 == 0, "pairs of weights per load");
  __shared__ __attribute__((aligned(16))) float ws[K0 * 2 * N];
  __shared__ __attribute__((aligned(16))) float xs[K0 * XS];
  __shared__ long long sidx[kTinRows];
  const int t = threadIdx.x, n = p.n, r0 = blockIdx.x * kTinRows;
  const int rows = min(kTinRows, n - r0);
  const long long* idx = p.idx + (p.idx_row ? (size_t)*p.idx_row * n : 0);
  if (t < kTinRows) sidx[t] = t < rows ? idx[r0 + t] : -1;
  const int net = t / TH, c0 = 2 * (t - net * TH), wc = net * N + c0;
  {
    const float* wr = p.W + (size_t)wc * K0;  // rows wc and wc + 1 of W viewed as [2 N, K0]
#pragma unroll 9
    for (int k = 0; k < K0; k += 2) {
      const float2 u = *reinterpret_cast<const float2*>(wr + k), v = *reinterpret_cast<const float2*>(wr + K0 + k);
      *reinterpret_cast<float2*>(&ws[k * 2 * N + wc]) = make_float2(u.x, v.x);
      *reinterpret_cast<float2*>(&ws[(k + 1) * 2 * N + wc]) = make_float2(u.y, v.y);
    }
  }
  __syncthreads();
  const long long nsrc = p.nsrc;
  const float nan = __builtin_nanf("");
  for (int e = t; e < kTinRows * K0; e += N) {  // observations: coalesced row reads and writes
    const int r = e / K0, k = e - r * K0;
    const long long s = sidx[r];
    const float v = (s >= 0 && s < nsrc) ? p.obs[(size_t)s * K0 + k] : nan;
    xs[k * XS + r] = v;
    if (r < rows) {
      p.o2[(size_t)(r0 + r) * K0 + k] = v;
      p.o2[((size_t)n + r0 + r) * K0 + k] = v;
    }
  }
  const int A = p.A;
  for (int e = t; e < rows * A; e += N) {
    const int r = e / A, k = e - r * A;
    const long long s = sidx[r];
    p.a[(size_t)(r0 + r) * A + k] = (s >= 0 && s < nsrc) ? p.act[(size_t)s * A + k] : nan;
  }
  if (t < rows) {
    const long long s = sidx[t];
    const bool ok = s >= 0 && s < nsrc;
    p.ol[r0 + t] = ok ? p.logp[s] : nan;
    p.r[r0 + t] = ok ? p.ret[s] : nan;
    p.ad[r0 + t] = ok ? p.adv[s] : nan;
  }
  __syncthreads();
  tw_f2 acc0[kTinRows / 2], acc1[kTinRows / 2];
#pragma unroll
  for (int i = 0; i < kTinRows / 2; i++) acc0[i] = acc1[i] = tw_f2{0.f, 0.f};
#pragma unroll 2
  for (int k = 0; k < K0; k++) {
    const float2 w = *reinterpret_cast<const float2*>(&ws[k * 2 * N + wc]);
#pragma unroll
    for (int q = 0; q < kTinRows / 4; q++) {
      const float4 xv = *reinterpret_cast<const float4*>(&xs[k * XS + 4 * q]);
      const tw_f2 lo{xv.x, xv.y}, hi{xv.z, xv.w};
      acc0[2 * q] = tw_fma(lo, w.x, acc0[2 * q]);
      acc0[2 * q + 1] = tw_fma(hi, w.x, acc0[2 * q + 1]);
      acc1[2 * q] = tw_fma(lo, w.y, acc1[2 * q]);
      acc1[2 * q + 1] = tw_fma(hi, w.y, acc1[2 * q + 1]);
    }
  }
  const float b0 = p.b[wc], b1 = p.b[wc + 1];
  float* hr = p.h + ((size_t)net * n + r0) * N + c0;
#pragma unroll
  for (int i = 0; i < kTinRows / 2; i++) {
    if (2 * i < rows)
      *reinterpret_cast<float2*>(hr + (size_t)(2 * i) * N) = make_float2(tanhf(acc0[i].x + b0), tanhf(acc1[i].x + b1));
    if (2 * i + 1 < rows)
      *reinterpret_cast<float2*>(hr + (size_t)(2 * i + 1) * N) =
          make_float2(tanhf(acc0[i].y + b0), tanhf(acc1[i].y + b1));
  }
}

// ------------------------------------------------------------------ output layers' backward
constexpr int kHbRows = 128;   // rows per block (= the weight-gradient / column-sum partial chunk)
constexpr int kHbCols = 128;   // columns per block: 32 quads
constexpr int kHbGroups = 8;   // row groups: thread t = quad t % 32, group t / 32
constexpr int kHbA = 21;       // instantiated output width (the humanoid's 21 actions)
constexpr int kHbDzStride = 24;  // LDS row stride of the staged dz rows (16-byte aligned)

struct TwinHeadBwdArgs {
  const float* dz;  // [2, n, A]: the output layers' dZ (mjl_twin_loss_head)
  const float* W;   // [2, A, N]: the output layers' weights
  const float* y;   // [2, n, N]: the last hidden layer's outputs tanh(.)
  float* dzh;       // out [2, n, N]: that layer's dZ = (dz W) (1 - y^2)
  float* cs;        // out [2, n / kHbRows, N]: its column sums per row chunk
  float* gw;        // out [2, n / kHbRows, A, N]: the output weight gradient dz^T y per row chunk
  int n, N;
};

template <int A>
__global__ __launch_bounds__(256) void twin_head_bwd_kernel(TwinHeadBwdArgs p) {
  __shared__ __attribute__((aligned(16))) float sdz[kHbRows * kHbDzStride];
  __shared__ float4 red[kHbGroups * A * 32];
  const int t = threadIdx.x, q = t & 31, g = t >> 5;
  const int chunk = blockIdx.x, net = blockIdx.z, n = p.n, N = p.N;
  const int col = blockIdx.y * kHbCols + 4 * q;
  const int r0 = chunk * kHbRows;
  const float* dzb = p.dz + ((size_t)net * n + r0) * A;
  for (int e = t; e < kHbRows * A; e += 256) {
    const int r = e / A, a = e - r * A;
    sdz[r * kHbDzStride + a] = dzb[e];
  }
  tw_f2 wl[A], wh[A];  // this thread's 4 columns of W_out
#pragma unroll
  for (int a = 0; a < A; a++) {
    const float4 w = *reinterpret_cast<const float4*>(p.W + ((size_t)net * A + a) * N + col);
    wl[a] = tw_f2{w.x, w.y};
    wh[a] = tw_f2{w.z, w.w};
  }
  __syncthreads();
  tw_f2 gl[A], gh[A];
#pragma unroll
  for (int a = 0; a < A; a++) gl[a] = gh[a] = tw_f2{0.f, 0.f};
  tw_f2 csl{0.f, 0.f}, csh{0.f, 0.f};
  const float* yb = p.y + ((size_t)net * n + r0) * N + col;
  float* zb = p.dzh + ((size_t)net * n + r0) * N + col;
  constexpr int U = 4;  // rows in flight per trip
  for (int r = g; r < kHbRows; r += U * kHbGroups) {
    float4 yv[U];
#pragma unroll
    for (int u = 0; u < U; u++) yv[u] = *reinterpret_cast<const float4*>(yb + (size_t)(r + u * kHbGroups) * N);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const float* d = &sdz[(r + u * kHbGroups) * kHbDzStride];
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
      *reinterpret_cast<float4*>(zb + (size_t)(r + u * kHbGroups) * N) = make_float4(zl.x, zl.y, zh.x, zh.y);
      csl += zl;
      csh += zh;
    }
  }
  // the 8 row groups' partials, summed in group order (fixed: deterministic)
  red[g * 32 + q] = make_float4(csl.x, csl.y, csh.x, csh.y);
  __syncthreads();
  if (t < 32) {
    float4 s = red[t];
    for (int k = 1; k < kHbGroups; k++) {
      const float4 v = red[k * 32 + t];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const int R = n / kHbRows;
    *reinterpret_cast<float4*>(p.cs + ((size_t)net * R + chunk) * N + blockIdx.y * kHbCols + 4 * t) = s;
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < A; a++) red[(g * A + a) * 32 + q] = make_float4(gl[a].x, gl[a].y, gh[a].x, gh[a].y);
  __syncthreads();
  const int S = n / kHbRows;
  for (int e = t; e < A * 32; e += 256) {
    const int a = e >> 5, qq = e & 31;
    float4 s = red[a * 32 + qq];
    for (int k = 1; k < kHbGroups; k++) {
      const float4 v = red[(k * A + a) * 32 + qq];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    *reinterpret_cast<float4*>(p.gw + (((size_t)net * S + chunk) * A + a) * N + blockIdx.y * kHbCols + 4 * qq) = s;
  }
}

}  // namespace mjl
