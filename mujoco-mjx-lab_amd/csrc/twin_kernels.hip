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
typedef float tw_f32x16 __attribute__((ext_vector_type(16)));

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

// A persistent grid of at most kTinBlocks workgroups of N threads (N / 64 waves), one net per workgroup
// (net = blockIdx & 1), each taking 32-row chunks blockIdx / 2, + gridDim / 2, ... Its net's input
// weights are staged ONCE per workgroup into LDS, row-major with an odd row stride (coalesced 16-byte
// loads, conflict-free writes and operand reads): 64 KB of LDS, two workgroups per CU. Per chunk
// every lane loads the row indices it needs itself (no LDS hand-off, so the observation loads issue
// right behind the index loads), writes the chunk transposed to LDS and its net's copy of the rows;
// then the N output columns in 32-wide tiles, wave w taking tiles w, w + N/64, ..., each as
// v_mfma_f32_32x32x2_f32 over K0 in steps of 2 with C = W X^T (A = the weight rows, lane l giving
// column l & 31 at k0 + (l >> 5); B = the gathered rows, lane l giving row l & 31): register v of lane
// l then holds C[(v & 3) + 8 (v >> 2) + 4 (l >> 5)][l & 31], i.e. lane l owns row l & 31 and 4
// consecutive columns per register quad, stored as 16-byte writes after the bias and tanh. The MFMA
// is an exact f32 fma chain in k order (deterministic). (Measured and replaced, per 8,192-row launch:
// vector-ALU versions 25-37 us; B operands read per lane from global memory 25.6 us — 4-byte reads over
// 32 weight rows missed L1; both nets per workgroup with 120 KB of LDS, one workgroup per CU,
// per-lane 4-byte stores 17.7-24 us. Where this one's 16.3-16.9 us go, by knocking parts out
// (tools/twin_micro.hip, profiles/r6/twin_micro.txt): ~6 us launch + weight staging + gather, ~4 us
// the MFMAs, ~6 us the 16.8 MB of H stores; a branch-free tanh in the epilogue changed nothing.)
constexpr int kTinBlocks = 512;
template <int K0, int N>
__global__ __launch_bounds__(N, 2) void twin_gather_in_kernel(TwinInArgs p) {
  constexpr int XS = kTinRows + 4;  // xs row stride
  constexpr int WS = K0 + 1;        // ws row stride (odd)
  constexpr int OBS_IT = (kTinRows * K0 + N - 1) / N;
  constexpr int ACT_IT = (kTinRows * 32 + N - 1) / N;  // A <= 32
  constexpr int KS = K0 / 2;                           // MFMA K steps
  constexpr int TPW = N / 32 / (N / 64);               // tiles per wave (2)
  constexpr int WQ = N * K0 / 4;                       // float4 of one net's W
  static_assert(K0 % 2 == 0 && (N * K0) % 4 == 0 && kTinRows == 32 && N % 64 == 0, "tile shape");
  __shared__ float ws[N * WS];
  __shared__ float xs[K0 * XS];
  const int t = threadIdx.x, n = p.n, A = p.A, net = blockIdx.x & 1;
  {  // this net's weights: W[net] [N, K0] row-major -> ws[col * WS + k] (= element e + col)
    const float4* W4 = reinterpret_cast<const float4*>(p.W + (size_t)net * N * K0);
    constexpr int IT = (WQ + N - 1) / N;
    float4 wv[IT];
#pragma unroll
    for (int i = 0; i < IT; i++) {
      const int q = t + i * N;
      wv[i] = q < WQ ? W4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < IT; i++) {
      const int q = t + i * N;
      if (q < WQ) {
        const float v4[4] = {wv[i].x, wv[i].y, wv[i].z, wv[i].w};
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const int e = 4 * q + c;
          ws[e + e / K0] = v4[c];
        }
      }
    }
  }
  const long long nsrc = p.nsrc;
  const float nan = __builtin_nanf("");
  const long long* idx = p.idx + (p.idx_row ? (size_t)*p.idx_row * n : 0);
  const int lane = t & 63, w = t >> 6, li = lane & 31, kh = lane >> 5;
  const int nchunk = (n + kTinRows - 1) / kTinRows, cstep = (int)(gridDim.x >> 1);
  float4 bq[TPW][4];  // this lane's bias quads (loop-invariant)
#pragma unroll
  for (int tt = 0; tt < TPW; tt++)
#pragma unroll
    for (int q = 0; q < 4; q++)
      bq[tt][q] = *reinterpret_cast<const float4*>(p.b + (size_t)net * N + (w * TPW + tt) * 32 + 8 * q + 4 * kh);
  for (int ch = (int)(blockIdx.x >> 1); ch < nchunk; ch += cstep) {
    const int r0 = ch * kTinRows, rows = min(kTinRows, n - r0);
    float ov[OBS_IT], av[ACT_IT];
#pragma unroll
    for (int i = 0; i < OBS_IT; i++) {
      const int e = t + i * N, r = e / K0, k = e - r * K0;
      const long long s = (e < kTinRows * K0 && r < rows) ? idx[r0 + r] : -1;
      ov[i] = (s >= 0 && s < nsrc) ? p.obs[(size_t)s * K0 + k] : nan;
    }
    if (net == 0) {
#pragma unroll
      for (int i = 0; i < ACT_IT; i++) {
        const int e = t + i * N, r = e / A, k = e - r * A;
        const long long s = e < rows * A ? idx[r0 + r] : -1;
        av[i] = (s >= 0 && s < nsrc) ? p.act[(size_t)s * A + k] : nan;
      }
    }
    float olv = nan, rv = nan, adv = nan;
    if (net == 0 && t < rows) {
      const long long s = idx[r0 + t];
      if (s >= 0 && s < nsrc) {
        olv = p.logp[s];
        rv = p.ret[s];
        adv = p.adv[s];
      }
    }
    __syncthreads();  // (the previous chunk's MFMAs are done with xs)
#pragma unroll
    for (int i = 0; i < OBS_IT; i++) {
      const int e = t + i * N, r = e / K0, k = e - r * K0;
      if (e < kTinRows * K0) {
        xs[k * XS + r] = ov[i];
        if (r < rows) p.o2[((size_t)net * n + r0 + r) * K0 + k] = ov[i];
      }
    }
    if (net == 0) {
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
    }
    __syncthreads();
#pragma unroll
    for (int tt = 0; tt < TPW; tt++) {
      const int c0 = (w * TPW + tt) * 32;  // the tile's first column
      const float* wr = &ws[(c0 + li) * WS + kh];
      tw_f32x16 acc;
#pragma unroll
      for (int v = 0; v < 16; v++) acc[v] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; s++)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[2 * s], xs[(2 * s + kh) * XS + li], acc, 0, 0, 0);
      if (li < rows) {
        float* hr = p.h + ((size_t)net * n + r0 + li) * N + c0 + 4 * kh;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const float4 b = bq[tt][q];
          *reinterpret_cast<float4*>(hr + 8 * q) = make_float4(tanhf(acc[4 * q] + b.x), tanhf(acc[4 * q + 1] + b.y),
                                                               tanhf(acc[4 * q + 2] + b.z), tanhf(acc[4 * q + 3] + b.w));
        }
      }
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
  constexpr int DZ_IT = (kHbRows * A + 255) / 256;
  float dv[DZ_IT];  // every load of the staging issued before the first LDS write
#pragma unroll
  for (int i = 0; i < DZ_IT; i++) {
    const int e = t + 256 * i;
    dv[i] = e < kHbRows * A ? dzb[e] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < DZ_IT; i++) {
    const int e = t + 256 * i, r = e / A, a = e - r * A;
    if (e < kHbRows * A) sdz[r * kHbDzStride + a] = dv[i];
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
