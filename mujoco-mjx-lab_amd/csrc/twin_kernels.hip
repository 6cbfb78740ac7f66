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

#include "ppo_loss_kernels.hip"  // wave_sum_dpp, kLog2Pi

namespace mjl {

typedef float tw_f2 __attribute__((ext_vector_type(2)));
typedef float tw_f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ tw_f2 tw_fma(tw_f2 a, float b, tw_f2 c) {
  return __builtin_elementwise_fma(a, tw_f2{b, b}, c);
}

// tanh without branches, for tiles on a launch's critical path: the device library's odd polynomial
// below |x| = 0.625, 1 - 2 / (e^{2|x|} + 1) above it (v_exp_f32, v_rcp_f32), both evaluated and one
// selected; within 3.6 ulp of tanhf over [-12, 12] (tools/twin_micro.hip). The library's tanhf
// branches per lane on |x|, so a wave holding both kinds of values runs both paths and their
// exec-mask bookkeeping (~35 instructions per value against ~15).
__device__ __forceinline__ float tw_tanh(float x) {
  const float ax = fabsf(x), x2 = x * x;
  float q = fmaf(__uint_as_float(0xbbbac73du), x2, __uint_as_float(0x3ca908c9u));
  q = fmaf(x2, q, __uint_as_float(0xbd5c1c4eu));
  q = fmaf(x2, q, __uint_as_float(0x3e088382u));
  q = fmaf(x2, q, __uint_as_float(0xbeaaaa99u));
  const float small = fmaf(x2, ax * q, ax);
  const float big = fmaf(-2.f, __builtin_amdgcn_rcpf(__expf(2.f * ax) + 1.f), 1.f);
  return copysignf(ax < 0.625f ? small : big, x);
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
  constexpr int WS = K0;            // ws row stride (K0 = 54: 54 col mod 64 banks are distinct over 32 lanes)
  constexpr int OBS_IT = (kTinRows * K0 + N - 1) / N;
  constexpr int ACT_IT = (kTinRows * 32 + N - 1) / N;  // A <= 32
  constexpr int KS = K0 / 2;                           // MFMA K steps
  constexpr int TPW = N / 32 / (N / 64);               // tiles per wave (2)
  static_assert(K0 % 2 == 0 && (N * K0) % 256 == 0 && kTinRows == 32 && N % 64 == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) float ws[N * WS];
  __shared__ float xs[K0 * XS];
  const int t = threadIdx.x, n = p.n, A = p.A, net = blockIdx.x & 1;
  {  // this net's weights W[net] [N, K0], row-major as they lie, by LDS-DMA (global_load_lds_dwordx4: 1 KB
     // per wave-instruction, no VGPRs, so the first chunk's gather issues behind it; the chunk's first
     // barrier retires it)
    const float* Wn = p.W + (size_t)net * N * K0;
    for (int i = t >> 6; i < N * K0 / 256; i += N / 64)
      __builtin_amdgcn_global_load_lds((const void*)(Wn + 256 * i + 4 * (t & 63)),
                                       (__attribute__((address_space(3))) void*)&ws[256 * i], 16, 0, 0);
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


// ------------------------------------------------------------------ fused head (forward + losses + backward)
// The twin update's head in ONE launch (train_ppo.py:204-220 for both nets' output layers, the last
// hidden layer's bias + tanh and its tanh backward): replaces the last hidden layer's bias + tanh pass,
// the output layers' batched GEMM, the loss launch (mjl_twin_loss_head) and the output backward
// (mjl_twin_head_bwd). A persistent grid of workgroups, one net each (net = blockIdx & 1), taking
// R-row chunks blockIdx / 2, + gridDim / 2, ...: the launch takes R = 32 with two workgroups per CU
// (75 KB of LDS each, at most kThBlocks); R = 64 (one per CU) measured slower at every size, and so
// did (R = 32) the first chunk's loads hoisted above the setup, the next chunk's issued during the
// current one and z on two accumulator chains (24.2-27.3 against 22.8 us at 8,192 rows: the live
// registers spill; profiles/r6/twin_micro.txt). Per chunk:
//   H = tanh(zh + bh) of the chunk into LDS (zh: the last hidden layer's bias-less GEMM output);
//   z = H W^T + bo on v_mfma_f32_32x32x2_f32 (2 K halves per 32-row tile, one wave each, summed in K
//     order through LDS);
//   per row (256 / R lanes, DPP sums): the policy's clipped surrogate as twin_loss_head_kernel (mean = tanh z,
//     the Gaussian log-prob with log_std clipped, ratio, torch.minimum's tie gradient, dz = d loss /
//     d z), or the value's dz = 2 (v - ret) / n in column 0;
//   the chunk's column sums (the loss, d loss / d log_std, the output bias gradient) added to the
//     workgroup's accumulators in chunk order;
//   dH = dz W on MFMA, dZ = dH (1 - H^2) stored and column-summed (the hidden bias gradient);
//   the output weight gradient dz^T H on MFMA, accumulated across the workgroup's chunks in registers.
// Per workgroup one partial of every reduction (block b of net k): lossp[b], glsp[b][A] (policy),
// biasp[k][b][A], cs[k][b][K], gw[k][b][A][K], summed over the workgroups in order by
// mjl_slice_sum_multi. Deterministic (fixed orders throughout).
constexpr int kThRows = 32;       // rows per chunk of the launch (two workgroups per CU)
constexpr int kThK = 256;         // instantiated last hidden width
constexpr int kThA = 21;          // instantiated output width
constexpr int kThBlocks = 512;    // at most this many workgroups
constexpr int kThHS = kThK + 4;   // hs / ws row stride (16-byte rows, 4 banks apart)
constexpr int kThZS = 33;         // sz row stride (32 output columns + 1)

struct TwinHeadArgs {
  const float* zh;  // [2, n, K]: the last hidden layer's bias-less pre-activation
  const float* bh;  // [2, K]: its bias
  const float* W;   // [2, A, K]: the output layers' weights
  const float* bo;  // [2, A]: their biases
  const float *log_std, *act, *old_logp, *adv, *ret;  // [A], [n, A], [n] x 3
  const float* adv_stats;                             // [n_minibatches, 2] (mean, std), read at *stats_row;
  const int* stats_row;                               // or NULL: merged from adv_part (adv_stats_kernel)
  const float* adv_part;
  int nb_adv;
  int n;
  float clip_eps, ent_coef, ls_lo, ls_hi;
  float* dzh;    // out [2, n, K]: dZ of the last hidden layer
  float* cs;     // out [2, S, K]: its column sums per workgroup
  float* gw;     // out [2, S, A, K]: the output weight gradient per workgroup
  float* lossp;  // out [S]: policy loss partials (workgroup 0 adds the entropy term)
  float* glsp;   // out [S, A]: d loss / d log_std partials
  float* biasp;  // out [2, S, A]: the output bias gradients
};

template <int A, int K, int R>
__global__ __launch_bounds__(256, 64 / R) void twin_head_kernel(TwinHeadArgs p) {
  static_assert(A <= 31 && K % 64 == 0 && K == 4 * 64, "tile shape: 4 waves x 2 column tiles of 32");
  static_assert(R == 32 || R == 64, "32 or 64 rows per chunk");
  constexpr int HS = kThHS, ZS = kThZS, NRT = R / 32, LPR = 256 / R;  // row tiles; lanes per loss row
  __shared__ __attribute__((aligned(16))) float hs[R * HS];  // H of the chunk
  __shared__ __attribute__((aligned(16))) float ws[A * HS];   // W_out rows (rows A..31 read as zero)
  constexpr int KP = 4 / NRT;                                 // K parts of z: every wave takes one (part, row tile)
  __shared__ float red[4 * 16 * 64];                          // z partials per wave; at the end, the csh sums
  __shared__ float sz[R * ZS];                                // z, then d, then dz (cols A..31 zero)
  __shared__ float sx[R * 32];                                // act, then the mean, then c_j
  __shared__ float srow[4][R];                                // old_logp, adv, ret, surr
  __shared__ float ivs[32];
  __shared__ float lss_s, mu_s, sd_s;
  __shared__ float acc_col[2 * 32 + 1];                       // c_j, dz column sums, loss: chunk order
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, li = lane & 31, kh = lane >> 5;
  const int net = blockIdx.x & 1, S = (int)(gridDim.x >> 1), blk = (int)(blockIdx.x >> 1), n = p.n;
  const int nchunk = (n + R - 1) / R;
  // ---- once per workgroup: W_out of this net, the log_std terms, the advantage statistics
  // (by LDS-DMA, global_load_lds_dwordx4: one 1-KB row per wave-instruction, no VGPRs, so the first
  // chunk's loads issue behind it; the chunk's first barrier retires it)
  static_assert(K == 64 * 4, "one W_out row per wave-instruction");
  for (int a = w; a < A; a += 4)
    __builtin_amdgcn_global_load_lds((const void*)(p.W + ((size_t)net * A + a) * K + 4 * lane),
                                     (__attribute__((address_space(3))) void*)&ws[a * HS], 16, 0, 0);
  if (w == 0) {
    const float ls = lane < A ? fminf(fmaxf(p.log_std[lane], p.ls_lo), p.ls_hi) : 0.f;  // networks.py:103
    if (lane < 32) ivs[lane] = lane < A ? expf(-2.f * ls) : 0.f;
    const float tot = wave_sum_dpp(lane < A ? 2.f * ls + kLog2Pi : 0.f);
    float mu, sdv;
    if (p.adv_stats) {
      const float* st = p.adv_stats + (p.stats_row ? 2 * (size_t)*p.stats_row : 0);
      mu = st[0];
      sdv = st[1];
    } else {
      adv_merge_wave(p.adv_part, p.nb_adv, lane, mu, sdv);
    }
    if (lane == 0) {
      lss_s = tot;
      mu_s = mu;
      sd_s = sdv;
    }
  }
  if (t < 2 * 32 + 1) acc_col[t] = 0.f;
  tw_f32x16 gwacc[2];
  float csacc[2] = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 2; c++)
#pragma unroll
    for (int v = 0; v < 16; v++) gwacc[c][v] = 0.f;
  const float4 bq = *reinterpret_cast<const float4*>(p.bh + (size_t)net * K + 4 * (t & (K / 4 - 1)));
  const float nf = (float)n;
  for (int ch = blk; ch < nchunk; ch += S) {
    const int r0 = ch * R, rows = min(R, n - r0);
    // ---- loads: the chunk's pre-activations, actions and per-row scalars, all issued together
    constexpr int QZ = R * K / 4 / 256;  // float4 of zh per thread (16)
    float4 zv[QZ];
#pragma unroll
    for (int i = 0; i < QZ; i++) {
      const int q = t + 256 * i, r = q / (K / 4), c4 = q - r * (K / 4);
      zv[i] = r < rows ? *reinterpret_cast<const float4*>(p.zh + ((size_t)net * n + r0 + r) * K + 4 * c4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    constexpr int QA = (R * 32 + 255) / 256;
    float av[QA];
    if (net == 0) {
#pragma unroll
      for (int i = 0; i < QA; i++) {
        const int e = t + 256 * i;
        av[i] = e < rows * A ? p.act[(size_t)r0 * A + e] : 0.f;
      }
    }
    float rv0 = 0.f, rv1 = 0.f, rv2 = 0.f;
    if (t < rows) {
      rv0 = p.old_logp[r0 + t];
      rv1 = p.adv[r0 + t];
      rv2 = p.ret[r0 + t];
    }
    __syncthreads();  // (the previous chunk's reads of hs / sz / sx are done)
#pragma unroll
    for (int i = 0; i < QZ; i++) {
      const int q = t + 256 * i, r = q / (K / 4), c4 = q - r * (K / 4);
      float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < rows)
        h = make_float4(tw_tanh(zv[i].x + bq.x), tw_tanh(zv[i].y + bq.y), tw_tanh(zv[i].z + bq.z),
                        tw_tanh(zv[i].w + bq.w));
      *reinterpret_cast<float4*>(&hs[r * HS + 4 * c4]) = h;
    }
    if (net == 0) {
#pragma unroll
      for (int i = 0; i < QA; i++) {
        const int e = t + 256 * i;
        if (e < rows * A) sx[(e / A) * 32 + e % A] = av[i];
      }
    }
    if (t < R) {
      srow[0][t] = rv0;
      srow[1][t] = rv1;
      srow[2][t] = rv2;
    }
    __syncthreads();
    // ---- z = H W^T: wave w takes row tile w % NRT and K part w / NRT (of KP)
    {
      const int rt = w % NRT, k0 = (w / NRT) * (K / KP);
      tw_f32x16 acc;
#pragma unroll
      for (int v = 0; v < 16; v++) acc[v] = 0.f;
      const float* ha = &hs[(32 * rt + li) * HS + k0 + kh];
      const float* wb = &ws[(li < A ? li : 0) * HS + k0 + kh];
      const bool wr = li < A;  // W_out rows A..31: zero
#pragma unroll 8
      for (int s = 0; s < K / (2 * KP); s++)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ha[2 * s], wr ? wb[2 * s] : 0.f, acc, 0, 0, 0);
#pragma unroll
      for (int v = 0; v < 16; v++) red[(w * 16 + v) * 64 + lane] = acc[v];
    }
    __syncthreads();
    // z[row][a] = the K parts in order (pairwise for 4) + bo (C[i][j] in register (i & 3) + 4 (i >> 3) of
    // lane j + 32 ((i >> 2) & 1))
    for (int e = t; e < R * 32; e += 256) {
      const int row = e >> 5, a = e & 31, rt = row >> 5, i = row & 31;
      const int v = (i & 3) + 4 * (i >> 3), L = a + 32 * ((i >> 2) & 1);
      auto part = [&](int k) { return red[((k * NRT + rt) * 16 + v) * 64 + L]; };
      const float zz = KP == 2 ? part(0) + part(1) : (part(0) + part(1)) + (part(2) + part(3));
      sz[row * ZS + a] = a < A ? zz + p.bo[net * A + a] : 0.f;
    }
    __syncthreads();
    // ---- per row: the losses and dz, LPR lanes per row (lane q of the row's group takes columns q,
    // q + LPR, ...; the row's log-density sum over the group by DPP, the same total in all its lanes)
    {
      const int r = t / LPR, q = t % LPR;
      float* zr = &sz[r * ZS];
      float* xr = &sx[r * 32];
      float surr = 0.f;
      if (r < rows) {
        if (net == 0) {
          float qs = 0.f;
          for (int j = q; j < A; j += LPR) {
            const float m = tanhf(zr[j]), d = xr[j] - m;
            zr[j] = d;
            xr[j] = m;
            qs += d * d * ivs[j];
          }
          qs += dpp_f<0xb1>(qs);                // quad_perm [1, 0, 3, 2]
          qs += dpp_f<0x4e>(qs);                // quad_perm [2, 3, 0, 1]
          if constexpr (LPR == 8) qs += dpp_f<0x141>(qs);  // row_half_mirror: the other quad of the 8
          const float logp = -0.5f * (qs + lss_s);
          const float ratio = expf(logp - srow[0][r]);
          const float an = (srow[1][r] - mu_s) / (sd_s + 1e-8f);
          const float lo = 1.f - p.clip_eps, hi = 1.f + p.clip_eps;
          const float rc = fminf(fmaxf(ratio, lo), hi);
          const float t1 = ratio * an, t2 = rc * an;
          surr = fminf(t1, t2);
          const float w1 = t1 < t2 ? 1.f : (t1 == t2 ? 0.5f : 0.f);
          const float w2 = t2 < t1 ? 1.f : (t1 == t2 ? 0.5f : 0.f);
          const float dratio = (-1.f / nf) * (w1 * an + ((ratio >= lo && ratio <= hi) ? w2 * an : 0.f));
          const float dlogp = dratio * ratio;
          for (int j = q; j < A; j += LPR) {
            const float d = zr[j], m = xr[j], iv = ivs[j];
            xr[j] = dlogp * (d * d * iv - 1.f);    // d logp / d s_j = q_j - 1
            zr[j] = dlogp * d * iv * (1.f - m * m);  // d loss / d z_j
          }
        } else {
          if (q == 0) zr[0] = 2.f * (zr[0] - srow[2][r]) / nf;  // value: d loss / d v (train_ppo.py:218-220)
          for (int j = (q == 0 ? LPR : q); j < A; j += LPR) zr[j] = 0.f;
        }
      } else {
        for (int j = q; j < 32; j += LPR) {
          zr[j] = 0.f;
          xr[j] = 0.f;
        }
      }
      if (q == 0) srow[3][r] = surr;
    }
    __syncthreads();
    // ---- the chunk's column sums into the workgroup's accumulators (rows in order, chunks in order)
    if (t < 2 * 32 + 1) {
      const bool pol = net == 0;
      const float* col = t == 2 * 32 ? srow[3] : t < 32 ? &sx[t] : &sz[t - 32];
      const int cstr = t == 2 * 32 ? 1 : (t < 32 ? 32 : ZS);
      const bool on = t == 2 * 32 ? pol : (t < 32 ? (pol && t < A) : (t - 32 < A));
      if (on) {
        float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
        for (int r = 0; r < R; r += 4) {
          p0 += col[r * cstr]; p1 += col[(r + 1) * cstr]; p2 += col[(r + 2) * cstr]; p3 += col[(r + 3) * cstr];
        }
        acc_col[t] += (p0 + p1) + (p2 + p3);
      }
    }
    // ---- dH = dz W, dZ = dH (1 - H^2): wave w takes column tiles 2w, 2w + 1 over both row tiles
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int ct = 2 * w + c, col = 32 * ct + li;
#pragma unroll
      for (int rt = 0; rt < NRT; rt++) {
        tw_f32x16 acc;
#pragma unroll
        for (int v = 0; v < 16; v++) acc[v] = 0.f;
#pragma unroll
        for (int s = 0; s < (A + 1) / 2; s++) {
          const int a = 2 * s + kh;  // W_out row a < A (row A of an odd A: zero)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sz[(32 * rt + li) * ZS + a], a < A ? ws[a * HS + col] : 0.f,
                                                     acc, 0, 0, 0);
        }
        float* out = p.dzh + ((size_t)net * n + r0) * K + col;
#pragma unroll
        for (int v = 0; v < 16; v++) {
          const int row = 32 * rt + (v & 3) + 8 * (v >> 2) + 4 * kh;
          const float y = hs[row * HS + col];
          const float dzv = acc[v] * (1.f - y * y);
          if (row < rows) out[(size_t)row * K] = dzv;
          csacc[c] += dzv;
        }
      }
    }
    // ---- the output weight gradient dz^T H, accumulated over the chunks: column tiles 2w, 2w + 1
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int col = 32 * (2 * w + c) + li;
#pragma unroll 8
      for (int s = 0; s < R / 2; s++)
        gwacc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(sz[(2 * s + kh) * ZS + li], hs[(2 * s + kh) * HS + col],
                                                        gwacc[c], 0, 0, 0);
    }
  }
  float (*csh)[K] = reinterpret_cast<float (*)[K]>(red);  // red is free after the last chunk's z sums
  // ---- the workgroup's partials
  const int nb = S;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const int col = 32 * (2 * w + c) + li;
#pragma unroll
    for (int v = 0; v < 16; v++) {
      const int a = (v & 3) + 8 * (v >> 2) + 4 * kh;
      if (a < A) p.gw[(((size_t)net * nb + blk) * A + a) * K + col] = gwacc[c][v];
    }
    csh[kh][col] = csacc[c];
  }
  __syncthreads();
  if (t < K) p.cs[((size_t)net * nb + blk) * K + t] = csh[0][t] + csh[1][t];
  if (net == 0) {
    if (t == 0) {
      float val = -acc_col[2 * 32] / nf;
      if (blk == 0) val -= p.ent_coef * (0.5f * ((float)A + lss_s) / (float)A);  // entropy, train_ppo.py:215
      p.lossp[blk] = val;
    }
    if (t < A) {
      const float ls = p.log_std[t];
      const float val = blk == 0 ? acc_col[t] - p.ent_coef / (float)A : acc_col[t];
      p.glsp[(size_t)blk * A + t] = (ls >= p.ls_lo && ls <= p.ls_hi) ? val : 0.f;
      p.biasp[(size_t)blk * A + t] = acc_col[32 + t];
    }
  } else if (t < A) {
    p.biasp[((size_t)nb + blk) * A + t] = t == 0 ? acc_col[32] : 0.f;
  }
}

}  // namespace mjl
