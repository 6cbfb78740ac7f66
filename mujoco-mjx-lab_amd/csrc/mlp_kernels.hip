// Dense-layer kernels of the PPO update (reference train_ppo.py:204-252: jax.value_and_grad of
// ppo_loss_fn / value_loss_fn through the src/networks.py:22-61 MLPs, 65,536-row minibatches), on the
// fp32 matrix cores (v_mfma_f32_32x32x2_f32: exact f32, a k-ordered fma chain per output).
//
//  mlp_fwd_kernel   Y = act(X W^T + b)          bias + tanh in the epilogue (no separate pass over Y)
//  mlp_dx_tanh_kernel  D = (G W) (1 - Y^2)     the input gradient with the lower layer's tanh' and its
//                   bias gradient's column-sum partials in the epilogue (the twin update's backward)
//  mlp_bwd_kernel   dZ = act'(G, Y) = G (1 - Y^2) (tanh) or G (identity), formed while the A tile is
//                   staged; writes dZ (for the weight gradient), its per-row-block column sums (the bias
//                   gradient, reduced in a fixed order by mjl_colsum) and dX = dZ W
// Layouts are torch's: X [M, K], Y / G / dZ [M, N], W [N, K] (nn.Linear.weight), all row-major fp32.
// The weight gradient dW = dZ^T X stays a split-K batched GEMM + sum (mjx_amd/ppo.py _FusedMLP).
//
// Tiling: a workgroup of WM x WN waves computes a BM x BN output tile over the reduction in steps of
// BK; each wave holds (BM / WM / 32) x (BN / WN / 32) accumulators of 32 x 32 (16 registers).
// Operand order: MFMA s of a step takes reduction index s from lanes 0-31 and s + BK/2 from lanes
// 32-63 (lane l: A[i = l & 31][k], B[k][j = l & 31]), so a lane's operands for four consecutive MFMAs
// are four consecutive k of ONE row of a row-major tile: the tiles are staged untransposed — X and
// G / Y rows as they lie in memory, W's rows as the B operand of the forward — with 16-B global loads
// and 16-B LDS stores, and read back as ds_read_b128 (row stride BK + 4 floats: the eight rows an
// 8-lane group reads land on disjoint banks); the backward's B (W, whose rows are the reduction
// index there) is staged k-major as it lies and read four b32 at a time. Each output is still a sum
// over every k of its row / column, in a fixed (permuted) order. Two LDS buffers and two register
// sets: tile s + 2's global loads are in flight while step s computes and tile s + 1 is stored.
// C layout (32x32, every dtype on gfx950): col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
#pragma once
#include <hip/hip_runtime.h>

namespace mjl {

constexpr int kMlpPad = 4;
typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { MLP_ACT_NONE = 0, MLP_ACT_TANH = 1 };

// Staging of one [R rows x BK] slice of a row-major source (rows r0.., reduction columns k0..) into
// registers, stored row-major into dst[r * (BK + pad) + k]. VEC: float4 loads along the reduction
// (the source's row stride, k0 and kmax multiples of 4, 16-B aligned base).
template <int R, int T, bool VEC, int BK> struct Stage {
  static constexpr int PER = R * BK / T / (VEC ? 4 : 1);
  static_assert(PER >= 1 && R * BK % (T * (VEC ? 4 : 1)) == 0, "tile / thread mapping");
  float v[PER * (VEC ? 4 : 1)];
  __device__ __forceinline__ void load(const float* __restrict__ src, long long ld, int r0, int rmax, int k0, int kmax,
                                       int tid) {
#pragma unroll
    for (int p = 0; p < PER; p++) {
      if constexpr (VEC) {
        const int q = tid + p * T, r = q / (BK / 4), kq = (q % (BK / 4)) * 4;
        const int gr = r0 + r, gk = k0 + kq;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gr < rmax && gk < kmax) x = *(const float4*)(src + (size_t)gr * ld + gk);
        v[4 * p] = x.x; v[4 * p + 1] = x.y; v[4 * p + 2] = x.z; v[4 * p + 3] = x.w;
      } else {
        const int q = tid + p * T, r = q / BK, k = q % BK;
        const int gr = r0 + r, gk = k0 + k;
        v[p] = (gr < rmax && gk < kmax) ? src[(size_t)gr * ld + gk] : 0.f;
      }
    }
  }
  __device__ __forceinline__ void store(float* dst, int tid) const {
#pragma unroll
    for (int p = 0; p < PER; p++) {
      if constexpr (VEC) {
        const int q = tid + p * T, r = q / (BK / 4), kq = (q % (BK / 4)) * 4;
        *(float4*)(dst + r * (BK + kMlpPad) + kq) = make_float4(v[4 * p], v[4 * p + 1], v[4 * p + 2], v[4 * p + 3]);
      } else {
        const int q = tid + p * T, r = q / BK, k = q % BK;
        dst[r * (BK + kMlpPad) + k] = v[p];
      }
    }
  }
};

// Staging of a [BK x C] slice of a row-major source whose rows ARE the reduction index (W [N, K] as
// the B operand of dX = dZ W), kept k-major: dst[k * (C + pad) + c]; float4 loads and stores along c.
template <int C, int T, int BK> struct StageK {
  static constexpr int PER = BK * C / T / 4;
  static_assert(PER >= 1 && BK * C % (T * 4) == 0, "tile / thread mapping");
  float4 v[PER];
  __device__ __forceinline__ void load(const float* __restrict__ src, long long ld, int k0, int kmax, int c0, int cmax,
                                       int tid) {
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const int q = tid + p * T, k = q / (C / 4), c = (q % (C / 4)) * 4;
      const int gk = k0 + k, gc = c0 + c;
      v[p] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gk < kmax && gc < cmax) v[p] = *(const float4*)(src + (size_t)gk * ld + gc);  // cmax % 4 == 0
    }
  }
  __device__ __forceinline__ void store(float* dst, int tid) const {
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const int q = tid + p * T, k = q / (C / 4), c = (q % (C / 4)) * 4;
      *(float4*)(dst + k * (C + kMlpPad) + c) = v[p];
    }
  }
};

// the wave's MFMAs over one staged step: acc[tm][tn] += sum_k A[i][k] B[k][j]. As[i][k] row-major
// (stride BK + pad); B either as Bs[j][k] row-major (BROW, the forward's W rows) or k-major Bs[k][j]
// (stride BN + pad, the backward's W as it lies). Lane l takes k from half (l >> 5) of the step, four
// k at a time (one ds_read_b128 of A per tile row; B one b128 or four b32), the next four's fragments
// loaded before the current four's MFMAs issue.
template <int BK, int BN, int TM, int TN, bool BROW>
__device__ __forceinline__ void mlp_mma_step(const float* As, const float* Bs, int wi, int wj, int lane,
                                             f32x16 (&acc)[TM][TN]) {
  constexpr int S = BK + kMlpPad, SBK = BN + kMlpPad;
  const int kh = (lane >> 5) * (BK / 2), il = lane & 31;
  float4 a[2][TM], b[2][TN];
  auto frag = [&](int buf, int k4) {
#pragma unroll
    for (int tm = 0; tm < TM; tm++) a[buf][tm] = *(const float4*)(As + (wi + tm * 32 + il) * S + kh + k4);
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
      if constexpr (BROW) {
        b[buf][tn] = *(const float4*)(Bs + (wj + tn * 32 + il) * S + kh + k4);
      } else {
        const float* bp = Bs + (kh + k4) * SBK + wj + tn * 32 + il;
        b[buf][tn] = make_float4(bp[0], bp[SBK], bp[2 * SBK], bp[3 * SBK]);
      }
    }
  };
  frag(0, 0);
#pragma unroll
  for (int k4 = 0; k4 < BK / 2; k4 += 4) {
    const int cur = (k4 >> 2) & 1;
    if (k4 + 4 < BK / 2) frag(cur ^ 1, k4 + 4);
#pragma unroll
    for (int e = 0; e < 4; e++)
#pragma unroll
      for (int tm = 0; tm < TM; tm++)
#pragma unroll
        for (int tn = 0; tn < TN; tn++)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cur][tm][e], b[cur][tn][e], acc[tm][tn], 0, 0, 0);
  }
}

// Y[M, N] = act(X[M, K] W[N, K]^T + b[N]); blockIdx.z selects one of a stack of such problems (the
// twin update's two nets: X at z * sx — sx = 0 for the shared observations —, W at z * sw, b at
// z * sbias, Y at z * sy; act = tanh when bit z of act_mask is set)
template <int BM, int BN, int WM, int WN, bool VECX, int BK = 32>
__global__ __launch_bounds__(WM * WN * 64) void mlp_fwd_kernel(const float* __restrict__ X, int ldx, long long sx,
                                                               const float* __restrict__ W, int ldw, long long sw,
                                                               const float* __restrict__ bias, int sbias,
                                                               float* __restrict__ Y, int ldy, long long sy, int M,
                                                               int N, int K, unsigned act_mask) {
  X += blockIdx.z * sx;
  W += blockIdx.z * sw;
  bias += blockIdx.z * sbias;
  Y += blockIdx.z * sy;
  const int act = (act_mask >> blockIdx.z) & 1u ? MLP_ACT_TANH : MLP_ACT_NONE;
  constexpr int T = WM * WN * 64, TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int SA = BM * (BK + kMlpPad), SB = BN * (BK + kMlpPad);
  __shared__ __attribute__((aligned(16))) float lds[2 * (SA + SB)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i0 = blockIdx.y * BM, j0 = blockIdx.x * BN;  // column tiles of one row block launch together
  const int wi = (wave / WN) * (BM / WM), wj = (wave % WN) * (BN / WN);
  f32x16 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; tm++)
#pragma unroll
    for (int tn = 0; tn < TN; tn++) acc[tm][tn] = f32x16{};
  // two register sets: tile s + 2's loads are in flight while step s computes and tile s + 1 (loaded
  // one step earlier) is stored
  Stage<BM, T, VECX, BK> sa[2];
  Stage<BN, T, VECX, BK> sb[2];
  const int nk = (K + BK - 1) / BK;
  sa[0].load(X, ldx, i0, M, 0, K, tid);
  sb[0].load(W, ldw, j0, N, 0, K, tid);
  if (nk > 1) {
    sa[1].load(X, ldx, i0, M, BK, K, tid);
    sb[1].load(W, ldw, j0, N, BK, K, tid);
  }
  sa[0].store(lds, tid);
  sb[0].store(lds + SA, tid);
  __syncthreads();
  auto step = [&](int s, Stage<BM, T, VECX, BK>& na, Stage<BN, T, VECX, BK>& nb,
                  Stage<BM, T, VECX, BK>& la, Stage<BN, T, VECX, BK>& lb) {
    const float* As = lds + (s & 1) * (SA + SB);
    if (s + 2 < nk) {
      la.load(X, ldx, i0, M, (s + 2) * BK, K, tid);
      lb.load(W, ldw, j0, N, (s + 2) * BK, K, tid);
    }
    mlp_mma_step<BK, BN, TM, TN, true>(As, As + SA, wi, wj, lane, acc);
    if (s + 1 < nk) {
      float* nx = lds + ((s + 1) & 1) * (SA + SB);
      na.store(nx, tid);
      nb.store(nx + SA, tid);
    }
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    step(s, sa[1], sb[1], sa[0], sb[0]);
    if (s + 1 < nk) step(s + 1, sa[0], sb[0], sa[1], sb[1]);
  }
#pragma unroll
  for (int tm = 0; tm < TM; tm++)
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
      const int col = j0 + wj + tn * 32 + (lane & 31);
      const float bc = col < N ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int row = i0 + wi + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M && col < N) {
          const float v = acc[tm][tn][r] + bc;
          Y[(size_t)row * ldy + col] = act == MLP_ACT_TANH ? tanhf(v) : v;
        }
      }
    }
}

// dZ = act'(G, Y) [M, N]; dX[M, K] = dZ W[N, K] (DX); column-sum partials of dZ per BM-row block:
// colpart[blockIdx.y, n] (fixed order: rows in 16-row groups, groups in order). VECG: float4 staging of
// G / Y (N % 4 == 0), else scalar (the heads: N = 21 or 1).
template <int BM, int BN, int WM, int WN, bool DX, bool VECG, int BK = 32>
__global__ __launch_bounds__(WM * WN * 64) void mlp_bwd_kernel(const float* __restrict__ G, const float* __restrict__ Y,
                                                               int ldg, const float* __restrict__ W, int ldw,
                                                               float* __restrict__ dZ, float* __restrict__ dX, int lddx,
                                                               float* __restrict__ colpart, int M, int N, int K, int act) {
  constexpr int T = WM * WN * 64, TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int S = BK + kMlpPad, SA = BM * S, SB = DX ? BK * (BN + kMlpPad) : 0;
  static_assert(T == 256 && BM % 16 == 0 && BM / 16 * BK <= 2 * T, "column-sum mapping");
  __shared__ __attribute__((aligned(16))) float lds[2 * (SA + SB) + (BM / 16) * BK];
  float* red = lds + 2 * (SA + SB);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i0 = blockIdx.y * BM, j0 = blockIdx.x * BN;
  const bool lead = blockIdx.x == 0;  // the column tile that writes dZ and the column sums
  const int wi = (wave / WN) * (BM / WM), wj = (wave % WN) * (BN / WN);
  f32x16 acc[TM][TN];
  if constexpr (DX) {
#pragma unroll
    for (int tm = 0; tm < TM; tm++)
#pragma unroll
      for (int tn = 0; tn < TN; tn++) acc[tm][tn] = f32x16{};
  }
  typedef Stage<BM, T, VECG, BK> SG;
  typedef StageK<BN, T, BK> SW;
  SG sg[2], sy[2];
  SW sw[2];
  const int nk = (N + BK - 1) / BK;
  // dZ of a staged slice, in the registers that hold G: written to global by the lead tile
  auto form = [&](SG& g_, const SG& y_, int k0) {
#pragma unroll
    for (int e = 0; e < SG::PER * (VECG ? 4 : 1); e++) {
      const float g = g_.v[e], y = y_.v[e];
      g_.v[e] = act == MLP_ACT_TANH ? g * (1.f - y * y) : g;
    }
    if (!lead) return;
#pragma unroll
    for (int p = 0; p < SG::PER; p++) {
      if constexpr (VECG) {
        const int q = tid + p * T, r = q / (BK / 4), kq = (q % (BK / 4)) * 4;
        const int gr = i0 + r, gk = k0 + kq;
        if (gr < M && gk < N)
          *(float4*)(dZ + (size_t)gr * ldg + gk) = make_float4(g_.v[4 * p], g_.v[4 * p + 1], g_.v[4 * p + 2], g_.v[4 * p + 3]);
      } else {
        const int q = tid + p * T, r = q / BK, k = q % BK;
        const int gr = i0 + r, gk = k0 + k;
        if (gr < M && gk < N) dZ[(size_t)gr * ldg + gk] = g_.v[p];
      }
    }
  };
  auto colsum = [&](const float* As, int k0) {  // 16-row group sums, then the groups in order
    if (!lead) return;
    for (int q = tid; q < (BM / 16) * BK; q += T) {
      const int k = q % BK, g = q / BK;
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 16; r++) s += As[(g * 16 + r) * S + k];
      red[g * BK + k] = s;
    }
    __syncthreads();
    if (tid < BK && k0 + tid < N) {
      float s = 0.f;
      for (int g = 0; g < BM / 16; g++) s += red[g * BK + tid];
      colpart[(size_t)blockIdx.y * N + k0 + tid] = s;
    }
  };
  auto load = [&](int t, SG& g_, SG& y_, SW& w_) {
    g_.load(G, ldg, i0, M, t * BK, N, tid);
    y_.load(Y, ldg, i0, M, t * BK, N, tid);
    if constexpr (DX) w_.load(W, ldw, t * BK, N, j0, K, tid);
  };
  auto put = [&](int t, SG& g_, const SG& y_, const SW& w_) {
    form(g_, y_, t * BK);
    float* nx = lds + (t & 1) * (SA + SB);
    g_.store(nx, tid);
    if constexpr (DX) w_.store(nx + SA, tid);
  };
  load(0, sg[0], sy[0], sw[0]);
  if (nk > 1) load(1, sg[1], sy[1], sw[1]);
  put(0, sg[0], sy[0], sw[0]);
  __syncthreads();
  auto step = [&](int s, SG& ng, SG& ny, SW& nw, SG& lg, SG& ly, SW& lw) {
    const float* As = lds + (s & 1) * (SA + SB);
    if (s + 2 < nk) load(s + 2, lg, ly, lw);
    if constexpr (DX) mlp_mma_step<BK, BN, TM, TN, false>(As, As + SA, wi, wj, lane, acc);
    colsum(As, s * BK);
    if (s + 1 < nk) put(s + 1, ng, ny, nw);
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    step(s, sg[1], sy[1], sw[1], sg[0], sy[0], sw[0]);
    if (s + 1 < nk) step(s + 1, sg[0], sy[0], sw[0], sg[1], sy[1], sw[1]);
  }
  if constexpr (DX) {
#pragma unroll
    for (int tm = 0; tm < TM; tm++)
#pragma unroll
      for (int tn = 0; tn < TN; tn++) {
        const int col = j0 + wj + tn * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int row = i0 + wi + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < M && col < K) dX[(size_t)row * lddx + col] = acc[tm][tn][r];
        }
      }
  }
}

// The backward's input-gradient GEMM with the tanh derivative of the layer below in its epilogue:
// D = (G W) (1 - Y^2) over a stack of problems (blockIdx.z): G [M, N] = dZ of this layer, W [N, K],
// Y [M, K] = the tanh output feeding this layer, D [M, K] = dZ of that layer (the dH = G W of autograd
// never reaches memory: the separate tanh-backward pass re-read it and Y). part[z][blockIdx.y][K]: the
// column sums of D over the block's BM rows (the lower layer's bias gradient, first stage): each lane
// sums its rows in order, the two half-waves pair up, then the WM row waves in order through LDS.
template <int BM, int BN, int WM, int WN, bool VECG, int BK = 32>
__global__ __launch_bounds__(WM * WN * 64) void mlp_dx_tanh_kernel(const float* __restrict__ G, long long sg,
                                                                   const float* __restrict__ W, long long sw,
                                                                   const float* __restrict__ Y, long long sy,
                                                                   float* __restrict__ D, float* __restrict__ part,
                                                                   int M, int N, int K) {
  G += blockIdx.z * sg;
  W += blockIdx.z * sw;
  Y += blockIdx.z * sy;
  D += blockIdx.z * sy;
  part += ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * K;
  constexpr int T = WM * WN * 64, TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int SA = BM * (BK + kMlpPad), SB = BK * (BN + kMlpPad);
  __shared__ __attribute__((aligned(16))) float lds[2 * (SA + SB)];
  __shared__ float red[WM][BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i0 = blockIdx.y * BM, j0 = blockIdx.x * BN;
  const int wr = wave / WN, wi = wr * (BM / WM), wj = (wave % WN) * (BN / WN);
  f32x16 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; tm++)
#pragma unroll
    for (int tn = 0; tn < TN; tn++) acc[tm][tn] = f32x16{};
  typedef Stage<BM, T, VECG, BK> SG;
  typedef StageK<BN, T, BK> SW;
  SG sa[2];
  SW sb[2];
  const int nk = (N + BK - 1) / BK;
  sa[0].load(G, N, i0, M, 0, N, tid);
  sb[0].load(W, K, 0, N, j0, K, tid);
  if (nk > 1) {
    sa[1].load(G, N, i0, M, BK, N, tid);
    sb[1].load(W, K, BK, N, j0, K, tid);
  }
  sa[0].store(lds, tid);
  sb[0].store(lds + SA, tid);
  __syncthreads();
  auto step = [&](int s, SG& na, SW& nb, SG& la, SW& lb) {
    const float* As = lds + (s & 1) * (SA + SB);
    if (s + 2 < nk) {
      la.load(G, N, i0, M, (s + 2) * BK, N, tid);
      lb.load(W, K, (s + 2) * BK, N, j0, K, tid);
    }
    mlp_mma_step<BK, BN, TM, TN, false>(As, As + SA, wi, wj, lane, acc);
    if (s + 1 < nk) {
      float* nx = lds + ((s + 1) & 1) * (SA + SB);
      na.store(nx, tid);
      nb.store(nx + SA, tid);
    }
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    step(s, sa[1], sb[1], sa[0], sb[0]);
    if (s + 1 < nk) step(s + 1, sa[0], sb[0], sa[1], sb[1]);
  }
  float cs[TN];
#pragma unroll
  for (int tn = 0; tn < TN; tn++) {
    cs[tn] = 0.f;
    const int col = j0 + wj + tn * 32 + (lane & 31);
#pragma unroll
    for (int tm = 0; tm < TM; tm++)
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int row = i0 + wi + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M && col < K) {
          const size_t o = (size_t)row * K + col;
          const float y = Y[o];
          const float d = acc[tm][tn][r] * (1.f - y * y);
          D[o] = d;
          cs[tn] += d;
        }
      }
    cs[tn] += __shfl_xor(cs[tn], 32);
    if (lane < 32) red[wr][wj + tn * 32 + lane] = cs[tn];
  }
  __syncthreads();
  for (int c = tid; c < BN; c += T) {
    if (j0 + c >= K) continue;
    float s = red[0][c];
#pragma unroll
    for (int q = 1; q < WM; q++) s += red[q][c];
    part[j0 + c] = s;
  }
}

}  // namespace mjl
