// Micro-benchmark of the in-wave dense Cholesky factor + solve used by the step kernel (nv = 27,
// one env per 64-lane wave, 2 waves per SIMD as in the step kernel). Diagnostic tool, not product.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/chol_micro tools/chol_micro.hip
// Prints mean s_memtime cycles per call for each variant and the max deviation from variant 0.
#include "../mujoco-mjx-lab_amd/csrc/step_kernels.hip"

#include <cstdio>
#include <vector>

using namespace mjl;
using D = DHum;
constexpr int NV = D::NV, LD = D::LD;

struct MicroWS {
  alignas(16) float S[NV * LD];
  alignas(16) float L[NV * LD];
  float invd[LD];
  float rhs[LD];
  float pad[(kLdsBudget - 2 * NV * LD * 4 - 2 * LD * 4) / 4];  // same LDS per wave as the step kernel
};

// Measured alternative (slower, kept for the record): the whole matrix resident in one
// v_mfma_f32_32x32x2_f32 accumulator, one rank-1 MFMA per column; 64-cycle MFMA latency per
// column, and both waves of a SIMD share its matrix core.
template <class D> INL f32x16 chol_acc_prep(f32x16 acc, bool add_acc, const LDSA float* src, float dg, int n,
                                            const LDSA float* rhs, int lane) {
  constexpr int NV = D::NV, LD = D::LD, R = NV;
  const int col = lane & 31, h = lane >> 5;
  const float rc = (col < n) ? rhs[col] : 0.f;
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int row = (v & 3) + 8 * (v >> 2) + 4 * h;
    float val;
    if (row < n && col < n) {
      val = src[row * LD + col] + (add_acc ? acc[v] : 0.f) + (row == col ? dg : 0.f);
    } else {
      val = (row == col && row < NV) ? 1.f : 0.f;
      if (row == R && col < n) val = rc;
      if (col == R && row < n) val = rhs[row];
    }
    acc[v] = -val;
  }
  return acc;
}

template <class D> INL float chol_acc_factor_solve(f32x16 acc, LDSA float* dst, LDSA float* invd_out, int lane) {
  constexpr int NV = D::NV, LD = D::LD, R = NV;
  static_assert(NV < 32, "the accumulator Cholesky keeps the right-hand side in column NV < 32");
  const int i = lane & 31, h = lane >> 5;
  float y = 0.f, invd = 1.f;
#pragma unroll
  for (int k = 0; k < NV; k++) {
    const int hk = (k >> 2) & 1, vk = (k & 3) + 4 * (k >> 3);
    const float piv = fmaxf(-rdlane(acc[vk], k + 32 * hk), 1e-30f);
    const float inv = __builtin_amdgcn_rsqf(piv);
    const float lv = acc[vk] * -inv;  // half hk, lane j: L[j][k] (j >= k), residue for j < k
    const float op = (h == hk) ? lv : 0.f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(op, op, acc, 0, 0, 0);
    const float yk = rdlane(lv, R + 32 * hk);
    if (h == hk && i < NV) dst[i * LD + k] = (i >= k) ? lv : 0.f;
    const bool sel = i == k;
    y = sel ? yk : y;
    invd = sel ? inv : invd;
  }
  if (lane < NV) invd_out[lane] = invd;
  SYNC();
  // back substitution L^T z = y: column i of L from the rows just written
  float lc[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) lc[k] = (i < k) ? dst[k * LD + i] : 0.f;
  float x = y;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) {
    const float zk = rdlane(x * invd, k);
    x = (i == k) ? zk : ((i < k) ? fmaf(-lc[k], zk, x) : x);
  }
  return x;
}

// Factor + solve in one pass, for the hot callers (M in forward / integrate, the Newton Hessian):
// L L^T = S (S: n x n SPD in LDS at src, stride LD), L written to dst (upper zeroed) with

template <int V> __global__ __launch_bounds__(64, 2) void kern(unsigned long long* tout, float* out, int reps) {
  __shared__ MicroWS Wsh;
  LDSA MicroWS& W = *(LDSA MicroWS*)&Wsh;
  const int lane = threadIdx.x, env = blockIdx.x;
  if (lane < NV) {
    float g[NV];
    for (int k = 0; k < NV; k++) g[k] = __sinf(0.37f * (env % 97) + 1.3f * lane + 0.71f * k);
    for (int j = 0; j < NV; j++) {
      float s = 0.f;
      for (int k = 0; k < NV; k++) s += g[k] * __sinf(0.37f * (env % 97) + 1.3f * j + 0.71f * k);
      W.S[lane * LD + j] = s / NV + (lane == j ? 1.f + 0.1f * lane : 0.f);
    }
    W.rhs[lane] = __cosf(0.5f * lane + env);
  }
  if (lane < LD) W.S[lane * LD + NV] = 0.f;
  SYNC();
  float x = 0.f;
  if constexpr (V == 5) chol_rows_factor_solve<D>(W.S, W.L, W.invd, NV, W.rhs, lane);
  if constexpr (V == 4) {
    if (lane < NV)
      for (int j = 0; j < NV; j++) W.L[lane * LD + j] = W.S[lane * LD + j];
    SYNC();
  }
  unsigned long long tot = 0;
  for (int r = 0; r < reps; r++) {
    SYNC();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) {
      x = chol_rows_factor_solve<D>(W.S, W.L, W.invd, NV, W.rhs, lane);
    } else if constexpr (V == 1) {
      x = chol_aug_factor_solve<D>(W.S, W.L, W.invd, NV, W.rhs, lane);
    } else if constexpr (V == 2) {
      f32x16 z = {};
      x = chol_acc_factor_solve<D>(chol_acc_prep<D>(z, false, W.S, 0.f, NV, W.rhs, lane), W.L, W.invd, lane);
    } else if constexpr (V == 4) {
      chol_factor<D>(W.S, W.invd, NV, lane);  // in place: restore S below (outside the timed region)
    } else if constexpr (V == 5) {
      x = chol_solve<D>(W.L, W.invd, (lane & 31) < NV ? W.rhs[lane & 31] : 0.f, lane);
    }
    SYNC();
    tot += __builtin_amdgcn_s_memtime() - t0;
    if constexpr (V == 4) {
      if (lane < NV)
        for (int j = 0; j < NV; j++) W.S[lane * LD + j] = W.L[lane * LD + j];
    }
  }
  if (lane == 0) tout[env] = tot / reps;
  out[env * 64 + lane] = x;
}

template <int V> void run(int B, const char* name, std::vector<float>* ref) {
  unsigned long long* t;
  float* o;
  hipMalloc(&t, B * 8);
  hipMalloc(&o, B * 64 * 4);
  kern<V><<<B, 64>>>(t, o, 2);
  hipDeviceSynchronize();
  kern<V><<<B, 64>>>(t, o, 8);
  hipDeviceSynchronize();
  std::vector<unsigned long long> th(B);
  std::vector<float> oh(B * 64);
  hipMemcpy(th.data(), t, B * 8, hipMemcpyDeviceToHost);
  hipMemcpy(oh.data(), o, B * 64 * 4, hipMemcpyDeviceToHost);
  double m = 0;
  for (auto v : th) m += v;
  m /= B;
  double dev = 0;
  if (ref && !ref->empty()) {
    for (int e = 0; e < B; e++)
      for (int l = 0; l < NV; l++) dev = fmax(dev, fabs(oh[e * 64 + l] - (*ref)[e * 64 + l]) / (1 + fabs((*ref)[e * 64 + l])));
  } else if (ref) {
    *ref = oh;
  }
  printf("%-34s %8.0f cycles/call   max rel dev vs rows %.2e\n", name, m, dev);
  hipFree(t);
  hipFree(o);
}

int main() {
  const int B = 2048;
  std::vector<float> ref;
  run<0>(B, "rows factor+solve (previous)", &ref);
  run<1>(B, "augmented rows factor+solve", &ref);
  run<2>(B, "accumulator factor+solve", &ref);
  run<4>(B, "rows factor only (chol_factor)", nullptr);
  run<5>(B, "rows solve only (chol_solve)", nullptr);
  return 0;
}
