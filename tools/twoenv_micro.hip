// Two envs per wave, priced on the step kernel's hottest dense routine: the
// augmented Cholesky factor + solve of one 27 x 27 SPD system (the Newton Hessian / M with the
// right-hand side riding along as row 27), as the product runs it — one env per 64-lane wave, row i
// in lanes i and i + 32 (the duplicated half feeds the MFMA trailing update) — against two envs per
// wave, env A on lanes 0-31 and env B on lanes 32-63:
//   V60: per-half broadcasts as two v_readlane + a select; trailing update on the two-block MFMA
//        v_mfma_f32_32x32x1_2b_f32 (block b = env b, rank-1 per instruction), one v_permlane32_swap
//        per accumulator pair hands each env's lanes both row halves;
//   V61: as V60, the column broadcasts through LDS (each lane writes its column-k element, every lane
//        reads its half's column with 16-byte broadcast reads: fewer instructions, LDS latency on the
//        column chain);
//   V62: as V60, the per-half broadcast as v_readlane + v_permlane32_swap (lane k of the upper half
//        reaches the lower half's register without a select).
// Diagnostic tool, not product. Reports per variant: s_memtime cycles per call (wave latency), kernel
// time per env-factor over B envs (throughput, HIP events), and the max deviation from the product.
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -fapprox-func -fno-slp-vectorize \
//          -o tools/twoenv_micro tools/twoenv_micro.hip
// Run:   tools/twoenv_micro [reps]     (B = 1024, 2048, 4096 envs)
#include "../mujoco-mjx-lab_amd/csrc/step_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace mjl;
using D = DHum;
constexpr int NV = D::NV, LD = D::LD, R = NV;
typedef float f32x32 __attribute__((ext_vector_type(32)));

struct EnvWS {  // one env's matrices (the product's layout: rows of stride LD)
  alignas(16) float S[NV * LD];
  alignas(16) float L[NV * LD];
  alignas(16) float invd[LD];
  alignas(16) float rhs[LD];
  alignas(16) float col[32];  // V61: the broadcast column
};

__device__ void make_system(LDSA EnvWS& W, int env, int i) {  // row i of env's system (lanes < NV)
  if (i < NV) {
    float g[NV];
    for (int k = 0; k < NV; k++) g[k] = __sinf(0.37f * (env % 97) + 1.3f * i + 0.71f * k);
    for (int j = 0; j < NV; j++) {
      float s = 0.f;
      for (int k = 0; k < NV; k++) s += g[k] * __sinf(0.37f * (env % 97) + 1.3f * j + 0.71f * k);
      W.S[i * LD + j] = s / NV + (i == j ? 1.f + 0.1f * i : 0.f);
    }
    W.rhs[i] = __cosf(0.5f * i + env);
    W.S[i * LD + NV] = 0.f;
  }
  if (i >= NV && i < LD) W.rhs[i] = 0.f;
}

// per-half broadcast of lane k of each 32-lane half
INL float hb_sel(float x, int k, bool hi) {
  const float a = rdlane(x, k), b = rdlane(x, k + 32);
  return hi ? b : a;
}
INL float hb_swap(float x, int k) {  // lane k (lower half) via readlane; lane k + 32 via the swap
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  // r[1]: lanes 0-31 hold lanes 32-63's x, lanes 32-63 their own: readlane of lane k from r[1] is the
  // upper half's lane k + 32; the lower half's comes from x itself
  const float a = rdlane(x, k), b = rdlane(__uint_as_float(r[1]), k);
  return (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 32) ? b : a;
}

template <int BV, int P0, int P1>
INL void panel2(float (&a)[LD], bool hi, LDSA float* col) {
#pragma unroll
  for (int k = P0; k < P1; k++) {
    float piv, s[P1];
    if constexpr (BV == 1) {  // LDS column: lane j writes a[k] to col[j] of its half, all read it back
      col[__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 31] = a[k];
      piv = col[k];
#pragma unroll
      for (int j = k + 1; j < P1; j++) s[j] = col[j];
    } else if constexpr (BV == 2) {
      piv = hb_swap(a[k], k);
#pragma unroll
      for (int j = k + 1; j < P1; j++) s[j] = hb_swap(a[k], j);
    } else {
      piv = hb_sel(a[k], k, hi);
#pragma unroll
      for (int j = k + 1; j < P1; j++) s[j] = hb_sel(a[k], j, hi);
    }
    const float inv = __builtin_amdgcn_rsqf(piv);
    a[k] *= inv;
    const float t = a[k] * inv;
#pragma unroll
    for (int j = k + 1; j < P1; j++) a[j] = fmaf(-t, s[j], a[j]);
  }
  if constexpr (P1 < NV) {
    f32x32 acc;
#pragma unroll
    for (int v = 0; v < 32; v++) acc[v] = 0.f;
#pragma unroll
    for (int k = P0; k < P1; k++) acc = __builtin_amdgcn_mfma_f32_32x32x1f32(a[k], a[k], acc, 0, 0, 0);
    float lo[16], hi16[16];
#pragma unroll
    for (int v = 0; v < 16; v++) {
      bool used = false;
#pragma unroll
      for (int j = P1; j < NV; j++) used |= ((j & 3) + 4 * (j >> 3)) == v;
      if (used) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[v]), __float_as_uint(acc[v + 16]), false, false);
        lo[v] = __uint_as_float(r[0]);
        hi16[v] = __uint_as_float(r[1]);
      }
    }
#pragma unroll
    for (int j = P1; j < NV; j++) {
      const int v = (j & 3) + 4 * (j >> 3);
      a[j] -= ((j >> 2) & 1) ? hi16[v] : lo[v];
    }
  }
}

// one env, the product's layout (row i in lanes i and i + 32), the factor's column broadcasts through
// LDS as in V61 (the back substitution keeps its readlane chain)
template <int P0, int P1> INL void panel1_lds(float (&a)[LD], int kh, LDSA float* col) {
#pragma unroll
  for (int k = P0; k < P1; k++) {
    col[__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 31] = a[k];
    const float piv = col[k];
    float s[P1];
#pragma unroll
    for (int j = k + 1; j < P1; j++) s[j] = col[j];
    const float inv = __builtin_amdgcn_rsqf(piv);
    a[k] *= inv;
    const float t = a[k] * inv;
#pragma unroll
    for (int j = k + 1; j < P1; j++) a[j] = fmaf(-t, s[j], a[j]);
  }
  if constexpr (P1 < NV) {
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; v++) acc[v] = 0.f;
#pragma unroll
    for (int t = P0 / 2; t < P1 / 2; t++) {
      const float op = kh ? a[2 * t + 1] : a[2 * t];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(op, op, acc, 0, 0, 0);
    }
    float lo[16], hi[16];
#pragma unroll
    for (int v = 0; v < 16; v++) {
      bool used = false;
#pragma unroll
      for (int j = P1; j < NV; j++) used |= ((j & 3) + 4 * (j >> 3)) == v;
      if (used) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[v]), __float_as_uint(acc[v]), false, false);
        lo[v] = __uint_as_float(r[0]);
        hi[v] = __uint_as_float(r[1]);
      }
    }
#pragma unroll
    for (int j = P1; j < NV; j++) {
      const int v = (j & 3) + 4 * (j >> 3);
      a[j] -= ((j >> 2) & 1) ? hi[v] : lo[v];
    }
  }
}

INL float factor_solve1_lds(LDSA EnvWS& W, int lane) {
  const int i = lane & 31, kh = lane >> 5;
  float a[LD];
  {
    const LDSA f32x4* rp = (const LDSA f32x4*)((i < NV) ? W.S + i * LD : W.rhs);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      const f32x4 v = rp[q];
#pragma unroll
      for (int e = 0; e < 4; e++) a[4 * q + e] = v[e];
    }
  }
  panel1_lds<0, 8>(a, kh, W.col);
  panel1_lds<8, 16>(a, kh, W.col);
  panel1_lds<16, NV>(a, kh, W.col);
  if (lane <= R) {
    LDSA f32x4* wp = (LDSA f32x4*)((i == R) ? W.invd : W.L + i * LD);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      f32x4 v;
      v[0] = a[4 * q]; v[1] = a[4 * q + 1]; v[2] = a[4 * q + 2]; v[3] = a[4 * q + 3];
      wp[q] = v;
    }
  }
  const int ic = (i < NV) ? i : 0;
  const float dg = W.L[ic * LD + ic], yv = W.invd[ic];
  float w[NV];
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) w[k] = W.L[k * LD + ic];
  const float y = (i < NV) ? yv : 0.f;
  const float invd = (i < NV) ? __builtin_amdgcn_rcpf(dg) : 1.f;
  if (lane < NV) W.invd[lane] = invd;
  const int io = opaque_int(i);
#pragma unroll
  for (int k = 0; k < NV; k++) w[k] = (io < k) ? w[k] * invd : 0.f;
  float x = y * invd;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) x = fmaf(-w[k], rdlane(x, k), x);
  return x;
}

// two envs: lane l holds row l & 31 of env l >> 5 (row R = the right-hand side)
template <int BV> INL float factor_solve2(LDSA EnvWS* E, int lane) {
  const int i = lane & 31;
  const bool hi = lane >= 32;
  LDSA EnvWS& W = E[hi ? 1 : 0];
  float a[LD];
  {
    const LDSA f32x4* rp = (const LDSA f32x4*)((i < NV) ? W.S + i * LD : W.rhs);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      const f32x4 v = rp[q];
#pragma unroll
      for (int e = 0; e < 4; e++) a[4 * q + e] = v[e];
    }
  }
  panel2<BV, 0, 8>(a, hi, W.col);
  panel2<BV, 8, 16>(a, hi, W.col);
  panel2<BV, 16, NV>(a, hi, W.col);
  if (i <= R) {
    LDSA f32x4* wp = (LDSA f32x4*)((i == R) ? W.invd : W.L + i * LD);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      f32x4 v;
      v[0] = a[4 * q]; v[1] = a[4 * q + 1]; v[2] = a[4 * q + 2]; v[3] = a[4 * q + 3];
      wp[q] = v;
    }
  }
  const int ic = (i < NV) ? i : 0;
  const float dg = W.L[ic * LD + ic], yv = W.invd[ic];
  float w[NV];
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) w[k] = W.L[k * LD + ic];
  const float y = (i < NV) ? yv : 0.f;
  const float invd = (i < NV) ? __builtin_amdgcn_rcpf(dg) : 1.f;
  if (i < NV) W.invd[i] = invd;
  const int io = opaque_int(i);
#pragma unroll
  for (int k = 0; k < NV; k++) w[k] = (io < k) ? w[k] * invd : 0.f;
  float x = y * invd;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) {
    const float xk = BV == 2 ? hb_swap(x, k) : hb_sel(x, k, hi);
    x = fmaf(-w[k], xk, x);
  }
  return x;
}

// V0: the product (one env per wave); V60-62: two envs per wave. Each wave runs `reps` calls.
template <int V> __global__ __launch_bounds__(64, 2) void kern(unsigned long long* tout, float* out, int reps) {
  constexpr int EPW = (V == 0 || V == 63) ? 1 : 2;  // envs per wave
  __shared__ EnvWS Wsh[EPW];
  LDSA EnvWS* E = (LDSA EnvWS*)Wsh;
  const int lane = threadIdx.x, wave = blockIdx.x;
  for (int e = 0; e < EPW; e++) {
    const int env = wave * EPW + e;
    make_system(E[e], env, lane);
  }
  SYNC();
  float x = 0.f;
  unsigned long long tot = 0;
  for (int r = 0; r < reps; r++) {
    SYNC();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) x = chol_aug_factor_solve<D, false>(E[0].S, E[0].L, E[0].invd, NV, E[0].rhs, lane);
    else if constexpr (V == 63) x = factor_solve1_lds(E[0], lane);
    else x = factor_solve2<V - 60>(E, lane);
    SYNC();
    tot += __builtin_amdgcn_s_memtime() - t0;
  }
  if (lane == 0) tout[wave] = tot / reps;
  // env e's solution x_i in out[env * 32 + i]
  if (EPW == 1) {
    if (lane < 32) out[wave * 32 + lane] = x;
  } else {
    out[(wave * 2 + (lane >> 5)) * 32 + (lane & 31)] = x;
  }
}

// lds_per_env > 0: pad each workgroup's LDS to lds_per_env bytes per env (the step kernel's 20 KB
// workspace: 2 envs per SIMD in either layout) -- the residency the real kernel would have
template <int V> void run(int B, int reps, const char* name, std::vector<float>* ref, int lds_per_env = 0) {
  constexpr int EPW = (V == 0 || V == 63) ? 1 : 2;
  const int waves = B / EPW;
  const size_t pad = lds_per_env > 0 ? (size_t)EPW * (lds_per_env - (int)sizeof(EnvWS)) : 0;
  unsigned long long* t;
  float* o;
  hipMalloc(&t, waves * 8);
  hipMalloc(&o, B * 32 * 4);
  kern<V><<<waves, 64, pad>>>(t, o, 2);  // warm-up
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  kern<V><<<waves, 64, pad>>>(t, o, reps);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> th(waves);
  std::vector<float> oh(B * 32);
  hipMemcpy(th.data(), t, waves * 8, hipMemcpyDeviceToHost);
  hipMemcpy(oh.data(), o, B * 32 * 4, hipMemcpyDeviceToHost);
  double m = 0;
  for (auto v : th) m += v;
  m /= waves;
  double dev = 0;
  if (ref && !ref->empty()) {
    for (int e = 0; e < B; e++)
      for (int l = 0; l < NV; l++)
        dev = fmax(dev, fabs(oh[e * 32 + l] - (*ref)[e * 32 + l]) / (1 + fabs((*ref)[e * 32 + l])));
  } else if (ref) {
    *ref = oh;
  }
  printf("B %5d  %-52s waves/SIMD %.2f  %7.0f cycles/call/wave  %7.2f ns per env-factor  max rel dev %.2e\n", B,
         name, pad ? fmin(waves / 1024.0, 2.0 / EPW) : waves / 1024.0, m, ms * 1e6 / ((double)reps * B), dev);
  hipFree(t);
  hipFree(o);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  for (int B : {1024, 2048, 4096}) {
    std::vector<float> ref;
    run<0>(B, reps, "product: one env per wave", &ref);
    run<60>(B, reps, "two envs per wave: readlane pair + select", &ref);
    run<61>(B, reps, "two envs per wave: LDS column broadcasts", &ref);
    run<62>(B, reps, "two envs per wave: readlane + permlane32_swap", &ref);
    run<63>(B, reps, "one env per wave: LDS column broadcasts", &ref);
    run<0>(B, reps, "product again", &ref);
  }
  // at the step kernel's residency: 20,480 bytes of LDS per env in both layouts (8 one-env or 4 two-env
  // waves per CU: two envs per SIMD either way; 4096 envs take two rounds in both)
  for (int B : {2048, 4096}) {
    std::vector<float> ref;
    run<0>(B, reps, "20 KB/env: product, one env per wave", &ref, 20480);
    run<61>(B, reps, "20 KB/env: two envs per wave, LDS broadcasts", &ref, 20480);
    run<0>(B, reps, "20 KB/env: product again", &ref, 20480);
  }
  return 0;
}
