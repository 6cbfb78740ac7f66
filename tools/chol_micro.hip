// Micro-benchmark of the in-wave dense factor + solve used by the step kernel (nv = 27, one env per
// 64-lane wave, 2 waves per SIMD as in the step kernel). Diagnostic tool, not product: candidate
// variants live here until one wins, then move into step_kernels.hip.
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -fapprox-func -fno-slp-vectorize \
//          -o tools/chol_micro tools/chol_micro.hip
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

// ---- candidate: LDL^T panels (no square roots: the multiplier L_ik = a_ik / d_k from one v_rcp
// of the pivot; the trailing update takes the scaled column as A and the saved unscaled column as
// B, sum_k L_ik a_jk = sum_k a_ik a_jk / d_k). Lane k captures 1 / d_k for the solves.
template <int LD, int NV, int P0, int P1> INL void ldl_panel(float (&a)[LD], float& dinv, int io, int kh) {
  float u[P1];
#pragma unroll
  for (int k = P0; k < P1; k++) {
    const float rp = fminf(__builtin_amdgcn_rcpf(rdlane(a[k], k)), 1e30f);
    float s[P1];
#pragma unroll
    for (int j = k + 1; j < P1; j++) s[j] = rdlane(a[k], j);
    u[k] = a[k];
    a[k] *= rp;  // lane i: L_ik
    dinv = (io == k) ? rp : dinv;
#pragma unroll
    for (int j = k + 1; j < P1; j++) a[j] = fmaf(-a[k], s[j], a[j]);
  }
  if constexpr (P1 < NV) {
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; v++) acc[v] = 0.f;
#pragma unroll
    for (int t2 = P0 / 2; t2 < P1 / 2; t2++) {
      const float opA = kh ? a[2 * t2 + 1] : a[2 * t2];
      const float opB = kh ? u[2 * t2 + 1] : u[2 * t2];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(opA, opB, acc, 0, 0, 0);
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
// LDL^T factor + solve: rows of unit L to dst, 1 / d to invd_out; lane R's augmented row ends as
// z = D^-1 L^-1 b, the back substitution runs on unit L^T (no scaling)
INL float ldl_aug_factor_solve(const LDSA float* src, LDSA float* dst, LDSA float* invd_out, const LDSA float* rhs,
                               int lane) {
  constexpr int R = NV;
  const int i = lane & 31, kh = lane >> 5;
  float a[LD];
  {
    const LDSA f32x4* rp = (const LDSA f32x4*)((i < NV) ? src + i * LD : rhs);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      const f32x4 v = rp[q];
#pragma unroll
      for (int e = 0; e < 4; e++) a[4 * q + e] = v[e];
    }
  }
  const int io = opaque_int(i);
  float dinv = 1.f;
  ldl_panel<LD, NV, 0, 8>(a, dinv, io, kh); ldl_panel<LD, NV, 8, 16>(a, dinv, io, kh);
  ldl_panel<LD, NV, 16, 24>(a, dinv, io, kh); ldl_panel<LD, NV, 24, NV>(a, dinv, io, kh);
  if (lane <= R) {
    LDSA f32x4* wp = (LDSA f32x4*)((i == R) ? invd_out : dst + i * LD);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      f32x4 v;
      v[0] = a[4 * q]; v[1] = a[4 * q + 1]; v[2] = a[4 * q + 2]; v[3] = a[4 * q + 3];
      wp[q] = v;
    }
  }
  const int ic = (i < NV) ? i : 0;
  const float zv = invd_out[ic];
  float w[NV];
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) w[k] = dst[k * LD + ic];
  if (lane < NV) invd_out[lane] = dinv;
#pragma unroll
  for (int k = 0; k < NV; k++) w[k] = (io < k) ? w[k] : 0.f;
  float x = (i < NV) ? zv : 0.f;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) x = fmaf(-w[k], rdlane(x, k), x);
  return x;
}

// ---- candidate: the product panel with the MFMA chain split over two accumulators
template <int LD, int NV, int P0, int P1> INL void chol_panel2(float (&a)[LD], int kh) {
#pragma unroll
  for (int k = P0; k < P1; k++) {
    const float inv = fminf(__builtin_amdgcn_rsqf(rdlane(a[k], k)), 1e15f);
    float s[P1];
#pragma unroll
    for (int j = k + 1; j < P1; j++) s[j] = rdlane(a[k], j);
    a[k] *= inv;
    const float t = a[k] * inv;
#pragma unroll
    for (int j = k + 1; j < P1; j++) a[j] = fmaf(-t, s[j], a[j]);
  }
  if constexpr (P1 < NV) {
    f32x16 acc0, acc1;
#pragma unroll
    for (int v = 0; v < 16; v++) { acc0[v] = 0.f; acc1[v] = 0.f; }
#pragma unroll
    for (int t = P0 / 2; t < P1 / 2; t++) {
      const float op = kh ? a[2 * t + 1] : a[2 * t];
      if ((t & 1) == 0) acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(op, op, acc0, 0, 0, 0);
      else acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(op, op, acc1, 0, 0, 0);
    }
    float lo[16], hi[16];
#pragma unroll
    for (int v = 0; v < 16; v++) {
      bool used = false;
#pragma unroll
      for (int j = P1; j < NV; j++) used |= ((j & 3) + 4 * (j >> 3)) == v;
      if (used) {
        const float cv = acc0[v] + acc1[v];
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(cv), __float_as_uint(cv), false, false);
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

// ---- candidate column-step variants of the product panel (CV 1: multiplier from v_rcp beside the
// v_rsq; CV 2: no pivot clamp; CV 3: both)
template <int LD, int NV, int P0, int P1, int CV> INL void chol_panel_cv(float (&a)[LD], int kh) {
#pragma unroll
  for (int k = P0; k < P1; k++) {
    const float piv = rdlane(a[k], k);
    const float inv = (CV & 2) ? __builtin_amdgcn_rsqf(piv) : fminf(__builtin_amdgcn_rsqf(piv), 1e15f);
    const float rp = (CV & 2) ? __builtin_amdgcn_rcpf(piv) : fminf(__builtin_amdgcn_rcpf(piv), 1e30f);
    float s[P1];
#pragma unroll
    for (int j = k + 1; j < P1; j++) s[j] = rdlane(a[k], j);
    if constexpr (CV & 4) {  // scaled broadcasts: a_ij -= L_ik (a_jk inv), one multiply deep
      a[k] *= inv;
#pragma unroll
      for (int j = k + 1; j < P1; j++) a[j] = fmaf(-a[k], s[j] * inv, a[j]);
    } else {
      float t;
      if constexpr (CV & 1) { t = a[k] * rp; a[k] *= inv; }
      else { a[k] *= inv; t = a[k] * inv; }
#pragma unroll
      for (int j = k + 1; j < P1; j++) a[j] = fmaf(-t, s[j], a[j]);
    }
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

// ---- candidate: 2x2 block pivots. Columns k and k + 1 from one set of broadcasts of the panel's
// state before column k: column k + 1's pivot and broadcasts after column k's update are formed
// from the uniform values (the same fma / mul sequence the column step runs in the lanes, so the
// result is bit-identical), which takes one readlane off the dependent chain per two columns.
template <int LD, int NV, int P0, int P1> INL void chol_panel_b2(float (&a)[LD], int kh) {
#pragma unroll
  for (int k = P0; k + 1 < P1; k += 2) {
    const float p = rdlane(a[k], k), b = rdlane(a[k], k + 1), c = rdlane(a[k + 1], k + 1);
    float s1[P1], s1b[P1], s2[P1];
#pragma unroll
    for (int j = k + 2; j < P1; j++) { s1[j] = rdlane(a[k], j); s1b[j] = rdlane(a[k + 1], j); }
    const float inv1 = __builtin_amdgcn_rsqf(p);
    const float tb = (b * inv1) * inv1;
    const float p2 = fmaf(-tb, b, c);
    const float inv2 = __builtin_amdgcn_rsqf(p2);
    a[k] *= inv1;
    const float t1 = a[k] * inv1;
    a[k + 1] = fmaf(-t1, b, a[k + 1]);
#pragma unroll
    for (int j = k + 2; j < P1; j++) {
      a[j] = fmaf(-t1, s1[j], a[j]);
      s2[j] = fmaf(-((s1[j] * inv1) * inv1), b, s1b[j]);
    }
    a[k + 1] *= inv2;
    const float t2 = a[k + 1] * inv2;
#pragma unroll
    for (int j = k + 2; j < P1; j++) a[j] = fmaf(-t2, s2[j], a[j]);
  }
  if constexpr ((P1 - P0) & 1) {
    constexpr int k = P1 - 1;
    const float inv = __builtin_amdgcn_rsqf(rdlane(a[k], k));
    a[k] *= inv;
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

// the product's factor + solve with a pluggable panel and optional stop after the factor
template <int PV, int SOLVE> INL float aug_variant(const LDSA float* src, LDSA float* dst, LDSA float* invd_out,
                                                   const LDSA float* rhs, int lane) {
  constexpr int R = NV;
  const int i = lane & 31, kh = lane >> 5;
  float a[LD];
  {
    const LDSA f32x4* rp = (const LDSA f32x4*)((i < NV) ? src + i * LD : rhs);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      const f32x4 v = rp[q];
#pragma unroll
      for (int e = 0; e < 4; e++) a[4 * q + e] = v[e];
    }
  }
  if constexpr (PV == 0) {
    chol_panel<LD, NV, 0, 8>(a, kh); chol_panel<LD, NV, 8, 16>(a, kh);
    chol_panel<LD, NV, 16, 24>(a, kh); chol_panel<LD, NV, 24, NV>(a, kh);
  } else if constexpr (PV == 1) {
    chol_panel2<LD, NV, 0, 8>(a, kh); chol_panel2<LD, NV, 8, 16>(a, kh);
    chol_panel2<LD, NV, 16, 24>(a, kh); chol_panel2<LD, NV, 24, NV>(a, kh);
  } else if constexpr (PV == 2) {
    chol_panel<LD, NV, 0, 6>(a, kh); chol_panel<LD, NV, 6, 12>(a, kh); chol_panel<LD, NV, 12, 18>(a, kh);
    chol_panel<LD, NV, 18, 24>(a, kh); chol_panel<LD, NV, 24, NV>(a, kh);
  } else if constexpr (PV == 3) {
    chol_panel<LD, NV, 0, 10>(a, kh); chol_panel<LD, NV, 10, 20>(a, kh); chol_panel<LD, NV, 20, NV>(a, kh);
  } else if constexpr (PV >= 21 && PV <= 27) {
    chol_panel_cv<LD, NV, 0, 8, PV - 20>(a, kh); chol_panel_cv<LD, NV, 8, 16, PV - 20>(a, kh);
    chol_panel_cv<LD, NV, 16, 24, PV - 20>(a, kh); chol_panel_cv<LD, NV, 24, NV, PV - 20>(a, kh);
  } else if constexpr (PV == 30) {
    chol_panel_cv<LD, NV, 0, 10, 2>(a, kh); chol_panel_cv<LD, NV, 10, 20, 2>(a, kh); chol_panel_cv<LD, NV, 20, NV, 2>(a, kh);
  } else if constexpr (PV == 31) {
    chol_panel_cv<LD, NV, 0, 12, 2>(a, kh); chol_panel_cv<LD, NV, 12, 24, 2>(a, kh); chol_panel_cv<LD, NV, 24, NV, 2>(a, kh);
  } else if constexpr (PV == 32) {
    chol_panel_cv<LD, NV, 0, 8, 2>(a, kh); chol_panel_cv<LD, NV, 8, 18, 2>(a, kh); chol_panel_cv<LD, NV, 18, NV, 2>(a, kh);
  } else if constexpr (PV == 33) {
    chol_panel_cv<LD, NV, 0, 14, 2>(a, kh); chol_panel_cv<LD, NV, 14, NV, 2>(a, kh);
  } else if constexpr (PV == 40) {
    chol_panel_cv<LD, NV, 0, 8, 2>(a, kh); chol_panel_cv<LD, NV, 8, 20, 2>(a, kh); chol_panel_cv<LD, NV, 20, NV, 2>(a, kh);
  } else if constexpr (PV == 41) {
    chol_panel_cv<LD, NV, 0, 6, 2>(a, kh); chol_panel_cv<LD, NV, 6, 16, 2>(a, kh); chol_panel_cv<LD, NV, 16, NV, 2>(a, kh);
  } else if constexpr (PV == 42) {
    chol_panel_cv<LD, NV, 0, 10, 2>(a, kh); chol_panel_cv<LD, NV, 10, 18, 2>(a, kh); chol_panel_cv<LD, NV, 18, NV, 2>(a, kh);
  } else if constexpr (PV == 43) {
    chol_panel_cv<LD, NV, 0, 8, 2>(a, kh); chol_panel_cv<LD, NV, 8, 16, 2>(a, kh); chol_panel_cv<LD, NV, 16, NV, 2>(a, kh);
  } else if constexpr (PV == 44) {
    chol_panel_cv<LD, NV, 0, 6, 2>(a, kh); chol_panel_cv<LD, NV, 6, 18, 2>(a, kh); chol_panel_cv<LD, NV, 18, NV, 2>(a, kh);
  } else if constexpr (PV == 45) {
    chol_panel_cv<LD, NV, 0, 8, 2>(a, kh); chol_panel_cv<LD, NV, 8, 18, 2>(a, kh); chol_panel_cv<LD, NV, 18, 24, 2>(a, kh); chol_panel_cv<LD, NV, 24, NV, 2>(a, kh);
  } else if constexpr (PV == 46) {
    chol_panel_cv<LD, NV, 0, 6, 2>(a, kh); chol_panel_cv<LD, NV, 6, 14, 2>(a, kh); chol_panel_cv<LD, NV, 14, NV, 2>(a, kh);
  } else if constexpr (PV == 47) {
    chol_panel_cv<LD, NV, 0, 10, 2>(a, kh); chol_panel_cv<LD, NV, 10, 16, 2>(a, kh); chol_panel_cv<LD, NV, 16, NV, 2>(a, kh);
  } else if constexpr (PV == 48) {
    chol_panel_cv<LD, NV, 0, 8, 2>(a, kh); chol_panel_cv<LD, NV, 8, 14, 2>(a, kh); chol_panel_cv<LD, NV, 14, 20, 2>(a, kh); chol_panel_cv<LD, NV, 20, NV, 2>(a, kh);
  } else if constexpr (PV == 50) {
    chol_panel_b2<LD, NV, 0, 8>(a, kh); chol_panel_b2<LD, NV, 8, 16>(a, kh); chol_panel_b2<LD, NV, 16, NV>(a, kh);
  } else if constexpr (PV == 51) {
    chol_panel_b2<LD, NV, 0, 10>(a, kh); chol_panel_b2<LD, NV, 10, 20>(a, kh); chol_panel_b2<LD, NV, 20, NV>(a, kh);
  } else if constexpr (PV == 52) {
    chol_panel_b2<LD, NV, 0, 6>(a, kh); chol_panel_b2<LD, NV, 6, 16>(a, kh); chol_panel_b2<LD, NV, 16, NV>(a, kh);
  } else if constexpr (PV == 53) {
    chol_panel_b2<LD, NV, 0, 8>(a, kh); chol_panel_b2<LD, NV, 8, 16>(a, kh); chol_panel_b2<LD, NV, 16, 24>(a, kh);
    chol_panel_b2<LD, NV, 24, NV>(a, kh);
  } else if constexpr (PV == 9) {  // no factor: load + store (+ solve) overhead only
  } else if constexpr (PV == 4) {
    chol_panel<LD, NV, 0, 4>(a, kh); chol_panel<LD, NV, 4, 8>(a, kh); chol_panel<LD, NV, 8, 12>(a, kh);
    chol_panel<LD, NV, 12, 16>(a, kh); chol_panel<LD, NV, 16, 20>(a, kh); chol_panel<LD, NV, 20, 24>(a, kh);
    chol_panel<LD, NV, 24, NV>(a, kh);
  }
  if (lane <= R) {
    LDSA f32x4* wp = (LDSA f32x4*)((i == R) ? invd_out : dst + i * LD);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      f32x4 v;
      v[0] = a[4 * q]; v[1] = a[4 * q + 1]; v[2] = a[4 * q + 2]; v[3] = a[4 * q + 3];
      wp[q] = v;
    }
  }
  if constexpr (SOLVE == 0) return 0.f;  // factor + store only
  const int ic = (i < NV) ? i : 0;
  const float dg = dst[ic * LD + ic], yv = invd_out[ic];
  float w[NV];
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) w[k] = dst[k * LD + ic];
  const float y = (i < NV) ? yv : 0.f;
  const float invd = (i < NV) ? __builtin_amdgcn_rcpf(dg) : 1.f;
  if (lane < NV) invd_out[lane] = invd;
  if constexpr (SOLVE == 2) {  // + the reloads, no back substitution
    float z = 0.f;
#pragma unroll
    for (int k = 0; k < NV; k++) z += w[k];
    return z + y * invd;
  }
  const int io = opaque_int(i);
#pragma unroll
  for (int k = 0; k < NV; k++) w[k] = (io < k) ? w[k] * invd : 0.f;
  float x = y * invd;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) x = fmaf(-w[k], rdlane(x, k), x);
  return x;
}

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
  if (lane >= NV && lane < LD) W.rhs[lane] = 0.f;
  SYNC();
  float x = 0.f;
  unsigned long long tot = 0;
  for (int r = 0; r < reps; r++) {
    SYNC();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) x = chol_aug_factor_solve<D, false>(W.S, W.L, W.invd, NV, W.rhs, lane);
    else if constexpr (V == 10) x = aug_variant<0, 0>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 11) x = aug_variant<1, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 12) x = aug_variant<2, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 13) x = aug_variant<3, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 14) x = aug_variant<4, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 20) x = ldl_aug_factor_solve(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 21) x = aug_variant<21, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 22) x = aug_variant<22, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 23) x = aug_variant<23, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 24) x = aug_variant<24, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 26) x = aug_variant<26, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 30) x = aug_variant<30, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 31) x = aug_variant<31, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 32) x = aug_variant<32, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 33) x = aug_variant<33, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 40) x = aug_variant<40, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 41) x = aug_variant<41, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 42) x = aug_variant<42, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 43) x = aug_variant<43, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 44) x = aug_variant<44, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 45) x = aug_variant<45, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 46) x = aug_variant<46, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 47) x = aug_variant<47, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 48) x = aug_variant<48, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 50) x = aug_variant<50, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 51) x = aug_variant<51, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 52) x = aug_variant<52, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 53) x = aug_variant<53, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 15) x = aug_variant<0, 1>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 16) x = aug_variant<0, 2>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 17) x = aug_variant<9, 0>(W.S, W.L, W.invd, W.rhs, lane);
    else if constexpr (V == 18) x = aug_variant<9, 1>(W.S, W.L, W.invd, W.rhs, lane);
    SYNC();
    tot += __builtin_amdgcn_s_memtime() - t0;
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
  printf("%-44s %8.0f cycles/call   max rel dev vs product %.2e\n", name, m, dev);
  hipFree(t);
  hipFree(o);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 2048;  // 2048: two waves per SIMD; 1024: one
  printf("B = %d\n", B);
  std::vector<float> ref;
  run<0>(B, "product chol_aug_factor_solve", &ref);
  run<15>(B, "product copy (panels 8)", &ref);
  run<10>(B, "factor + store (panels 8)", nullptr);
  run<16>(B, "factor + store + reloads (no back subst)", nullptr);
  run<17>(B, "load + store only (no factor)", nullptr);
  run<18>(B, "load + store + reload + back subst (no factor)", nullptr);
  run<11>(B, "panels 8, two MFMA accumulators", &ref);
  run<12>(B, "panels 6", &ref);
  run<13>(B, "panels 10", &ref);
  run<14>(B, "panels 4", &ref);
  run<20>(B, "LDL^T factor + solve", &ref);
  run<21>(B, "column step: rcp multiplier", &ref);
  run<22>(B, "column step: no pivot clamp", &ref);
  run<23>(B, "column step: rcp multiplier, no clamp", &ref);
  run<24>(B, "column step: scaled broadcasts", &ref);
  run<26>(B, "column step: scaled broadcasts, no clamp", &ref);
  run<30>(B, "no clamp, panels 10/20", &ref);
  run<31>(B, "no clamp, panels 12/24", &ref);
  run<32>(B, "no clamp, panels 8/18", &ref);
  run<33>(B, "no clamp, panels 14", &ref);
  run<40>(B, "no clamp, panels 8/20", &ref);
  run<41>(B, "no clamp, panels 6/16", &ref);
  run<42>(B, "no clamp, panels 10/18", &ref);
  run<43>(B, "no clamp, panels 8/16", &ref);
  run<44>(B, "no clamp, panels 6/18", &ref);
  run<45>(B, "no clamp, panels 8/18/24", &ref);
  run<46>(B, "no clamp, panels 6/14", &ref);
  run<47>(B, "no clamp, panels 10/16", &ref);
  run<48>(B, "no clamp, panels 8/14/20", &ref);
  run<50>(B, "2x2 block pivots, panels 8/16", &ref);
  run<51>(B, "2x2 block pivots, panels 10/20", &ref);
  run<52>(B, "2x2 block pivots, panels 6/16", &ref);
  run<53>(B, "2x2 block pivots, panels 8/16/24", &ref);
  run<0>(B, "product again", &ref);
  return 0;
}
