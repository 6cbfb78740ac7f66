// Micro-benchmark of the step kernel's two factor + solve routines on the humanoid's dof tree:
// the dense panel Cholesky (chol_aug_factor_solve) and the tree-ordered L'DL (tree_factor_solve),
// one env per 64-lane wave, B waves (2048: two per SIMD as in the step kernel; 1024: one), on
// tree-patterned SPD matrices S = L0' L0 + diag (L0 with the tree's ancestor pattern, like M).
// Prints mean s_memtime cycles per call and the max relative error against a host fp64 solve.
// Diagnostic tool, not product.
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -fapprox-func -fno-slp-vectorize \
//          -o tools/tree_chol_micro tools/tree_chol_micro.hip
#include "../mujoco-mjx-lab_amd/csrc/step_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <type_traits>

namespace mjl {
// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E)
template <int B, int E, class F> INL void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}


// ---------------------------------------------------------------------------------------------
// tree-ordered factor + solve (the two reference humanoids' dof tree). Measured in the step kernel
// in round 5 (MJL_TREE=1 instantiation, profiles/r5/): no faster than the dense panels there --
// speed test 58.13 vs 58.27 us, pooled env step 90.5 vs 88.2 us at 2048 envs, 79.6 vs 78.3 us at
// 1024 -- so it lives here, not in the product ("tree-ordered factor").
// ---------------------------------------------------------------------------------------------
// The dof tree of humanoid.xml / humanoid_mjx.xml (dof_parentid): a trunk of 9 dofs (the free
// joint's 6, then abdomen z, y, x) and four chains hanging off it -- the legs (6 dofs each, parent
// dof 8) and the arms (3 each, parent dof 5). The mass matrix has exactly the tree's pattern (entry
// (i, j) is nonzero only when one dof is an ancestor of the other), so do M + dt diag(damping) and
// the Newton Hessian M + J'DJ whenever no active row couples two branches (every row's J lies on one
// body chain: floor contacts, joint limits, the hamstring tendons). Eliminating the dofs leaves
// first (MuJoCo's mj_factorM order, M = L' D L) makes no fill, and the four chains are independent:
// 15 dependent columns instead of 27.
struct HumTree {
  static constexpr int NV = 27, TN = 9, NBR = 4;
  static constexpr int bs[NBR] = {9, 15, 21, 24};   // first dof of each chain
  static constexpr int be[NBR] = {15, 21, 24, 27};  // one past its last dof
  static constexpr int bp[NBR] = {8, 8, 5, 5};      // the trunk dof it hangs off
  static constexpr int len(int b) { return be[b] - bs[b]; }
  static constexpr int parent(int d) {  // dof_parentid of this tree
    if (d < TN) return d - 1;
    for (int b = 0; b < NBR; b++)
      if (d == bs[b]) return bp[b];
    return d - 1;
  }
};

// L' D L = S (S: the tree-patterned SPD matrix in LDS at src, stride LD; ADD: plus the symmetric
// MFMA-layout addend C, as chol_aug_factor_solve), returns S^-1 rhs with row i's value in lanes i
// and i + 32; `scratch` (LD floats of LDS) carries the forward substitution's result between lanes.
// Nothing is stored: the callers that use it only need the solution (the Newton direction,
// qacc_smooth, the implicit-integration update).
//
// Layout: lane l holds row l & 31 of S in registers a[0..LD) (the whole row, both triangles), and
// the right-hand side rides along as one more row R = NV (lane R: a[j] = rhs_j). Eliminating dof k
// (pivot d_k = S'[k][k], broadcast of row k by v_readlane) updates S'[i][j] -= S'[i][k] S'[k][j] / d_k
// for i, j in k's ancestors -- lane i's multiplier t = a[k] / d_k is nonzero only on the ancestors'
// lanes (and lane R, whose row update is the forward substitution), so one VALU op per column j
// updates every row at once.
//  1. chains, leaves first, the four chains' columns interleaved: each elimination updates only its
//     own chain's columns on the VALU; its update of the trunk columns -- every lane's a[j], j in the
//     trunk -- is deferred to one rank-18 product C[j][i] = sum_k a_j[k] t_i[k] on the matrix cores
//     (the legs' columns pairwise in one v_mfma_f32_32x32x2_f32 per elimination step, the arms' in a
//     second accumulator), so a chain elimination's VALU work is the chain's own columns only;
//  2. the trunk, dofs 8 .. 0, on the VALU;
//  3. lane R's row (z = L'^-1 rhs) through `scratch` to the lanes, x = D^-1 z, then L x = that,
//     ancestors first: the trunk's 9 columns, then the four chains' columns on four registers (no
//     false dependency between the chains), each lane keeping its own value at its own step.
template <int V> using IC = std::integral_constant<int, V>;
template <class D, class T, bool ADD> INL float tree_factor_solve(const LDSA float* src, LDSA float* scratch,
                                                                 const LDSA float* rhs, int lane, f32x16 C = {}) {
  constexpr int NV = D::NV, LD = D::LD, R = NV, TN = T::TN;
  static_assert(NV == T::NV && NV < 32 && LD > NV && LD % 4 == 0, "tree factor: the humanoid instantiation");
  static_assert(T::NBR == 4 && T::len(0) == T::len(1) && T::len(2) == T::len(3) && T::len(2) <= T::len(0),
                "chains paired legs / arms for the deferred trunk update");
  static_assert(TN <= 12, "trunk rows within the extracted MFMA registers");
  const int i = lane & 31, kh = lane >> 5;
  float a[LD];
  if constexpr (ADD) {
#pragma unroll
    for (int v = 0; v < 16; v++) {
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(C[v]), __float_as_uint(C[v]), false, false);
      const int j0 = (v & 3) + 8 * (v >> 2);
      if (j0 < LD) a[j0] = __uint_as_float(r[0]);
      if (j0 + 4 < LD) a[j0 + 4] = __uint_as_float(r[1]);
    }
  }
  {  // row i of S (lanes i < NV), the right-hand side as row R (lanes >= NV; kept by lane R)
    const LDSA f32x4* rp = (const LDSA f32x4*)((i < NV) ? src + i * LD : rhs);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      const f32x4 v = rp[q];
#pragma unroll
      for (int e = 0; e < 4; e++) a[4 * q + e] = ADD ? a[4 * q + e] + v[e] : v[e];
    }
  }
  // the lane's row index for the masks, with row R ordered before every dof (it is updated by
  // every elimination and never eliminated); opaque: the compares stay at their uses
  const int io = opaque_int(i == R ? -1 : i);
  float dinv = 1.f;  // 1 / d of the lane's own dof
  auto eliminate = [&](auto kc, auto j0c, auto j1c) {  // dof k: update columns [j0, j1) of its ancestors
    constexpr int k = decltype(kc)::value, j0 = decltype(j0c)::value, j1 = decltype(j1c)::value;
    const float inv = __builtin_amdgcn_rcpf(rdlane(a[k], k));
    float s[LD];
#pragma unroll
    for (int j = j0; j < j1; j++) s[j] = rdlane(a[j], k);
    const float t = (io < k) ? a[k] * inv : 0.f;
#pragma unroll
    for (int j = j0; j < j1; j++) a[j] = fmaf(-t, s[j], a[j]);
    dinv = (io == k) ? inv : dinv;
    return t;
  };
  // 1. the chains, leaves first; deferred trunk update C[j][i] = sum_k a_j[k] t_i[k]
  f32x16 accL, accA;
#pragma unroll
  for (int v = 0; v < 16; v++) { accL[v] = 0.f; accA[v] = 0.f; }
  constexpr int L0 = T::len(0), L2 = T::len(2);
  static_for<0, L0>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    constexpr int k0 = T::be[0] - 1 - s, k1 = T::be[1] - 1 - s;
    const float t0 = eliminate(IC<k0>{}, IC<T::bs[0]>{}, IC<k0>{});
    const float t1 = eliminate(IC<k1>{}, IC<T::bs[1]>{}, IC<k1>{});
    accL = __builtin_amdgcn_mfma_f32_32x32x2f32(kh ? a[k1] : a[k0], kh ? t1 : t0, accL, 0, 0, 0);
    if constexpr (s < L2) {
      constexpr int k2 = T::be[2] - 1 - s, k3 = T::be[3] - 1 - s;
      const float t2 = eliminate(IC<k2>{}, IC<T::bs[2]>{}, IC<k2>{});
      const float t3 = eliminate(IC<k3>{}, IC<T::bs[3]>{}, IC<k3>{});
      accA = __builtin_amdgcn_mfma_f32_32x32x2f32(kh ? a[k3] : a[k2], kh ? t3 : t2, accA, 0, 0, 0);
    }
  });
  {  // a[j] -= C[j][lane] for the trunk columns (C layout: row j of column l & 31 in half (j >> 2) & 1,
     // register (j & 3) + 4 (j >> 3); one v_permlane32_swap hands each lane both halves)
    float lo[4], hi[4];
#pragma unroll
    for (int v = 0; v < 4 * ((TN + 7) / 8); v++) {
      const int vv = v;  // registers 0..3 (rows 0-7), 4..7 (rows 8-15)
      const float c = accL[vv] + accA[vv];
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(c), __float_as_uint(c), false, false);
      if (vv < 4) { lo[vv] = __uint_as_float(r[0]); hi[vv] = __uint_as_float(r[1]); }
      else {
#pragma unroll
        for (int j = 8; j < TN; j++)
          if ((j & 3) + 4 == vv) a[j] -= ((j >> 2) & 1) ? __uint_as_float(r[1]) : __uint_as_float(r[0]);
      }
    }
#pragma unroll
    for (int j = 0; j < (TN < 8 ? TN : 8); j++) a[j] -= ((j >> 2) & 1) ? hi[j & 3] : lo[j & 3];
  }
  // 2. the trunk (a chain: every lower dof is an ancestor)
  static_for<0, TN>([&](auto sc) {
    constexpr int k = TN - 1 - decltype(sc)::value;
    (void)eliminate(IC<k>{}, IC<0>{}, IC<k>{});
  });
  // 3. z = lane R's row, x = D^-1 z, then L x = that (L[i][j] = a_i[j] / d_i, j an ancestor of i)
  if (lane == R) {
    LDSA f32x4* wp = (LDSA f32x4*)scratch;
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      f32x4 v;
      v[0] = a[4 * q]; v[1] = a[4 * q + 1]; v[2] = a[4 * q + 2]; v[3] = a[4 * q + 3];
      wp[q] = v;
    }
  }
  // (same wave: the LDS store completes before the read)
  const float z = scratch[i < NV ? i : 0];
  float x = (i < NV) ? z * dinv : 0.f, xf = x;
#pragma unroll
  for (int j = 0; j < NV; j++) a[j] *= dinv;  // rows of L (lanes past a finished dof's step may take
                                              // junk updates: each lane keeps its value at its own step)
  static_for<0, TN>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const float xj = rdlane(x, j);
    xf = (io == j) ? xj : xf;
    x = fmaf(-a[j], xj, x);
  });
  float xb[T::NBR];
#pragma unroll
  for (int b = 0; b < T::NBR; b++) xb[b] = x;
  static_for<0, L0>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<0, T::NBR>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      if constexpr (s < T::len(b)) {
        constexpr int j = T::bs[b] + s;
        const float xj = rdlane(xb[b], j);
        xf = (io == j) ? xj : xf;
        xb[b] = fmaf(-a[j], xj, xb[b]);
      }
    });
  });
  return xf;
}

}  // namespace mjl

using namespace mjl;
using D = DHum;
constexpr int NV = D::NV, LD = D::LD, NMAT = 97;

struct MicroWS {
  alignas(16) float S[NV * LD];
  alignas(16) float L[NV * LD];
  float invd[LD];
  float rhs[LD];
  float pad[(kLdsBudget - 2 * NV * LD * 4 - 2 * LD * 4) / 4];  // same LDS per wave as the step kernel
};

template <int V> __global__ __launch_bounds__(64, 2) void kern(const float* mats, const float* rhss, const float* diag,
                                                               unsigned long long* tout, float* out, int reps) {
  __shared__ MicroWS Wsh;
  LDSA MicroWS& W = *(LDSA MicroWS*)&Wsh;
  const int lane = threadIdx.x, env = blockIdx.x, mi = env % NMAT;
  for (int e = lane; e < NV * LD; e += 64) W.S[e] = mats[(size_t)mi * NV * LD + e];
  if (lane < LD) W.rhs[lane] = rhss[mi * LD + lane];
  // the implicit-integration addend dt * diag(damping) in the MFMA C layout (ADD variants)
  f32x16 C;
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int v = 0; v < 16; v++) C[v] = ((v & 3) + 8 * (v >> 2) + 4 * h == c && c < NV) ? diag[c] : 0.f;
  SYNC();
  float x = 0.f;
  unsigned long long tot = 0;
  for (int r = 0; r < reps; r++) {
    SYNC();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) x = chol_aug_factor_solve<D, false>(W.S, W.L, W.invd, NV, W.rhs, lane);
    else if constexpr (V == 1) x = tree_factor_solve<D, HumTree, false>(W.S, W.invd, W.rhs, lane);
    else if constexpr (V == 2) x = chol_aug_factor_solve<D, true>(W.S, W.L, W.invd, NV, W.rhs, lane, C);
    else if constexpr (V == 3) x = tree_factor_solve<D, HumTree, true>(W.S, W.invd, W.rhs, lane, C);
    SYNC();
    tot += __builtin_amdgcn_s_memtime() - t0;
  }
  if (lane == 0) tout[env] = tot / reps;
  out[env * 64 + lane] = x;
}

// host: tree-patterned SPD matrices and fp64 solutions
static void host_mats(std::vector<float>& S, std::vector<float>& rhs, std::vector<float>& diag,
                      std::vector<double>& sol0, std::vector<double>& sol1) {
  S.assign((size_t)NMAT * NV * LD, 0.f);
  rhs.assign((size_t)NMAT * LD, 0.f);
  diag.assign(32, 0.f);
  sol0.assign((size_t)NMAT * NV, 0.0);
  sol1.assign((size_t)NMAT * NV, 0.0);
  for (int d = 0; d < NV; d++) diag[d] = 0.002f * (1 + d % 5);
  srand(12345);
  auto rnd = [] { return (double)rand() / RAND_MAX * 2 - 1; };
  for (int m = 0; m < NMAT; m++) {
    std::vector<double> L0(NV * NV, 0.0), A(NV * NV, 0.0);
    for (int k = 0; k < NV; k++) {
      L0[k * NV + k] = 0.3 + std::fabs(rnd());
      for (int p = HumTree::parent(k); p >= 0; p = HumTree::parent(p)) L0[k * NV + p] = 0.5 * rnd();
    }
    for (int i = 0; i < NV; i++)
      for (int j = 0; j < NV; j++) {
        double s = 0;
        for (int k = 0; k < NV; k++) s += L0[k * NV + i] * L0[k * NV + j];
        A[i * NV + j] = s + (i == j ? 0.05 : 0.0);
      }
    for (int i = 0; i < NV; i++)
      for (int j = 0; j < NV; j++) S[(size_t)m * NV * LD + i * LD + j] = (float)A[i * NV + j];
    for (int i = 0; i < NV; i++) rhs[m * LD + i] = (float)rnd();
    for (int add = 0; add < 2; add++) {  // fp64 solve of the fp32-rounded system (Gaussian elimination)
      std::vector<double> B(NV * (NV + 1));
      for (int i = 0; i < NV; i++) {
        for (int j = 0; j < NV; j++) B[i * (NV + 1) + j] = S[(size_t)m * NV * LD + i * LD + j] + (add && i == j ? diag[i] : 0.f);
        B[i * (NV + 1) + NV] = rhs[m * LD + i];
      }
      for (int k = 0; k < NV; k++)
        for (int i = k + 1; i < NV; i++) {
          double f = B[i * (NV + 1) + k] / B[k * (NV + 1) + k];
          for (int j = k; j <= NV; j++) B[i * (NV + 1) + j] -= f * B[k * (NV + 1) + j];
        }
      std::vector<double>& sol = add ? sol1 : sol0;
      for (int i = NV - 1; i >= 0; i--) {
        double s = B[i * (NV + 1) + NV];
        for (int j = i + 1; j < NV; j++) s -= B[i * (NV + 1) + j] * sol[m * NV + j];
        sol[m * NV + i] = s / B[i * (NV + 1) + i];
      }
    }
  }
}

template <int V> void run(int B, const char* name, const float* dS, const float* dr, const float* dd,
                          const std::vector<double>& sol) {
  unsigned long long* t;
  float* o;
  hipMalloc(&t, B * 8);
  hipMalloc(&o, B * 64 * 4);
  kern<V><<<B, 64>>>(dS, dr, dd, t, o, 2);
  hipDeviceSynchronize();
  kern<V><<<B, 64>>>(dS, dr, dd, t, o, 8);
  hipDeviceSynchronize();
  std::vector<unsigned long long> th(B);
  std::vector<float> oh(B * 64);
  hipMemcpy(th.data(), t, B * 8, hipMemcpyDeviceToHost);
  hipMemcpy(oh.data(), o, B * 64 * 4, hipMemcpyDeviceToHost);
  double m = 0, dev = 0;
  for (auto v : th) m += v;
  m /= B;
  for (int e = 0; e < B; e++) {
    double mx = 0;
    for (int l = 0; l < NV; l++) mx = fmax(mx, fabs(sol[(e % NMAT) * NV + l]));
    for (int h = 0; h < 2; h++)
      for (int l = 0; l < NV; l++)
        dev = fmax(dev, fabs(oh[e * 64 + 32 * h + l] - sol[(e % NMAT) * NV + l]) / (1e-6 + mx));
  }
  printf("%-40s %8.0f cycles/call   max |x - x64| / max|x64| %.2e\n", name, m, dev);
  hipFree(t);
  hipFree(o);
}

int main(int argc, char** argv) {
  std::vector<float> S, r, dg;
  std::vector<double> s0, s1;
  host_mats(S, r, dg, s0, s1);
  float *dS, *dr, *dd;
  hipMalloc(&dS, S.size() * 4);
  hipMalloc(&dr, r.size() * 4);
  hipMalloc(&dd, dg.size() * 4);
  hipMemcpy(dS, S.data(), S.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dr, r.data(), r.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dd, dg.data(), dg.size() * 4, hipMemcpyHostToDevice);
  for (int B : {2048, 1024}) {
    printf("B = %d\n", B);
    run<0>(B, "dense panels (product)", dS, dr, dd, s0);
    run<1>(B, "tree L'DL", dS, dr, dd, s0);
    run<2>(B, "dense panels + diag addend", dS, dr, dd, s1);
    run<3>(B, "tree L'DL + diag addend", dS, dr, dd, s1);
    run<0>(B, "dense panels (again)", dS, dr, dd, s0);
  }
  return 0;
}
