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
