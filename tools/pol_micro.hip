// Times the fused rollout policy (csrc/ppo_kernels.hip policy_rollout_kernel: obs normalisation, the
// 54 -> 256 x 3 -> 21 tanh MLP on MFMA, sampling and log-density) alone on synthetic data at 1024 and
// 2048 envs, and a stamped copy (tools/pol_stamped.inc, tools/gen_pol_stamped.py) that prints the
// cycles of each phase for workgroup 6's waves 0 and 15. Diagnostic tool, not product.
// Build: python3 tools/gen_pol_stamped.py && hipcc -O2 -std=c++17 --offload-arch=gfx950 -fapprox-func \
//          -fno-slp-vectorize -o tools/pol_micro tools/pol_micro.hip
#include "../mujoco-mjx-lab_amd/csrc/ppo_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace mjl {
#include "pol4_kernel.inc"
#pragma clang fp contract(off)
#include "pol_stamped.inc"
#pragma clang fp contract(on)
}  // namespace mjl
using namespace mjl;

static float* dev_rand(size_t n, unsigned seed, float scale) {
  std::vector<float> h(n);
  unsigned s = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; i++) {
    s = s * 1664525u + 1013904223u;
    h[i] = scale * ((float)(s >> 8) / 16777216.f * 2.f - 1.f);
  }
  float* d;
  (void)hipMalloc(&d, n * 4);
  (void)hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  return d;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  PolicyDims pd{};
  pd.nlayer = 4; pd.obs_dim = 54; pd.act_dim = 21;
  const int K[4] = {64, 256, 256, 256}, N[4] = {256, 256, 256, 32};
  long long off = 0;
  for (int l = 0; l < 4; l++) { pd.K[l] = K[l]; pd.N[l] = N[l]; pd.off[l] = off; off += (long long)K[l] * N[l] + N[l]; }
  float* params = dev_rand(off, 1, 0.06f);
  float* mean = dev_rand(54, 2, 0.1f);
  std::vector<float> hv(54, 1.f);
  float* var;
  (void)hipMalloc(&var, 54 * 4);
  (void)hipMemcpy(var, hv.data(), 54 * 4, hipMemcpyHostToDevice);
  float* log_std = dev_rand(21, 3, 0.5f);
  unsigned long long* st;
  (void)hipMalloc(&st, 64 * 8);
  for (int B : {1024, 2048}) {
    float* obs = dev_rand((size_t)B * 54, 4, 2.f);
    float* eps = dev_rand((size_t)B * 21, 5, 1.f);
    float *act, *lp;
    (void)hipMalloc(&act, (size_t)B * 21 * 4);
    (void)hipMalloc(&lp, (size_t)B * 4);
    const dim3 grid((B + 15) / 16), block(64 * kPolWaves);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 10; i++)
      hipLaunchKernelGGL(policy_rollout_kernel, grid, block, 0, 0, obs, mean, var, 10.f, params, pd, log_std, eps, B, act, lp);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < reps; i++)
      hipLaunchKernelGGL(policy_rollout_kernel, grid, block, 0, 0, obs, mean, var, 10.f, params, pd, log_std, eps, B, act, lp);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("B %5d  policy_rollout_kernel %8.2f us\n", B, 1000.f * ms / reps);
    {  // the 4-env layout: same bits, time
      std::vector<float> a16((size_t)B * 21), l16(B), a4((size_t)B * 21), l4(B);
      (void)hipMemcpy(a16.data(), act, a16.size() * 4, hipMemcpyDeviceToHost);
      (void)hipMemcpy(l16.data(), lp, l16.size() * 4, hipMemcpyDeviceToHost);
      (void)hipMemset(act, 0, a16.size() * 4);
      const dim3 g4((B + 3) / 4), b4(64 * kPol4Waves);
      for (int i = 0; i < 10; i++)
        hipLaunchKernelGGL(policy_rollout4_kernel, g4, b4, 0, 0, obs, mean, var, 10.f, params, pd, log_std, eps, B, act, lp);
      (void)hipEventRecord(e0, 0);
      for (int i = 0; i < reps; i++)
        hipLaunchKernelGGL(policy_rollout4_kernel, g4, b4, 0, 0, obs, mean, var, 10.f, params, pd, log_std, eps, B, act, lp);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms4;
      (void)hipEventElapsedTime(&ms4, e0, e1);
      (void)hipMemcpy(a4.data(), act, a4.size() * 4, hipMemcpyDeviceToHost);
      (void)hipMemcpy(l4.data(), lp, l4.size() * 4, hipMemcpyDeviceToHost);
      size_t diff = 0;
      double md = 0;
      for (size_t i = 0; i < a4.size(); i++) { diff += a4[i] != a16[i]; md = fmax(md, fabs(a4[i] - a16[i])); }
      for (int i = 0; i < B; i++) { diff += l4[i] != l16[i]; md = fmax(md, fabs(l4[i] - l16[i])); }
      printf("B %5d  policy_rollout4_kernel %8.2f us  (outputs differing from the 16-env kernel: %zu, max |diff| %.3g)\n",
             B, 1000.f * ms4 / reps, diff, md);
      (void)hipMemset(st, 0, 64 * 8);
      for (int i = 0; i < reps; i++)
        hipLaunchKernelGGL(pol4_stamped, g4, b4, 0, 0, st, obs, mean, var, 10.f, params, pd, log_std, eps, B, act, lp);
      (void)hipDeviceSynchronize();
      unsigned long long h4[64];
      (void)hipMemcpy(h4, st, 64 * 8, hipMemcpyDeviceToHost);
      const char* nm4[13] = {"prologue", "L0 mfma", "L0 bar", "L1 mfma", "L1 bar", "L2 mfma", "L2 bar", "L3 mfma", "L3 bar", "-", "-", "-", "head"};
      for (int w = 0; w < 2; w++) {
        printf("   4-env wave %d cycles:", w ? 3 : 0);
        for (int i = 0; i < 13; i++)
          if (nm4[i][0] != '-') printf(" %s %llu |", nm4[i], h4[16 * w + i] / reps);
        printf("\n");
      }
    }
    (void)hipMemset(st, 0, 64 * 8);
    for (int i = 0; i < reps; i++)
      hipLaunchKernelGGL(pol_stamped, grid, block, 0, 0, st, obs, mean, var, 10.f, params, pd, log_std, eps, B, act, lp);
    (void)hipDeviceSynchronize();
    unsigned long long h[64];
    (void)hipMemcpy(h, st, 64 * 8, hipMemcpyDeviceToHost);
    const char* nm[13] = {"prologue", "L0 mfma", "L0 bar", "L1 mfma", "L1 bar", "L2 mfma", "L2 bar", "L3 mfma", "L3 bar", "-", "-", "-", "head"};
    for (int w = 0; w < 2; w++) {
      printf("   wave %2d cycles:", w ? 15 : 0);
      for (int i = 0; i < 13; i++)
        if (nm[i][0] != '-') printf(" %s %llu |", nm[i], h[16 * w + i] / reps);
      printf("\n");
    }
  }
  return 0;
}
