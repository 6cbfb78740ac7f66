// Times the twin update's fused thin-end launches (csrc/twin_kernels.hip) alone at C5's 8,192-row
// per-rank minibatch (and C3's 65,536), synthetic data: the gather + input layer
// (mjl_twin_gather_in's kernel) and the output backward + last tanh backward (mjl_twin_head_bwd's).
// Diagnostic tool, not product. HIP events around 200 back-to-back launches per kernel.
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -fapprox-func -fno-slp-vectorize \
//          -o tools/twin_micro tools/twin_micro.hip
#include "../mujoco-mjx-lab_amd/csrc/twin_kernels.hip"
#include "../mujoco-mjx-lab_amd/csrc/ppo_loss_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace mjl;




static float* dev_rand(size_t n, unsigned seed, float scale) {
  std::vector<float> h(n);
  unsigned s = seed * 2654435761u + 1u;
  for (size_t i = 0; i < n; i++) {
    s = s * 1664525u + 1013904223u;
    h[i] = scale * ((s >> 8) * (1.0f / 16777216.0f) * 2.f - 1.f);
  }
  float* d;
  (void)hipMalloc(&d, n * 4);
  (void)hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  return d;
}

template <class F> float time_ms(F launch, int reps) {
  for (int i = 0; i < 5; i++) launch();
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; i++) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  constexpr int K0 = kTinK0, N = kTinN, A = kHbA;
  const long long nsrc = 262144;  // one C5 rank's rollout rows (1024 x 256)
  float* obs = dev_rand(nsrc * K0, 1, 1.f);
  float* act = dev_rand(nsrc * A, 2, 1.f);
  float* lp = dev_rand(nsrc, 3, 1.f);
  float* rt = dev_rand(nsrc, 4, 1.f);
  float* av = dev_rand(nsrc, 5, 1.f);
  float* W0 = dev_rand(2 * N * K0, 6, 0.1f);
  float* b0 = dev_rand(2 * N, 7, 0.1f);
  float* Wo = dev_rand(2 * A * N, 8, 0.1f);
  for (int M : {8192, 65536}) {
    std::vector<long long> hidx(M);
    for (int i = 0; i < M; i++) hidx[i] = ((long long)i * 7919) % nsrc;
    long long* idx;
    (void)hipMalloc(&idx, M * 8);
    (void)hipMemcpy(idx, hidx.data(), M * 8, hipMemcpyHostToDevice);
    float *o2, *a, *ol, *r, *ad, *h, *dz, *y, *dzh, *cs, *gw;
    (void)hipMalloc(&o2, 2ull * M * K0 * 4);
    (void)hipMalloc(&a, 1ull * M * A * 4);
    (void)hipMalloc(&ol, M * 4);
    (void)hipMalloc(&r, M * 4);
    (void)hipMalloc(&ad, M * 4);
    (void)hipMalloc(&h, 2ull * M * N * 4);
    dz = dev_rand(2ull * M * A, 9, 0.01f);
    y = dev_rand(2ull * M * N, 10, 0.9f);
    (void)hipMalloc(&dzh, 2ull * M * N * 4);
    (void)hipMalloc(&cs, 2ull * (M / kHbRows) * N * 4);
    (void)hipMalloc(&gw, 2ull * (M / kHbRows) * A * N * 4);
    TwinInArgs pi{idx, nullptr, M, A, nsrc, obs, act, lp, rt, av, o2, a, ol, r, ad, W0, b0, h};
    const float t_in = time_ms([&] {
      const int nblk = 2 * ((M + kTinRows - 1) / kTinRows);
      hipLaunchKernelGGL((twin_gather_in_kernel<K0, N>), dim3(nblk < kTinBlocks ? nblk : kTinBlocks), dim3(N), 0, 0, pi);
    }, reps);
    TwinHeadBwdArgs ph{dz, Wo, y, dzh, cs, gw, M, N};
    const float t_hb = time_ms([&] {
      hipLaunchKernelGGL(twin_head_bwd_kernel<A>, dim3(M / kHbRows, N / kHbCols, 2), dim3(256), 0, 0, ph);
    }, reps);
    {  // the twin loss head (mjl_twin_loss_head's kernel) at 64 and 128 rows per block
      float *z = dev_rand(2ull * M * A, 11, 0.5f), *lstd = dev_rand(A, 12, 0.3f), *st = dev_rand(2, 13, 1.f);
      float *lp2, *glsp, *biasp, *dzl;
      int* row;
      (void)hipMalloc(&lp2, 4 * (M / 64 + 1));
      (void)hipMalloc(&glsp, 4ull * (M / 64 + 1) * A);
      (void)hipMalloc(&biasp, 8ull * (M / 64 + 1) * A);
      (void)hipMalloc(&dzl, 8ull * M * A);
      (void)hipMalloc(&row, 4);
      (void)hipMemset(row, 0, 4);
      const float t64 = time_ms([&] {
        hipLaunchKernelGGL(twin_loss_head_kernel<64>, dim3(M / 64), dim3(128), 0, 0, z, lstd, act, lp, av, rt, M, A, 0.2f,
                           0.01f, nullptr, 0, st, row, -20.f, 2.f, b0, dzl, lp2, glsp, biasp);
      }, reps);
      const float t128 = time_ms([&] {
        hipLaunchKernelGGL(twin_loss_head_kernel<128>, dim3(M / 128), dim3(256), 0, 0, z, lstd, act, lp, av, rt, M, A,
                           0.2f, 0.01f, nullptr, 0, st, row, -20.f, 2.f, b0, dzl, lp2, glsp, biasp);
      }, reps);
      printf("M %6d  twin_loss_head  RB 64: %7.2f us   RB 128: %7.2f us\n", M, t64 * 1e3, t128 * 1e3);
    }
    {  // the fused head (mjl_twin_head's kernel), statistics from a table row
      float *zh = dev_rand(2ull * M * N, 14, 1.f), *lstd = dev_rand(A, 12, 0.3f), *st = dev_rand(2, 13, 1.f);
      float *dzh2, *cs2, *gw2, *lossp2, *glsp2, *biasp2;
      int* row;
      const int S = (M / kThRows) < kThBlocks / 2 ? (M / kThRows) : kThBlocks / 2;
      (void)hipMalloc(&dzh2, 8ull * M * N);
      (void)hipMalloc(&cs2, 8ull * S * N);
      (void)hipMalloc(&gw2, 8ull * S * A * N);
      (void)hipMalloc(&lossp2, 4ull * S);
      (void)hipMalloc(&glsp2, 4ull * S * A);
      (void)hipMalloc(&biasp2, 8ull * S * A);
      (void)hipMalloc(&row, 4);
      (void)hipMemset(row, 0, 4);
      TwinHeadArgs ha{zh, b0, Wo, b0, lstd, act, lp, av, rt, st, row, nullptr, 0, M, 0.2f, 0.01f, -20.f, 2.f,
                      dzh2, cs2, gw2, lossp2, glsp2, biasp2};
      const float th = time_ms([&] {
        hipLaunchKernelGGL((twin_head_kernel<kThA, kThK>), dim3(2 * S), dim3(256), 0, 0, ha);
      }, reps);
      printf("M %6d  twin_head (fused forward + losses + backward)  %7.2f us\n", M, th * 1e3);
    }
    const double in_bytes = 2.0 * M * N * 4 + 3.0 * M * K0 * 4, hb_bytes = 4.0 * M * N * 4;
    printf("M %6d  gather_in %7.2f us (%5.1f TFLOP/s, %5.2f TB/s)   head_bwd %7.2f us (%5.2f TB/s)\n", M, t_in * 1e3,
           2.0 * M * K0 * 2 * N / (t_in * 1e-3) / 1e12, in_bytes / (t_in * 1e-3) / 1e12, t_hb * 1e3,
           hb_bytes / (t_hb * 1e-3) / 1e12);
    (void)hipFree(idx);
  }
  return 0;
}
