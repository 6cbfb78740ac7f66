// Micro-benchmark of the PPO update's dense-layer kernels (csrc/mlp_kernels.hip) at the update's
// shape (M = 65,536 rows, 256 x 256 layers): tile / K-step variants of mlp_fwd_kernel and
// mlp_bwd_kernel, each checked against a float64 reference on sampled rows, timed with hipEvents.
// Diagnostic tool, not product: the winner's parameters go into capi.hip's launchers.
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -fapprox-func -fno-slp-vectorize -x hip \
//          -o tools/mlp_micro tools/mlp_micro.cpp
#include "../mujoco-mjx-lab_amd/csrc/mlp_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace mjl;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static const int M = 65536, N = 256, K = 256;
static int g_act = 1, g_K = 256;

template <class F> static float time_ms(F f, int reps = 20) {
  for (int i = 0; i < 3; i++) f();
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

static double check_fwd(const std::vector<float>& x, const std::vector<float>& w, const std::vector<float>& bias,
                        const float* dY) {
  std::vector<float> y((size_t)M * N);
  CK(hipMemcpy(y.data(), dY, y.size() * 4, hipMemcpyDeviceToHost));
  double worst = 0;
  for (int i = 0; i < M; i += 997) {
    for (int j = 0; j < N; j++) {
      double s = bias[j], sa = std::fabs(bias[j]);
      for (int k = 0; k < K; k++) { s += (double)x[(size_t)i * K + k] * w[(size_t)j * K + k]; sa += std::fabs((double)x[(size_t)i * K + k] * w[(size_t)j * K + k]); }
      worst = std::fmax(worst, std::fabs(std::tanh(s) - y[(size_t)i * N + j]) / (sa + 1e-30));
    }
  }
  return worst;
}

static double check_bwd(const std::vector<float>& g, const std::vector<float>& yv, const std::vector<float>& w,
                        const float* dX) {
  std::vector<float> dx((size_t)M * K);
  CK(hipMemcpy(dx.data(), dX, dx.size() * 4, hipMemcpyDeviceToHost));
  double worst = 0;
  for (int i = 0; i < M; i += 997) {
    for (int j = 0; j < K; j++) {
      double s = 0, sa = 0;
      for (int n = 0; n < N; n++) {
        const double z = (double)g[(size_t)i * N + n] * (1.0 - (double)yv[(size_t)i * N + n] * yv[(size_t)i * N + n]);
        s += z * w[(size_t)n * K + j];
        sa += std::fabs(z * w[(size_t)n * K + j]);
      }
      worst = std::fmax(worst, std::fabs(s - dx[(size_t)i * K + j]) / (sa + 1e-30));
    }
  }
  return worst;
}

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;  // run one variant (counter passes)
  int vid = 0;
  std::vector<float> x((size_t)M * K), w((size_t)N * K), bias(N), g((size_t)M * N), yv((size_t)M * N);
  srand(1);
  auto u = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& v : x) v = u();
  for (auto& v : w) v = u() * 0.1f;
  for (auto& v : bias) v = u() * 0.1f;
  for (auto& v : g) v = u();
  for (auto& v : yv) v = std::tanh(u());
  float *dx_in, *dw, *db, *dy, *dg, *dyv, *ddz, *ddx, *dpart;
  CK(hipMalloc(&dx_in, x.size() * 4)); CK(hipMalloc(&dw, w.size() * 4)); CK(hipMalloc(&db, N * 4));
  CK(hipMalloc(&dy, (size_t)M * N * 4)); CK(hipMalloc(&dg, g.size() * 4)); CK(hipMalloc(&dyv, yv.size() * 4));
  CK(hipMalloc(&ddz, (size_t)M * N * 4)); CK(hipMalloc(&ddx, (size_t)M * K * 4)); CK(hipMalloc(&dpart, (size_t)(M / 128 + 1) * N * 4));
  CK(hipMemcpy(dx_in, x.data(), x.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bias.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dg, g.data(), g.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dyv, yv.data(), yv.size() * 4, hipMemcpyHostToDevice));
  const double flops = 2.0 * M * N * K;
#define FWD(BM, BN, WM, WN, BK)                                                                                    \
  if (only < 0 || only == vid++) {                                                                                 \
    dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM);                                                              \
    auto f = [&] { hipLaunchKernelGGL((mlp_fwd_kernel<BM, BN, WM, WN, true, BK>), grid, dim3(WM * WN * 64), 0, 0, \
                                      dx_in, K, dw, K, db, dy, N, M, N, K, 1); };                                  \
    CK(hipMemset(dy, 0, (size_t)M * N * 4));                                                                       \
    const float ms = time_ms(f);                                                                                   \
    printf("fwd BM %3d BN %3d waves %dx%d BK %2d: %8.2f us  %6.1f TFLOP/s  max rel err %.2e\n", BM, BN, WM, WN, BK,  \
           ms * 1e3, flops / (ms * 1e-3) / 1e12, check_fwd(x, w, bias, dy));                                       \
  }
#define BWD(BM, BN, WM, WN, BK)                                                                                    \
  if (only < 0 || only == vid++) {                                                                                 \
    dim3 grid((K + BN - 1) / BN, (M + BM - 1) / BM);                                                              \
    auto f = [&] { hipLaunchKernelGGL((mlp_bwd_kernel<BM, BN, WM, WN, true, true, BK>), grid, dim3(WM * WN * 64), \
                                      0, 0, dg, dyv, N, dw, K, ddz, ddx, K, dpart, M, N, K, 1); };                  \
    CK(hipMemset(ddx, 0, (size_t)M * K * 4));                                                                      \
    const float ms = time_ms(f);                                                                                   \
    printf("bwd BM %3d BN %3d waves %dx%d BK %2d: %8.2f us  %6.1f TFLOP/s  max rel err %.2e\n", BM, BN, WM, WN, BK,  \
           ms * 1e3, flops / (ms * 1e-3) / 1e12, check_bwd(g, yv, w, ddx));                                        \
  }
  FWD(128, 128, 2, 2, 32)
  {  // the same tile without the tanh epilogue, and over a 4x longer reduction (prologue / epilogue share)
    dim3 grid(N / 128, M / 128);
    auto f0 = [&] { hipLaunchKernelGGL((mlp_fwd_kernel<128, 128, 2, 2, true, 32>), grid, dim3(256), 0, 0, dx_in, K, dw, K, db, dy, N, M, N, K, 0); };
    const float ms0 = time_ms(f0);
    printf("fwd 128x128x32 no tanh: %8.2f us  %6.1f TFLOP/s\n", ms0 * 1e3, flops / (ms0 * 1e-3) / 1e12);
    float *xb, *wb;
    const int K4 = 1024, M4 = M / 4;
    CK(hipMalloc(&xb, (size_t)M4 * K4 * 4)); CK(hipMalloc(&wb, (size_t)N * K4 * 4));
    CK(hipMemset(xb, 0, (size_t)M4 * K4 * 4)); CK(hipMemset(wb, 0, (size_t)N * K4 * 4));
    dim3 g4(N / 128, M4 / 128);
    auto f4 = [&] { hipLaunchKernelGGL((mlp_fwd_kernel<128, 128, 2, 2, true, 32>), g4, dim3(256), 0, 0, xb, K4, wb, K4, db, dy, N, M4, N, K4, 1); };
    const float ms4 = time_ms(f4);
    printf("fwd 128x128x32 M=%d K=%d: %8.2f us  %6.1f TFLOP/s (zero operands)\n", M4, K4, ms4 * 1e3, 2.0 * M4 * N * K4 / (ms4 * 1e-3) / 1e12);
    CK(hipFree(xb)); CK(hipFree(wb));
  }
  FWD(128, 128, 2, 2, 64)
  FWD(128, 128, 2, 2, 16)
  FWD(128, 256, 2, 2, 32)
  FWD(128, 256, 2, 2, 16)
  FWD(256, 128, 2, 2, 16)
  FWD(256, 256, 2, 2, 16)
  FWD(128, 256, 1, 4, 16)
  BWD(128, 128, 2, 2, 32)
  BWD(128, 128, 2, 2, 16)
  BWD(128, 256, 2, 2, 32)
  BWD(128, 256, 2, 2, 16)
  BWD(256, 256, 2, 2, 16)
  return 0;
}
