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

namespace mjl {
// the twin loss head with s_memtime stamps (block 7, thread 0) at its phase boundaries
template <int RB>
__global__ __launch_bounds__(2 * RB) void lh_stamped(unsigned long long* stamps, 
    const float* __restrict__ z, const float* __restrict__ log_std, const float* __restrict__ act,
    const float* __restrict__ old_logp, const float* __restrict__ adv, const float* __restrict__ ret, int n, int A,
    float clip_eps, float ent_coef, const float* __restrict__ adv_part, int nb_adv,
    const float* __restrict__ adv_stats, const int* __restrict__ stats_row, float ls_lo, float ls_hi,
    const float* __restrict__ bias, float* __restrict__ dz, float* __restrict__ lossp, float* __restrict__ glsp,
    float* __restrict__ biasp) {
  if (threadIdx.x == 0 && blockIdx.x == 7) stamps[0] = __builtin_amdgcn_s_memtime();
  // 2 RB threads: all of them stage the block's rows element-wise (and, bias given, form the means:
  // half the per-thread chain of tanh's a thread-per-row pass had); the row passes run on the first
  // RB (waves 0 .. NW - 1), thread t = row t
  constexpr int NW = RB / 64, TB = 2 * RB;
  __shared__ float sd[RB * kLossMaxA];  // a - mean of the block's rows (row-major), then dz[0]
  __shared__ float sm[RB * kLossMaxA];  // the mean
  __shared__ float sgv[RB];             // dz[1][:, 0]
  __shared__ float wred[NW][2 * kLossMaxA + 2];
  __shared__ float ivs[kLossMaxA], lsd[kLossMaxA], lss;
  __shared__ float mu_s, sd_s;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, r0 = blockIdx.x * RB, i = r0 + t;
  const int rows = min(RB, n - r0), cnt = rows * A;
  const size_t base = (size_t)r0 * A;
  const float* mean = z;
  const float* v = z + (size_t)n * A;
  const bool in = t < RB && t < rows;
  const float olp = in ? old_logp[i] : 0.f, adv_i = in ? adv[i] : 0.f;
  const float gv = in ? 2.f * (v[(size_t)i * A] + (bias ? bias[A] : 0.f) - ret[i]) / (float)n : 0.f;
  if (threadIdx.x == 0 && blockIdx.x == 7) stamps[1] = __builtin_amdgcn_s_memtime();
  {
    // element e = t + k TB: its column advances by TB mod A per trip (no divide per element)
    const int step = TB % A;
    int e = t, j = t % A;
    auto col_next = [&](int c) { c += step; return c >= A ? c - A : c; };
    constexpr int U = 4;
    for (; e + (U - 1) * TB < cnt; e += U * TB) {
      float a[U], m[U];
      int jj[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        a[u] = act[base + e + u * TB];
        m[u] = mean[base + e + u * TB];
        jj[u] = j;
        j = col_next(j);
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const float mu = bias ? tanhf(m[u] + bias[jj[u]]) : m[u];
        sm[e + u * TB] = mu;
        sd[e + u * TB] = a[u] - mu;
      }
    }
    for (; e < cnt; e += TB) {
      const float mu = bias ? tanhf(mean[base + e] + bias[j]) : mean[base + e];
      sm[e] = mu;
      sd[e] = act[base + e] - mu;
      j = col_next(j);
    }
  }
  if (t < RB) sgv[t] = gv;
  if (threadIdx.x == 0 && blockIdx.x == 7) stamps[2] = __builtin_amdgcn_s_memtime();
  if (t < A) {
    const float ls = fminf(fmaxf(log_std[t], ls_lo), ls_hi);  // networks.py:103's clip
    lsd[t] = ls;
    ivs[t] = expf(-2.f * ls);
  }
  if (w == (NW > 1 ? 1 : 0)) {  // the advantage statistics
    float mu, sdv;
    if (adv_stats) {
      const float* st = adv_stats + (stats_row ? 2 * (size_t)*stats_row : 0);
      mu = st[0]; sdv = st[1];
    }
    else adv_merge_wave(adv_part, nb_adv, lane, mu, sdv);
    if (lane == 0) { mu_s = mu; sd_s = sdv; }
  }
  __syncthreads();
  if (t == 0) {
    float s = 0.f;
    for (int j = 0; j < A; j++) s += 2.f * lsd[j] + kLog2Pi;
    lss = s;
  }
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 7) stamps[3] = __builtin_amdgcn_s_memtime();
  float* dr = sd + (in ? t : 0) * A;
  const float* mr = sm + (in ? t : 0) * A;
  float qs = 0.f;
  // the row waves only: a staging-only wave (w >= NW) is never `in`, so its qs would be discarded; the
  // guard only skips that benign read of row 0's sd (thread 0 may be writing it)
  if (w < NW)
    for (int j = 0; j < A; j++) qs += dr[j] * dr[j] * ivs[j];
  float surr = 0.f, dlogp = 0.f;
  if (threadIdx.x == 0 && blockIdx.x == 7) stamps[4] = __builtin_amdgcn_s_memtime();
  if (in) {
    const float logp = -0.5f * (qs + lss);
    const float ratio = expf(logp - olp);
    const float an = (adv_i - mu_s) / (sd_s + 1e-8f);
    const float lo = 1.f - clip_eps, hi = 1.f + clip_eps;
    const float rc = fminf(fmaxf(ratio, lo), hi);
    const float t1 = ratio * an, t2 = rc * an;
    surr = fminf(t1, t2);
    const float w1 = t1 < t2 ? 1.f : (t1 == t2 ? 0.5f : 0.f);
    const float w2 = t2 < t1 ? 1.f : (t1 == t2 ? 0.5f : 0.f);
    const float dratio = (-1.f / (float)n) * (w1 * an + ((ratio >= lo && ratio <= hi) ? w2 * an : 0.f));
    dlogp = dratio * ratio;
  }
  if (w < NW) {  // the row waves
  const float ssum = wave_sum_dpp(surr);
  if (lane == 0) wred[w][0] = ssum;
  for (int j = 0; j < A; j++) {
    const float d = dr[j], m = mr[j];
    const float c = wave_sum_dpp(in ? dlogp * (d * d * ivs[j] - 1.f) : 0.f);  // d logp / d s_j = q_j - 1
    const float g = in ? dlogp * d * ivs[j] * (1.f - m * m) : 0.f;          // d loss / d z_j
    const float cz = wave_sum_dpp(g);
    if (in) dr[j] = g;  // (row t's a - mean is read by thread t only)
    if (lane == 0) { wred[w][1 + j] = c; wred[w][1 + A + j] = cz; }
  }
  const float gsum = wave_sum_dpp(gv);
  if (lane == 0) wred[w][1 + 2 * A] = gsum;
  }
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 7) stamps[5] = __builtin_amdgcn_s_memtime();
  float* dz0 = dz + base;
  float* dz1 = dz + (size_t)n * A + base;
  {
    const int rstep = TB / A, cstep = TB % A;
    int r = t / A, c = t - (t / A) * A;
    for (int e = t; e < cnt; e += TB) {
      dz0[e] = sd[e];
      dz1[e] = c == 0 ? sgv[r] : 0.f;
      r += rstep;
      c += cstep;
      if (c >= A) { c -= A; r++; }
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 7) stamps[6] = __builtin_amdgcn_s_memtime();
  const int nb = gridDim.x, b = blockIdx.x;
  if (t <= 2 * A + 1) {
    float acc = wred[0][t];
#pragma unroll
    for (int k = 1; k < NW; k++) acc += wred[k][t];
    if (t == 0) {
      float val = -acc / (float)n;
      if (b == 0) val -= ent_coef * (0.5f * ((float)A + lss) / (float)A);  // entropy, train_ppo.py:215
      lossp[b] = val;
    } else if (t <= A) {
      const int j = t - 1;
      const float ls = log_std[j];
      const float val = b == 0 ? acc - ent_coef / (float)A : acc;
      glsp[(size_t)b * A + j] = (ls >= ls_lo && ls <= ls_hi) ? val : 0.f;
    } else if (t <= 2 * A) {
      biasp[(size_t)b * A + (t - 1 - A)] = acc;
    } else {
      biasp[((size_t)nb + b) * A] = acc;
    }
  }
  if (t >= 1 && t < A) biasp[((size_t)nb + b) * A + t] = 0.f;
  if (threadIdx.x == 0 && blockIdx.x == 7) stamps[7] = __builtin_amdgcn_s_memtime();
}

}  // namespace mjl



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
      unsigned long long* stp;
      (void)hipMalloc(&stp, 64);
      for (int rep = 0; rep < 3; rep++)
        hipLaunchKernelGGL(lh_stamped<64>, dim3(M / 64), dim3(128), 0, 0, stp, z, lstd, act, lp, av, rt, M, A, 0.2f,
                           0.01f, nullptr, 0, st, row, -20.f, 2.f, b0, dzl, lp2, glsp, biasp);
      (void)hipDeviceSynchronize();
      unsigned long long hs[8];
      (void)hipMemcpy(hs, stp, 64, hipMemcpyDeviceToHost);
      printf("   loss head block 7 phases (cycles): loads %llu | staging %llu | stats+lss %llu | qs %llu | column sums %llu | dz %llu | partials %llu\n",
             hs[1] - hs[0], hs[2] - hs[1], hs[3] - hs[2], hs[4] - hs[3], hs[5] - hs[4], hs[6] - hs[5], hs[7] - hs[6]);
    }
    const double in_bytes = 2.0 * M * N * 4 + 3.0 * M * K0 * 4, hb_bytes = 4.0 * M * N * 4;
    printf("M %6d  gather_in %7.2f us (%5.1f TFLOP/s, %5.2f TB/s)   head_bwd %7.2f us (%5.2f TB/s)\n", M, t_in * 1e3,
           2.0 * M * K0 * 2 * N / (t_in * 1e-3) / 1e12, in_bytes / (t_in * 1e-3) / 1e12, t_hb * 1e3,
           hb_bytes / (t_hb * 1e-3) / 1e12);
    (void)hipFree(idx);
  }
  return 0;
}
