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
// the fused head with s_memtime stamps (workgroup 6, thread 0), cycles accumulated per phase
template <int A, int K, int R>
__global__ __launch_bounds__(256, 64 / R) void th_stamped(TwinHeadArgs p, unsigned long long* stamps) {
  unsigned long long tq = __builtin_amdgcn_s_memtime();
  auto STMP = [&](int i) { if (threadIdx.x == 0 && blockIdx.x == 6) { const unsigned long long x = __builtin_amdgcn_s_memtime(); stamps[i] += x - tq; tq = x; } };
  static_assert(A <= 31 && K % 64 == 0 && K == 4 * 64, "tile shape: 4 waves x 2 column tiles of 32");
  static_assert(R == 32 || R == 64, "32 or 64 rows per chunk");
  constexpr int HS = kThHS, ZS = kThZS, NRT = R / 32, LPR = 256 / R;  // row tiles; lanes per loss row
  __shared__ __attribute__((aligned(16))) float hs[R * HS];  // H of the chunk
  __shared__ __attribute__((aligned(16))) float ws[A * HS];   // W_out rows (rows A..31 read as zero)
  constexpr int KP = 4 / NRT;                                 // K parts of z: every wave takes one (part, row tile)
  __shared__ float red[4 * 16 * 64];                          // z partials per wave; at the end, the csh sums
  __shared__ float sz[R * ZS];                                // z, then d, then dz (cols A..31 zero)
  __shared__ float sx[R * 32];                                // act, then the mean, then c_j
  __shared__ float srow[4][R];                                // old_logp, adv, ret, surr
  __shared__ float ivs[32];
  __shared__ float lss_s, mu_s, sd_s;
  __shared__ float acc_col[2 * 32 + 1];                       // c_j, dz column sums, loss: chunk order
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, li = lane & 31, kh = lane >> 5;
  const int net = blockIdx.x & 1, S = (int)(gridDim.x >> 1), blk = (int)(blockIdx.x >> 1), n = p.n;
  const int nchunk = (n + R - 1) / R;
  // ---- once per workgroup: W_out of this net, the log_std terms, the advantage statistics
  // (by LDS-DMA, global_load_lds_dwordx4: one 1-KB row per wave-instruction, no VGPRs, so the first
  // chunk's loads issue behind it; the chunk's first barrier retires it)
  static_assert(K == 64 * 4, "one W_out row per wave-instruction");
  for (int a = w; a < A; a += 4)
    __builtin_amdgcn_global_load_lds((const void*)(p.W + ((size_t)net * A + a) * K + 4 * lane),
                                     (__attribute__((address_space(3))) void*)&ws[a * HS], 16, 0, 0);
  if (w == 0) {
    const float ls = lane < A ? fminf(fmaxf(p.log_std[lane], p.ls_lo), p.ls_hi) : 0.f;  // networks.py:103
    if (lane < 32) ivs[lane] = lane < A ? expf(-2.f * ls) : 0.f;
    const float tot = wave_sum_dpp(lane < A ? 2.f * ls + kLog2Pi : 0.f);
    float mu, sdv;
    if (p.adv_stats) {
      const float* st = p.adv_stats + (p.stats_row ? 2 * (size_t)*p.stats_row : 0);
      mu = st[0];
      sdv = st[1];
    } else {
      adv_merge_wave(p.adv_part, p.nb_adv, lane, mu, sdv);
    }
    if (lane == 0) {
      lss_s = tot;
      mu_s = mu;
      sd_s = sdv;
    }
  }
  if (t < 2 * 32 + 1) acc_col[t] = 0.f;
  tw_f32x16 gwacc[2];
  float csacc[2] = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 2; c++)
#pragma unroll
    for (int v = 0; v < 16; v++) gwacc[c][v] = 0.f;
  const float4 bq = *reinterpret_cast<const float4*>(p.bh + (size_t)net * K + 4 * (t & (K / 4 - 1)));
  const float nf = (float)n;
  STMP(0);
  for (int ch = blk; ch < nchunk; ch += S) {
    const int r0 = ch * R, rows = min(R, n - r0);
    // ---- loads: the chunk's pre-activations, actions and per-row scalars, all issued together
    constexpr int QZ = R * K / 4 / 256;  // float4 of zh per thread (16)
    float4 zv[QZ];
#pragma unroll
    for (int i = 0; i < QZ; i++) {
      const int q = t + 256 * i, r = q / (K / 4), c4 = q - r * (K / 4);
      zv[i] = r < rows ? *reinterpret_cast<const float4*>(p.zh + ((size_t)net * n + r0 + r) * K + 4 * c4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    constexpr int QA = (R * 32 + 255) / 256;
    float av[QA];
    if (net == 0) {
#pragma unroll
      for (int i = 0; i < QA; i++) {
        const int e = t + 256 * i;
        av[i] = e < rows * A ? p.act[(size_t)r0 * A + e] : 0.f;
      }
    }
    float rv0 = 0.f, rv1 = 0.f, rv2 = 0.f;
    if (t < rows) {
      rv0 = p.old_logp[r0 + t];
      rv1 = p.adv[r0 + t];
      rv2 = p.ret[r0 + t];
    }
    __syncthreads();  // (the previous chunk's reads of hs / sz / sx are done)
#pragma unroll
    for (int i = 0; i < QZ; i++) {
      const int q = t + 256 * i, r = q / (K / 4), c4 = q - r * (K / 4);
      float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < rows)
        h = make_float4(tw_tanh(zv[i].x + bq.x), tw_tanh(zv[i].y + bq.y), tw_tanh(zv[i].z + bq.z),
                        tw_tanh(zv[i].w + bq.w));
      *reinterpret_cast<float4*>(&hs[r * HS + 4 * c4]) = h;
    }
    if (net == 0) {
#pragma unroll
      for (int i = 0; i < QA; i++) {
        const int e = t + 256 * i;
        if (e < rows * A) sx[(e / A) * 32 + e % A] = av[i];
      }
    }
    if (t < R) {
      srow[0][t] = rv0;
      srow[1][t] = rv1;
      srow[2][t] = rv2;
    }
    __syncthreads();
  STMP(1);
    // ---- z = H W^T: wave w takes row tile w % NRT and K part w / NRT (of KP)
    {
      const int rt = w % NRT, k0 = (w / NRT) * (K / KP);
      tw_f32x16 acc;
#pragma unroll
      for (int v = 0; v < 16; v++) acc[v] = 0.f;
      const float* ha = &hs[(32 * rt + li) * HS + k0 + kh];
      const float* wb = &ws[(li < A ? li : 0) * HS + k0 + kh];
      const bool wr = li < A;  // W_out rows A..31: zero
#pragma unroll 8
      for (int s = 0; s < K / (2 * KP); s++)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ha[2 * s], wr ? wb[2 * s] : 0.f, acc, 0, 0, 0);
#pragma unroll
      for (int v = 0; v < 16; v++) red[(w * 16 + v) * 64 + lane] = acc[v];
    }
    __syncthreads();
  STMP(2);
    // z[row][a] = the K parts in order (pairwise for 4) + bo (C[i][j] in register (i & 3) + 4 (i >> 3) of
    // lane j + 32 ((i >> 2) & 1))
    for (int e = t; e < R * 32; e += 256) {
      const int row = e >> 5, a = e & 31, rt = row >> 5, i = row & 31;
      const int v = (i & 3) + 4 * (i >> 3), L = a + 32 * ((i >> 2) & 1);
      auto part = [&](int k) { return red[((k * NRT + rt) * 16 + v) * 64 + L]; };
      const float zz = KP == 2 ? part(0) + part(1) : (part(0) + part(1)) + (part(2) + part(3));
      sz[row * ZS + a] = a < A ? zz + p.bo[net * A + a] : 0.f;
    }
    __syncthreads();
  STMP(3);
    // ---- per row: the losses and dz, LPR lanes per row (lane q of the row's group takes columns q,
    // q + LPR, ...; the row's log-density sum over the group by DPP, the same total in all its lanes)
    {
      const int r = t / LPR, q = t % LPR;
      float* zr = &sz[r * ZS];
      float* xr = &sx[r * 32];
      float surr = 0.f;
      if (r < rows) {
        if (net == 0) {
          float qs = 0.f;
          for (int j = q; j < A; j += LPR) {
            const float m = tanhf(zr[j]), d = xr[j] - m;
            zr[j] = d;
            xr[j] = m;
            qs += d * d * ivs[j];
          }
          qs += dpp_f<0xb1>(qs);                // quad_perm [1, 0, 3, 2]
          qs += dpp_f<0x4e>(qs);                // quad_perm [2, 3, 0, 1]
          if constexpr (LPR == 8) qs += dpp_f<0x141>(qs);  // row_half_mirror: the other quad of the 8
          const float logp = -0.5f * (qs + lss_s);
          const float ratio = expf(logp - srow[0][r]);
          const float an = (srow[1][r] - mu_s) / (sd_s + 1e-8f);
          const float lo = 1.f - p.clip_eps, hi = 1.f + p.clip_eps;
          const float rc = fminf(fmaxf(ratio, lo), hi);
          const float t1 = ratio * an, t2 = rc * an;
          surr = fminf(t1, t2);
          const float w1 = t1 < t2 ? 1.f : (t1 == t2 ? 0.5f : 0.f);
          const float w2 = t2 < t1 ? 1.f : (t1 == t2 ? 0.5f : 0.f);
          const float dratio = (-1.f / nf) * (w1 * an + ((ratio >= lo && ratio <= hi) ? w2 * an : 0.f));
          const float dlogp = dratio * ratio;
          for (int j = q; j < A; j += LPR) {
            const float d = zr[j], m = xr[j], iv = ivs[j];
            xr[j] = dlogp * (d * d * iv - 1.f);    // d logp / d s_j = q_j - 1
            zr[j] = dlogp * d * iv * (1.f - m * m);  // d loss / d z_j
          }
        } else {
          if (q == 0) zr[0] = 2.f * (zr[0] - srow[2][r]) / nf;  // value: d loss / d v (train_ppo.py:218-220)
          for (int j = (q == 0 ? LPR : q); j < A; j += LPR) zr[j] = 0.f;
        }
      } else {
        for (int j = q; j < 32; j += LPR) {
          zr[j] = 0.f;
          xr[j] = 0.f;
        }
      }
      if (q == 0) srow[3][r] = surr;
    }
    __syncthreads();
  STMP(4);
    // ---- the chunk's column sums into the workgroup's accumulators (rows in order, chunks in order)
    if (t < 2 * 32 + 1) {
      const bool pol = net == 0;
      const float* col = t == 2 * 32 ? srow[3] : t < 32 ? &sx[t] : &sz[t - 32];
      const int cstr = t == 2 * 32 ? 1 : (t < 32 ? 32 : ZS);
      const bool on = t == 2 * 32 ? pol : (t < 32 ? (pol && t < A) : (t - 32 < A));
      if (on) {
        float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
        for (int r = 0; r < R; r += 4) {
          p0 += col[r * cstr]; p1 += col[(r + 1) * cstr]; p2 += col[(r + 2) * cstr]; p3 += col[(r + 3) * cstr];
        }
        acc_col[t] += (p0 + p1) + (p2 + p3);
      }
    }
  STMP(5);
    // ---- dH = dz W, dZ = dH (1 - H^2): wave w takes column tiles 2w, 2w + 1 over both row tiles
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int ct = 2 * w + c, col = 32 * ct + li;
#pragma unroll
      for (int rt = 0; rt < NRT; rt++) {
        tw_f32x16 acc;
#pragma unroll
        for (int v = 0; v < 16; v++) acc[v] = 0.f;
#pragma unroll
        for (int s = 0; s < (A + 1) / 2; s++) {
          const int a = 2 * s + kh;  // W_out row a < A (row A of an odd A: zero)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sz[(32 * rt + li) * ZS + a], a < A ? ws[a * HS + col] : 0.f,
                                                     acc, 0, 0, 0);
        }
        float* out = p.dzh + ((size_t)net * n + r0) * K + col;
#pragma unroll
        for (int v = 0; v < 16; v++) {
          const int row = 32 * rt + (v & 3) + 8 * (v >> 2) + 4 * kh;
          const float y = hs[row * HS + col];
          const float dzv = acc[v] * (1.f - y * y);
          if (row < rows) out[(size_t)row * K] = dzv;
          csacc[c] += dzv;
        }
      }
    }
  STMP(6);
    // ---- the output weight gradient dz^T H, accumulated over the chunks: column tiles 2w, 2w + 1
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int col = 32 * (2 * w + c) + li;
#pragma unroll 8
      for (int s = 0; s < R / 2; s++)
        gwacc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(sz[(2 * s + kh) * ZS + li], hs[(2 * s + kh) * HS + col],
                                                        gwacc[c], 0, 0, 0);
    }
  STMP(7);
  }
  float (*csh)[K] = reinterpret_cast<float (*)[K]>(red);  // red is free after the last chunk's z sums
  // ---- the workgroup's partials
  const int nb = S;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const int col = 32 * (2 * w + c) + li;
#pragma unroll
    for (int v = 0; v < 16; v++) {
      const int a = (v & 3) + 8 * (v >> 2) + 4 * kh;
      if (a < A) p.gw[(((size_t)net * nb + blk) * A + a) * K + col] = gwacc[c][v];
    }
    csh[kh][col] = csacc[c];
  }
  __syncthreads();
  if (t < K) p.cs[((size_t)net * nb + blk) * K + t] = csh[0][t] + csh[1][t];
  STMP(8);
  if (net == 0) {
    if (t == 0) {
      float val = -acc_col[2 * 32] / nf;
      if (blk == 0) val -= p.ent_coef * (0.5f * ((float)A + lss_s) / (float)A);  // entropy, train_ppo.py:215
      p.lossp[blk] = val;
    }
    if (t < A) {
      const float ls = p.log_std[t];
      const float val = blk == 0 ? acc_col[t] - p.ent_coef / (float)A : acc_col[t];
      p.glsp[(size_t)blk * A + t] = (ls >= p.ls_lo && ls <= p.ls_hi) ? val : 0.f;
      p.biasp[(size_t)blk * A + t] = acc_col[32 + t];
    }
  } else if (t < A) {
    p.biasp[((size_t)nb + blk) * A + t] = t == 0 ? acc_col[32] : 0.f;
  }
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
    }
    for (int R : {32, 64}) {  // the fused head (mjl_twin_head's kernel), statistics from a table row
      float *zh = dev_rand(2ull * M * N, 14, 1.f), *lstd = dev_rand(A, 12, 0.3f), *st = dev_rand(2, 13, 1.f);
      float *dzh2, *cs2, *gw2, *lossp2, *glsp2, *biasp2;
      int* row;
      const int cap = (R == 32 ? 512 : 256) / 2;
      const int S = (M / R) < cap ? (M / R) : cap;
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
        if (R == 32) hipLaunchKernelGGL((twin_head_kernel<kThA, kThK, 32>), dim3(2 * S), dim3(256), 0, 0, ha);
        else hipLaunchKernelGGL((twin_head_kernel<kThA, kThK, 64>), dim3(2 * S), dim3(256), 0, 0, ha);
      }, reps);
      printf("M %6d  twin_head R %d (fused forward + losses + backward)  %7.2f us\n", M, R, th * 1e3);
      unsigned long long* stp;
      (void)hipMalloc(&stp, 16 * 8);
      (void)hipMemset(stp, 0, 16 * 8);
      if (R == 32) hipLaunchKernelGGL((th_stamped<kThA, kThK, 32>), dim3(2 * S), dim3(256), 0, 0, ha, stp);
      else hipLaunchKernelGGL((th_stamped<kThA, kThK, 64>), dim3(2 * S), dim3(256), 0, 0, ha, stp);
      unsigned long long hs[16];
      (void)hipMemcpy(hs, stp, 16 * 8, hipMemcpyDeviceToHost);
      printf("   head workgroup 6 cycles: setup %llu | loads+H %llu | z MFMA %llu | z sum %llu | losses %llu | col sums %llu | dH %llu | dW %llu | partials %llu\n",
             hs[0], hs[1], hs[2], hs[3], hs[4], hs[5], hs[6], hs[7], hs[8]);
    }
    const double in_bytes = 2.0 * M * N * 4 + 3.0 * M * K0 * 4, hb_bytes = 4.0 * M * N * 4;
    printf("M %6d  gather_in %7.2f us (%5.1f TFLOP/s, %5.2f TB/s)   head_bwd %7.2f us (%5.2f TB/s)\n", M, t_in * 1e3,
           2.0 * M * K0 * 2 * N / (t_in * 1e-3) / 1e12, in_bytes / (t_in * 1e-3) / 1e12, t_hb * 1e3,
           hb_bytes / (t_hb * 1e-3) / 1e12);
    (void)hipFree(idx);
  }
  return 0;
}
