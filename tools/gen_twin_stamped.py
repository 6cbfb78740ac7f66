"""Writes the stamped copy of csrc/twin_kernels.hip's fused head (th_stamped: s_memtime stamps per phase,
workgroup 6, thread 0) into tools/twin_micro.hip between its markers."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "mujoco-mjx-lab_amd/csrc/twin_kernels.hip")).read()
a = src.index("template <int A, int K, int R>\n__global__ __launch_bounds__(256, 64 / R) void twin_head_kernel(TwinHeadArgs p) {")
b = src.index("}  // namespace mjl", a)
k = src[a:b]
k = k.replace("void twin_head_kernel(TwinHeadArgs p) {", "void th_stamped(TwinHeadArgs p, unsigned long long* stamps) {\n"
              "  unsigned long long tq = __builtin_amdgcn_s_memtime();\n"
              "  auto STMP = [&](int i) { if (threadIdx.x == 0 && blockIdx.x == 6) { const unsigned long long x = "
              "__builtin_amdgcn_s_memtime(); stamps[i] += x - tq; tq = x; } };", 1)


def ins(after, i):
    global k
    idx = k.index(after) + len(after)
    k = k[:idx] + f"\n  STMP({i});" + k[idx:]


ins("  const float nf = (float)n;", 0)
ins("      srow[2][t] = rv2;\n    }\n    __syncthreads();", 1)
ins("      for (int v = 0; v < 16; v++) red[(w * 16 + v) * 64 + lane] = acc[v];\n    }\n    __syncthreads();", 2)
ins("      sz[row * ZS + a] = a < A ? zz + p.bo[net * A + a] : 0.f;\n    }\n    __syncthreads();", 3)
ins("      if (q == 0) srow[3][r] = surr;\n    }\n    __syncthreads();", 4)
ins("        acc_col[t] += (p0 + p1) + (p2 + p3);\n      }\n    }", 5)
ins("          csacc[c] += dzv;\n        }\n      }\n    }", 6)
ins("                                                        gwacc[c], 0, 0, 0);\n    }", 7)
k = k.replace("  if (t < K) p.cs[((size_t)net * nb + blk) * K + t] = csh[0][t] + csh[1][t];",
              "  if (t < K) p.cs[((size_t)net * nb + blk) * K + t] = csh[0][t] + csh[1][t];\n  STMP(8);")
p = os.path.join(ROOT, "tools/twin_micro.hip")
s = open(p).read()
a = s.index("template <int A, int K, int R>\n__global__ __launch_bounds__(256, 64 / R) void th_stamped")
b = s.index("}  // namespace mjl", a)
open(p, "w").write(s[:a] + k + s[b:])
