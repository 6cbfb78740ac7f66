// Prints v_mfma_f32_4x4x1_16b_f32's operand / result layout and the CBSZ/ABID A broadcast on the
// GPU: a = lane (A values), b = 1000 * lane (B values); with one nonzero per operand the product
// names the lanes that fed each output register.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void probe(float* out, int mode) {
  const int lane = threadIdx.x;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  // mode 0: only lane 5 has a (=1), all b = lane + 1 -> which outputs see a from lane 5
  // mode 1: a = 1 everywhere, only lane 9 has b (=1)
  // mode 2: broadcast cbsz 4 abid 3: a = lane + 1 everywhere, b = 1 -> which lane's a reached each block
  if (mode == 0) c = __builtin_amdgcn_mfma_f32_4x4x1f32(lane == 5 ? 1.f : 0.f, (float)(lane + 1), c, 0, 0, 0);
  if (mode == 1) c = __builtin_amdgcn_mfma_f32_4x4x1f32(1.f, lane == 9 ? 1.f : 0.f, c, 0, 0, 0);
  if (mode == 2) c = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(lane + 1), 1.f, c, 4, 3, 0);
  for (int r = 0; r < 4; r++) out[lane * 4 + r] = c[r];
}
int main() {
  float* d;
  hipMalloc(&d, 256 * 4);
  float h[256];
  for (int mode = 0; mode < 3; mode++) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
    printf("mode %d:", mode);
    for (int l = 0; l < 64; l++)
      for (int r = 0; r < 4; r++)
        if (h[l * 4 + r] != 0.f && (mode != 2 || l < 12)) printf(" L%d.r%d=%g", l, r, h[l * 4 + r]);
    printf("\n");
  }
  return 0;
}
