// development probe: does v_mfma_f32_16x16x32_bf16 keep fp32 denormal results?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out, float s) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(i == 0 ? s : 0.f); b[i] = (__bf16)(i == 0 ? s : 0.f); }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  out[threadIdx.x] = c[0];
}
int main() {
  float* d;
  if (hipMalloc(&d, 64 * 4) != hipSuccess) return 1;
  const float ss[] = {0x1p-70f, 0x1p-64f, 0x1p-63f, 0x1p-75f};
  for (float s : ss) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, s);
    float h[64]; if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    unsigned bits; memcpy(&bits, &h[0], 4);
    printf("s=%a  s*s=%a  mfma lane0=%a bits=0x%08x\n", s, (double)s * s, h[0], bits);
  }
  return 0;
}
