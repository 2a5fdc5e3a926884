// development probe: where does global_load_lds_dwordx4 with an instruction
// offset put its data?  (does `offset:N` advance the LDS destination as well
// as the global source?)  One wave DMAs 1 KiB from src + lane*16 + N into LDS
// at M0 = 4096; the kernel dumps the whole 8 KiB LDS window.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int OFF>
__global__ void k(const unsigned* src, unsigned* out) {
  __shared__ unsigned lds[2048];
  for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = 0xdeadbeefu;
  __syncthreads();
  const unsigned char* g = (const unsigned char*)src + threadIdx.x * 16;
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)((__attribute__((address_space(3))) unsigned*)lds) + 4096u);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off offset:%2\n\ts_waitcnt vmcnt(0)"
               :
               : "v"(g), "s"(m0), "i"(OFF)
               : "memory", "m0");
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 64) out[i] = lds[i];
}
int main() {
  unsigned *src, *out;
  if (hipMalloc(&src, 16384) != hipSuccess || hipMalloc(&out, 8192) != hipSuccess) return 1;
  unsigned h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = i;  // word index = byte offset / 4
  if (hipMemcpy(src, h, 16384, hipMemcpyHostToDevice) != hipSuccess) return 1;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, src, out);
    else hipLaunchKernelGGL(k<1024>, dim3(1), dim3(64), 0, 0, src, out);
    unsigned o[2048];
    if (hipMemcpy(o, out, 8192, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int first = -1, last = -1;
    for (int i = 0; i < 2048; ++i)
      if (o[i] != 0xdeadbeefu) { if (first < 0) first = i; last = i; }
    printf("offset %d: LDS bytes written [%d, %d], first value = src word %u (byte %u), last = src word %u\n",
           pass ? 1024 : 0, first * 4, last * 4 + 3, first >= 0 ? o[first] : 0, first >= 0 ? o[first] * 4 : 0,
           last >= 0 ? o[last] : 0);
  }
  return 0;
}
