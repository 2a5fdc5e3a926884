// Shared helpers for the libasr HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/asr.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

#define ASR_LDS __attribute__((address_space(3)))

namespace asr {

// thread-local error message (asr_last_error)
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

inline int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(ASR_E_HIP, "%s: %s", what, hipGetErrorString(e));
  return ASR_OK;
}

#define ASR_TRY(expr)            \
  do {                           \
    int _rc = (expr);            \
    if (_rc != ASR_OK) return _rc; \
  } while (0)

#define ASR_LAUNCH_CHECK(name) ASR_TRY(::asr::hip_check(hipGetLastError(), name))

int cu_count();

// A network / stage workspace must live on the current device: its layout (the
// weight-gradient slab rows, hence every offset after them) follows the CU
// count of the device current when it was sized, and the kernels size their
// grids by the device current at launch.  ASR_E_WORKSPACE, before any launch,
// when ws is not device memory of the current device.
int check_ws_device(const void* ws, const char* who);

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// One launch of the balanced bf16 weight pack for several layer sets (the
// multi-stage net's stages, asr_stages.hip): one workgroup per layer, so the
// stages' packs run side by side (asr_theta.hip, k_theta_to_w_pack_bal).
struct PackJob {
  const float* theta;
  long theta_stride;
  int L, C;
  const int32_t* w_src;
  float gamma;
  void* w;
  long w_stride;
  // asr_param_map's theta_dst of a map known to pair its entries (3by3, general): theta read
  // coalesced and no pairing check; nullptr: the entries gathered through w_src and checked
  const int32_t* theta_dst;
  long n_theta;
};
constexpr int kMaxPackJobs = 16;
int theta_to_w_bf16_jobs(const PackJob* jobs, int njobs, hipStream_t s);

// Slab layout of the pair-local C=64 stacked backward (k_bwd3_stack<..., PAIR>,
// asr_block_mfma.hip): for an antisymmetric operator every theta pulls back
// D(t,i,o) = dW[t][i][o] - dW[8-t][o][i] (tap t = 3ky+kx), and the slab holds
// 74 16x16 fp32 tiles of D, element (r, c) of tile T at T*256 + ((r/4)*16 + c)*4 + r%4:
//   T = 16p + 4a + b (p < 4):  D(p, 16a + r, 16b + c)
//   T = 64 + k (tap-4 cross pairs (a', b') = kPairTap4A/B[k]):  D(4, 16a' + r, 16b' + c)
//   T = 70 + c (tap-4 self tiles): X = dW[4] tile (c, c), raw for even c, transposed for odd c
// then db [64].  pair_encode turns one entry (e = (t*C + i)*C + o, neg) of a theta's
// (e, mirror(e)) pair into 1 or 2 (slab index << 1 | neg) entries.
struct PairSlabLayout {
  static constexpr int kTap4 = 64, kSelf = 70, kTiles = 74, E = kTiles * 256, ES = E + 64;
};
__host__ __device__ inline int pair_slab_index(int T, int r, int c) { return T * 256 + ((r >> 2) * 16 + c) * 4 + (r & 3); }
// tap-4 cross pairs (a', b'), k = 3h + p for the waves (p < 3, h) of k_bwd3_stack<PAIR>
__host__ __device__ inline int pair_tap4_a(int k) { return k < 3 ? (k == 0 ? 1 : k == 1 ? 2 : 3) : (k == 3 ? 3 : k == 4 ? 1 : 0); }
__host__ __device__ inline int pair_tap4_b(int k) { return k < 3 ? (k == 2 ? 1 : 0) : (k == 5 ? 3 : 2); }
__host__ __device__ inline int pair_encode(long e, int neg, int C, int32_t* out) {
  const int t = (int)(e / ((long)C * C)), i = (int)((e / C) % C), o = (int)(e % C);
  if (t < 4) {
    out[0] = (pair_slab_index(t * 16 + (i >> 4) * 4 + (o >> 4), i & 15, o & 15) << 1) | neg;
    return 1;
  }
  if (t > 4) {  // D(t, i, o) = -D(8-t, o, i)
    out[0] = (pair_slab_index((8 - t) * 16 + (o >> 4) * 4 + (i >> 4), o & 15, i & 15) << 1) | (neg ^ 1);
    return 1;
  }
  const int a = i >> 4, b = o >> 4;
  if (a != b) {
    for (int k = 0; k < 6; ++k) {
      if (pair_tap4_a(k) == a && pair_tap4_b(k) == b) {
        out[0] = (pair_slab_index(PairSlabLayout::kTap4 + k, i & 15, o & 15) << 1) | neg;
        return 1;
      }
      if (pair_tap4_a(k) == b && pair_tap4_b(k) == a) {  // D(4, i, o) = -D(4, o, i)
        out[0] = (pair_slab_index(PairSlabLayout::kTap4 + k, o & 15, i & 15) << 1) | (neg ^ 1);
        return 1;
      }
    }
    return 0;
  }
  // self tile: D = X[i][o] - X[o][i]; stored raw (a even) or transposed (a odd)
  const int T = PairSlabLayout::kSelf + a, ri = i & 15, ro = o & 15;
  const bool tr = (a & 1) != 0;
  out[0] = (pair_slab_index(T, tr ? ro : ri, tr ? ri : ro) << 1) | neg;
  out[1] = (pair_slab_index(T, tr ? ri : ro, tr ? ro : ri) << 1) | (neg ^ 1);
  return 2;
}

// ---- device helpers --------------------------------------------------------

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }
template <typename T>
__device__ __forceinline__ T from_f32(float v);
template <>
__device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// two fp32 -> packed bf16 pair, round to nearest even (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned pk_bf16_rn(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t v = {(bf16)a, (bf16)b};
  return __builtin_bit_cast(unsigned, v);
}

// The wait states of a v_mfma_f32_16x16x4_f32 result (10 on gfx950), spent on
// the straight line right after the MFMA chain, before the epilogue's first
// branch.  hipcc (ROCm 7.2) pads a join block for its longer predecessor
// only: where an epilogue branch skips a few instructions, the join read the
// accumulator 2 states early (k_conv32 forward) or 5-7 early (a
// persistent-band k_conv32).  sched_barrier keeps the nops
// between the chain and the code after it; tests/test_isa.py
// (tools/asm_mfma_audit.py) checks every path of the compiled kernels.
__device__ __forceinline__ void mfma_f32_settle() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 9");
  __builtin_amdgcn_sched_barrier(0);
}

// the same for a v_mfma_f32_16x16x32_bf16 result (8 wait states)
__device__ __forceinline__ void mfma_bf16_settle() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7");
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace asr
